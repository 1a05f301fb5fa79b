/*
 * dtmpc.h — C ABI of the MI355X-native batched differentiable tube-MPC hot path.
 *
 * The reference (lmcggg/differentiable-tube-mpc) has no FFI: its solver boundary is a
 * Python-closure boundary (core/ddp.py:102-117, core/ddp.py:317-329) fed by closures built in
 * core/tube_mpc.py:814-957.  This header replaces those closures with a TYPED problem
 * specification (Dubins + DBaS barrier state + circle obstacles + diagonal quadratic costs + box
 * controls) that the HIP kernels in libdtmpc.so consume for a whole batch of independent
 * trajectories at once.  Every entry point below names the reference function it replaces.
 *
 * Conventions (all entry points):
 *   - dtype: DTMPC_F32 or DTMPC_F64; every `void*` array argument holds that scalar type.
 *   - Batched arrays are SoA "step-major, trajectory-minor": element (k, f, i) of an array with
 *     F fields per step lives at index (k*F + f)*B + i.  Trajectory i of the batch is one
 *     independent copy of the reference's single-trajectory problem.
 *   - All array pointers are DEVICE pointers owned by the caller; nothing is allocated inside
 *     (scratch comes from caller-provided workspaces sized by the *_workspace_bytes queries).
 *   - Launches are asynchronous on the given hipStream_t (`stream`, NULL = default stream);
 *     entry points are re-entrant across streams.
 *   - Return value: DTMPC_OK or DTMPC_ERR_BAD_ARG / DTMPC_ERR_HIP for launch-time failures.
 *     Numerical failures are reported per trajectory through `status` words (bit flags
 *     DTMPC_ST_*), which the host maps to the reference's exceptions (FloatingPointError for
 *     non-finite values, core/ddp.py:138-159; RuntimeError when line search yields nothing,
 *     core/ddp.py:298-299).
 */
#ifndef DTMPC_H
#define DTMPC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DTMPC_ABI_VERSION 7
#define DTMPC_MAX_OBS 16
#define DTMPC_MAX_ALPHAS 8
#define DTMPC_MAX_HORIZON 512
#define DTMPC_LOG_FIELDS 18 /* rows of dtmpc_tube_state.log */
#define DTMPC_GEN_LOG_FIELDS 12 /* rows of dtmpc_general_state.log */
#define DTMPC_GEN_SUMS 25 /* L, ancillary raw-theta grads (11), nominal raw-theta-bar grads (12),
                             healthy-trajectory count */
#define DTMPC_TUBE_SUMS 8 /* L, gQ(3), gR(2), gqb, healthy-trajectory count */

/* scalar type of the arrays */
enum { DTMPC_F32 = 0, DTMPC_F64 = 1 };

/* obstacle aggregation for the safety function h (core/systems/dubins_aug_jac.py:96-112) */
enum {
  DTMPC_OBS_SMOOTHMIN = 0, /* h = -(1/beta) LSE(-beta h_i), dubins_obstacles.py:41-92 */
  DTMPC_OBS_MIN = 1,       /* h = min_i h_i, argmin subgradient, dubins_obstacles.py:95-117 */
  DTMPC_OBS_SINGLE = 2,    /* one circle (obstacle 0), dubins_obstacles.py:16-38 */
  DTMPC_OBS_NONE = 3       /* h = 1 (run_nominal.py:256) */
};

/* barrier used in the DBaS dynamics b' = B(h(f(x,u))) - gamma (B(h(x)) - b)  (core/barrier.py:75-108).
 * The linearisation always differentiates the relaxed inverse barrier, exactly as the
 * reference does (core/systems/dubins_aug_jac.py:116-122). */
enum { DTMPC_BARRIER_INVERSE = 0, DTMPC_BARRIER_LOG = 1 };

/* stage/terminal cost family */
enum {
  DTMPC_COST_TARGET = 0, /* nominal: sum Q (x-x*)^2 + R u^2 + qb b^2 (core/tube_mpc.py:823-842) */
  DTMPC_COST_TRACK = 1   /* ancillary: sum Q (x-xref_k)^2 + R (u-uref_k)^2 + qb b^2 (core/tube_mpc.py:875-894) */
};

/* return codes */
enum {
  DTMPC_OK = 0,
  DTMPC_ERR_BAD_ARG = 3,
  DTMPC_ERR_HIP = 4
};

/* per-trajectory status bits */
enum {
  DTMPC_ST_NONFINITE = 1,    /* FloatingPointError in the reference */
  DTMPC_ST_NO_CANDIDATE = 2  /* RuntimeError("iLQR line search failed ...") */
};

/* Problem specification: system + environment + DBaS (core/tube_mpc.py:680-721). */
typedef struct dtmpc_spec {
  int32_t horizon;          /* N (configs/dubins.yaml:13) */
  int32_t n_obstacles;      /* M <= DTMPC_MAX_OBS */
  int32_t obs_aggregation;  /* DTMPC_OBS_* */
  int32_t barrier_type;     /* DTMPC_BARRIER_* */
  double dt;                /* DubinsConfig.dt (core/systems/dubins.py:14) */
  double u_min[2];          /* BoxClampControl.u_min (core/control.py:56) */
  double u_max[2];
  double active_tol;        /* BoxClampControl.active_tol = 1e-8 (core/control.py:59) */
  double obs_beta;          /* smooth-min temperature (configs/dubins.yaml:59) */
  double obs_cx[DTMPC_MAX_OBS];
  double obs_cy[DTMPC_MAX_OBS];
  double obs_r[DTMPC_MAX_OBS];
  double dbas_alpha;        /* DBaSConfig.alpha (core/barrier.py:29) */
  double dbas_gamma;        /* DBaSConfig.gamma, in [-1, 1] */
  double dbas_eps;          /* DBaSConfig.eps */
  double h_offset;          /* constraint tightening s of the nominal MPC: the DBaS dynamics use
                               h(x) - s (core/tube_mpc.py:151-153, 232-238); the linearisation
                               differentiates the untightened h (core/tube_mpc.py:282-286).  0 for
                               every other caller. */
} dtmpc_spec;

/* Quadratic stage/terminal cost (core/cost_derivs.py:58-146 + caller overrides in
 * core/tube_mpc.py:837-842, 890-894 and run_nominal.py:297-324). */
typedef struct dtmpc_cost {
  int32_t kind;             /* DTMPC_COST_* */
  int32_t wrap_angle;       /* 1: heading error wrapped to (-pi, pi] (run_nominal.py:32-34, 297-324) */
  double Q[3];
  double R[2];
  double Qf[3];             /* terminal weight; the paper ancillary passes Qf = Q (core/tube_mpc.py:885, 891) */
  double qb;
  double target[3];         /* DTMPC_COST_TARGET only */
} dtmpc_cost;

/* ILQRConfig (core/ddp.py:12-20) */
typedef struct dtmpc_ilqr_cfg {
  int32_t max_iter;
  int32_t n_alphas;         /* <= DTMPC_MAX_ALPHAS */
  double tol;               /* early exit when |J_prev - J_best| < tol; tol < 0 = fixed iterations */
  double reg;               /* Quu regulariser (core/ddp.py:136, 239) */
  double alphas[DTMPC_MAX_ALPHAS];
} dtmpc_ilqr_cfg;

/* Online adaptation of the ancillary weights (core/tube_mpc.py:746-752, 978-984). */
typedef struct dtmpc_adapt_cfg {
  double lr_eta;
  double momentum;
  double q_min;             /* Qa >= 0 */
  double r_min;             /* Ra >= 1e-4 */
  double qb_min, qb_max;    /* qba in [0, 1] */
} dtmpc_adapt_cfg;

/* Algorithm-2 closed-loop tube step configuration (core/tube_mpc.py:803-1023). */
typedef struct dtmpc_tube_cfg {
  dtmpc_cost nominal;       /* fixed nominal cost */
  dtmpc_ilqr_cfg nom_ilqr;
  dtmpc_ilqr_cfg aux_ilqr;
  int32_t disturbance;      /* 0: w injected by the caller, 1: counter-based Philox on device */
  int32_t write_log;        /* 1: write the per-step log record (see dtmpc_tube_state.log) */
  uint64_t seed;            /* Philox key (disturbance == 1) */
  double w_low[3];
  double w_high[3];
  double grad_bound;        /* health policy of the shared update: a trajectory whose DOC gradient row
                               [gQ, gR, gqb] has a component of magnitude above grad_bound (or a
                               non-finite one) drops out of the batch sums like a flagged trajectory;
                               <= 0 disables the magnitude bound, but a row with a non-finite component
                               is always left out (one NaN row would make the batch mean NaN).  The
                               count left out this way is the global batch minus the healthy count
                               (partials slot 7) minus the flagged trajectories (TubeMPC
                               .bound_dropped_count) */
} dtmpc_tube_cfg;

/* Device-resident closed-loop state; all SoA [fields][B] unless stated, caller-owned. */
typedef struct dtmpc_tube_state {
  void* x;          /* [3][B] plant state x_t */
  void* b;          /* [B]    plant barrier state b_t */
  void* xbar;       /* [3][B] nominal state */
  void* bbar;       /* [B] */
  void* Xnom;       /* [N+1][4][B] nominal optimal tape (written) */
  void* Unom;       /* [N][2][B]  in: nominal warm start, out: shifted warm start */
  void* Xaux;       /* [N+1][4][B] ancillary optimal tape (written) */
  void* Uaux;       /* [N][2][B]  in: ancillary warm start, out: shifted warm start */
  void* work;       /* dtmpc_tube_workspace_bytes() scratch */
  const void* theta;/* [6] ancillary weights Qa(3), Ra(2), qba (shared by the batch) */
  void* partials;   /* [n_partials][8] per-workgroup sums over the HEALTHY trajectories (status 0
                       after this step and a gradient row within cfg->grad_bound): L, gQ(3), gR(2),
                       gqb, and their count */
  void* log;        /* [18][B] or NULL: x(3) u(2) xbar(3) ubar(2) b L gQ(3) gR(2) gqb of step t
                       (the gradient rows are the trajectory's own contribution before any
                       status masking) */
  int32_t* status;  /* [B] DTMPC_ST_* bits (OR-accumulated) */
  int32_t* iters;   /* [2][B] nominal / ancillary iterations used, or NULL */
  int32_t lanes;    /* lanes per trajectory, fixed when the state is built: dtmpc_tube_lanes_dtype(B, dtype) (the
                       precision's rule; dtmpc_tube_lanes(B) is the f32 rule) */
  int32_t phase;    /* ABI 6 (was padding, 0): which part of the step dtmpc_tube_step launches -- 0 the whole step;
                       1 the nominal solve alone (theta-independent, core/tube_mpc.py:813-857); 2 the rest (the
                       ancillary solve with the current theta, sensitivity, gradient sums, plant), after a phase-1
                       launch of the same step on the same state.  Splitting lets a multi-rank caller run the
                       previous step's theta all-reduce and update beside the nominal solve (TubeMPC, SURVEY.md
                       §5); fused kernel only (dtmpc_tube_split_supported) */
  int64_t n_partials; /* rows of `partials`; must be >= dtmpc_tube_partials_count(B, lanes) */
  int64_t chunk;    /* trajectories per launch of the f32 fast kernel, fixed when the state is built:
                       dtmpc_tube_chunk(horizon, lanes) */
  int64_t work_bytes; /* size of `work`; must be >=
                         dtmpc_tube_workspace_bytes(dtype, horizon, B, lanes, chunk) */
  int8_t* choices;  /* [nom_ilqr.max_iter + aux_ilqr.max_iter][B] or NULL: the decision record of the
                       step -- per iteration of the nominal, then the ancillary solve, the
                       original position of the winning line-search alpha (core/ddp.py:293, strict <,
                       first wins), -1 for iterations not run */
  void* costs;      /* [nom_ilqr.max_iter + aux_ilqr.max_iter][8][B] (dtype) or NULL: the costs behind the
                       decisions -- every line-search candidate's cost J (core/ddp.py:286-291) by
                       original alpha position, the alpha = 0 candidate's the current tape's; only the
                       candidates that ran are written (pre-fill it, e.g. with NaN).  Written by the fused
                       kernels only (diagnostics / the tie-aware parity
                       gate, tests/_common.py); the generic kernel leaves it untouched */
} dtmpc_tube_state;

int dtmpc_abi_version(void);
const char* dtmpc_last_error(void);

/* Device count visible to the library (0 when no GPU). */
int dtmpc_device_count(void);

/* ---- KAT-level entry points (per-kernel parity) --------------------------------------- */

/* rollout with f = DBaS-augmented Dubins step:
 *   replaces core/ddp.py:89-99 `rollout` with f = f_hat_nom (core/tube_mpc.py:816-821),
 *   i.e. core/barrier.py:75-108 `dbas_step` over core/systems/dubins.py:26-45 `dubins_step`.
 *   x0 [4][B], U [N][2][B] (used as given, not clamped), X [N+1][4][B] out. */
int dtmpc_dbas_rollout(int dtype, const dtmpc_spec* spec, int64_t B,
                       const void* x0, const void* U, void* X, void* stream);

/* b0 = B(h(x0)) for each trajectory: replaces core/barrier.py:111-120 `dbas_init_b0`.
 *   x [3][B] (or the first 3 fields of any [F][B] array with F >= 3 via x), b [B] out. */
int dtmpc_dbas_init(int dtype, const dtmpc_spec* spec, int64_t B, const void* x, void* b,
                    void* stream);

/* Per-step linearisation + cost derivatives along a tape:
 *   replaces core/systems/dubins_aug_jac.py:61-139 `dubins_augmented_jacobian` and
 *   core/cost_derivs.py:58-146 (`*_cost_derivs_u`, `*_terminal_derivs`).
 *   A [N][16][B] (row-major 4x4), Bm [N][8][B] (row-major 4x2),
 *   lx [N+1][4][B] (k = N is phi_x), lu [N][2][B].  Xref [N+1][3][B] / Uref [N][2][B] are read
 *   only for DTMPC_COST_TRACK (may be NULL otherwise). */
int dtmpc_linearize(int dtype, const dtmpc_spec* spec, const dtmpc_cost* cost, int64_t B,
                    const void* X, const void* U, const void* Xref, const void* Uref,
                    void* A, void* Bm, void* lx, void* lu, void* stream);

/* ---- solver entry points -------------------------------------------------------------- */

/* Box-clamped iLQR with line search (all alphas, best-of, strict <) and per-trajectory tol exit:
 *   replaces core/ddp.py:102-307 `ilqr_solve` for the typed problem.
 *   x0 [4][B]; U [N][2][B] in: V_init (clamped first, core/ddp.py:127-129), out: V*;
 *   X [N+1][4][B] out: X*; K [N][8][B] / kff [N][2][B] out: gains of the last backward pass (scratch
 *   of the solve, required); iters [B] out (may be NULL); status [B] out (OR-accumulated);
 *   choices [cfg->max_iter][B] out or NULL: the winning line-search alpha's original position per
 *   iteration (core/ddp.py:293), -1 for iterations not run. */
int dtmpc_ilqr_solve(int dtype, const dtmpc_spec* spec, const dtmpc_cost* cost,
                     const dtmpc_ilqr_cfg* cfg, int64_t B, const void* x0,
                     const void* Xref, const void* Uref, void* X, void* U,
                     void* K, void* kff, int32_t* iters, int32_t* status, int8_t* choices,
                     void* stream);

/* Workspace bytes of dtmpc_ilqr_solve_ws for B trajectories at `lanes` per trajectory (0: the
 * dtmpc_tube_lanes(B) default; 1, 2 or 4), for DTMPC_F32 and DTMPC_F64 alike (both precisions have the
 * fused solver: csrc/dtmpc_fast_ilqr.hip, csrc/dtmpc_fast64_ilqr.hip); 0 for bad arguments. */
size_t dtmpc_ilqr_workspace_bytes(int dtype, int32_t horizon, int64_t B, int32_t lanes);

/* dtmpc_ilqr_solve (same arrays, same results contract) through the fused solver of the tube step
 * on the fast configuration -- f32 or f64, smooth-min obstacles (1..8), relaxed inverse barrier,
 * h_offset 0, six non-zero line-search alphas (plus at most one alpha = 0) -- with `lanes` lanes per
 * trajectory (0: default) and a caller-owned workspace of dtmpc_ilqr_workspace_bytes; any other
 * configuration (DTMPC_FAST=0 in the environment, or DTMPC_FAST64=0 for f64) runs dtmpc_ilqr_solve's
 * generic kernel (dtmpc_ilqr_fused_eligible says which).  costs (or NULL): [max_iter][8][B] every
 * line-search candidate's cost by alpha position as dtmpc_tube_state.costs (fused solver only; only the
 * candidates that ran are written).
 * max_iter = 0: K and kff are written as zeros
 * (no backward pass ran), as the generic kernel leaves the zeroed arrays the package passes.
 * Replaces core/ddp.py:102-307 `ilqr_solve` (the batched nominal DDP of BASELINE config 2). */
/* 1 when dtmpc_ilqr_solve_ws runs the fused solver for this problem / cost / config in this precision
 * (and the environment's DTMPC_FAST / DTMPC_FAST64 switches), 0 when it falls to dtmpc_ilqr_solve's
 * generic kernel.  Host-only (no device call). */
int32_t dtmpc_ilqr_fused_eligible(int dtype, const dtmpc_spec* spec, const dtmpc_cost* cost,
                                  const dtmpc_ilqr_cfg* cfg);

int dtmpc_ilqr_solve_ws(int dtype, const dtmpc_spec* spec, const dtmpc_cost* cost,
                        const dtmpc_ilqr_cfg* cfg, int64_t B, const void* x0,
                        const void* Xref, const void* Uref, void* X, void* U,
                        void* K, void* kff, int32_t* iters, int32_t* status, int8_t* choices,
                        void* costs, int32_t lanes, void* work, size_t work_bytes, void* stream);

/* Scratch bytes for dtmpc_ddp_sensitivity. */
size_t dtmpc_sensitivity_workspace_bytes(int dtype, int32_t horizon, int64_t B, int32_t want_lambda);

/* DDP-structured KKT sensitivity with active set (paper Appendix G):
 *   replaces core/ddp.py:317-427 `ddp_sensitivity` driven by the paper-mode upper-loss closures
 *   core/tube_mpc.py:924-957 (g_x = [2(x - xbar_k), 2 b], g_u = 0, terminal likewise).
 *   X/U: ancillary optimum; Xbar [N+1][3][B]: nominal states of the upper loss;
 *   Xref/Uref: ancillary cost references (DTMPC_COST_TRACK), cost: ancillary cost.
 *   dX [N+1][4][B], dU [N][2][B], dlam [N+1][4][B] (NULL skips delta_lambda). */
int dtmpc_ddp_sensitivity(int dtype, const dtmpc_spec* spec, const dtmpc_cost* cost, int64_t B,
                          const void* X, const void* U, const void* Xref, const void* Uref,
                          const void* Xbar, void* dX, void* dU, void* dlam, void* work,
                          int32_t* status, void* stream);

/* Upper loss and analytic DOC gradient per trajectory:
 *   replaces core/tube_mpc.py:915-919 (L) and :963-976 (gQ, gR, gqb).
 *   out [7][B]: L, gQ(3), gR(2), gqb. */
int dtmpc_doc_grad(int dtype, int32_t horizon, int64_t B, const void* Xaux, const void* Uaux,
                   const void* Xnom, const void* Unom, const void* dX, const void* dU,
                   void* out, void* stream);

/* ---- fused closed-loop step (Algorithm 2 body) ----------------------------------------- */

/* Trajectories per launch of the f32 fast kernel: its per-lane workspace records stay below 2^31 bytes
 * (one buffer resource); the environment variable DTMPC_FAST_CHUNK (a smaller chunk, for the tests of
 * the chunked launch) is read here only.  Resolved ONCE, when the caller builds its state
 * (dtmpc_tube_state.chunk); dtmpc_tube_step never reads it. */
int64_t dtmpc_tube_chunk(int32_t horizon, int32_t lanes);
/* Scratch bytes for dtmpc_tube_step at `lanes` lanes per trajectory and `chunk` (dtmpc_tube_chunk).
 * 0 if lanes is not a supported count or chunk is not one dtmpc_tube_chunk can return. */
size_t dtmpc_tube_workspace_bytes(int dtype, int32_t horizon, int64_t B, int32_t lanes, int64_t chunk);
/* Lanes per trajectory the fused step uses for a batch of B on the current device (lane slots =
 * CUs x 4 SIMDs x 64, 65,536 on MI355X): 4 while 8 B <= slots (B <= 8,192: one line-search pair per
 * lane, candidate tapes kept instead of a commit pass), 2 while 2 B <= slots (paired line search),
 * else 1 (one wave per SIMD at the benchmark batch); the environment variable DTMPC_TUBE_LANES=1|2|4
 * overrides.  Resolved ONCE, when the caller builds its state (dtmpc_tube_state.lanes);
 * dtmpc_tube_step never reads the environment. */
int32_t dtmpc_tube_lanes(int64_t B);
/* dtmpc_tube_lanes for a precision (ABI 6): DTMPC_F32 as dtmpc_tube_lanes; DTMPC_F64 4 while 4 B <= slots
 * (B <= 16,384 on MI355X), 2 while 2 B <= slots (B <= 32,768; round 6), else 1 -- the f64 step is
 * instruction-bound, so the split line search pays for the duplicated recursion up to half the lane slots.  The default of dtmpc_ilqr_workspace_bytes /
 * dtmpc_ilqr_solve_ws (lanes = 0) follows their dtype the same way.  0 for a bad dtype. */
int32_t dtmpc_tube_lanes_dtype(int64_t B, int dtype);
/* Number of per-workgroup partial records dtmpc_tube_step writes for B trajectories at `lanes`
 * lanes per trajectory (0 if lanes is not a supported count): one per workgroup of 256 threads, or of
 * 64 threads while B x lanes is below the device's wave slots (CUs x 4 SIMDs x 64). */
int64_t dtmpc_tube_partials_count(int64_t B, int32_t lanes);

/* One closed-loop step for every trajectory (core/tube_mpc.py:803-1023 loop body):
 *   nominal iLQR -> ancillary iLQR tracking it -> upper loss -> sensitivity -> DOC gradient
 *   (per-workgroup sums into state->partials) -> plant step with disturbance -> nominal
 *   propagation -> warm-start shift.  theta is READ (the update happens in
 *   dtmpc_theta_update after the cross-rank sum).  w: [3][B] injected disturbance
 *   (cfg->disturbance == 0) or NULL.  global_offset / step index key the Philox stream so that
 *   every sharding of a global batch sees identical disturbances. */
int dtmpc_tube_step(int dtype, const dtmpc_spec* spec, const dtmpc_tube_cfg* cfg, int64_t B,
                    int64_t global_offset, int64_t step, const dtmpc_tube_state* state,
                    const void* w, void* stream);
/* 1 when dtmpc_tube_step runs the fused kernel for this problem / config / precision and lane count, which is
 * what a phase split (dtmpc_tube_state.phase = 1, 2) needs; 0 otherwise.  Host-only. */
int32_t dtmpc_tube_split_supported(int dtype, const dtmpc_spec* spec, const dtmpc_tube_cfg* cfg, int32_t lanes);
/* ABI 7: 1 when a phase split of THIS batch is possible -- dtmpc_tube_split_supported, and B within one launch chunk of
 * the precision (the nominal records of the whole batch stay in the workspace between the two launches; f64 records
 * are twice as large, so its chunk is min(chunk, about half the f32 maximum)).  dtmpc_tube_step refuses a phase != 0
 * launch for which this is 0.  Host-only. */
int32_t dtmpc_tube_split_ok(int dtype, const dtmpc_spec* spec, const dtmpc_tube_cfg* cfg, int64_t B, int32_t lanes,
                            int64_t chunk);

/* Episode start of the fused closed loop in one launch (core/tube_mpc.py:770-779; the reference's
 * run_closed_loop_experiment sets x = x_bar = x0, b = b_bar = B(h(x0)), zero warm starts and its
 * initial adaptation weights): x0 [B][3] trajectory-major; writes state->x, xbar [3][B], b, bbar [B],
 * Unom, Uaux [N][2][B] (zero), status [B] (zero), theta [6] = theta0 [6] and vel [6] = 0. */
int dtmpc_tube_reset(int dtype, const dtmpc_spec* spec, int64_t B, const void* x0,
                     const dtmpc_tube_state* state, const void* theta0, void* theta, void* vel,
                     void* stream);

/* Fixed-order sum of the per-workgroup partial records: sums [8] (L, gQ(3), gR(2), gqb, count). */
int dtmpc_partials_reduce(int dtype, int64_t n_partials, const void* partials, void* sums,
                          void* stream);

/* Momentum + projected update of the shared ancillary weights (core/tube_mpc.py:978-984) with
 * the batch-mean gradient g = sums[1:7] * inv_batch, or, for inv_batch <= 0, the mean over the
 * healthy trajectories g = sums[1:7] / sums[7] (g = 0 when none is healthy: a flagged trajectory
 * -- the reference raises there -- drops out of the mean instead of pulling it toward zero).
 * theta [6] and velocity [6] in/out. */
int dtmpc_theta_update(int dtype, const dtmpc_adapt_cfg* cfg, double inv_batch, const void* sums,
                       void* theta, void* velocity, void* stream);


/* ---- general (softplus / tanh parameterised) IFT path ------------------------------------ */
/*
 * core/tube_mpc.py:40-663 with adapt_nominal (or paper_dubins_mode off): every weight and DBaS
 * parameter is a raw, unconstrained value mapped through core/params.py:9-59 --
 * Q = softplus(Q_raw), R, Qf, q_b likewise, alpha = softplus(alpha_raw) + 1e-6,
 * gamma = tanh(gamma_raw), tightening s = softplus(tight_raw) -- and both the ancillary theta and
 * the nominal theta-bar adapt by the IFT gradient (core/ift.py:35-92), the nominal one through the
 * ancillary's gradient w.r.t. its reference trajectory (core/tube_mpc.py:509-584).
 *
 * Raw parameter vector layout ([12] per parameter set): */
enum {
  DTMPC_P_Q = 0,      /* Q_raw[3] */
  DTMPC_P_R = 3,      /* R_raw[2] */
  DTMPC_P_QF = 5,     /* Qf_raw[3] */
  DTMPC_P_QB = 8,     /* qb_raw */
  DTMPC_P_ALPHA = 9,  /* alpha_raw */
  DTMPC_P_GAMMA = 10, /* gamma_raw */
  DTMPC_P_TIGHT = 11, /* tight_raw (nominal theta-bar only; ignored for the ancillary set) */
  DTMPC_P_COUNT = 12
};

/* Scratch bytes for dtmpc_ddp_sensitivity_upper. */
size_t dtmpc_sensitivity_upper_workspace_bytes(int dtype, int32_t horizon, int64_t B);

/* DDP-structured KKT sensitivity with ARBITRARY upper-level gradients:
 *   replaces core/ddp.py:317-427 `ddp_sensitivity` with upper_grad_x / upper_grad_u /
 *   upper_grad_xN given as arrays (the nominal solve of core/tube_mpc.py:523-554 feeds
 *   [dL/dX_ref, 0] and dL/dU_ref from the ancillary IFT).
 *   gX [N+1][4][B] (row N = upper_grad_xN), gU [N][2][B]; dX [N+1][4][B], dU [N][2][B],
 *   dlam [N+1][4][B] (NULL skips delta_lambda). */
int dtmpc_ddp_sensitivity_upper(int dtype, const dtmpc_spec* spec, const dtmpc_cost* cost, int64_t B,
                                const void* X, const void* U, const void* gX, const void* gU,
                                void* dX, void* dU, void* dlam, void* work, int32_t* status,
                                void* stream);

/* IFT gradient w.r.t. the raw parameters, in closed form:
 *   replaces core/ift.py:35-92 `ift_gradient` for the typed problem, with the closures of
 *   core/tube_mpc.py:461-500 (cost->kind = DTMPC_COST_TRACK: ancillary, also dL/dX_ref, dL/dU_ref)
 *   or :556-585 (DTMPC_COST_TARGET: nominal, with the tightening).  The weights and DBaS
 *   parameters are taken from theta_raw (host [12]) through core/params.py, not from cost/spec;
 *   cost supplies kind and target, spec the system, obstacles, barrier type and eps.
 *   X, U, dX, dU, dlam: optimum and its sensitivity (dtmpc_ddp_sensitivity*).
 *   g_theta [12][B] out (row DTMPC_P_TIGHT is 0 for the ancillary), g_xref [N+1][3][B] and
 *   g_uref [N][2][B] out for DTMPC_COST_TRACK (either may be NULL). */
int dtmpc_ift_gradient(int dtype, const dtmpc_spec* spec, const dtmpc_cost* cost,
                       const double* theta_raw, int64_t B, const void* X, const void* U,
                       const void* dX, const void* dU, const void* dlam, const void* Xref,
                       const void* Uref, void* g_theta, void* g_xref, void* g_uref, void* stream);

/* Closed-loop configuration of the general path (core/tube_mpc.py:48-188). */
typedef struct dtmpc_general_cfg {
  double target[3];          /* DubinsConfig.x_target of the nominal cost */
  dtmpc_ilqr_cfg nom_ilqr;   /* ILQRConfig(max_iter=nominal_max_iter, reg=ilqr_reg) (:161) */
  dtmpc_ilqr_cfg aux_ilqr;   /* ILQRConfig(max_iter=aux_max_iter, reg=ilqr_reg) (:162) */
  int32_t adapt_nominal;     /* (:108) */
  int32_t adapt_ancillary;   /* (:109) */
  int32_t project_params;    /* _project (:192-237) */
  int32_t disturbance;       /* 0: injected w, 1: device Philox (as dtmpc_tube_cfg) */
  int32_t write_log;
  int32_t pad_;
  uint64_t seed;
  double w_low[3];
  double w_high[3];
  double lr_eta;             /* (:178) */
  double momentum;           /* (:181) */
  double clip_norm;          /* grad_clip_norm, per parameter tensor; <= 0 disables (:180) */
} dtmpc_general_cfg;

/* Device-resident state of the general closed loop; SoA [fields][B] unless stated. */
typedef struct dtmpc_general_state {
  void* x;          /* [3][B] */
  void* b;          /* [B] */
  void* xbar;       /* [3][B] */
  void* bbar;       /* [B] */
  void* Xnom;       /* [N+1][4][B] */
  void* Unom;       /* [N][2][B] warm start in / optimum out (shifted by dtmpc_general_plant) */
  void* Xaux;       /* [N+1][4][B] */
  void* Uaux;       /* [N][2][B] */
  void* work;       /* dtmpc_general_workspace_bytes() scratch */
  void* theta;      /* [2][12] raw parameters, row 0 ancillary theta, row 1 nominal theta-bar
                       (shared by the batch; updated in place by dtmpc_general_update) */
  void* velocity;   /* [2][12] momentum buffers */
  void* partials;   /* [n_partials][25] per-workgroup sums over the healthy trajectories */
  void* sums;       /* [25] batch sums (after the cross-rank all-reduce) */
  void* gout;       /* [25][B] or NULL: each trajectory's own L (always) and raw gradients
                       (0 for a flagged trajectory), row 24 = 1 if healthy */
  void* log;        /* [12][B] or NULL: x(3) u(2) xbar(3) ubar(2) b L of step t */
  int32_t* status;  /* [B] */
  int32_t* iters;   /* [2][B] or NULL */
  int64_t n_partials; /* rows of `partials`; must be >= dtmpc_general_partials_count(B) */
} dtmpc_general_state;

size_t dtmpc_general_workspace_bytes(int dtype, int32_t horizon, int64_t B);
/* Number of per-workgroup partial records dtmpc_general_step writes (one lane per trajectory). */
int64_t dtmpc_general_partials_count(int64_t B);

/* Solves + sensitivities + IFT gradients for every trajectory (core/tube_mpc.py:217-584):
 * nominal iLQR with theta-bar -> ancillary iLQR tracking it with theta -> upper loss ->
 * ancillary sensitivity -> ancillary IFT (theta, X_ref, U_ref) -> [adapt_nominal] nominal
 * sensitivity driven by the reference gradients -> nominal IFT (theta-bar); per-workgroup sums of
 * [L, g_theta(11), g_theta_bar(12), count] over the healthy trajectories into state->partials.
 * theta is read only. */
int dtmpc_general_step(int dtype, const dtmpc_spec* spec, const dtmpc_general_cfg* cfg, int64_t B,
                       const dtmpc_general_state* state, void* stream);

/* Fixed-order sum of n_partials records of `width` values each into sums[width]. */
int dtmpc_partials_reduce_n(int dtype, int64_t n_partials, int32_t width, const void* partials,
                            void* sums, void* stream);

/* Momentum / clipped / projected update of theta and theta-bar with the batch-mean gradient
 * g = state->sums * inv_batch, or for inv_batch <= 0 the healthy-trajectory mean
 * g = state->sums / state->sums[24] (core/tube_mpc.py:239-255, 507-508, 584). */
int dtmpc_general_update(int dtype, const dtmpc_spec* spec, const dtmpc_general_cfg* cfg,
                         double inv_batch, const dtmpc_general_state* state, void* stream);

/* Plant step with the UPDATED parameters, nominal propagation, log, warm-start shift
 * (core/tube_mpc.py:589-624).  w: [3][B] injected (cfg->disturbance == 0) or NULL. */
int dtmpc_general_plant(int dtype, const dtmpc_spec* spec, const dtmpc_general_cfg* cfg, int64_t B,
                        int64_t global_offset, int64_t step, const dtmpc_general_state* state,
                        const void* w, void* stream);

/* ---- receding-horizon nominal MPC (run_nominal.py:204-415) --------------------------------- */

size_t dtmpc_receding_workspace_bytes(int dtype, int32_t horizon, int64_t B);

/* B independent runs of run_nominal_receding, the whole task horizon H in one launch: per step
 * iLQR (cost: nominal, usually wrap_angle = 1, run_nominal.py:297-324) from [x_t, b_t] with the
 * shifted warm start -> u0 -> x_{t+1} = f_hat(x_t, u0) -> exits: collision when the true
 * min_i h_i(x_t) <= 0 (:388-397), success when ||x_t[:2] - target[:2]|| <= success_radius
 * (:399-403).  x0 [3][B] (b0 = B(h(x0)) is derived, :279); U [N][2][B] warm start in (the reference
 * uses v = v_max, omega = 0, :368-369), last shifted plan out; log [H][6][B] out: x(3), u0(2), b of
 * every recorded step (rows past h_ran untouched); h_ran / success_t (-1: none) / collided [B] out;
 * status [B] OR-accumulated (a failed solve ends that trajectory's run, where the reference raises).
 * The paper configuration (smooth-min obstacles, relaxed inverse barrier, six non-zero alphas + 0) runs the
 * tube step's fused solver with the wrapped cost compiled in (csrc/dtmpc_fast.hip receding_fast_kernel, f32
 * and f64); anything else, and DTMPC_FAST=0 / DTMPC_FAST64=0, the generic receding_kernel. */
int dtmpc_nominal_receding(int dtype, const dtmpc_spec* spec, const dtmpc_cost* cost,
                           const dtmpc_ilqr_cfg* cfg, int64_t B, int32_t H, double success_radius,
                           const void* x0, void* U, void* log, int32_t* h_ran, int32_t* success_t,
                           int32_t* collided, int32_t* status, void* work, void* stream);
/* dtmpc_nominal_receding with iters [B] out (ABI 6; may be NULL): each run's total iLQR iterations over its
 * receding steps -- the receding leg of bench.py prices its algorithmic bytes by them (7,652 B
 * per nominal iteration in f32). */
int dtmpc_nominal_receding_it(int dtype, const dtmpc_spec* spec, const dtmpc_cost* cost,
                              const dtmpc_ilqr_cfg* cfg, int64_t B, int32_t H, double success_radius,
                              const void* x0, void* U, void* log, int32_t* h_ran, int32_t* success_t,
                              int32_t* collided, int32_t* status, int32_t* iters, void* work, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* DTMPC_H */
