/*
 * oracle_impl.h — TEST INFRASTRUCTURE ONLY (the parity checker and the CPU baseline).
 *
 * Plain-C restatement of the reference hot path (lmcggg/differentiable-tube-mpc), one
 * trajectory at a time, written to follow the reference's PyTorch code operation by operation.
 * It is included twice by dtmpc_oracle.c: once with REAL=double (suffix _f64) and once with
 * REAL=float (suffix _f32).  Nothing in the product path (libdtmpc.so, the Python package)
 * links, imports or calls this code; only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg do.
 *
 * Parity pinning: tests/test_oracle_golden.py checks every function here against golden
 * vectors produced by running the reference itself (tests/golden/make_golden.py).
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

#define CAT_(a, b) a##b
#define CAT(a, b) CAT_(a, b)
#define FN(name) CAT(name, SUFFIX)
#define SPEC_T CAT(ospec, SUFFIX)
#define COST_T CAT(ocost, SUFFIX)

typedef struct {
  int N, M, agg, barrier;
  REAL dt, umin[2], umax[2], active_tol;
  REAL neg_beta, neg_inv_beta;
  REAL cx[DTMPC_MAX_OBS], cy[DTMPC_MAX_OBS], r2[DTMPC_MAX_OBS];
  REAL alpha, gamma, eps;
  REAL tight; /* h offset of the DBaS dynamics (nominal tightening, core/tube_mpc.py:151-153) */
} SPEC_T;

typedef struct {
  int kind, wrap;
  REAL Q[3], R[2], Qf[3], qb, target[3];
} COST_T;

static void FN(spec_from)(const dtmpc_spec* s, SPEC_T* o) {
  o->N = s->horizon;
  o->M = s->n_obstacles;
  o->agg = s->obs_aggregation;
  o->barrier = s->barrier_type;
  o->dt = (REAL)s->dt;
  for (int a = 0; a < 2; ++a) {
    o->umin[a] = (REAL)s->u_min[a];
    o->umax[a] = (REAL)s->u_max[a];
  }
  o->active_tol = (REAL)s->active_tol;
  o->neg_beta = (REAL)(-s->obs_beta);               /* (-beta) * H, dubins_obstacles.py:65 */
  o->neg_inv_beta = (REAL)(-(1.0 / s->obs_beta));   /* -(1.0/beta) * lse, dubins_obstacles.py:68 */
  for (int i = 0; i < s->n_obstacles && i < DTMPC_MAX_OBS; ++i) {
    o->cx[i] = (REAL)s->obs_cx[i];
    o->cy[i] = (REAL)s->obs_cy[i];
    o->r2[i] = (REAL)(s->obs_r[i] * s->obs_r[i]);  /* obs.radius ** 2 (python float) */
  }
  o->alpha = (REAL)s->dbas_alpha;
  o->gamma = (REAL)s->dbas_gamma;
  o->eps = (REAL)s->dbas_eps;
  o->tight = (REAL)s->h_offset;
}

static void FN(cost_from)(const dtmpc_cost* c, COST_T* o) {
  o->kind = c->kind;
  o->wrap = c->wrap_angle;
  for (int i = 0; i < 3; ++i) {
    o->Q[i] = (REAL)c->Q[i];
    o->Qf[i] = (REAL)c->Qf[i];
    o->target[i] = (REAL)c->target[i];
  }
  o->R[0] = (REAL)c->R[0];
  o->R[1] = (REAL)c->R[1];
  o->qb = (REAL)c->qb;
}

static int FN(isfin)(REAL v) { return isfinite(v) ? 1 : 0; }

/* torch.clamp: NaN propagates (core/control.py:61-64) */
static REAL FN(clampv)(REAL v, REAL lo, REAL hi) {
  if (v < lo) return lo;
  if (v > hi) return hi;
  return v;
}

/* ---- safety function h (core/systems/dubins_obstacles.py) ------------------------------ */

/* h_circle_obstacle :16-30 */
static REAL FN(h_circle)(const SPEC_T* s, int i, REAL px, REAL py) {
  REAL dx = px - s->cx[i];
  REAL dy = py - s->cy[i];
  return dx * dx + dy * dy - s->r2[i];
}

/* h(x) and its gradient d h / d(px, py) (theta derivative is 0).
 *   smoothmin: h_multi_circle_obstacles :41-69 and grad_h_multi_circle_obstacles :72-92
 *   min:       h_min_circle_obstacles :95-106 and grad_h_min_circle_obstacles :109-117
 *   single:    h_circle_obstacle :16-30 and grad_h_circle_obstacle :33-38
 *   none:      h = 1 (run_nominal.py:256), gradient 0 */
static REAL FN(h_eval)(const SPEC_T* s, REAL px, REAL py, REAL* gx, REAL* gy) {
  if (s->agg == DTMPC_OBS_NONE || s->M == 0) {
    *gx = 0;
    *gy = 0;
    return (REAL)1;
  }
  if (s->agg == DTMPC_OBS_SINGLE) {
    *gx = (REAL)2 * (px - s->cx[0]);
    *gy = (REAL)2 * (py - s->cy[0]);
    return FN(h_circle)(s, 0, px, py);
  }
  REAL hs[DTMPC_MAX_OBS];
  for (int i = 0; i < s->M; ++i) hs[i] = FN(h_circle)(s, i, px, py);
  if (s->agg == DTMPC_OBS_MIN) {
    int am = 0;
    for (int i = 1; i < s->M; ++i)
      if (hs[i] < hs[am]) am = i; /* torch.argmin: first minimum */
    *gx = (REAL)2 * (px - s->cx[am]);
    *gy = (REAL)2 * (py - s->cy[am]);
    return hs[am];
  }
  /* smooth-min: stable log-sum-exp */
  REAL z[DTMPC_MAX_OBS];
  for (int i = 0; i < s->M; ++i) z[i] = s->neg_beta * hs[i];
  REAL zmax = z[0];
  for (int i = 1; i < s->M; ++i)
    if (z[i] > zmax) zmax = z[i];
  REAL se = 0;
  REAL e[DTMPC_MAX_OBS];
  for (int i = 0; i < s->M; ++i) {
    e[i] = M_EXP(z[i] - zmax);
    se += e[i];
  }
  REAL lse = zmax + M_LOG(se);
  /* gradient: softmax(-beta h_i) weighted sum of 2 (p - c_i) */
  REAL g0 = 0, g1 = 0;
  for (int i = 0; i < s->M; ++i) {
    REAL w = e[i] / se;
    g0 += w * ((REAL)2 * (px - s->cx[i]));
    g1 += w * ((REAL)2 * (py - s->cy[i]));
  }
  *gx = g0;
  *gy = g1;
  return s->neg_inv_beta * lse;
}

/* ---- barriers (core/barrier.py, core/systems/dubins_aug_jac.py) -------------------------- */

/* relaxed_inverse_barrier_B_alpha core/barrier.py:36-59 with alpha_eff = max(alpha, eps) */
static REAL FN(barrier_relaxed)(const SPEC_T* s, REAL z) {
  REAL a = s->alpha > s->eps ? s->alpha : s->eps;
  if (z >= a) {
    REAL zc = z < s->eps ? s->eps : z;
    return (REAL)1 / zc;
  }
  REAL diff = z - a;
  REAL a2 = a * a;
  return ((REAL)1 / a - diff / a2) + (diff * diff) / (a2 * a);
}

/* _dB_relaxed_inv_dz core/systems/dubins_aug_jac.py:31-40 */
static REAL FN(dbarrier_relaxed)(const SPEC_T* s, REAL z) {
  REAL a = s->alpha > s->eps ? s->alpha : s->eps;
  if (z >= a) {
    REAL zc = z < s->eps ? s->eps : z;
    return (REAL)(-1) / (zc * zc);
  }
  REAL diff = z - a;
  REAL a2 = a * a;
  return -((REAL)1 / a2) + ((REAL)2 * diff) / (a2 * a);
}

/* barrier used by the DBaS dynamics (core/barrier.py:99-106); log branch is barrier_B :62-72 */
static REAL FN(barrier_dyn)(const SPEC_T* s, REAL z) {
  if (s->barrier == DTMPC_BARRIER_LOG) {
    REAL zc = z < s->eps ? s->eps : z;
    return -M_LOG(zc);
  }
  return FN(barrier_relaxed)(s, z);
}

/* ---- dynamics ---------------------------------------------------------------------------- */

/* dubins_step core/systems/dubins.py:26-45 */
static void FN(dubins)(const SPEC_T* s, const REAL* x, const REAL* u, REAL* xn) {
  REAL c = M_COS(x[2]), sn = M_SIN(x[2]);
  REAL dv = s->dt * u[0];
  xn[0] = x[0] + dv * c;
  xn[1] = x[1] + dv * sn;
  xn[2] = x[2] + s->dt * u[1];
}

/* dbas_step core/barrier.py:75-108 as f_hat (core/tube_mpc.py:816-821): xh = [x, b] */
static void FN(fhat)(const SPEC_T* s, const REAL* xh, const REAL* u, REAL* xhn) {
  REAL gx, gy;
  FN(dubins)(s, xh, u, xhn);
  /* h_nom(x) = h(x) - s for the tightened nominal (core/tube_mpc.py:235-238); s = 0 otherwise */
  REAL hn = FN(h_eval)(s, xhn[0], xhn[1], &gx, &gy) - s->tight;
  REAL hc = FN(h_eval)(s, xh[0], xh[1], &gx, &gy) - s->tight;
  REAL Bn = FN(barrier_dyn)(s, hn);
  REAL Bc = FN(barrier_dyn)(s, hc);
  xhn[3] = Bn - s->gamma * (Bc - xh[3]);
}

/* dubins_augmented_jacobian core/systems/dubins_aug_jac.py:61-139 (+ dubins_f_jac :42-58).
 * A row-major 4x4, Bm row-major 4x2. */
static void FN(aug_jac)(const SPEC_T* s, const REAL* xh, const REAL* u, REAL* A, REAL* Bm) {
  REAL dt = s->dt;
  REAL c = M_COS(xh[2]), sn = M_SIN(xh[2]);
  REAL v = u[0];
  REAL A3[9] = {1, 0, -dt * v * sn, 0, 1, dt * v * c, 0, 0, 1};
  REAL B3[6] = {dt * c, 0, dt * sn, 0, 0, dt};
  REAL xn[3];
  FN(dubins)(s, xh, u, xn);
  REAL dhc[3], dhn[3];
  REAL hc = FN(h_eval)(s, xh[0], xh[1], &dhc[0], &dhc[1]);
  REAL hn = FN(h_eval)(s, xn[0], xn[1], &dhn[0], &dhn[1]);
  dhc[2] = 0;
  dhn[2] = 0;
  REAL dBc = FN(dbarrier_relaxed)(s, hc);
  REAL dBn = FN(dbarrier_relaxed)(s, hn);
  REAL r[3], gc[3];
  for (int i = 0; i < 3; ++i) {
    r[i] = dBn * dhn[i];
    gc[i] = s->gamma * dBc * dhc[i];
  }
  memset(A, 0, 16 * sizeof(REAL));
  memset(Bm, 0, 8 * sizeof(REAL));
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) A[i * 4 + j] = A3[i * 3 + j];
    for (int j = 0; j < 2; ++j) Bm[i * 2 + j] = B3[i * 2 + j];
  }
  for (int j = 0; j < 3; ++j) {
    REAL acc = 0;
    for (int i = 0; i < 3; ++i) acc += r[i] * A3[i * 3 + j];
    A[12 + j] = acc - gc[j];
  }
  A[15] = s->gamma;
  for (int j = 0; j < 2; ++j) {
    REAL acc = 0;
    for (int i = 0; i < 3; ++i) acc += r[i] * B3[i * 2 + j];
    Bm[6 + j] = acc;
  }
}

/* ---- costs ------------------------------------------------------------------------------- */

/* _wrap_angle run_nominal.py:32-34 */
static REAL FN(wrap)(REAL e) { return M_ATAN2(M_SIN(e), M_COS(e)); }

/* stage cost: nominal core/tube_mpc.py:823-827 (wrapped: run_nominal.py:297-302),
 * tracking core/tube_mpc.py:875-880 */
static REAL FN(stage_cost)(const COST_T* c, const REAL* xh, const REAL* u, const REAL* xr,
                           const REAL* ur) {
  REAL dx[3], du[2];
  if (c->kind == DTMPC_COST_TRACK) {
    for (int i = 0; i < 3; ++i) dx[i] = xh[i] - xr[i];
    for (int a = 0; a < 2; ++a) du[a] = u[a] - ur[a];
  } else {
    for (int i = 0; i < 3; ++i) dx[i] = xh[i] - c->target[i];
    if (c->wrap) dx[2] = FN(wrap)(dx[2]);
    du[0] = u[0];
    du[1] = u[1];
  }
  REAL sq = 0, sr = 0;
  for (int i = 0; i < 3; ++i) sq += c->Q[i] * dx[i] * dx[i];
  for (int a = 0; a < 2; ++a) sr += c->R[a] * du[a] * du[a];
  return sq + sr + c->qb * (xh[3] * xh[3]);
}

/* terminal cost: core/tube_mpc.py:829-832, 882-885; run_nominal.py:304-309 */
static REAL FN(term_cost)(const COST_T* c, const REAL* xh, const REAL* xr) {
  REAL dx[3];
  for (int i = 0; i < 3; ++i) dx[i] = xh[i] - (c->kind == DTMPC_COST_TRACK ? xr[i] : c->target[i]);
  if (c->kind != DTMPC_COST_TRACK && c->wrap) dx[2] = FN(wrap)(dx[2]);
  REAL sq = 0;
  for (int i = 0; i < 3; ++i) sq += c->Qf[i] * dx[i] * dx[i];
  return sq + c->qb * (xh[3] * xh[3]);
}

/* tracking/target error used by the derivatives: nominal_cost_derivs_u (core/cost_derivs.py:58-76)
 * with the wrapped target of run_nominal.py:311-315 (target_k[2] = x2 - wrap(x2 - t2)). */
static void FN(deriv_dx)(const COST_T* c, const REAL* xh, const REAL* xr, REAL* dx) {
  if (c->kind == DTMPC_COST_TRACK) {
    for (int i = 0; i < 3; ++i) dx[i] = xh[i] - xr[i];
    return;
  }
  REAL t2 = c->target[2];
  if (c->wrap) t2 = xh[2] - FN(wrap)(xh[2] - c->target[2]);
  dx[0] = xh[0] - c->target[0];
  dx[1] = xh[1] - c->target[1];
  dx[2] = xh[2] - t2;
}

/* l_x, l_u (l_xx = diag(2Q, 2qb), l_uu = diag(2R), l_ux = 0)
 * core/cost_derivs.py:58-76 (nominal) and :110-130 (auxiliary) */
static void FN(stage_derivs)(const COST_T* c, const REAL* xh, const REAL* u, const REAL* xr,
                             const REAL* ur, REAL* lx, REAL* lu) {
  REAL dx[3];
  FN(deriv_dx)(c, xh, xr, dx);
  for (int i = 0; i < 3; ++i) lx[i] = ((REAL)2 * c->Q[i]) * dx[i];
  lx[3] = ((REAL)2 * c->qb) * xh[3];
  for (int a = 0; a < 2; ++a)
    lu[a] = ((REAL)2 * c->R[a]) * (c->kind == DTMPC_COST_TRACK ? (u[a] - ur[a]) : u[a]);
}

/* phi_x (phi_xx = diag(2Qf, 2qb)): core/cost_derivs.py:133-146 + overrides
 * core/tube_mpc.py:837-842, 890-894, run_nominal.py:317-324 */
static void FN(term_derivs)(const COST_T* c, const REAL* xh, const REAL* xr, REAL* lx) {
  REAL dx[3];
  FN(deriv_dx)(c, xh, xr, dx);
  for (int i = 0; i < 3; ++i) lx[i] = ((REAL)2 * c->Qf[i]) * dx[i];
  lx[3] = ((REAL)2 * c->qb) * xh[3];
}

/* ---- 2x2 solves -------------------------------------------------------------------------- */

/* torch.linalg.solve on a 2x2 system: LU with partial pivoting, nrhs columns.  M row-major 2x2,
 * rhs/out row-major 2 x nrhs. */
static void FN(solve2)(const REAL* M, const REAL* rhs, int nrhs, REAL* out) {
  REAL a00 = M[0], a01 = M[1], a10 = M[2], a11 = M[3];
  int sw = M_FABS(a10) > M_FABS(a00);
  if (sw) {
    REAL t;
    t = a00; a00 = a10; a10 = t;
    t = a01; a01 = a11; a11 = t;
  }
  REAL l = a10 / a00;
  REAL u11 = a11 - l * a01;
  for (int j = 0; j < nrhs; ++j) {
    REAL r0 = sw ? rhs[nrhs + j] : rhs[j];
    REAL r1 = sw ? rhs[j] : rhs[nrhs + j];
    REAL y1 = r1 - l * r0;
    REAL x1 = y1 / u11;
    REAL x0 = (r0 - a01 * x1) / a00;
    out[j] = x0;
    out[nrhs + j] = x1;
  }
}

/* _solve_reduced core/ddp.py:23-60: active rows are zero, free block solved */
static void FN(solve_reduced)(const REAL* M, const REAL* rhs, int nrhs, const int* act, REAL* out) {
  if (!act[0] && !act[1]) {
    FN(solve2)(M, rhs, nrhs, out);
    return;
  }
  for (int j = 0; j < 2 * nrhs; ++j) out[j] = 0;
  if (act[0] && act[1]) return;
  int f = act[0] ? 1 : 0;
  REAL a = M[f * 2 + f];
  for (int j = 0; j < nrhs; ++j) out[f * nrhs + j] = rhs[f * nrhs + j] / a;
}

/* ---- Riccati (core/ddp.py:213-254) -------------------------------------------------------- */

/* One backward step.  Inputs: A (4x4), Bm (4x2), lx, lu, l_xx = diag(lxx_d), l_uu = diag(luu_d),
 * Vx, Vxx (in/out).  Outputs K (2x4), kff (2).  Returns 0 if every checked quantity is finite. */
static int FN(riccati_step)(const REAL* A, const REAL* Bm, const REAL* lx, const REAL* lu,
                            const REAL* lxx_d, const REAL* luu_d, REAL reg, REAL* Vx, REAL* Vxx,
                            REAL* K, REAL* kff) {
  REAL Qx[4], Qu[2], AtV[16], Qxx[16], BtV[8], Qux[8], Quu[4], Qreg[4];
  for (int i = 0; i < 4; ++i) {
    REAL acc = 0;
    for (int j = 0; j < 4; ++j) acc += A[j * 4 + i] * Vx[j];
    Qx[i] = lx[i] + acc;
  }
  for (int a = 0; a < 2; ++a) {
    REAL acc = 0;
    for (int j = 0; j < 4; ++j) acc += Bm[j * 2 + a] * Vx[j];
    Qu[a] = lu[a] + acc;
  }
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) {
      REAL acc = 0;
      for (int m = 0; m < 4; ++m) acc += A[m * 4 + i] * Vxx[m * 4 + j];
      AtV[i * 4 + j] = acc;
    }
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) {
      REAL acc = 0;
      for (int m = 0; m < 4; ++m) acc += AtV[i * 4 + m] * A[m * 4 + j];
      Qxx[i * 4 + j] = (i == j ? lxx_d[i] : (REAL)0) + acc;
    }
  for (int a = 0; a < 2; ++a)
    for (int j = 0; j < 4; ++j) {
      REAL acc = 0;
      for (int m = 0; m < 4; ++m) acc += Bm[m * 2 + a] * Vxx[m * 4 + j];
      BtV[a * 4 + j] = acc;
    }
  for (int a = 0; a < 2; ++a)
    for (int j = 0; j < 4; ++j) {
      REAL acc = 0;
      for (int m = 0; m < 4; ++m) acc += BtV[a * 4 + m] * A[m * 4 + j];
      Qux[a * 4 + j] = (REAL)0 + acc; /* l_ux = 0 */
    }
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 2; ++b) {
      REAL acc = 0;
      for (int m = 0; m < 4; ++m) acc += BtV[a * 4 + m] * Bm[m * 2 + b];
      Quu[a * 2 + b] = (a == b ? luu_d[a] : (REAL)0) + acc;
    }
  int ok = 1;
  for (int j = 0; j < 4; ++j) ok &= FN(isfin)(Quu[j]);
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 2; ++b) Qreg[a * 2 + b] = Quu[a * 2 + b] + (a == b ? reg : (REAL)0);
  REAL Ks[8], ks[2];
  FN(solve2)(Qreg, Qux, 4, Ks);
  FN(solve2)(Qreg, Qu, 1, ks);
  for (int j = 0; j < 8; ++j) {
    K[j] = -Ks[j];
    ok &= FN(isfin)(K[j]);
  }
  for (int a = 0; a < 2; ++a) {
    kff[a] = -ks[a];
    ok &= FN(isfin)(kff[a]);
  }
  /* V_x = Q_x + K^T Q_uu k + K^T Q_u + Q_xu k   (core/ddp.py:251) */
  REAL KtQuu[8];
  for (int i = 0; i < 4; ++i)
    for (int b = 0; b < 2; ++b) {
      REAL acc = 0;
      for (int a = 0; a < 2; ++a) acc += K[a * 4 + i] * Quu[a * 2 + b];
      KtQuu[i * 2 + b] = acc;
    }
  for (int i = 0; i < 4; ++i) {
    REAL t1 = 0, t2 = 0, t3 = 0;
    for (int b = 0; b < 2; ++b) t1 += KtQuu[i * 2 + b] * kff[b];
    for (int a = 0; a < 2; ++a) t2 += K[a * 4 + i] * Qu[a];
    for (int a = 0; a < 2; ++a) t3 += Qux[a * 4 + i] * kff[a];
    Vx[i] = Qx[i] + t1 + t2 + t3;
    ok &= FN(isfin)(Vx[i]);
  }
  /* V_xx = Q_xx + K^T Q_uu K + K^T Q_ux + Q_xu K   (core/ddp.py:252) */
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j) {
      REAL m1 = 0, m2 = 0, m3 = 0;
      for (int b = 0; b < 2; ++b) m1 += KtQuu[i * 2 + b] * K[b * 4 + j];
      for (int a = 0; a < 2; ++a) m2 += K[a * 4 + i] * Qux[a * 4 + j];
      for (int a = 0; a < 2; ++a) m3 += Qux[a * 4 + i] * K[a * 4 + j];
      Vxx[i * 4 + j] = Qxx[i * 4 + j] + m1 + m2 + m3;
      ok &= FN(isfin)(Vxx[i * 4 + j]);
    }
#ifdef ORACLE_SYM_VXX
  /* test variant (liboracle_sym.so): V_xx mirrored from its upper triangle -- equal in exact arithmetic to
   * the reference's full update (core/ddp.py:252), a different rounding of it.  Deep in the relaxed
   * barrier's quadratic branch (B's barrier row ~1e10) Q_uu is numerically rank one in f32 and the gains
   * are rounding noise; whether that noise overflows within the horizon depends on the evaluation order
   * (tests/test_gpu_receding.py::test_receding_f32_failure_set_vs_oracle) */
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < i; ++j) Vxx[i * 4 + j] = Vxx[j * 4 + i];
#endif
  return ok ? 0 : 1;
}

/* ---- rollouts ------------------------------------------------------------------------------ */

/* rollout core/ddp.py:89-99 */
static void FN(rollout1)(const SPEC_T* s, const REAL* x0, const REAL* V, REAL* X) {
  int N = s->N;
  for (int f = 0; f < 4; ++f) X[f] = x0[f];
  for (int k = 0; k < N; ++k) FN(fhat)(s, X + 4 * k, V + 2 * k, X + 4 * (k + 1));
}

static REAL FN(traj_cost)(const SPEC_T* s, const COST_T* c, const REAL* X, const REAL* V,
                          const REAL* Xr, const REAL* Ur) {
  int N = s->N;
  REAL J = 0;
  for (int k = 0; k < N; ++k)
    J += FN(stage_cost)(c, X + 4 * k, V + 2 * k, Xr ? Xr + 3 * k : NULL, Ur ? Ur + 2 * k : NULL);
  return J + FN(term_cost)(c, X + 4 * N, Xr ? Xr + 3 * N : NULL);
}

/* ---- iLQR (core/ddp.py:102-307) ------------------------------------------------------------ */

/* work: >= (2*(N+1)*4 + 2*2*N) REALs. Returns status bits; *iters = iterations run.  choice (or NULL):
 * the line search's winning alpha position of iteration it at choice[it * cstride] (the decision record
 * of SURVEY.md §8c; iterations not run are left as the caller set them).  ccost (or NULL): the cost of
 * every line-search candidate, alpha position ia of iteration it at ccost[(it * 8 + ia) * cstride] (the
 * candidates' costs behind each decision: the tie-aware decision gate of tests/_common.py). */
static int FN(ilqr1)(const SPEC_T* s, const COST_T* c, const dtmpc_ilqr_cfg* cfg, const REAL* x0,
                     const REAL* Xr, const REAL* Ur, REAL* X, REAL* V, REAL* K, REAL* kff,
                     int* iters, REAL* work, signed char* choice, long long cstride, REAL* ccost) {
  int N = s->N;
  REAL reg = (REAL)cfg->reg, tol = (REAL)cfg->tol;
  REAL* Xc = work;
  REAL* Vc = Xc + 4 * (N + 1);
  REAL* Xb = Vc + 2 * N;
  REAL* Vb = Xb + 4 * (N + 1);
  *iters = 0;
  /* V = ctrl.clamp(V_init); X = rollout(x0, V)  :127-131 */
  for (int k = 0; k < N; ++k)
    for (int a = 0; a < 2; ++a) V[2 * k + a] = FN(clampv)(V[2 * k + a], s->umin[a], s->umax[a]);
  FN(rollout1)(s, x0, V, X);
  int have_prev = 0;
  REAL prev = 0;
  REAL lxx_d[4], luu_d[2];
  for (int i = 0; i < 3; ++i) lxx_d[i] = (REAL)2 * c->Q[i];
  lxx_d[3] = (REAL)2 * c->qb;
  for (int a = 0; a < 2; ++a) luu_d[a] = (REAL)2 * c->R[a];
  REAL pxx_d[4];
  for (int i = 0; i < 3; ++i) pxx_d[i] = (REAL)2 * c->Qf[i];
  pxx_d[3] = (REAL)2 * c->qb;
  for (int it = 0; it < cfg->max_iter; ++it) {
    *iters = it + 1;
    /* derivatives along the tape + cost (finite checks only)  :172-205 */
    REAL cost = 0;
    for (int k = 0; k < N; ++k) {
      for (int f = 0; f < 4; ++f)
        if (!FN(isfin)(X[4 * k + f])) return DTMPC_ST_NONFINITE;
      for (int a = 0; a < 2; ++a)
        if (!FN(isfin)(V[2 * k + a])) return DTMPC_ST_NONFINITE;
      cost += FN(stage_cost)(c, X + 4 * k, V + 2 * k, Xr ? Xr + 3 * k : NULL, Ur ? Ur + 2 * k : NULL);
      if (!FN(isfin)(cost)) return DTMPC_ST_NONFINITE;
    }
    /* backward pass :208-254 */
    REAL Vx[4], Vxx[16];
    FN(term_derivs)(c, X + 4 * N, Xr ? Xr + 3 * N : NULL, Vx);
    memset(Vxx, 0, sizeof(Vxx));
    for (int i = 0; i < 4; ++i) Vxx[i * 5] = pxx_d[i];
    for (int f = 0; f < 4; ++f)
      if (!FN(isfin)(Vx[f])) return DTMPC_ST_NONFINITE;
    cost += FN(term_cost)(c, X + 4 * N, Xr ? Xr + 3 * N : NULL);
    if (!FN(isfin)(cost)) return DTMPC_ST_NONFINITE;
    for (int k = N - 1; k >= 0; --k) {
      REAL A[16], Bm[8], lx[4], lu[2];
      FN(aug_jac)(s, X + 4 * k, V + 2 * k, A, Bm);
      for (int j = 0; j < 16; ++j)
        if (!FN(isfin)(A[j])) return DTMPC_ST_NONFINITE;
      for (int j = 0; j < 8; ++j)
        if (!FN(isfin)(Bm[j])) return DTMPC_ST_NONFINITE;
      FN(stage_derivs)(c, X + 4 * k, V + 2 * k, Xr ? Xr + 3 * k : NULL, Ur ? Ur + 2 * k : NULL, lx, lu);
      if (FN(riccati_step)(A, Bm, lx, lu, lxx_d, luu_d, reg, Vx, Vxx, K + 8 * k, kff + 2 * k))
        return DTMPC_ST_NONFINITE;
    }
    /* forward pass with line search :256-301 */
    int have_best = 0, best_ia = -1;
    REAL best = 0;
    for (int ia = 0; ia < cfg->n_alphas; ++ia) {
      REAL al = (REAL)cfg->alphas[ia];
      for (int f = 0; f < 4; ++f) Xc[f] = x0[f];
      for (int k = 0; k < N; ++k) {
        REAL dx[4], u[2];
        for (int f = 0; f < 4; ++f) dx[f] = Xc[4 * k + f] - X[4 * k + f];
        for (int a = 0; a < 2; ++a) {
          REAL du = kff[2 * k + a];
          REAL acc = 0;
          for (int f = 0; f < 4; ++f) acc += K[8 * k + 4 * a + f] * dx[f];
          du = du + acc;
          u[a] = FN(clampv)(V[2 * k + a] + al * du, s->umin[a], s->umax[a]);
          Vc[2 * k + a] = u[a];
        }
        FN(fhat)(s, Xc + 4 * k, u, Xc + 4 * (k + 1));
      }
      for (int j = 0; j < 4 * (N + 1); ++j)
        if (!FN(isfin)(Xc[j])) return DTMPC_ST_NONFINITE;
      for (int j = 0; j < 2 * N; ++j)
        if (!FN(isfin)(Vc[j])) return DTMPC_ST_NONFINITE;
      REAL J = FN(traj_cost)(s, c, Xc, Vc, Xr, Ur);
      if (ccost && ia < 8) ccost[((long long)it * 8 + ia) * cstride] = J;
      if (!FN(isfin)(J)) return DTMPC_ST_NONFINITE;
      if (!have_best || J < best) {
        have_best = 1;
        best = J;
        best_ia = ia;
        memcpy(Xb, Xc, sizeof(REAL) * 4 * (N + 1));
        memcpy(Vb, Vc, sizeof(REAL) * 2 * N);
      }
    }
    if (!have_best) return DTMPC_ST_NO_CANDIDATE;
    if (choice) choice[(long long)it * cstride] = (signed char)best_ia;
    memcpy(X, Xb, sizeof(REAL) * 4 * (N + 1));
    memcpy(V, Vb, sizeof(REAL) * 2 * N);
    /* :303-305 */
    if (have_prev && M_FABS(prev - best) < tol) break;
    have_prev = 1;
    prev = best;
  }
  return 0;
}

/* ---- DDP sensitivity (core/ddp.py:317-427) with the paper upper loss (core/tube_mpc.py:932-944) */

/* Upper gradients: gX [N+1][4] / gU [N][2] when given (core/ddp.py:322-324 closures as arrays),
 * else the paper upper loss g_x = [2(x - xbar_k), 2 b], g_u = 0. */
static int FN(sens1)(const SPEC_T* s, const COST_T* c, const REAL* X, const REAL* V,
                     const REAL* Xr, const REAL* Ur, const REAL* Xbar, const REAL* gX,
                     const REAL* gU, REAL* dX, REAL* dV, REAL* dlam, REAL* work) {
  (void)Ur;
  int N = s->N;
  REAL* Aseq = work;               /* N*16 */
  REAL* Bseq = Aseq + 16 * N;      /* N*8 */
  REAL* Kseq = Bseq + 8 * N;       /* N*8 */
  REAL* kseq = Kseq + 8 * N;       /* N*2 */
  REAL* Vxxs = kseq + 2 * N;       /* (N+1)*16 */
  REAL* tVxs = Vxxs + 16 * (N + 1);/* (N+1)*4 */
  int* act = (int*)(tVxs + 4 * (N + 1)); /* N*2 */
  int ok = 1;
  REAL lxx_d[4], luu_d[2], pxx_d[4];
  for (int i = 0; i < 3; ++i) lxx_d[i] = (REAL)2 * c->Q[i];
  lxx_d[3] = (REAL)2 * c->qb;
  for (int a = 0; a < 2; ++a) luu_d[a] = (REAL)2 * c->R[a];
  for (int i = 0; i < 3; ++i) pxx_d[i] = (REAL)2 * c->Qf[i];
  pxx_d[3] = (REAL)2 * c->qb;
  (void)Xr;
  for (int k = 0; k < N; ++k) FN(aug_jac)(s, X + 4 * k, V + 2 * k, Aseq + 16 * k, Bseq + 8 * k);
  /* backward, reg 1e-9 :362-410 */
  REAL Vxx[16], tVx[4];
  memset(Vxx, 0, sizeof(Vxx));
  for (int i = 0; i < 4; ++i) Vxx[5 * i] = pxx_d[i];
  if (gX) {
    for (int i = 0; i < 4; ++i) tVx[i] = gX[4 * N + i];
  } else {
    for (int i = 0; i < 3; ++i) tVx[i] = (REAL)2 * (X[4 * N + i] - Xbar[3 * N + i]);
    tVx[3] = (REAL)2 * X[4 * N + 3];
  }
  memcpy(Vxxs + 16 * N, Vxx, sizeof(Vxx));
  memcpy(tVxs + 4 * N, tVx, sizeof(tVx));
  REAL reg = (REAL)1e-9;
  for (int k = N - 1; k >= 0; --k) {
    const REAL* A = Aseq + 16 * k;
    const REAL* Bm = Bseq + 8 * k;
    REAL AtV[16], Qxx[16], Qxu[8], Qux[8], Quu[4], BtV[8], tQu[2], tQx[4], Qreg[4];
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) {
        REAL acc = 0;
        for (int m = 0; m < 4; ++m) acc += A[m * 4 + i] * Vxx[m * 4 + j];
        AtV[i * 4 + j] = acc;
      }
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) {
        REAL acc = 0;
        for (int m = 0; m < 4; ++m) acc += AtV[i * 4 + m] * A[m * 4 + j];
        Qxx[i * 4 + j] = (i == j ? lxx_d[i] : (REAL)0) + acc;
      }
    /* Q_xu = l_ux^T + A^T V_xx B */
    for (int i = 0; i < 4; ++i)
      for (int b = 0; b < 2; ++b) {
        REAL acc = 0;
        for (int m = 0; m < 4; ++m) acc += AtV[i * 4 + m] * Bm[m * 2 + b];
        Qxu[i * 2 + b] = (REAL)0 + acc;
      }
    for (int a = 0; a < 2; ++a)
      for (int j = 0; j < 4; ++j) {
        REAL acc = 0;
        for (int m = 0; m < 4; ++m) acc += Bm[m * 2 + a] * Vxx[m * 4 + j];
        BtV[a * 4 + j] = acc;
      }
    for (int a = 0; a < 2; ++a)
      for (int j = 0; j < 4; ++j) {
        REAL acc = 0;
        for (int m = 0; m < 4; ++m) acc += BtV[a * 4 + m] * A[m * 4 + j];
        Qux[a * 4 + j] = (REAL)0 + acc;
      }
    for (int a = 0; a < 2; ++a)
      for (int b = 0; b < 2; ++b) {
        REAL acc = 0;
        for (int m = 0; m < 4; ++m) acc += BtV[a * 4 + m] * Bm[m * 2 + b];
        Quu[a * 2 + b] = (a == b ? luu_d[a] : (REAL)0) + acc;
      }
    /* g_u = 0, g_x = [2(x - xbar_k), 2 b] */
    REAL gx[4], gu[2] = {0, 0};
    if (gX) {
      for (int i = 0; i < 4; ++i) gx[i] = gX[4 * k + i];
      gu[0] = gU[2 * k];
      gu[1] = gU[2 * k + 1];
    } else {
      for (int i = 0; i < 3; ++i) gx[i] = (REAL)2 * (X[4 * k + i] - Xbar[3 * k + i]);
      gx[3] = (REAL)2 * X[4 * k + 3];
    }
    for (int a = 0; a < 2; ++a) {
      REAL acc = 0;
      for (int m = 0; m < 4; ++m) acc += Bm[m * 2 + a] * tVx[m];
      tQu[a] = gu[a] + acc;
    }
    for (int i = 0; i < 4; ++i) {
      REAL acc = 0;
      for (int m = 0; m < 4; ++m) acc += A[m * 4 + i] * tVx[m];
      tQx[i] = gx[i] + acc;
    }
    for (int a = 0; a < 2; ++a)
      for (int b = 0; b < 2; ++b) Qreg[a * 2 + b] = Quu[a * 2 + b] + (a == b ? reg : (REAL)0);
    int* ak = act + 2 * k;
    for (int a = 0; a < 2; ++a) {
      REAL u = V[2 * k + a];
      ak[a] = (u <= s->umin[a] + s->active_tol) || (u >= s->umax[a] - s->active_tol);
    }
    REAL Ks[8], ks[2];
    FN(solve_reduced)(Qreg, Qux, 4, ak, Ks);
    FN(solve_reduced)(Qreg, tQu, 1, ak, ks);
    REAL* Kk = Kseq + 8 * k;
    REAL* kk = kseq + 2 * k;
    for (int j = 0; j < 8; ++j) Kk[j] = -Ks[j];
    for (int a = 0; a < 2; ++a) kk[a] = -ks[a];
    /* tilde_V_x = tilde_Q_x + Q_xu k ; V_xx = Q_xx + Q_xu K   :403-404 */
    for (int i = 0; i < 4; ++i) {
      REAL acc = 0;
      for (int b = 0; b < 2; ++b) acc += Qxu[i * 2 + b] * kk[b];
      tVx[i] = tQx[i] + acc;
    }
    for (int i = 0; i < 4; ++i)
      for (int j = 0; j < 4; ++j) {
        REAL acc = 0;
        for (int b = 0; b < 2; ++b) acc += Qxu[i * 2 + b] * Kk[b * 4 + j];
        Vxx[i * 4 + j] = Qxx[i * 4 + j] + acc;
      }
    memcpy(Vxxs + 16 * k, Vxx, sizeof(Vxx));
    memcpy(tVxs + 4 * k, tVx, sizeof(tVx));
  }
  /* forward :413-425 */
  for (int f = 0; f < 4; ++f) dX[f] = 0;
  for (int k = 0; k < N; ++k) {
    const REAL* Kk = Kseq + 8 * k;
    const REAL* kk = kseq + 2 * k;
    const REAL* dxk = dX + 4 * k;
    for (int a = 0; a < 2; ++a) {
      REAL acc = 0;
      for (int f = 0; f < 4; ++f) acc += Kk[a * 4 + f] * dxk[f];
      dV[2 * k + a] = act[2 * k + a] ? (REAL)0 : kk[a] + acc;
    }
    const REAL* A = Aseq + 16 * k;
    const REAL* Bm = Bseq + 8 * k;
    for (int i = 0; i < 4; ++i) {
      REAL a1 = 0, a2 = 0;
      for (int f = 0; f < 4; ++f) a1 += A[i * 4 + f] * dxk[f];
      for (int b = 0; b < 2; ++b) a2 += Bm[i * 2 + b] * dV[2 * k + b];
      dX[4 * (k + 1) + i] = a1 + a2;
    }
    if (dlam) {
      const REAL* W = Vxxs + 16 * k;
      for (int i = 0; i < 4; ++i) {
        REAL acc = 0;
        for (int f = 0; f < 4; ++f) acc += W[i * 4 + f] * dxk[f];
        dlam[4 * k + i] = tVxs[4 * k + i] + acc;
      }
    }
  }
  if (dlam) {
    const REAL* W = Vxxs + 16 * N;
    for (int i = 0; i < 4; ++i) {
      REAL acc = 0;
      for (int f = 0; f < 4; ++f) acc += W[i * 4 + f] * dX[4 * N + f];
      dlam[4 * N + i] = tVxs[4 * N + i] + acc;
    }
  }
  for (int j = 0; j < 4 * (N + 1); ++j) ok &= FN(isfin)(dX[j]);
  for (int j = 0; j < 2 * N; ++j) ok &= FN(isfin)(dV[j]);
  return ok ? 0 : DTMPC_ST_NONFINITE;
}

/* upper loss + analytic DOC gradient core/tube_mpc.py:915-919, 963-976.  out[7] */
static void FN(docgrad1)(int N, const REAL* Xa, const REAL* Ua, const REAL* Xn, const REAL* Un,
                         const REAL* dX, const REAL* dU, REAL* out) {
  REAL L1 = 0, L2 = 0, gQ[3] = {0, 0, 0}, gR[2] = {0, 0}, gqb = 0;
  for (int k = 0; k <= N; ++k) {
    for (int i = 0; i < 3; ++i) {
      REAL d = Xa[4 * k + i] - Xn[4 * k + i];
      L1 += d * d;
    }
    L2 += Xa[4 * k + 3] * Xa[4 * k + 3];
  }
  for (int k = 0; k < N; ++k) {
    for (int i = 0; i < 3; ++i) gQ[i] += (REAL)2 * (Xa[4 * k + i] - Xn[4 * k + i]) * dX[4 * k + i];
    for (int a = 0; a < 2; ++a) gR[a] += (REAL)2 * (Ua[2 * k + a] - Un[2 * k + a]) * dU[2 * k + a];
    gqb += (REAL)2 * Xa[4 * k + 3] * dX[4 * k + 3];
  }
  for (int i = 0; i < 3; ++i) gQ[i] = gQ[i] + (REAL)2 * (Xa[4 * N + i] - Xn[4 * N + i]) * dX[4 * N + i];
  gqb = gqb + (REAL)2 * Xa[4 * N + 3] * dX[4 * N + 3];
  out[0] = L1 + L2;
  out[1] = gQ[0];
  out[2] = gQ[1];
  out[3] = gQ[2];
  out[4] = gR[0];
  out[5] = gR[1];
  out[6] = gqb;
}

/* disturbance w = low + (high - low) * U[0,1) (core/systems/dubins.py:59-67) from the shared
 * counter-based Philox stream keyed by (global trajectory index, step) */
static void FN(philox_w)(const dtmpc_tube_cfg* cfg, long long gidx, long long step, REAL* w) {
  uint32_t r[4];
  dtmpc_philox_uniform_bits(cfg->seed, (uint64_t)gidx, (uint64_t)step, r);
  for (int f = 0; f < 3; ++f) {
    REAL u = (REAL)(r[f] >> 8) * (REAL)(1.0 / 16777216.0);
    REAL lo = (REAL)cfg->w_low[f], hi = (REAL)cfg->w_high[f];
    w[f] = lo + (hi - lo) * u;
  }
}

/* ---- SoA gather/scatter ------------------------------------------------------------------- */

static void FN(gather)(const REAL* src, int rows, int F, long long B, long long i, REAL* dst) {
  for (int k = 0; k < rows; ++k)
    for (int f = 0; f < F; ++f) dst[k * F + f] = src[((long long)k * F + f) * B + i];
}
static void FN(scatter)(const REAL* src, int rows, int F, long long B, long long i, REAL* dst) {
  for (int k = 0; k < rows; ++k)
    for (int f = 0; f < F; ++f) dst[((long long)k * F + f) * B + i] = src[k * F + f];
}
/* gather the first 3 of 4 fields (x part of x_hat) as an Xref [rows][3] */
static void FN(gather_x3)(const REAL* src4, int rows, long long B, long long i, REAL* dst) {
  for (int k = 0; k < rows; ++k)
    for (int f = 0; f < 3; ++f) dst[k * 3 + f] = src4[((long long)k * 4 + f) * B + i];
}

/* ---- exported batched entry points (SoA layout, as include/dtmpc.h) ---------------------- */

void FN(oracle_h_eval)(const dtmpc_spec* sp, long long n, const REAL* px, const REAL* py, REAL* h,
                       REAL* gx, REAL* gy) {
  SPEC_T s;
  FN(spec_from)(sp, &s);
  for (long long i = 0; i < n; ++i) h[i] = FN(h_eval)(&s, px[i], py[i], &gx[i], &gy[i]);
}

void FN(oracle_barrier)(const dtmpc_spec* sp, long long n, const REAL* z, REAL* Bdyn, REAL* Brel,
                        REAL* dB) {
  SPEC_T s;
  FN(spec_from)(sp, &s);
  for (long long i = 0; i < n; ++i) {
    Bdyn[i] = FN(barrier_dyn)(&s, z[i]);
    Brel[i] = FN(barrier_relaxed)(&s, z[i]);
    dB[i] = FN(dbarrier_relaxed)(&s, z[i]);
  }
}

/* one DBaS step for n independent (x_hat, u) pairs, AoS [n][4], [n][2] */
void FN(oracle_fhat)(const dtmpc_spec* sp, long long n, const REAL* xh, const REAL* u, REAL* xhn) {
  SPEC_T s;
  FN(spec_from)(sp, &s);
  for (long long i = 0; i < n; ++i) FN(fhat)(&s, xh + 4 * i, u + 2 * i, xhn + 4 * i);
}

/* augmented jacobian for n pairs, AoS: A [n][16], Bm [n][8] */
void FN(oracle_aug_jac)(const dtmpc_spec* sp, long long n, const REAL* xh, const REAL* u, REAL* A,
                        REAL* Bm) {
  SPEC_T s;
  FN(spec_from)(sp, &s);
  for (long long i = 0; i < n; ++i) FN(aug_jac)(&s, xh + 4 * i, u + 2 * i, A + 16 * i, Bm + 8 * i);
}

void FN(oracle_dbas_rollout)(const dtmpc_spec* sp, long long B, const REAL* x0, const REAL* U,
                             REAL* X) {
  SPEC_T s;
  FN(spec_from)(sp, &s);
  int N = s.N;
  REAL* x0a = (REAL*)malloc(sizeof(REAL) * 4);
  REAL* Va = (REAL*)malloc(sizeof(REAL) * 2 * N);
  REAL* Xa = (REAL*)malloc(sizeof(REAL) * 4 * (N + 1));
  for (long long i = 0; i < B; ++i) {
    FN(gather)(x0, 1, 4, B, i, x0a);
    FN(gather)(U, N, 2, B, i, Va);
    FN(rollout1)(&s, x0a, Va, Xa);
    FN(scatter)(Xa, N + 1, 4, B, i, X);
  }
  free(x0a);
  free(Va);
  free(Xa);
}

void FN(oracle_linearize)(const dtmpc_spec* sp, const dtmpc_cost* cp, long long B, const REAL* X,
                          const REAL* U, const REAL* Xref, const REAL* Uref, REAL* A, REAL* Bm,
                          REAL* lx, REAL* lu) {
  SPEC_T s;
  COST_T c;
  FN(spec_from)(sp, &s);
  FN(cost_from)(cp, &c);
  int N = s.N;
  for (long long i = 0; i < B; ++i) {
    for (int k = 0; k <= N; ++k) {
      REAL xh[4], u[2], xr[3], ur[2], Ak[16], Bk[8], lxk[4], luk[2];
      for (int f = 0; f < 4; ++f) xh[f] = X[((long long)k * 4 + f) * B + i];
      if (c.kind == DTMPC_COST_TRACK)
        for (int f = 0; f < 3; ++f) xr[f] = Xref[((long long)k * 3 + f) * B + i];
      if (k == N) {
        FN(term_derivs)(&c, xh, xr, lxk);
        for (int f = 0; f < 4; ++f) lx[((long long)k * 4 + f) * B + i] = lxk[f];
        break;
      }
      for (int a = 0; a < 2; ++a) u[a] = U[((long long)k * 2 + a) * B + i];
      if (c.kind == DTMPC_COST_TRACK)
        for (int a = 0; a < 2; ++a) ur[a] = Uref[((long long)k * 2 + a) * B + i];
      FN(aug_jac)(&s, xh, u, Ak, Bk);
      FN(stage_derivs)(&c, xh, u, xr, ur, lxk, luk);
      for (int f = 0; f < 16; ++f) A[((long long)k * 16 + f) * B + i] = Ak[f];
      for (int f = 0; f < 8; ++f) Bm[((long long)k * 8 + f) * B + i] = Bk[f];
      for (int f = 0; f < 4; ++f) lx[((long long)k * 4 + f) * B + i] = lxk[f];
      for (int a = 0; a < 2; ++a) lu[((long long)k * 2 + a) * B + i] = luk[a];
    }
  }
}

/* choices (or NULL): [max_iter][B] winning alpha position per iteration, -1 where none ran;
 * costs (or NULL): [max_iter][8][B] every line-search candidate's cost by alpha position (NaN: not run) */
void FN(oracle_ilqr_solve_ex)(const dtmpc_spec* sp, const dtmpc_cost* cp, const dtmpc_ilqr_cfg* cfg,
                              long long B, const REAL* x0, const REAL* Xref, const REAL* Uref,
                              REAL* X, REAL* U, REAL* K, REAL* kff, int* iters, int* status,
                              signed char* choices, REAL* costs, int nthreads) {
  SPEC_T s;
  COST_T c;
  FN(spec_from)(sp, &s);
  FN(cost_from)(cp, &c);
  int N = s.N;
  if (nthreads < 1) nthreads = 1;
#pragma omp parallel num_threads(nthreads)
  {
    size_t per = (size_t)(4 + 4 * (N + 1) + 2 * N + 3 * (N + 1) + 2 * N + 8 * N + 2 * N +
                          2 * (4 * (N + 1) + 2 * N));
    REAL* buf = (REAL*)malloc(sizeof(REAL) * per);
    REAL* x0a = buf;
    REAL* Xa = x0a + 4;
    REAL* Va = Xa + 4 * (N + 1);
    REAL* Xr = Va + 2 * N;
    REAL* Ur = Xr + 3 * (N + 1);
    REAL* Ka = Ur + 2 * N;
    REAL* ka = Ka + 8 * N;
    REAL* wk = ka + 2 * N;
#pragma omp for schedule(dynamic, 1)
    for (long long i = 0; i < B; ++i) {
      FN(gather)(x0, 1, 4, B, i, x0a);
      FN(gather)(U, N, 2, B, i, Va);
      if (c.kind == DTMPC_COST_TRACK) {
        FN(gather)(Xref, N + 1, 3, B, i, Xr);
        FN(gather)(Uref, N, 2, B, i, Ur);
      }
      memset(Ka, 0, sizeof(REAL) * 8 * N);
      memset(ka, 0, sizeof(REAL) * 2 * N);
      int it = 0;
      if (choices)
        for (int j = 0; j < cfg->max_iter; ++j) choices[(long long)j * B + i] = -1;
      if (costs)
        for (int j = 0; j < cfg->max_iter * 8; ++j) costs[(long long)j * B + i] = (REAL)NAN;
      int st = FN(ilqr1)(&s, &c, cfg, x0a, c.kind == DTMPC_COST_TRACK ? Xr : NULL,
                         c.kind == DTMPC_COST_TRACK ? Ur : NULL, Xa, Va, Ka, ka, &it, wk,
                         choices ? choices + i : NULL, B, costs ? costs + i : NULL);
      FN(scatter)(Xa, N + 1, 4, B, i, X);
      FN(scatter)(Va, N, 2, B, i, U);
      if (K) FN(scatter)(Ka, N, 8, B, i, K);
      if (kff) FN(scatter)(ka, N, 2, B, i, kff);
      if (iters) iters[i] = it;
      if (status) status[i] |= st;
    }
    free(buf);
  }
}

void FN(oracle_ddp_sensitivity)(const dtmpc_spec* sp, const dtmpc_cost* cp, long long B,
                                const REAL* X, const REAL* U, const REAL* Xref, const REAL* Uref,
                                const REAL* Xbar, REAL* dX, REAL* dU, REAL* dlam, int* status,
                                int nthreads) {
  SPEC_T s;
  COST_T c;
  FN(spec_from)(sp, &s);
  FN(cost_from)(cp, &c);
  (void)Xref;
  (void)Uref;
  int N = s.N;
  if (nthreads < 1) nthreads = 1;
#pragma omp parallel num_threads(nthreads)
  {
    size_t per = (size_t)(4 * (N + 1) + 2 * N + 3 * (N + 1) + 4 * (N + 1) + 2 * N + 4 * (N + 1) +
                          16 * N + 8 * N + 8 * N + 2 * N + 16 * (N + 1) + 4 * (N + 1) + 2 * N + 8);
    REAL* buf = (REAL*)malloc(sizeof(REAL) * per + sizeof(int) * 2 * N + 64);
    REAL* Xa = buf;
    REAL* Va = Xa + 4 * (N + 1);
    REAL* Xb = Va + 2 * N;
    REAL* dXa = Xb + 3 * (N + 1);
    REAL* dVa = dXa + 4 * (N + 1);
    REAL* dla = dVa + 2 * N;
    REAL* wk = dla + 4 * (N + 1);
#pragma omp for schedule(dynamic, 1)
    for (long long i = 0; i < B; ++i) {
      FN(gather)(X, N + 1, 4, B, i, Xa);
      FN(gather)(U, N, 2, B, i, Va);
      FN(gather)(Xbar, N + 1, 3, B, i, Xb);
      int st = FN(sens1)(&s, &c, Xa, Va, NULL, NULL, Xb, NULL, NULL, dXa, dVa, dlam ? dla : NULL, wk);
      FN(scatter)(dXa, N + 1, 4, B, i, dX);
      FN(scatter)(dVa, N, 2, B, i, dU);
      if (dlam) FN(scatter)(dla, N + 1, 4, B, i, dlam);
      if (status) status[i] |= st;
    }
    free(buf);
  }
}

void FN(oracle_doc_grad)(int N, long long B, const REAL* Xa, const REAL* Ua, const REAL* Xn,
                         const REAL* Un, const REAL* dX, const REAL* dU, REAL* out) {
  REAL* xa = (REAL*)malloc(sizeof(REAL) * (2 * 4 * (N + 1) + 2 * 2 * N + 4 * (N + 1) + 2 * N + 8));
  REAL* ua = xa + 4 * (N + 1);
  REAL* xn = ua + 2 * N;
  REAL* un = xn + 4 * (N + 1);
  REAL* dx = un + 2 * N;
  REAL* du = dx + 4 * (N + 1);
  REAL o[7];
  for (long long i = 0; i < B; ++i) {
    FN(gather)(Xa, N + 1, 4, B, i, xa);
    FN(gather)(Ua, N, 2, B, i, ua);
    FN(gather)(Xn, N + 1, 4, B, i, xn);
    FN(gather)(Un, N, 2, B, i, un);
    FN(gather)(dX, N + 1, 4, B, i, dx);
    FN(gather)(dU, N, 2, B, i, du);
    FN(docgrad1)(N, xa, ua, xn, un, dx, du, o);
    for (int j = 0; j < 7; ++j) out[(long long)j * B + i] = o[j];
  }
  free(xa);
}

/* Algorithm-2 loop body per trajectory (core/tube_mpc.py:813-1023), theta read-only.
 * State arrays SoA as dtmpc_tube_state (host memory).  gout [7][B] per-trajectory L, gQ, gR, gqb.
 * log [18][B] (may be NULL).  w [3][B] (may be NULL when cfg->disturbance == 1). */
/* choices (or NULL): [nom max_iter + aux max_iter][B] winning alpha position per iteration of the
 * nominal, then the ancillary solve, -1 where none ran; costs (or NULL): [nom + aux max_iter][8][B] the
 * candidates' costs of every line search by alpha position (NaN: not run) */
void FN(oracle_tube_step_ex)(const dtmpc_spec* sp, const dtmpc_tube_cfg* cfg, long long B,
                             long long goff, long long step, REAL* x, REAL* b, REAL* xbar,
                             REAL* bbar, REAL* Xnom, REAL* Unom, REAL* Xaux, REAL* Uaux,
                             const REAL* theta, const REAL* w, REAL* gout, REAL* log, int* status,
                             int* iters, signed char* choices, REAL* costs, int nthreads) {
  SPEC_T s;
  COST_T cn, ca;
  FN(spec_from)(sp, &s);
  FN(cost_from)(&cfg->nominal, &cn);
  int N = s.N;
  ca.kind = DTMPC_COST_TRACK;
  ca.wrap = 0;
  for (int i = 0; i < 3; ++i) {
    ca.Q[i] = theta[i];
    ca.Qf[i] = theta[i];
    ca.target[i] = 0;
  }
  ca.R[0] = theta[3];
  ca.R[1] = theta[4];
  ca.qb = theta[5];
  if (nthreads < 1) nthreads = 1;
#pragma omp parallel num_threads(nthreads)
  {
    size_t per = (size_t)(8 + 2 * 4 * (N + 1) + 2 * 2 * N + 3 * (N + 1) + 8 * N + 2 * N +
                          2 * (4 * (N + 1) + 2 * N) + 4 * (N + 1) + 2 * N + 16 * N + 8 * N +
                          8 * N + 2 * N + 16 * (N + 1) + 4 * (N + 1) + 2 * N + 64);
    REAL* buf = (REAL*)malloc(sizeof(REAL) * per + sizeof(int) * 2 * N + 64);
    REAL* x0 = buf;
    REAL* Xn = x0 + 8;
    REAL* Vn = Xn + 4 * (N + 1);
    REAL* Xa = Vn + 2 * N;
    REAL* Va = Xa + 4 * (N + 1);
    REAL* Xr = Va + 2 * N;
    REAL* Ka = Xr + 3 * (N + 1);
    REAL* ka = Ka + 8 * N;
    REAL* wk = ka + 2 * N;
    REAL* dXa = wk + 2 * (4 * (N + 1) + 2 * N);
    REAL* dVa = dXa + 4 * (N + 1);
    REAL* wk2 = dVa + 2 * N;
#pragma omp for schedule(dynamic, 1)
    for (long long i = 0; i < B; ++i) {
      int st = 0, itn = 0, ita = 0;
      REAL xs[3], xb[3], bs = b[i], bb = bbar[i];
      for (int f = 0; f < 3; ++f) {
        xs[f] = x[(long long)f * B + i];
        xb[f] = xbar[(long long)f * B + i];
      }
      /* nominal solve from [xbar, bbar] :813-857 */
      x0[0] = xb[0]; x0[1] = xb[1]; x0[2] = xb[2]; x0[3] = bb;
      FN(gather)(Unom, N, 2, B, i, Vn);
      if (choices)
        for (int j = 0; j < cfg->nom_ilqr.max_iter + cfg->aux_ilqr.max_iter; ++j) choices[(long long)j * B + i] = -1;
      if (costs)
        for (int j = 0; j < (cfg->nom_ilqr.max_iter + cfg->aux_ilqr.max_iter) * 8; ++j)
          costs[(long long)j * B + i] = (REAL)NAN;
      st |= FN(ilqr1)(&s, &cn, &cfg->nom_ilqr, x0, NULL, NULL, Xn, Vn, Ka, ka, &itn, wk,
                      choices ? choices + i : NULL, B, costs ? costs + i : NULL);
      /* ancillary solve tracking the nominal :863-909 */
      for (int k = 0; k <= N; ++k)
        for (int f = 0; f < 3; ++f) Xr[3 * k + f] = Xn[4 * k + f];
      x0[0] = xs[0]; x0[1] = xs[1]; x0[2] = xs[2]; x0[3] = bs;
      FN(gather)(Uaux, N, 2, B, i, Va);
      st |= FN(ilqr1)(&s, &ca, &cfg->aux_ilqr, x0, Xr, Vn, Xa, Va, Ka, ka, &ita, wk,
                      choices ? choices + (long long)cfg->nom_ilqr.max_iter * B + i : NULL, B,
                      costs ? costs + (long long)cfg->nom_ilqr.max_iter * 8 * B + i : NULL);
      /* sensitivity + DOC gradient :915-976 */
      st |= FN(sens1)(&s, &ca, Xa, Va, Xr, Vn, Xr, NULL, NULL, dXa, dVa, NULL, wk2);
      REAL o[7];
      FN(docgrad1)(N, Xa, Va, Xn, Vn, dXa, dVa, o);
      /* a flagged (non-finite) trajectory contributes nothing to the shared gradient */
      for (int j = 0; j < 7; ++j) gout[(long long)j * B + i] = st ? (REAL)0 : o[j];
      /* plant + nominal propagation :990-1001 */
      REAL u[2] = {Va[0], Va[1]}, ub[2] = {Vn[0], Vn[1]};
      REAL ww[3];
      if (w) {
        for (int f = 0; f < 3; ++f) ww[f] = w[(long long)f * B + i];
      } else {
        FN(philox_w)(cfg, goff + i, step, ww);
      }
      REAL xh[4] = {xs[0], xs[1], xs[2], bs}, xhn[4], xbh[4] = {xb[0], xb[1], xb[2], bb}, xbn[4];
      FN(fhat)(&s, xh, u, xhn);
      FN(fhat)(&s, xbh, ub, xbn);
      if (log) {
        for (int f = 0; f < 3; ++f) log[(long long)f * B + i] = xs[f];
        log[3 * B + i] = u[0];
        log[4 * B + i] = u[1];
        for (int f = 0; f < 3; ++f) log[(long long)(5 + f) * B + i] = xb[f];
        log[8 * B + i] = ub[0];
        log[9 * B + i] = ub[1];
        log[10 * B + i] = bs;
        for (int j = 0; j < 7; ++j) log[(long long)(11 + j) * B + i] = o[j];
      }
      for (int f = 0; f < 3; ++f) {
        x[(long long)f * B + i] = xhn[f] + ww[f];
        xbar[(long long)f * B + i] = xbn[f];
      }
      b[i] = xhn[3];
      bbar[i] = xbn[3];
      /* outputs + warm-start shift :1015-1020 */
      FN(scatter)(Xn, N + 1, 4, B, i, Xnom);
      FN(scatter)(Xa, N + 1, 4, B, i, Xaux);
      for (int k = 0; k < N; ++k) {
        int src = k + 1 < N ? k + 1 : N - 1;
        for (int a = 0; a < 2; ++a) {
          Unom[((long long)k * 2 + a) * B + i] = Vn[2 * src + a];
          Uaux[((long long)k * 2 + a) * B + i] = Va[2 * src + a];
        }
      }
      if (status) status[i] |= st;
      if (iters) {
        iters[i] = itn;
        iters[B + i] = ita;
      }
    }
    free(buf);
  }
}

void FN(oracle_tube_step)(const dtmpc_spec* sp, const dtmpc_tube_cfg* cfg, long long B,
                          long long goff, long long step, REAL* x, REAL* b, REAL* xbar,
                          REAL* bbar, REAL* Xnom, REAL* Unom, REAL* Xaux, REAL* Uaux,
                          const REAL* theta, const REAL* w, REAL* gout, REAL* log, int* status,
                          int* iters, int nthreads) {
  FN(oracle_tube_step_ex)(sp, cfg, B, goff, step, x, b, xbar, bbar, Xnom, Unom, Xaux, Uaux, theta, w, gout, log,
                          status, iters, NULL, NULL, nthreads);
}

void FN(oracle_ilqr_solve)(const dtmpc_spec* sp, const dtmpc_cost* cp, const dtmpc_ilqr_cfg* cfg,
                           long long B, const REAL* x0, const REAL* Xref, const REAL* Uref,
                           REAL* X, REAL* U, REAL* K, REAL* kff, int* iters, int* status,
                           int nthreads) {
  FN(oracle_ilqr_solve_ex)(sp, cp, cfg, B, x0, Xref, Uref, X, U, K, kff, iters, status, NULL, NULL, nthreads);
}

/* momentum + projected update core/tube_mpc.py:978-984 with g = sums[1:7] * inv_batch, or for
 * inv_batch <= 0 the mean over the healthy trajectories counted in sums[7] (dtmpc_theta_update) */
void FN(oracle_theta_update)(const dtmpc_adapt_cfg* cfg, double inv_batch, const REAL* sums,
                             REAL* theta, REAL* vel) {
  REAL mom = (REAL)cfg->momentum, eta = (REAL)cfg->lr_eta;
  REAL ib = (REAL)inv_batch;
  if (!(inv_batch > 0)) ib = sums[7] > 0 ? (REAL)1 / sums[7] : (REAL)0;
  for (int j = 0; j < 6; ++j) {
    REAL g = sums[1 + j] * ib;
    vel[j] = mom * vel[j] + g;
    REAL t = theta[j] - eta * vel[j];
    if (j < 3) {
      REAL lo = (REAL)cfg->q_min;
      theta[j] = t < lo ? lo : t;
    } else if (j < 5) {
      REAL lo = (REAL)cfg->r_min;
      theta[j] = t < lo ? lo : t;
    } else {
      theta[j] = FN(clampv)(t, (REAL)cfg->qb_min, (REAL)cfg->qb_max);
    }
  }
}

#include "oracle_general.h"

/* Tanh-box control map and stage-cost derivatives in the decision variable v, along a tape.
 *   u(v)      = u_min + (u_max - u_min) * (tanh(v) + 1) * 0.5     core/control.py:22-27
 *   du/dv     = ((u_max - u_min) * 0.5) * (1 - tanh(v)^2)         core/control.py:29-35
 *   d2u/dv2   = scale * ((-2 tanh(v)) * sech2)                    core/cost_derivs.py:16-24
 *   nominal   l_x = [2Q dx, 2qb b], l_v = 2R u du/dv,             core/cost_derivs.py:27-55
 *             l_vv = 2R (du/dv^2 + u d2u/dv2)   (dx = x - target)
 *   auxiliary the same with u - u_ref in place of u, dx = x - x_ref  core/cost_derivs.py:79-107
 * (l_xx = diag(2Q, 2qb) and l_vx = 0 are constants of the cost.)  Each product is rounded in the
 * order torch evaluates the reference's expression.  SoA in/out; any output may be NULL. */
void FN(oracle_tanh_cost_derivs)(const dtmpc_spec* sp, const dtmpc_cost* cp, long long B, const REAL* X,
                                 const REAL* Vd, const REAL* Xref, const REAL* Uref, REAL* U, REAL* dU,
                                 REAL* lx, REAL* lv, REAL* lvv) {
  SPEC_T s;
  COST_T c;
  FN(spec_from)(sp, &s);
  FN(cost_from)(cp, &c);
  const int N = s.N;
  const int trk = c.kind == DTMPC_COST_TRACK;
  for (long long i = 0; i < B; ++i)
    for (int k = 0; k < N; ++k) {
      REAL xh[4], dx[3];
      for (int f = 0; f < 4; ++f) xh[f] = X[((long long)k * 4 + f) * B + i];
      for (int f = 0; f < 3; ++f)
        dx[f] = xh[f] - (trk ? Xref[((long long)k * 3 + f) * B + i] : c.target[f]);
      for (int f = 0; f < 3; ++f)
        if (lx) lx[((long long)k * 4 + f) * B + i] = ((REAL)2 * c.Q[f]) * dx[f];
      if (lx) lx[((long long)k * 4 + 3) * B + i] = ((REAL)2 * c.qb) * xh[3];
      for (int a = 0; a < 2; ++a) {
        const long long o = ((long long)k * 2 + a) * B + i;
        const REAL v = Vd[o];
        const REAL th = M_TANH(v);
        const REAL w = s.umax[a] - s.umin[a];
        const REAL u = s.umin[a] + (w * (th + (REAL)1)) * (REAL)0.5;
        const REAL scale = w * (REAL)0.5;
        const REAL sech2 = (REAL)1 - th * th;
        const REAL du_dv = scale * sech2;
        const REAL d2u = scale * (((REAL)-2 * th) * sech2);
        const REAL e = trk ? u - Uref[o] : u;
        const REAL r2 = (REAL)2 * c.R[a];
        if (U) U[o] = u;
        if (dU) dU[o] = du_dv;
        if (lv) lv[o] = (r2 * e) * du_dv;
        if (lvv) lvv[o] = r2 * (du_dv * du_dv + e * d2u);
      }
    }
}

/* total_cost core/ocp.py:63-85 with the typed stage / terminal costs (FN(traj_cost)): J = sum_k l_k + phi_N
 * per trajectory, SoA tapes in (X [N+1][4][B], U [N][2][B], refs only for TRACK). */
void FN(oracle_tape_cost)(const dtmpc_spec* sp, const dtmpc_cost* cp, long long B, const REAL* X, const REAL* U,
                          const REAL* Xref, const REAL* Uref, REAL* J) {
  SPEC_T s;
  COST_T c;
  FN(spec_from)(sp, &s);
  FN(cost_from)(cp, &c);
  const int N = s.N, trk = c.kind == DTMPC_COST_TRACK;
  REAL* Xa = (REAL*)malloc(sizeof(REAL) * 4 * (N + 1));
  REAL* Ua = (REAL*)malloc(sizeof(REAL) * 2 * N);
  REAL* Xr = (REAL*)malloc(sizeof(REAL) * 3 * (N + 1));
  REAL* Ur = (REAL*)malloc(sizeof(REAL) * 2 * N);
  for (long long i = 0; i < B; ++i) {
    FN(gather)(X, N + 1, 4, B, i, Xa);
    FN(gather)(U, N, 2, B, i, Ua);
    if (trk) {
      FN(gather)(Xref, N + 1, 3, B, i, Xr);
      FN(gather)(Uref, N, 2, B, i, Ur);
    }
    J[i] = FN(traj_cost)(&s, &c, Xa, Ua, trk ? Xr : NULL, trk ? Ur : NULL);
  }
  free(Xa);
  free(Ua);
  free(Xr);
  free(Ur);
}

#undef SPEC_T
#undef COST_T
