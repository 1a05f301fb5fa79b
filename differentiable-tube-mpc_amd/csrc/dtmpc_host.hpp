// dtmpc_host.hpp — host-side helpers shared by the translation units of libdtmpc.so:
// C struct -> typed device descriptor conversion, argument checks, launch error reporting.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

#include "../../include/dtmpc.h"
#include "dtmpc_general.hpp"

namespace dtmpc {

constexpr int kBlock = 256;

// Line-search candidate counts the kernels are instantiated for (1..8).  -DDTMPC_NA_ONLY=n builds
// only n (experiment variants of the library: a quarter of the compile time; other counts then
// return DTMPC_ERR_BAD_ARG).
#ifdef DTMPC_NA_ONLY
#define DTMPC_NA_CASES(C) C(DTMPC_NA_ONLY)
#else
#define DTMPC_NA_CASES(C) C(1) C(2) C(3) C(4) C(5) C(6) C(7) C(8)
#endif

// ---------------------------------------------------------------------------------------------
// host-side conversion of the C structs into the typed device descriptors
template <typename T>
inline DSpec<T> make_spec(const dtmpc_spec& p) {
  DSpec<T> s;
  std::memset(&s, 0, sizeof(s));
  s.N = p.horizon;
  s.M = p.n_obstacles;
  s.agg = p.obs_aggregation;
  s.barrier = p.barrier_type;
  s.dt = T(p.dt);
  s.umin0 = T(p.u_min[0]);
  s.umin1 = T(p.u_min[1]);
  s.umax0 = T(p.u_max[0]);
  s.umax1 = T(p.u_max[1]);
  s.active_tol = T(p.active_tol);
  s.neg_beta = T(-p.obs_beta);
  s.neg_inv_beta = T(-(1.0 / p.obs_beta));
  s.alpha = T(p.dbas_alpha);
  s.gamma = T(p.dbas_gamma);
  s.eps = T(p.dbas_eps);
  s.tight = T(p.h_offset);
  for (int i = 0; i < p.n_obstacles && i < DTMPC_MAX_OBS; ++i) {
    s.cx[i] = T(p.obs_cx[i]);
    s.cy[i] = T(p.obs_cy[i]);
    s.r2[i] = T(p.obs_r[i] * p.obs_r[i]);
  }
  return s;
}

template <typename T>
inline DCost<T> make_cost(const dtmpc_cost& c) {
  DCost<T> o;
  o.kind = c.kind;
  o.wrap = c.wrap_angle;
  o.Q0 = T(c.Q[0]);
  o.Q1 = T(c.Q[1]);
  o.Q2 = T(c.Q[2]);
  o.R0 = T(c.R[0]);
  o.R1 = T(c.R[1]);
  o.Qf0 = T(c.Qf[0]);
  o.Qf1 = T(c.Qf[1]);
  o.Qf2 = T(c.Qf[2]);
  o.qb = T(c.qb);
  o.t0 = T(c.target[0]);
  o.t1 = T(c.target[1]);
  o.t2 = T(c.target[2]);
  return o;
}

template <typename T>
inline DIlqr<T> make_ilqr(const dtmpc_ilqr_cfg& c) {
  DIlqr<T> o;
  std::memset(&o, 0, sizeof(o));
  o.max_iter = c.max_iter;
  o.na = c.n_alphas;
  o.tol = T(c.tol);
  o.reg = T(c.reg);
  for (int a = 0; a < DTMPC_MAX_ALPHAS; ++a) o.alphas[a] = T(c.alphas[a]);
  o.zpos = -1;
  o.nc = 0;
  for (int a = 0; a < c.n_alphas; ++a) {
    if (c.alphas[a] == 0.0) {
      if (o.zpos < 0) o.zpos = a;
    } else {
      o.cpos[o.nc] = a;
      o.calphas[o.nc] = T(c.alphas[a]);
      ++o.nc;
    }
  }
  if (o.nc == 0) {  // only zero alphas: roll them out like any other candidate
    o.zpos = -1;
    o.nc = c.n_alphas;
    for (int a = 0; a < c.n_alphas; ++a) {
      o.cpos[a] = a;
      o.calphas[a] = T(c.alphas[a]);
    }
  }
  return o;
}

template <typename T>
__device__ __forceinline__ Col<T> col(void* p, int64_t i, int B) {
  Col<T> c;
  c.base = reinterpret_cast<T*>(p);
  c.ld = (unsigned)B;
  c.lane = (unsigned)i;
  return c;
}
template <typename T>
__device__ __forceinline__ Col<T> col(const void* p, int64_t i, int B) {
  return col<T>(const_cast<void*>(p), i, B);
}

// last-error text, shared by every translation unit of libdtmpc.so (inline function static)
inline char* err_buf() {
  static thread_local char buf[512] = "";
  return buf;
}

inline int set_err(int code, const char* msg) {
  std::snprintf(err_buf(), 512, "%s", msg);
  return code;
}

inline int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    std::snprintf(err_buf(), 512, "%s: %s", what, hipGetErrorString(e));
    return DTMPC_ERR_HIP;
  }
  return DTMPC_OK;
}

inline int check_spec(const dtmpc_spec* s, int64_t B) {
  if (!s) return set_err(DTMPC_ERR_BAD_ARG, "spec is NULL");
  if (s->horizon < 1 || s->horizon > DTMPC_MAX_HORIZON) return set_err(DTMPC_ERR_BAD_ARG, "horizon out of range");
  if (s->n_obstacles < 0 || s->n_obstacles > DTMPC_MAX_OBS) return set_err(DTMPC_ERR_BAD_ARG, "n_obstacles out of range");
  if (s->obs_aggregation < 0 || s->obs_aggregation > DTMPC_OBS_NONE) return set_err(DTMPC_ERR_BAD_ARG, "bad obs_aggregation");
  if (s->barrier_type != DTMPC_BARRIER_INVERSE && s->barrier_type != DTMPC_BARRIER_LOG) return set_err(DTMPC_ERR_BAD_ARG, "bad barrier_type");
  if (s->dbas_alpha < 0) return set_err(DTMPC_ERR_BAD_ARG, "alpha must be >= 0");
  if (!(s->dbas_gamma >= -1.0 && s->dbas_gamma <= 1.0)) return set_err(DTMPC_ERR_BAD_ARG, "gamma must be in [-1, 1]");
  if (s->obs_aggregation == DTMPC_OBS_SMOOTHMIN && !(s->obs_beta > 0)) return set_err(DTMPC_ERR_BAD_ARG, "obs_beta must be > 0");
  if (B < 1) return set_err(DTMPC_ERR_BAD_ARG, "batch must be >= 1");
  // 32-bit in-kernel offsets: (rows * fields) * B must fit
  if ((int64_t)(s->horizon + 1) * 20 * B >= (int64_t)1 << 31) return set_err(DTMPC_ERR_BAD_ARG, "batch too large for 32-bit tape offsets");
  return DTMPC_OK;
}

inline int check_ilqr(const dtmpc_ilqr_cfg* c) {
  if (!c) return set_err(DTMPC_ERR_BAD_ARG, "ilqr cfg is NULL");
  if (c->n_alphas < 1 || c->n_alphas > DTMPC_MAX_ALPHAS) return set_err(DTMPC_ERR_BAD_ARG, "n_alphas out of range");
  if (c->max_iter < 0) return set_err(DTMPC_ERR_BAD_ARG, "max_iter must be >= 0");
  return DTMPC_OK;
}

inline int check_cost(const dtmpc_cost* c, const void* Xref, const void* Uref) {
  if (!c) return set_err(DTMPC_ERR_BAD_ARG, "cost is NULL");
  if (c->kind != DTMPC_COST_TARGET && c->kind != DTMPC_COST_TRACK) return set_err(DTMPC_ERR_BAD_ARG, "bad cost kind");
  if (c->kind == DTMPC_COST_TRACK && (!Xref || !Uref)) return set_err(DTMPC_ERR_BAD_ARG, "tracking cost needs Xref and Uref");
  return DTMPC_OK;
}

inline dim3 grid_for(int64_t B) { return dim3((unsigned)((B + kBlock - 1) / kBlock)); }

// Threads per workgroup of the fused kernels (tube step, standalone iLQR, general solves) for B
// trajectories at `lanes`: 64 -- one wave per workgroup, so the waves spread over every CU -- while the
// launch has fewer waves than the device has SIMDs, else 256.  (A 256-thread launch of 4,096 trajectories
// at four lanes puts its 256 waves on 64 CUs, four per CU, and leaves 192 CUs idle.)  The tube step's
// partial-sum rows are per workgroup: dtmpc_tube_partials_count follows this rule.
// -D DTMPC_TUBE_SMALL_BLOCK=0: always 256 (A/B builds).
int tube_block(int64_t B, int lanes);

// the specialised tube step of the paper configuration (dtmpc_fast.hip)
bool tube_fast_eligible(int dtype, const dtmpc_spec* sp, const dtmpc_tube_cfg* cf);
// largest chunk (trajectories per launch) whose per-lane records fit one buffer resource at `lanes`
int64_t tube_fast_chunk_max(int N, int lanes);
size_t tube_fast_workspace_bytes(int N, int64_t B, int lanes, int64_t chunk);
int launch_tube_fast(const dtmpc_spec* sp, const dtmpc_tube_cfg* cf, int64_t B, int64_t goff, int64_t step,
                     const dtmpc_tube_state* S, const void* w, hipStream_t st);
// the same tube step in f64 (dtmpc_fast64.hip: dtmpc_fast.hip with real = double); its chunk is clamped to
// tube_fast_chunk_max64 at launch
bool tube_fast_eligible64(int dtype, const dtmpc_spec* sp, const dtmpc_tube_cfg* cf);
// false for the f64 instantiations the fused step does not run: none since round 5 v3 (DTMPC_FAST64_L4G=0, an A/B
// switch, routes the general gain records at four lanes to the generic f64 kernel)
bool tube_fast_lanes_ok64(const dtmpc_spec* sp, int lanes);
int64_t tube_fast_chunk_max64(int N, int lanes);
size_t tube_fast_workspace_bytes64(int N, int64_t B, int lanes, int64_t chunk);
int launch_tube_fast64(const dtmpc_spec* sp, const dtmpc_tube_cfg* cf, int64_t B, int64_t goff, int64_t step,
                       const dtmpc_tube_state* S, const void* w, hipStream_t st);
// the standalone batched iLQR on the same configuration (dtmpc_ilqr_solve_ws)
bool ilqr_fast_eligible(int dtype, const dtmpc_spec* sp, const dtmpc_cost* c, const dtmpc_ilqr_cfg* cf);
size_t ilqr_fast_workspace_bytes(int N, int64_t B, int lanes);
int launch_ilqr_fast(const dtmpc_spec* sp, const dtmpc_cost* cp, const dtmpc_ilqr_cfg* cf, int64_t B, const void* x0,
                     const void* Xref, const void* Uref, void* X, void* U, void* K, void* kff, int* iters, int* status,
                     signed char* choices, void* costs, int lanes, void* work, size_t work_bytes, hipStream_t st);
// ... and in f64 (dtmpc_fast64_ilqr.hip)
bool ilqr_fast_eligible64(int dtype, const dtmpc_spec* sp, const dtmpc_cost* c, const dtmpc_ilqr_cfg* cf);
size_t ilqr_fast_workspace_bytes64(int N, int64_t B, int lanes);
int launch_ilqr_fast64(const dtmpc_spec* sp, const dtmpc_cost* cp, const dtmpc_ilqr_cfg* cf, int64_t B, const void* x0,
                       const void* Xref, const void* Uref, void* X, void* U, void* K, void* kff, int* iters, int* status,
                       signed char* choices, void* costs, int lanes, void* work, size_t work_bytes, hipStream_t st);
// the receding-horizon driver on the same solver (dtmpc_nominal_receding), f32 and f64 (dtmpc_fast*_ilqr.hip)
bool receding_fast_eligible(int dtype, const dtmpc_spec* sp, const dtmpc_cost* c, const dtmpc_ilqr_cfg* cf);
size_t receding_fast_workspace_bytes(int N, int64_t B);
int launch_receding_fast(const dtmpc_spec* sp, const dtmpc_cost* cp, const dtmpc_ilqr_cfg* cf, int64_t B, int H,
                         double success_r, const void* x0, void* U, void* log, int* h_ran, int* success_t,
                         int* collided, int* status, int* iters, void* work, hipStream_t st);
bool receding_fast_eligible64(int dtype, const dtmpc_spec* sp, const dtmpc_cost* c, const dtmpc_ilqr_cfg* cf);
size_t receding_fast_workspace_bytes64(int N, int64_t B);
int launch_receding_fast64(const dtmpc_spec* sp, const dtmpc_cost* cp, const dtmpc_ilqr_cfg* cf, int64_t B, int H,
                           double success_r, const void* x0, void* U, void* log, int* h_ran, int* success_t,
                           int* collided, int* status, int* iters, void* work, hipStream_t st);
// the general path's two solves on the same solver (dtmpc_general_step); per-trajectory solve status to sst
bool general_fast_eligible(int dtype, const dtmpc_spec* sp, const dtmpc_general_cfg* cf);
int launch_general_solve_fast(const dtmpc_spec* sp, const dtmpc_general_cfg* cf, int64_t B,
                              const dtmpc_general_state* S, int* sst, hipStream_t st);
// ... and in f64 (dtmpc_fast64_general.hip)
bool general_fast_eligible64(int dtype, const dtmpc_spec* sp, const dtmpc_general_cfg* cf);
int launch_general_solve_fast64(const dtmpc_spec* sp, const dtmpc_general_cfg* cf, int64_t B,
                                const dtmpc_general_state* S, int* sst, hipStream_t st);

}  // namespace dtmpc
