// dtmpc_receding.hip — batched receding-horizon nominal MPC (run_nominal.py:204-415): B independent
// closed loops (iLQR with the angle-wrapped nominal cost -> apply u0 -> DBaS plant step -> collision /
// success exits -> warm-start shift), the WHOLE task horizon in one launch.  One lane per trajectory;
// a lane whose run has ended (collision, success, failure) simply stops, so early exits cost nothing
// for the others and there is no host round trip per step.
#include <hip/hip_runtime.h>

#include <cstring>

#include "../../include/dtmpc.h"
#include "dtmpc_host.hpp"

namespace dtmpc {

template <typename T>
struct RecedingArgs {
  int B, H;
  T success_r;   // success radius (run_nominal.py:382)
  const T* x0;   // [3][B]
  T* U;          // [N][2][B] warm start in, last shifted plan out
  T* X;          // [N+1][4][B] scratch (the current plan)
  T* K;          // [N][8][B]
  T* kf;         // [N][2][B]
  T* log;        // [H][6][B]
  int* h_ran;
  int* success_t;
  int* collided;
  int* status;
  int* iters;  // [B] total iLQR iterations of each run, or NULL
};

// true min_i h_i(x) over the circles (run_nominal.py:390-396)
template <typename T>
__device__ __forceinline__ T h_true_min(const DSpec<T>& s, T px, T py) {
  T m = h_circle_exact(s, 0, px, py);
  for (int i = 1; i < s.M; ++i) m = m_min(m, h_circle_exact(s, i, px, py));
  return m;
}

template <typename T, int NA>
__global__ void __launch_bounds__(kBlock) receding_kernel(DSpec<T> s, DCost<T> c, DIlqr<T> cfg, RecedingArgs<T> a) {
  const int B = a.B;
  const int N = s.N;
  int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= B) return;
  const size_t nb = (size_t)B;
  Col<T> X = col<T>(a.X, i, B), U = col<T>(a.U, i, B), K = col<T>(a.K, i, B), kf = col<T>(a.kf, i, B),
         lg = col<T>(a.log, i, B);
  Col<T> none = col<T>((void*)nullptr, i, B);
  const bool has_obs = s.agg != DTMPC_OBS_NONE && s.M > 0;
  T x[4] = {a.x0[i], a.x0[nb + i], a.x0[2 * nb + i], T(0)};
  x[3] = barrier_of_state(s, x[0], x[1]);  // dbas_init_b0 (:279)
  int st = 0, ran = a.H, sidx = -1, coll = 0, itot = 0;
  Prof pr;
  for (int t = 0; t < a.H; ++t) {
    int it = 0;
    st |= ilqr_traj<T, NA>(s, c, cfg, x, X, U, GainsSoA<T>{K, kf}, none, 0, none, it, pr, 0);
    itot += it;
    T u0[1] = {U.at(0, 2, 0)}, u1[1] = {U.at(0, 2, 1)};
    lg.at(t, 6, 0) = x[0];
    lg.at(t, 6, 1) = x[1];
    lg.at(t, 6, 2) = x[2];
    lg.at(t, 6, 3) = u0[0];
    lg.at(t, 6, 4) = u1[0];
    lg.at(t, 6, 5) = x[3];
    if (st) {
      ran = t + 1;
      break;
    }
    if (has_obs && h_true_min(s, x[0], x[1]) <= T(0)) {  // collision (:388-397)
      coll = 1;
      ran = t + 1;
      break;
    }
    T ex = x[0] - c.t0, ey = x[1] - c.t1;
    if (sqrt(ex * ex + ey * ey) <= a.success_r) {  // success: ||x[:2] - target[:2]|| <= r (:399-403)
      sidx = t;
      ran = t + 1;
      break;
    }
    // x <- f_hat(x, u0) (:377-378), U <- [U[1:], U[-1]] (:405-406)
    T p0[1] = {x[0]}, p1[1] = {x[1]}, p2[1] = {x[2]}, pb[1] = {x[3]};
    T Bc[1] = {barrier_of_state(s, x[0], x[1])};
    fhat_vec<T, 1>(s, p0, p1, p2, pb, u0, u1, Bc);
    x[0] = p0[0];
    x[1] = p1[0];
    x[2] = p2[0];
    x[3] = pb[0];
    for (int k = 0; k + 1 < N; ++k) {
      U.at(k, 2, 0) = U.at(k + 1, 2, 0);
      U.at(k, 2, 1) = U.at(k + 1, 2, 1);
    }
  }
  a.h_ran[i] = ran;
  a.success_t[i] = sidx;
  a.collided[i] = coll;
  a.status[i] |= st;
  if (a.iters) a.iters[i] = itot;
}

template <typename T>
static int launch_receding(const dtmpc_spec* sp, const dtmpc_cost* cp, const dtmpc_ilqr_cfg* cf, int64_t B, int H,
                           double success_r, const void* x0, void* U, void* log, int* h_ran, int* success_t,
                           int* collided, int* status, int* iters, void* work, hipStream_t st) {
  DSpec<T> s = make_spec<T>(*sp);
  DCost<T> c = make_cost<T>(*cp);
  DIlqr<T> cfg = make_ilqr<T>(*cf);
  const int N = sp->horizon;
  const size_t nb = (size_t)B;
  RecedingArgs<T> a;
  std::memset(&a, 0, sizeof(a));
  a.B = (int)B;
  a.H = H;
  a.success_r = T(success_r);
  a.x0 = (const T*)x0;
  a.U = (T*)U;
  a.X = (T*)work;
  a.K = a.X + (size_t)(N + 1) * 4 * nb;
  a.kf = a.K + (size_t)N * 8 * nb;
  a.log = (T*)log;
  a.h_ran = h_ran;
  a.success_t = success_t;
  a.collided = collided;
  a.status = status;
  a.iters = iters;
  switch (cfg.nc) {
#define CASE(n)                                                                                     \
  case n: hipLaunchKernelGGL((receding_kernel<T, n>), grid_for(B), dim3(kBlock), 0, st, s, c, cfg, a); break;
    DTMPC_NA_CASES(CASE)
#undef CASE
    default: return set_err(DTMPC_ERR_BAD_ARG, "n_alphas out of range");
  }
  return check_launch("receding_kernel");
}

}  // namespace dtmpc

using namespace dtmpc;

extern "C" {

size_t dtmpc_receding_workspace_bytes(int dtype, int32_t horizon, int64_t B) {
  if (horizon < 1 || B < 1) return 0;
  size_t el = dtype == DTMPC_F64 ? 8 : 4;
  const size_t generic = el * ((size_t)(horizon + 1) * 4 + (size_t)horizon * 10) * (size_t)B;
  // the fused driver's records (csrc/dtmpc_fast.hip receding_fast_kernel) need more: the larger of the two
  const size_t fused = dtype == DTMPC_F64 ? receding_fast_workspace_bytes64(horizon, B) : receding_fast_workspace_bytes(horizon, B);
  return generic > fused ? generic : fused;
}

int dtmpc_nominal_receding_it(int dtype, const dtmpc_spec* spec, const dtmpc_cost* cost, const dtmpc_ilqr_cfg* cfg,
                              int64_t B, int32_t H, double success_radius, const void* x0, void* U, void* log,
                              int32_t* h_ran, int32_t* success_t, int32_t* collided, int32_t* status, int32_t* iters,
                              void* work, void* stream) {
  int e = check_spec(spec, B);
  if (e) return e;
  if ((e = check_ilqr(cfg))) return e;
  if (!cost || cost->kind != DTMPC_COST_TARGET) return set_err(DTMPC_ERR_BAD_ARG, "cost must be DTMPC_COST_TARGET");
  if (H < 1) return set_err(DTMPC_ERR_BAD_ARG, "H must be >= 1");
  if ((int64_t)H * 6 * B >= (int64_t)1 << 31) return set_err(DTMPC_ERR_BAD_ARG, "H * B too large for 32-bit log offsets");
  if (!x0 || !U || !log || !h_ran || !success_t || !collided || !status || !work)
    return set_err(DTMPC_ERR_BAD_ARG, "NULL array");
  hipStream_t st = (hipStream_t)stream;
  // the paper configuration on the fused solver (DTMPC_FAST=0 / DTMPC_FAST64=0: the generic one below)
  if (receding_fast_eligible(dtype, spec, cost, cfg))
    return launch_receding_fast(spec, cost, cfg, B, H, success_radius, x0, U, log, h_ran, success_t, collided, status,
                                iters, work, st);
  if (receding_fast_eligible64(dtype, spec, cost, cfg))
    return launch_receding_fast64(spec, cost, cfg, B, H, success_radius, x0, U, log, h_ran, success_t, collided,
                                  status, iters, work, st);
  if (dtype == DTMPC_F32)
    return launch_receding<float>(spec, cost, cfg, B, H, success_radius, x0, U, log, h_ran, success_t, collided, status,
                                  iters, work, st);
  if (dtype == DTMPC_F64)
    return launch_receding<double>(spec, cost, cfg, B, H, success_radius, x0, U, log, h_ran, success_t, collided,
                                   status, iters, work, st);
  return set_err(DTMPC_ERR_BAD_ARG, "bad dtype");
}

int dtmpc_nominal_receding(int dtype, const dtmpc_spec* spec, const dtmpc_cost* cost, const dtmpc_ilqr_cfg* cfg,
                           int64_t B, int32_t H, double success_radius, const void* x0, void* U, void* log,
                           int32_t* h_ran, int32_t* success_t, int32_t* collided, int32_t* status, void* work,
                           void* stream) {
  return dtmpc_nominal_receding_it(dtype, spec, cost, cfg, B, H, success_radius, x0, U, log, h_ran, success_t, collided,
                                   status, nullptr, work, stream);
}

}  // extern "C"
