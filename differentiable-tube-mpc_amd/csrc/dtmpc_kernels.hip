// dtmpc_kernels.hip — HIP kernels (gfx950) + the C ABI of include/dtmpc.h.
//
// One lane = one trajectory; 256-lane workgroups; grid = ceil(B / 256).  All arrays are SoA
// [step][field][B] (include/dtmpc.h), so lane i of a wave touches element i of every 256 B line.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "../../include/dtmpc.h"
#include "dtmpc_host.hpp"

namespace dtmpc {

// ---------------------------------------------------------------------------------------------
// KAT-level kernels

template <typename T>
__global__ void __launch_bounds__(kBlock) rollout_kernel(DSpec<T> s, int B, const void* x0,
                                                         const void* U, void* X) {
  int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= B) return;
  Col<T> cx0 = col<T>(x0, i, B);
  T xs[4] = {cx0.at(0, 4, 0), cx0.at(0, 4, 1), cx0.at(0, 4, 2), cx0.at(0, 4, 3)};
  rollout_traj(s, xs, col<T>(X, i, B), col<T>(U, i, B));
}

template <typename T>
__global__ void __launch_bounds__(kBlock) dbas_init_kernel(DSpec<T> s, int B, const T* x, T* b) {
  int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= B) return;
  b[i] = barrier_of_state(s, x[i], x[(size_t)B + i]);
}

// episode start of the fused closed loop in one launch (core/tube_mpc.py:770-779): x = xbar = x0 (given
// trajectory-major [B][3], the reference's layout), b = bbar = B(h(x0)), zero warm starts (both
// [N][2][B] tapes: each lane clears its own column), status 0; lane 0 restores theta and clears the
// momentum
template <typename T>
__global__ void __launch_bounds__(kBlock) tube_reset_kernel(DSpec<T> s, int B, const T* x0, T* x, T* b, T* xbar,
                                                            T* bbar, T* Unom, T* Uaux, int* status,
                                                            const T* theta0, T* theta, T* vel) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i == 0)
    for (int j = 0; j < 6; ++j) {
      theta[j] = theta0[j];
      vel[j] = T(0);
    }
  if (i >= B) return;
  const size_t nb = (size_t)B;
  const T p0 = x0[3 * (size_t)i], p1 = x0[3 * (size_t)i + 1], p2 = x0[3 * (size_t)i + 2];
  x[i] = xbar[i] = p0;
  x[nb + i] = xbar[nb + i] = p1;
  x[2 * nb + i] = xbar[2 * nb + i] = p2;
  b[i] = bbar[i] = barrier_of_state(s, p0, p1);
  for (int r = 0; r < 2 * s.N; ++r) {
    Unom[r * nb + i] = T(0);
    Uaux[r * nb + i] = T(0);
  }
  status[i] = 0;
}

// dense A [N][16], Bm [N][8], lx [N+1][4], lu [N][2] (dubins_augmented_jacobian + cost derivs)
template <typename T>
__global__ void __launch_bounds__(kBlock) linearize_kernel(DSpec<T> s, DCost<T> c, int B,
                                                           const void* Xp, const void* Up,
                                                           const void* Xrp, const void* Urp,
                                                           void* Ap, void* Bp, void* lxp, void* lup) {
  int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= B) return;
  const int N = s.N;
  Col<T> X = col<T>(Xp, i, B), U = col<T>(Up, i, B), Xr = col<T>(Xrp, i, B), Ur = col<T>(Urp, i, B);
  Col<T> A = col<T>(Ap, i, B), Bm = col<T>(Bp, i, B), LX = col<T>(lxp, i, B), LU = col<T>(lup, i, B);
  T lxx[4], luu[2], pxx[4];
  cost_diag(c, lxx, luu, pxx);
  T r0, r1, r2, d0, d1, d2;
  for (int k = 0; k < N; ++k) {
    T x0 = X.at(k, 4, 0), x1 = X.at(k, 4, 1), x2 = X.at(k, 4, 2), xb = X.at(k, 4, 3);
    T u0 = U.at(k, 2, 0), u1 = U.at(k, 2, 1);
    T sn, cs;
    m_sincos(x2, &sn, &cs);
    T gxk, gyk, gxn, gyn;
    T hk = h_grad(s, x0, x1, gxk, gyk);
    T dv = s.dt * u0;
    T n0 = x0 + dv * cs, n1 = x1 + dv * sn;
    T hn = h_grad(s, n0, n1, gxn, gyn);
    Jac<T> J = make_jac(s, sn, cs, u0, gxk, gyk, dbarrier_relaxed(s, hk), gxn, gyn,
                        dbarrier_relaxed(s, hn));
    T Ad[16] = {T(1), T(0), J.a02, T(0), T(0), T(1), J.a12, T(0),
                T(0), T(0), T(1),  T(0), J.a30, J.a31, J.a32, J.g};
    T Bd[8] = {J.b00, T(0), J.b10, T(0), T(0), J.b21, J.b30, J.b31};
#pragma unroll
    for (int j = 0; j < 16; ++j) A.at(k, 16, j) = Ad[j];
#pragma unroll
    for (int j = 0; j < 8; ++j) Bm.at(k, 8, j) = Bd[j];
    load_ref(c, Xr, 3, k, r0, r1, r2);
    deriv_dx(c, x0, x1, x2, r0, r1, r2, d0, d1, d2);
    LX.at(k, 4, 0) = lxx[0] * d0;
    LX.at(k, 4, 1) = lxx[1] * d1;
    LX.at(k, 4, 2) = lxx[2] * d2;
    LX.at(k, 4, 3) = lxx[3] * xb;
    T q0, q1;
    load_uref(c, Ur, k, q0, q1);
    if (c.kind == DTMPC_COST_TRACK) {
      LU.at(k, 2, 0) = luu[0] * (u0 - q0);
      LU.at(k, 2, 1) = luu[1] * (u1 - q1);
    } else {
      LU.at(k, 2, 0) = luu[0] * u0;
      LU.at(k, 2, 1) = luu[1] * u1;
    }
  }
  load_ref(c, Xr, 3, N, r0, r1, r2);
  deriv_dx(c, T(X.at(N, 4, 0)), T(X.at(N, 4, 1)), T(X.at(N, 4, 2)), r0, r1, r2, d0, d1, d2);
  LX.at(N, 4, 0) = pxx[0] * d0;
  LX.at(N, 4, 1) = pxx[1] * d1;
  LX.at(N, 4, 2) = pxx[2] * d2;
  LX.at(N, 4, 3) = pxx[3] * X.at(N, 4, 3);
}

// ---------------------------------------------------------------------------------------------
// solver kernels

template <typename T, int NA>
__global__ void __launch_bounds__(kBlock) ilqr_kernel(DSpec<T> s, DCost<T> c, DIlqr<T> cfg, int B,
                                                      const void* x0p, const void* Xrp,
                                                      const void* Urp, void* Xp, void* Up,
                                                      void* Kp, void* kfp, int* iters, int* status,
                                                      signed char* choices) {
  int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= B) return;
  Col<T> cx0 = col<T>(x0p, i, B);
  T x0[4] = {cx0.at(0, 4, 0), cx0.at(0, 4, 1), cx0.at(0, 4, 2), cx0.at(0, 4, 3)};
  int it = 0;
  Prof pr;
  pr.start();
  int st = ilqr_traj<T, NA>(s, c, cfg, x0, col<T>(Xp, i, B), col<T>(Up, i, B),
                            GainsSoA<T>{col<T>(Kp, i, B), col<T>(kfp, i, B)}, col<T>(Xrp, i, B), 3,
                            col<T>(Urp, i, B), it, pr, 0, 0, choices ? choices + i : nullptr, (size_t)B);
  pr.flush();
  if (iters) iters[i] = it;
  if (status) status[i] |= st;
}

template <typename T, bool LAMBDA>
__global__ void __launch_bounds__(kBlock) sens_kernel(DSpec<T> s, DCost<T> c, int B, const void* Xp,
                                                      const void* Up, const void* Xrp,
                                                      const void* Urp, const void* Xbp, void* dXp,
                                                      void* dUp, void* dLp, void* work,
                                                      int* status) {
  int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= B) return;
  const int N = s.N;
  T* w = reinterpret_cast<T*>(work);
  const size_t nb = (size_t)B;
  void* Kp = w;
  void* kfp = w + (size_t)N * 8 * nb;
  void* ABp = w + (size_t)N * 10 * nb;
  void* VVp = w + (size_t)N * 20 * nb;
  int st = sens_traj<T, LAMBDA, true, false>(
      s, c, col<T>(Xp, i, B), col<T>(Up, i, B), col<T>(Xrp, i, B), 3, col<T>(Urp, i, B),
      col<T>(Xbp, i, B), 3, col<T>(Kp, i, B), col<T>(kfp, i, B), col<T>(ABp, i, B),
      col<T>(VVp, i, B), col<T>(dXp, i, B), col<T>(dUp, i, B), col<T>(dLp, i, B), nullptr);
  if (status) status[i] |= st;
}

// upper loss + DOC gradient per trajectory (core/tube_mpc.py:915-919, 963-976); out [7][B]
template <typename T>
__global__ void __launch_bounds__(kBlock) docgrad_kernel(int N, int B, const void* Xap,
                                                         const void* Uap, const void* Xnp,
                                                         const void* Unp, const void* dXp,
                                                         const void* dUp, void* outp) {
  int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= B) return;
  Col<T> Xa = col<T>(Xap, i, B), Ua = col<T>(Uap, i, B), Xn = col<T>(Xnp, i, B),
         Un = col<T>(Unp, i, B), dX = col<T>(dXp, i, B), dU = col<T>(dUp, i, B),
         o = col<T>(outp, i, B);
  T L1 = 0, L2 = 0, g0 = 0, g1 = 0, g2 = 0, r0 = 0, r1 = 0, gb = 0;
  for (int k = 0; k <= N; ++k) {
    T e0 = Xa.at(k, 4, 0) - Xn.at(k, 4, 0), e1 = Xa.at(k, 4, 1) - Xn.at(k, 4, 1),
      e2 = Xa.at(k, 4, 2) - Xn.at(k, 4, 2), bb = Xa.at(k, 4, 3);
    L1 += e0 * e0 + e1 * e1 + e2 * e2;
    L2 += bb * bb;
    g0 += T(2) * e0 * dX.at(k, 4, 0);
    g1 += T(2) * e1 * dX.at(k, 4, 1);
    g2 += T(2) * e2 * dX.at(k, 4, 2);
    gb += T(2) * bb * dX.at(k, 4, 3);
    if (k < N) {
      r0 += T(2) * (Ua.at(k, 2, 0) - Un.at(k, 2, 0)) * dU.at(k, 2, 0);
      r1 += T(2) * (Ua.at(k, 2, 1) - Un.at(k, 2, 1)) * dU.at(k, 2, 1);
    }
  }
  o.at(0, 1, 0) = L1 + L2;
  o.at(1, 1, 0) = g0;
  o.at(2, 1, 0) = g1;
  o.at(3, 1, 0) = g2;
  o.at(4, 1, 0) = r0;
  o.at(5, 1, 0) = r1;
  o.at(6, 1, 0) = gb;
}

// ---------------------------------------------------------------------------------------------
// fused closed-loop step (core/tube_mpc.py:803-1023 loop body)

template <typename T>
struct TubeArgs {
  int B;
  int64_t goff, step;
  T* x;
  T* b;
  T* xbar;
  T* bbar;
  T* Xnom;
  T* Unom;
  T* Xaux;
  T* Uaux;
  T* work;
  const T* theta;
  T* partials;
  T* log;
  int* status;
  int* iters;
  const T* w;
  int disturbance, write_log;
  uint64_t seed;
  T wlo[3], whi[3];
  signed char* choices;  // [nom max_iter + aux max_iter][B] or NULL
  T gbound;              // health bound on the gradient row (+inf: none)
};


// Lanes per trajectory, chosen per batch when the caller builds its state (dtmpc_tube_lanes; the
// generic kernel below takes LPT = 1 or 2, the f32 fast kernel 1, 2 or 4).  At the benchmark batch
// (65,536 trajectories) one lane per trajectory is exactly one wave per SIMD; two lanes (paired line
// search: each lane of a pair rolls out half the candidates, the rest of the step is computed
// identically by both) measured 8.27 vs 7.54 ms there -- the duplicated work outweighs the overlap.
// Below the lane slots the machine is mostly idle and the step is ONE wave's latency, which more lanes
// per trajectory cut: 4 lanes while 8 B <= (SIMDs x 64) lane slots of the current device (MI355X: 256
// CUs x 4 SIMDs x 64 = 65,536, i.e. B <= 8,192: measured 2.22 / 2.30 ms at B = 4,096 / 8,192 against
// 2.92 / 2.93 at two lanes; at B = 16,384 four lanes fill every SIMD with duplicated backward work and
// lose, 3.76 vs 3.06 ms), 2 while 2 B <= slots (B <= 32,768).  The generic
// kernel runs a 4-lane state with LPT = 2.  DTMPC_TUBE_LANES=1|2|4 (environment) forces a count, for
// the parity tests; it is read by dtmpc_tube_lanes only, i.e. once, when the caller builds its state
// (state->lanes).  Without a device (host-side tests) the MI355X count is assumed.
static int64_t lane_slots() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      cus <= 0) {
    (void)hipGetLastError();
    cus = 256;
  }
  return (int64_t)cus * 4 * 64;
}

#ifndef DTMPC_TUBE_SMALL_BLOCK
#define DTMPC_TUBE_SMALL_BLOCK 1
#endif
int tube_block(int64_t B, int lanes) {
  return (DTMPC_TUBE_SMALL_BLOCK && B * lanes < lane_slots()) ? 64 : kBlock;
}

// f64 (round 5): the fused f64 step is instruction-bound at every batch (no packed f64 VALU), so four lanes --
// the line search split four ways, the linearisation shared -- pay for their duplicated Riccati recursion up to
// 4 B <= slots (B <= 16,384: 8.11 ms at four lanes vs 8.83 at two, profiles/r04/f64_lanes_v5.txt); round 6: two lanes
// while 2 B <= slots (B = 32,768: 7.36 ms at two lanes vs 9.87 at one, profiles/r06/f64_lanes_v1.txt), above it one
// lane (B = 65,536: 11.45 ms vs 14.95 at two).
static int tube_lanes_default(int64_t B, int dtype = DTMPC_F32) {
  const char* e = getenv("DTMPC_TUBE_LANES");
  if (e && (e[0] == '1' || e[0] == '2' || e[0] == '4') && e[1] == 0) return e[0] - '0';
  const int64_t slots = lane_slots();
  if (dtype == DTMPC_F64) return 4 * B <= slots ? 4 : 2 * B <= slots ? 2 : 1;
  return 8 * B <= slots ? 4 : 2 * B <= slots ? 2 : 1;
}

// One wave per SIMD is all either form gets (the two-lane form runs only at small batches), so the
// full 512-register budget, no spill.
template <typename T, int NA, int LPT>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(1, 1)))
tube_step_kernel(DSpec<T> s_arg, DCost<T> cn, DIlqr<T> cfn, DIlqr<T> cfa, TubeArgs<T> a) {
  __shared__ T red[kBlock / 64][DTMPC_TUBE_SUMS];
  DSpec<T> s = s_arg;
#ifdef DTMPC_OBS_REGS
  obs_pin(s);  // obstacle table in VGPRs for the whole step (obs_tab)
#endif
  const int B = a.B;
  const int N = s.N;
  const int gl = blockIdx.x * kBlock + threadIdx.x;
  const int i = gl / LPT, hl = gl % LPT;
  T acc[DTMPC_TUBE_SUMS] = {T(0), T(0), T(0), T(0), T(0), T(0), T(0), T(0)};
  if (i < B) {
    const size_t nb = (size_t)B;
    Col<T> Xn = col<T>(a.Xnom, i, B), Un = col<T>(a.Unom, i, B), Xa = col<T>(a.Xaux, i, B),
           Ua = col<T>(a.Uaux, i, B);
    Col<T> K = col<T>(a.work, i, B), kf = col<T>(a.work + (size_t)N * 8 * nb, i, B),
           AB = col<T>(a.work + (size_t)N * 10 * nb, i, B);
    T x0 = a.x[i], x1 = a.x[nb + i], x2 = a.x[2 * nb + i], xb = a.b[i];
    T y0 = a.xbar[i], y1 = a.xbar[nb + i], y2 = a.xbar[2 * nb + i], yb = a.bbar[i];
    int st = 0, itn = 0, ita = 0;
    // nominal MPC solve (fixed weights) :813-857
    T xn0[4] = {y0, y1, y2, yb};
    Col<T> none = col<T>((void*)nullptr, i, B);
    Prof pr;
    pr.start();
    // the iLQR gains: per-lane contiguous (GainsAoS) in their own region of the workspace.  It must
    // not overlap the sensitivity's SoA scratch (K / kf / AB above): an AoS block of lane i covers
    // SoA cells of other lanes, which other waves may be writing in their sensitivity pass meanwhile.
    const GainsAoS<T> gains{a.work + (size_t)N * 20 * nb, a.work + (size_t)N * 28 * nb, (unsigned)B,
                            (unsigned)i};
    st |= ilqr_traj<T, NA, LPT>(s, cn, cfn, xn0, Xn, Un, gains, none, 0, none, itn, pr, 0, hl,
                                a.choices ? a.choices + i : nullptr, nb);
    // ancillary MPC tracking the nominal plan :863-909 (terminal weight Qa, :885, :891)
    DCost<T> ca;
    ca.kind = DTMPC_COST_TRACK;
    ca.wrap = 0;
    ca.Q0 = ca.Qf0 = a.theta[0];
    ca.Q1 = ca.Qf1 = a.theta[1];
    ca.Q2 = ca.Qf2 = a.theta[2];
    ca.R0 = a.theta[3];
    ca.R1 = a.theta[4];
    ca.qb = a.theta[5];
    ca.t0 = ca.t1 = ca.t2 = T(0);
    T xa0[4] = {x0, x1, x2, xb};
    pr.mark(8);
    st |= ilqr_traj<T, NA, LPT>(s, ca, cfa, xa0, Xa, Ua, gains, Xn, 4, Un, ita, pr, 4, hl,
                                a.choices ? a.choices + (size_t)cfn.max_iter * nb + i : nullptr, nb);
    pr.mark(8);
    // upper loss, DOC sensitivity and analytic gradient :915-976
    st |= sens_traj<T, false, false, true>(s, ca, Xa, Ua, Xn, 4, Un, Xn, 4, K, kf, AB, none, none,
                                           none, none, acc);
    pr.mark(9);
    // plant step with disturbance, nominal propagation :990-1001
    T u0 = Ua.at(0, 2, 0), u1 = Ua.at(0, 2, 1);
    T v0 = Un.at(0, 2, 0), v1 = Un.at(0, 2, 1);
    T w[3];
    if (a.disturbance == 0) {
      w[0] = a.w[i];
      w[1] = a.w[nb + i];
      w[2] = a.w[2 * nb + i];
    } else {
      uint32_t r[4];
      philox4x32_10(a.seed, (uint64_t)(a.goff + i), (uint64_t)a.step, r);
#pragma unroll
      for (int f = 0; f < 3; ++f) {
        T u = T(r[f] >> 8) * T(1.0 / 16777216.0);
        w[f] = a.wlo[f] + (a.whi[f] - a.wlo[f]) * u;
      }
    }
    if (a.write_log) {
      T* lg = a.log;
      lg[i] = x0;
      lg[nb + i] = x1;
      lg[2 * nb + i] = x2;
      lg[3 * nb + i] = u0;
      lg[4 * nb + i] = u1;
      lg[5 * nb + i] = y0;
      lg[6 * nb + i] = y1;
      lg[7 * nb + i] = y2;
      lg[8 * nb + i] = v0;
      lg[9 * nb + i] = v1;
      lg[10 * nb + i] = xb;
#pragma unroll
      for (int j = 0; j < 7; ++j) lg[(11 + j) * nb + i] = acc[j];
    }
    {
      T p0[1] = {x0}, p1[1] = {x1}, p2[1] = {x2}, pb[1] = {xb}, q0[1] = {u0}, q1[1] = {u1};
      T Bc[1] = {barrier_of_state(s, x0, x1)};
      fhat_vec<T, 1>(s, p0, p1, p2, pb, q0, q1, Bc);
      a.x[i] = p0[0] + w[0];
      a.x[nb + i] = p1[0] + w[1];
      a.x[2 * nb + i] = p2[0] + w[2];
      a.b[i] = pb[0];
    }
    {
      T p0[1] = {y0}, p1[1] = {y1}, p2[1] = {y2}, pb[1] = {yb}, q0[1] = {v0}, q1[1] = {v1};
      T Bc[1] = {barrier_of_state(s, y0, y1)};
      fhat_vec<T, 1>(s, p0, p1, p2, pb, q0, q1, Bc);
      a.xbar[i] = p0[0];
      a.xbar[nb + i] = p1[0];
      a.xbar[2 * nb + i] = p2[0];
      a.bbar[i] = pb[0];
    }
    // warm-start shift V <- [V[1:], V[-1]]  :1015-1020
    for (int k = 0; k + 1 < N; ++k) {
      Un.at(k, 2, 0) = Un.at(k + 1, 2, 0);
      Un.at(k, 2, 1) = Un.at(k + 1, 2, 1);
      Ua.at(k, 2, 0) = Ua.at(k + 1, 2, 0);
      Ua.at(k, 2, 1) = Ua.at(k + 1, 2, 1);
    }
    // batch sums over the healthy trajectories only (L and gradients, and their count in slot 7):
    // a flagged trajectory drops out of the mean; a pair counts once
    acc[7] = T(1);
    bool within = true;  // every gradient component within the health bound (NaN fails)
    for (int j = 1; j < 7; ++j) within = within && (m_abs(acc[j]) <= a.gbound);
    if (st || hl != 0 || !within) {
#pragma unroll
      for (int j = 0; j < DTMPC_TUBE_SUMS; ++j) acc[j] = T(0);
    }
    a.status[i] |= st;
    if (a.iters) {
      a.iters[i] = itn;
      a.iters[nb + i] = ita;
    }
    pr.mark(10);
    pr.flush();
  }
  // fixed-order workgroup sum of [L, gQ, gR, gqb, count]
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < DTMPC_TUBE_SUMS; ++j) {
    T v = wave_sum(acc[j]);
    if (lane == 0) red[wv][j] = v;
  }
  __syncthreads();
  if (threadIdx.x < DTMPC_TUBE_SUMS) {
    T v = T(0);
#pragma unroll
    for (int q = 0; q < kBlock / 64; ++q) v += red[q][threadIdx.x];
    a.partials[(size_t)blockIdx.x * DTMPC_TUBE_SUMS + threadIdx.x] = v;
  }
}

template <typename T>
__global__ void __launch_bounds__(kBlock) partials_reduce_kernel(int64_t n, const T* p, T* sums) {
  __shared__ T red[kBlock][8];
  T v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int64_t r = threadIdx.x; r < n; r += kBlock)
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] += p[r * 8 + j];
#pragma unroll
  for (int j = 0; j < 8; ++j) red[threadIdx.x][j] = v[j];
  __syncthreads();
  for (int h = kBlock / 2; h > 0; h >>= 1) {
    if ((int)threadIdx.x < h)
#pragma unroll
      for (int j = 0; j < 8; ++j) red[threadIdx.x][j] += red[threadIdx.x + h][j];
    __syncthreads();
  }
  if (threadIdx.x < 8) sums[threadIdx.x] = red[0][threadIdx.x];
}

// momentum + projected update (core/tube_mpc.py:978-984); inv_batch <= 0: mean over the healthy
// trajectories counted in sums[7]
template <typename T>
__global__ void theta_update_kernel(T mom, T eta, T qmin, T rmin, T qbmin, T qbmax, T inv_batch,
                                    const T* sums, T* theta, T* vel) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  if (!(inv_batch > T(0))) inv_batch = sums[7] > T(0) ? T(1) / sums[7] : T(0);
  for (int j = 0; j < 6; ++j) {
    T g = sums[1 + j] * inv_batch;
    vel[j] = mom * vel[j] + g;
    T t = theta[j] - eta * vel[j];
    if (j < 3)
      theta[j] = t < qmin ? qmin : t;
    else if (j < 5)
      theta[j] = t < rmin ? rmin : t;
    else
      theta[j] = clampv(t, qbmin, qbmax);
  }
}

// ---------------------------------------------------------------------------------------------
// host dispatch

template <typename T, int NA>
static void launch_ilqr_na(const DSpec<T>& s, const DCost<T>& c, const DIlqr<T>& cfg, int B,
                           const void* x0, const void* Xref, const void* Uref, void* X, void* U,
                           void* K, void* kff, int* iters, int* status, signed char* choices, hipStream_t st) {
  hipLaunchKernelGGL((ilqr_kernel<T, NA>), grid_for(B), dim3(kBlock), 0, st, s, c, cfg, B, x0, Xref,
                     Uref, X, U, K, kff, iters, status, choices);
}

template <typename T>
static int launch_ilqr(const dtmpc_spec* sp, const dtmpc_cost* cp, const dtmpc_ilqr_cfg* cf,
                       int64_t B, const void* x0, const void* Xref, const void* Uref, void* X,
                       void* U, void* K, void* kff, int* iters, int* status, signed char* choices,
                       hipStream_t st) {
  DSpec<T> s = make_spec<T>(*sp);
  DCost<T> c = make_cost<T>(*cp);
  DIlqr<T> cfg = make_ilqr<T>(*cf);
  switch (cfg.nc) {  // rolled-out candidates (alpha = 0 is taken from the previous iteration)
#define CASE(n) \
  case n: launch_ilqr_na<T, n>(s, c, cfg, (int)B, x0, Xref, Uref, X, U, K, kff, iters, status, choices, st); break;
    DTMPC_NA_CASES(CASE)
#undef CASE
    default: return set_err(DTMPC_ERR_BAD_ARG, "n_alphas out of range");
  }
  return check_launch("ilqr_kernel");
}

template <typename T>
static int launch_tube(const dtmpc_spec* sp, const dtmpc_tube_cfg* cf, int64_t B, int64_t goff,
                       int64_t step, const dtmpc_tube_state* S, const void* w, hipStream_t st) {
  const int lpt = S->lanes == 1 ? 1 : 2;  // a 4-lane state runs the generic kernel at two lanes
  DSpec<T> s = make_spec<T>(*sp);
  DCost<T> cn = make_cost<T>(cf->nominal);
  DIlqr<T> cfn = make_ilqr<T>(cf->nom_ilqr), cfa = make_ilqr<T>(cf->aux_ilqr);
  TubeArgs<T> a;
  std::memset(&a, 0, sizeof(a));
  a.B = (int)B;
  a.goff = goff;
  a.step = step;
  a.x = (T*)S->x;
  a.b = (T*)S->b;
  a.xbar = (T*)S->xbar;
  a.bbar = (T*)S->bbar;
  a.Xnom = (T*)S->Xnom;
  a.Unom = (T*)S->Unom;
  a.Xaux = (T*)S->Xaux;
  a.Uaux = (T*)S->Uaux;
  a.work = (T*)S->work;
  a.theta = (const T*)S->theta;
  a.partials = (T*)S->partials;
  a.log = (T*)S->log;
  a.status = S->status;
  a.iters = S->iters;
  a.w = (const T*)w;
  a.choices = (signed char*)S->choices;
  a.gbound = cf->grad_bound > 0 ? T(cf->grad_bound) : T(__builtin_inf());
  a.disturbance = cf->disturbance;
  a.write_log = (cf->write_log && S->log) ? 1 : 0;
  a.seed = cf->seed;
  for (int f = 0; f < 3; ++f) {
    a.wlo[f] = T(cf->w_low[f]);
    a.whi[f] = T(cf->w_high[f]);
  }
  // the fused kernel runs both solves with one line-search width (same alphas, checked)
  switch (cfn.nc) {
#define CASE(n)                                                                                     \
  case n:                                                                                           \
    if (lpt == 2)                                                                                   \
      hipLaunchKernelGGL((tube_step_kernel<T, n, 2>), grid_for(B * 2), dim3(kBlock), 0, st, s, cn, cfn, cfa, a); \
    else                                                                                            \
      hipLaunchKernelGGL((tube_step_kernel<T, n, 1>), grid_for(B), dim3(kBlock), 0, st, s, cn, cfn, cfa, a); \
    break;
    DTMPC_NA_CASES(CASE)
#undef CASE
    default: return set_err(DTMPC_ERR_BAD_ARG, "n_alphas out of range");
  }
  {  // the partial rows past this grid's (a 4-lane state, or small-batch 64-thread rows): zero, so the
     // reduction of all dtmpc_tube_partials_count rows holds
    const int64_t r0 = (B * lpt + kBlock - 1) / kBlock, r1 = dtmpc_tube_partials_count(B, S->lanes);
    if (r1 > r0 && hipMemsetAsync((T*)S->partials + r0 * DTMPC_TUBE_SUMS, 0, (size_t)(r1 - r0) * DTMPC_TUBE_SUMS * sizeof(T), st) != hipSuccess)
      return check_launch("partials tail");
  }
  return check_launch("tube_step_kernel");
}

}  // namespace dtmpc

using namespace dtmpc;

extern "C" {

#ifdef DTMPC_PROFILE
// profiling builds only (not part of include/dtmpc.h): read / clear the phase-cycle accumulators
int dtmpc_prof_read(void* host16) {
  return hipMemcpyFromSymbol(host16, HIP_SYMBOL(dtmpc::g_prof), 16 * sizeof(unsigned long long)) ==
                 hipSuccess
             ? 0
             : 1;
}
int dtmpc_prof_reset(void) {
  unsigned long long z[16] = {0};
  return hipMemcpyToSymbol(HIP_SYMBOL(dtmpc::g_prof), z, sizeof(z)) == hipSuccess ? 0 : 1;
}
#endif

int dtmpc_abi_version(void) { return DTMPC_ABI_VERSION; }

const char* dtmpc_last_error(void) { return err_buf(); }

int dtmpc_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

int dtmpc_dbas_rollout(int dtype, const dtmpc_spec* spec, int64_t B, const void* x0, const void* U,
                       void* X, void* stream) {
  int e = check_spec(spec, B);
  if (e) return e;
  if (!x0 || !U || !X) return set_err(DTMPC_ERR_BAD_ARG, "NULL array");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DTMPC_F32)
    hipLaunchKernelGGL(rollout_kernel<float>, grid_for(B), dim3(kBlock), 0, st, make_spec<float>(*spec), (int)B, x0, U, X);
  else if (dtype == DTMPC_F64)
    hipLaunchKernelGGL(rollout_kernel<double>, grid_for(B), dim3(kBlock), 0, st, make_spec<double>(*spec), (int)B, x0, U, X);
  else
    return set_err(DTMPC_ERR_BAD_ARG, "bad dtype");
  return check_launch("rollout_kernel");
}

int dtmpc_dbas_init(int dtype, const dtmpc_spec* spec, int64_t B, const void* x, void* b,
                    void* stream) {
  int e = check_spec(spec, B);
  if (e) return e;
  if (!x || !b) return set_err(DTMPC_ERR_BAD_ARG, "NULL array");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DTMPC_F32)
    hipLaunchKernelGGL(dbas_init_kernel<float>, grid_for(B), dim3(kBlock), 0, st, make_spec<float>(*spec), (int)B, (const float*)x, (float*)b);
  else if (dtype == DTMPC_F64)
    hipLaunchKernelGGL(dbas_init_kernel<double>, grid_for(B), dim3(kBlock), 0, st, make_spec<double>(*spec), (int)B, (const double*)x, (double*)b);
  else
    return set_err(DTMPC_ERR_BAD_ARG, "bad dtype");
  return check_launch("dbas_init_kernel");
}

int dtmpc_tube_reset(int dtype, const dtmpc_spec* spec, int64_t B, const void* x0, const dtmpc_tube_state* S,
                     const void* theta0, void* theta, void* vel, void* stream) {
  int e = check_spec(spec, B);
  if (e) return e;
  if (!x0 || !S || !theta0 || !theta || !vel) return set_err(DTMPC_ERR_BAD_ARG, "NULL argument");
  if (!S->x || !S->b || !S->xbar || !S->bbar || !S->Unom || !S->Uaux || !S->status)
    return set_err(DTMPC_ERR_BAD_ARG, "NULL state array");
  hipStream_t st = (hipStream_t)stream;
#define RESET(T)                                                                                          \
  hipLaunchKernelGGL(tube_reset_kernel<T>, grid_for(B), dim3(kBlock), 0, st, make_spec<T>(*spec), (int)B,   \
                     (const T*)x0, (T*)S->x, (T*)S->b, (T*)S->xbar, (T*)S->bbar, (T*)S->Unom, (T*)S->Uaux,   \
                     S->status, (const T*)theta0, (T*)theta, (T*)vel)
  if (dtype == DTMPC_F32)
    RESET(float);
  else if (dtype == DTMPC_F64)
    RESET(double);
  else
    return set_err(DTMPC_ERR_BAD_ARG, "bad dtype");
#undef RESET
  return check_launch("tube_reset_kernel");
}

int dtmpc_linearize(int dtype, const dtmpc_spec* spec, const dtmpc_cost* cost, int64_t B,
                    const void* X, const void* U, const void* Xref, const void* Uref, void* A,
                    void* Bm, void* lx, void* lu, void* stream) {
  int e = check_spec(spec, B);
  if (e) return e;
  if ((e = check_cost(cost, Xref, Uref))) return e;
  if (!X || !U || !A || !Bm || !lx || !lu) return set_err(DTMPC_ERR_BAD_ARG, "NULL array");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DTMPC_F32)
    hipLaunchKernelGGL(linearize_kernel<float>, grid_for(B), dim3(kBlock), 0, st, make_spec<float>(*spec), make_cost<float>(*cost), (int)B, X, U, Xref, Uref, A, Bm, lx, lu);
  else if (dtype == DTMPC_F64)
    hipLaunchKernelGGL(linearize_kernel<double>, grid_for(B), dim3(kBlock), 0, st, make_spec<double>(*spec), make_cost<double>(*cost), (int)B, X, U, Xref, Uref, A, Bm, lx, lu);
  else
    return set_err(DTMPC_ERR_BAD_ARG, "bad dtype");
  return check_launch("linearize_kernel");
}

int dtmpc_ilqr_solve(int dtype, const dtmpc_spec* spec, const dtmpc_cost* cost,
                     const dtmpc_ilqr_cfg* cfg, int64_t B, const void* x0, const void* Xref,
                     const void* Uref, void* X, void* U, void* K, void* kff, int32_t* iters,
                     int32_t* status, int8_t* choices, void* stream) {
  int e = check_spec(spec, B);
  if (e) return e;
  if ((e = check_cost(cost, Xref, Uref))) return e;
  if ((e = check_ilqr(cfg))) return e;
  if (!x0 || !X || !U || !K || !kff || !status) return set_err(DTMPC_ERR_BAD_ARG, "NULL array");
  hipStream_t st = (hipStream_t)stream;
  signed char* ch = (signed char*)choices;
  if (dtype == DTMPC_F32) return launch_ilqr<float>(spec, cost, cfg, B, x0, Xref, Uref, X, U, K, kff, iters, status, ch, st);
  if (dtype == DTMPC_F64) return launch_ilqr<double>(spec, cost, cfg, B, x0, Xref, Uref, X, U, K, kff, iters, status, ch, st);
  return set_err(DTMPC_ERR_BAD_ARG, "bad dtype");
}

size_t dtmpc_ilqr_workspace_bytes(int dtype, int32_t horizon, int64_t B, int32_t lanes) {
  if (dtype != DTMPC_F32 && dtype != DTMPC_F64) return 0;
  if (horizon < 1 || horizon > DTMPC_MAX_HORIZON || B < 1) return 0;
  if (lanes == 0) lanes = tube_lanes_default(B, dtype);
  if (lanes != 1 && lanes != 2 && lanes != 4) return 0;
  return dtype == DTMPC_F64 ? ilqr_fast_workspace_bytes64(horizon, B, lanes) : ilqr_fast_workspace_bytes(horizon, B, lanes);
}

int32_t dtmpc_ilqr_fused_eligible(int dtype, const dtmpc_spec* spec, const dtmpc_cost* cost,
                                  const dtmpc_ilqr_cfg* cfg) {
  if (!spec || !cost || !cfg) return 0;
  return (ilqr_fast_eligible(dtype, spec, cost, cfg) || ilqr_fast_eligible64(dtype, spec, cost, cfg)) ? 1 : 0;
}

int dtmpc_ilqr_solve_ws(int dtype, const dtmpc_spec* spec, const dtmpc_cost* cost,
                        const dtmpc_ilqr_cfg* cfg, int64_t B, const void* x0, const void* Xref,
                        const void* Uref, void* X, void* U, void* K, void* kff, int32_t* iters,
                        int32_t* status, int8_t* choices, void* costs, int32_t lanes, void* work,
                        size_t work_bytes, void* stream) {
  int e = check_spec(spec, B);
  if (e) return e;
  if ((e = check_cost(cost, Xref, Uref))) return e;
  if ((e = check_ilqr(cfg))) return e;
  if (!x0 || !X || !U || !K || !kff || !status) return set_err(DTMPC_ERR_BAD_ARG, "NULL array");
  if (lanes == 0) lanes = tube_lanes_default(B, dtype);
  if (lanes != 1 && lanes != 2 && lanes != 4) return set_err(DTMPC_ERR_BAD_ARG, "lanes must be 0, 1, 2 or 4");
  if (ilqr_fast_eligible(dtype, spec, cost, cfg))
    return launch_ilqr_fast(spec, cost, cfg, B, x0, Xref, Uref, X, U, K, kff, iters, status, (signed char*)choices,
                            costs, lanes, work, work_bytes, (hipStream_t)stream);
  if (ilqr_fast_eligible64(dtype, spec, cost, cfg))
    return launch_ilqr_fast64(spec, cost, cfg, B, x0, Xref, Uref, X, U, K, kff, iters, status, (signed char*)choices,
                              costs, lanes, work, work_bytes, (hipStream_t)stream);
  return dtmpc_ilqr_solve(dtype, spec, cost, cfg, B, x0, Xref, Uref, X, U, K, kff, iters, status, choices, stream);
}

size_t dtmpc_sensitivity_workspace_bytes(int dtype, int32_t horizon, int64_t B, int32_t want_lambda) {
  size_t el = dtype == DTMPC_F64 ? 8 : 4;
  size_t per = (size_t)horizon * 20 + (want_lambda ? (size_t)(horizon + 1) * 20 : 0);
  return el * per * (size_t)B;
}

int dtmpc_ddp_sensitivity(int dtype, const dtmpc_spec* spec, const dtmpc_cost* cost, int64_t B,
                          const void* X, const void* U, const void* Xref, const void* Uref,
                          const void* Xbar, void* dX, void* dU, void* dlam, void* work,
                          int32_t* status, void* stream) {
  int e = check_spec(spec, B);
  if (e) return e;
  if ((e = check_cost(cost, Xref, Uref))) return e;
  if (!X || !U || !Xbar || !dX || !dU || !work || !status) return set_err(DTMPC_ERR_BAD_ARG, "NULL array");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DTMPC_F32) {
    DSpec<float> s = make_spec<float>(*spec);
    DCost<float> c = make_cost<float>(*cost);
    if (dlam)
      hipLaunchKernelGGL((sens_kernel<float, true>), grid_for(B), dim3(kBlock), 0, st, s, c, (int)B, X, U, Xref, Uref, Xbar, dX, dU, dlam, work, status);
    else
      hipLaunchKernelGGL((sens_kernel<float, false>), grid_for(B), dim3(kBlock), 0, st, s, c, (int)B, X, U, Xref, Uref, Xbar, dX, dU, dlam, work, status);
  } else if (dtype == DTMPC_F64) {
    DSpec<double> s = make_spec<double>(*spec);
    DCost<double> c = make_cost<double>(*cost);
    if (dlam)
      hipLaunchKernelGGL((sens_kernel<double, true>), grid_for(B), dim3(kBlock), 0, st, s, c, (int)B, X, U, Xref, Uref, Xbar, dX, dU, dlam, work, status);
    else
      hipLaunchKernelGGL((sens_kernel<double, false>), grid_for(B), dim3(kBlock), 0, st, s, c, (int)B, X, U, Xref, Uref, Xbar, dX, dU, dlam, work, status);
  } else {
    return set_err(DTMPC_ERR_BAD_ARG, "bad dtype");
  }
  return check_launch("sens_kernel");
}

int dtmpc_doc_grad(int dtype, int32_t horizon, int64_t B, const void* Xaux, const void* Uaux,
                   const void* Xnom, const void* Unom, const void* dX, const void* dU, void* out,
                   void* stream) {
  if (horizon < 1 || horizon > DTMPC_MAX_HORIZON || B < 1) return set_err(DTMPC_ERR_BAD_ARG, "bad sizes");
  if (!Xaux || !Uaux || !Xnom || !Unom || !dX || !dU || !out) return set_err(DTMPC_ERR_BAD_ARG, "NULL array");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DTMPC_F32)
    hipLaunchKernelGGL(docgrad_kernel<float>, grid_for(B), dim3(kBlock), 0, st, horizon, (int)B, Xaux, Uaux, Xnom, Unom, dX, dU, out);
  else if (dtype == DTMPC_F64)
    hipLaunchKernelGGL(docgrad_kernel<double>, grid_for(B), dim3(kBlock), 0, st, horizon, (int)B, Xaux, Uaux, Xnom, Unom, dX, dU, out);
  else
    return set_err(DTMPC_ERR_BAD_ARG, "bad dtype");
  return check_launch("docgrad_kernel");
}

int64_t dtmpc_tube_chunk(int32_t horizon, int32_t lanes) {
  if (horizon < 1 || horizon > DTMPC_MAX_HORIZON || (lanes != 1 && lanes != 2 && lanes != 4)) return 0;
  int64_t c = tube_fast_chunk_max(horizon, lanes);
  if (const char* e = getenv("DTMPC_FAST_CHUNK")) {
    const int64_t v = atoll(e) / kBlock * kBlock;
    if (v > 0 && v < c) c = v;
  }
  return c;
}

size_t dtmpc_tube_workspace_bytes(int dtype, int32_t horizon, int64_t B, int32_t lanes, int64_t chunk) {
  if (horizon < 1 || horizon > DTMPC_MAX_HORIZON || B < 1 || (lanes != 1 && lanes != 2 && lanes != 4)) return 0;
  if (chunk < kBlock || chunk % kBlock || chunk > tube_fast_chunk_max(horizon, lanes)) return 0;
  size_t el = dtype == DTMPC_F64 ? 8 : 4;
  // generic kernel: sensitivity K / kf / AB (SoA, 20) + iLQR gains (AoS, 10) values per step;
  // the f32 fast kernel: its per-lane records for one chunk (dtmpc_fast.hip)
  const size_t gen = el * (size_t)horizon * 30 * (size_t)B;
  size_t fast = 0;
  if (dtype == DTMPC_F32) {
    fast = tube_fast_workspace_bytes(horizon, B, lanes, chunk);
  } else {  // f64 records: at most tube_fast_chunk_max64 trajectories per launch chunk
    const int64_t c64 = tube_fast_chunk_max64(horizon, lanes);
    fast = tube_fast_workspace_bytes64(horizon, B, lanes, chunk < c64 ? chunk : c64);
  }
  return gen > fast ? gen : fast;
}

int32_t dtmpc_tube_lanes(int64_t B) { return tube_lanes_default(B); }
int32_t dtmpc_tube_lanes_dtype(int64_t B, int dtype) {
  if (dtype != DTMPC_F32 && dtype != DTMPC_F64) return 0;
  return tube_lanes_default(B, dtype);
}

int64_t dtmpc_tube_partials_count(int64_t B, int32_t lanes) {
  if (B < 1 || (lanes != 1 && lanes != 2 && lanes != 4)) return 0;
  const int64_t bs = tube_block(B, lanes);
  return (B * lanes + bs - 1) / bs;
}

int dtmpc_tube_step(int dtype, const dtmpc_spec* spec, const dtmpc_tube_cfg* cfg, int64_t B,
                    int64_t global_offset, int64_t step, const dtmpc_tube_state* state,
                    const void* w, void* stream) {
  int e = check_spec(spec, B);
  if (e) return e;
  if (!cfg || !state) return set_err(DTMPC_ERR_BAD_ARG, "NULL cfg/state");
  if ((e = check_ilqr(&cfg->nom_ilqr)) || (e = check_ilqr(&cfg->aux_ilqr))) return e;
  if (cfg->nom_ilqr.n_alphas != cfg->aux_ilqr.n_alphas)
    return set_err(DTMPC_ERR_BAD_ARG, "nominal and ancillary line searches must have the same width");
  for (int a = 0; a < cfg->nom_ilqr.n_alphas; ++a)
    if (cfg->nom_ilqr.alphas[a] != cfg->aux_ilqr.alphas[a])
      return set_err(DTMPC_ERR_BAD_ARG, "nominal and ancillary alphas must match");
  if (cfg->nominal.kind != DTMPC_COST_TARGET) return set_err(DTMPC_ERR_BAD_ARG, "nominal cost must be DTMPC_COST_TARGET");
  const dtmpc_tube_state* S = state;
  if (!S->x || !S->b || !S->xbar || !S->bbar || !S->Xnom || !S->Unom || !S->Xaux || !S->Uaux ||
      !S->work || !S->theta || !S->partials || !S->status)
    return set_err(DTMPC_ERR_BAD_ARG, "NULL state array");
  if (S->lanes != 1 && S->lanes != 2 && S->lanes != 4) return set_err(DTMPC_ERR_BAD_ARG, "state->lanes must be 1, 2 or 4");
  if (S->n_partials < dtmpc_tube_partials_count(B, S->lanes))
    return set_err(DTMPC_ERR_BAD_ARG, "state->n_partials < dtmpc_tube_partials_count(B, lanes)");
  {
    // the workspace the caller allocated must hold what this launch addresses (chunk and lanes come from
    // the state, never from the environment)
    const size_t need = dtmpc_tube_workspace_bytes(dtype, spec->horizon, B, S->lanes, S->chunk);
    if (need == 0) return set_err(DTMPC_ERR_BAD_ARG, "state->chunk is not a chunk dtmpc_tube_chunk(horizon, lanes) returns");
    if (S->work_bytes < 0 || (size_t)S->work_bytes < need)
      return set_err(DTMPC_ERR_BAD_ARG, "state->work_bytes < dtmpc_tube_workspace_bytes(dtype, horizon, B, lanes, chunk)");
  }
  if (cfg->disturbance == 0 && !w) return set_err(DTMPC_ERR_BAD_ARG, "injected disturbance w is NULL");
  if (cfg->disturbance != 0 && cfg->disturbance != 1) return set_err(DTMPC_ERR_BAD_ARG, "bad disturbance mode");
  if (S->phase < 0 || S->phase > 2) return set_err(DTMPC_ERR_BAD_ARG, "state->phase must be 0, 1 or 2");
  if (S->phase != 0 && !dtmpc_tube_split_ok(dtype, spec, cfg, B, S->lanes, S->chunk))
    return set_err(DTMPC_ERR_BAD_ARG, "a split step (state->phase 1 / 2) needs the fused kernel and B within one launch "
                                      "chunk of the precision (dtmpc_tube_split_ok)");
  hipStream_t st = (hipStream_t)stream;
  if (tube_fast_eligible(dtype, spec, cfg)) return launch_tube_fast(spec, cfg, B, global_offset, step, S, w, st);
  if (tube_fast_eligible64(dtype, spec, cfg) && tube_fast_lanes_ok64(spec, S->lanes))
    return launch_tube_fast64(spec, cfg, B, global_offset, step, S, w, st);
  if (dtype == DTMPC_F32) return launch_tube<float>(spec, cfg, B, global_offset, step, S, w, st);
  if (dtype == DTMPC_F64) return launch_tube<double>(spec, cfg, B, global_offset, step, S, w, st);
  return set_err(DTMPC_ERR_BAD_ARG, "bad dtype");
}

int32_t dtmpc_tube_split_supported(int dtype, const dtmpc_spec* spec, const dtmpc_tube_cfg* cfg, int32_t lanes) {
  if (!spec || !cfg) return 0;
  return (tube_fast_eligible(dtype, spec, cfg) ||
          (tube_fast_eligible64(dtype, spec, cfg) && tube_fast_lanes_ok64(spec, lanes))) ? 1 : 0;
}

// ABI 7: the split needs the nominal records of the WHOLE batch between the two launches, i.e. one launch
// chunk -- the precision's own chunk: f64 records are twice as large, so launch_tube_fast64 clamps the state's chunk to
// tube_fast_chunk_max64, about half the f32 one
int32_t dtmpc_tube_split_ok(int dtype, const dtmpc_spec* spec, const dtmpc_tube_cfg* cfg, int64_t B, int32_t lanes,
                            int64_t chunk) {
  if (!dtmpc_tube_split_supported(dtype, spec, cfg, lanes) || B < 1 || chunk < 1) return 0;
  int64_t c = chunk;
  if (dtype == DTMPC_F64) {
    const int64_t c64 = tube_fast_chunk_max64(spec->horizon, lanes);
    c = c < c64 ? c : c64;
  } else {
    const int64_t c32 = tube_fast_chunk_max(spec->horizon, lanes);
    c = c < c32 ? c : c32;
  }
  return B <= c ? 1 : 0;
}

int dtmpc_partials_reduce(int dtype, int64_t n, const void* partials, void* sums, void* stream) {
  if (n < 1 || !partials || !sums) return set_err(DTMPC_ERR_BAD_ARG, "bad partials");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DTMPC_F32)
    hipLaunchKernelGGL(partials_reduce_kernel<float>, dim3(1), dim3(kBlock), 0, st, n, (const float*)partials, (float*)sums);
  else if (dtype == DTMPC_F64)
    hipLaunchKernelGGL(partials_reduce_kernel<double>, dim3(1), dim3(kBlock), 0, st, n, (const double*)partials, (double*)sums);
  else
    return set_err(DTMPC_ERR_BAD_ARG, "bad dtype");
  return check_launch("partials_reduce_kernel");
}

int dtmpc_theta_update(int dtype, const dtmpc_adapt_cfg* c, double inv_batch, const void* sums,
                       void* theta, void* vel, void* stream) {
  if (!c || !sums || !theta || !vel) return set_err(DTMPC_ERR_BAD_ARG, "NULL argument");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DTMPC_F32)
    hipLaunchKernelGGL(theta_update_kernel<float>, dim3(1), dim3(64), 0, st, (float)c->momentum, (float)c->lr_eta, (float)c->q_min, (float)c->r_min, (float)c->qb_min, (float)c->qb_max, (float)inv_batch, (const float*)sums, (float*)theta, (float*)vel);
  else if (dtype == DTMPC_F64)
    hipLaunchKernelGGL(theta_update_kernel<double>, dim3(1), dim3(64), 0, st, c->momentum, c->lr_eta, c->q_min, c->r_min, c->qb_min, c->qb_max, inv_batch, (const double*)sums, (double*)theta, (double*)vel);
  else
    return set_err(DTMPC_ERR_BAD_ARG, "bad dtype");
  return check_launch("theta_update_kernel");
}

}  // extern "C"
