// dtmpc_general.hip — HIP kernels (gfx950) + C ABI of the GENERAL IFT path (include/dtmpc.h,
// "general" section): core/tube_mpc.py:40-663 with softplus / tanh parameterised weights and DBaS
// parameters, both MPCs adapting.  Device bodies in dtmpc_general.hpp; one lane per trajectory.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstring>

#include "../../include/dtmpc.h"
#include "dtmpc_host.hpp"

namespace dtmpc {

template <typename T>
struct Raw12 {
  T v[DTMPC_P_COUNT];
};

// ---------------------------------------------------------------------------------------------
// stand-alone entry points

// ddp_sensitivity with array upper gradients (core/ddp.py:317-427)
template <typename T, bool LAMBDA>
__global__ void __launch_bounds__(kBlock) sens_upper_kernel(DSpec<T> s, DCost<T> c, int B, const void* Xp,
                                                            const void* Up, const void* gXp, const void* gUp,
                                                            void* dXp, void* dUp, void* dLp, void* work,
                                                            int* status) {
  int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= B) return;
  const int N = s.N;
  T* w = reinterpret_cast<T*>(work);
  const size_t nb = (size_t)B;
  Col<T> K = col<T>(w, i, B), kf = col<T>(w + (size_t)N * 8 * nb, i, B), AB = col<T>(w + (size_t)N * 10 * nb, i, B),
         VV = col<T>(w + (size_t)N * 20 * nb, i, B), VF = col<T>(w + ((size_t)N * 20 + (size_t)(N + 1) * 5) * nb, i, B);
  Col<T> none = col<T>((void*)nullptr, i, B);
  GPar<T> p;  // unused without the IFT
  int st = sens_ift_traj<T, kUpperArrays, false, true, LAMBDA>(
      s, c, p, col<T>(Xp, i, B), col<T>(Up, i, B), none, 3, none, none, 3, col<T>(gXp, i, B), col<T>(gUp, i, B), K,
      kf, AB, VV, VF, none, col<T>(dXp, i, B), col<T>(dUp, i, B), col<T>(dLp, i, B), nullptr);
  if (status) status[i] |= st;
}

// ift_gradient on a given optimum + sensitivity (core/ift.py:35-92)
template <typename T>
__global__ void __launch_bounds__(kBlock) ift_kernel(DSpec<T> s, DCost<T> c, Raw12<T> raw, int B, const void* Xp,
                                                     const void* Up, const void* dXp, const void* dUp,
                                                     const void* dLp, const void* Xrp, const void* Urp, void* gp,
                                                     void* gxrp, void* gurp) {
  int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= B) return;
  const int N = s.N;
  const bool track = c.kind == DTMPC_COST_TRACK;
  GPar<T> p = gpar_from(raw.v, !track);
  DSpec<T> sp = gspec(s, p);
  Col<T> X = col<T>(Xp, i, B), U = col<T>(Up, i, B), dX = col<T>(dXp, i, B), dU = col<T>(dUp, i, B),
         dL = col<T>(dLp, i, B), Xr = col<T>(Xrp, i, B), Ur = col<T>(Urp, i, B), G = col<T>(gp, i, B),
         Gx = col<T>(gxrp, i, B), Gu = col<T>(gurp, i, B);
  IftAcc<T> A;
  A.zero();
  for (int k = 0; k < N; ++k) {
    T xk[4] = {X.at(k, 4, 0), X.at(k, 4, 1), X.at(k, 4, 2), X.at(k, 4, 3)};
    T uk[2] = {U.at(k, 2, 0), U.at(k, 2, 1)};
    T dxk[4] = {dX.at(k, 4, 0), dX.at(k, 4, 1), dX.at(k, 4, 2), dX.at(k, 4, 3)};
    T duk[2] = {dU.at(k, 2, 0), dU.at(k, 2, 1)};
    T r[3] = {c.t0, c.t1, c.t2}, q[2] = {T(0), T(0)};
    if (track) {
      r[0] = Xr.at(k, 3, 0);
      r[1] = Xr.at(k, 3, 1);
      r[2] = Xr.at(k, 3, 2);
      q[0] = Ur.at(k, 2, 0);
      q[1] = Ur.at(k, 2, 1);
      if (gxrp) {
        Gx.at(k, 3, 0) = -(T(2) * p.Q[0]) * dxk[0];
        Gx.at(k, 3, 1) = -(T(2) * p.Q[1]) * dxk[1];
        Gx.at(k, 3, 2) = -(T(2) * p.Q[2]) * dxk[2];
      }
      if (gurp) {
        Gu.at(k, 2, 0) = -(T(2) * p.R[0]) * duk[0];
        Gu.at(k, 2, 1) = -(T(2) * p.R[1]) * duk[1];
      }
    }
    ift_step(sp, xk, uk, dxk, duk, T(dL.at(k + 1, 4, 3)), r, q, A);
  }
  T xN[4] = {X.at(N, 4, 0), X.at(N, 4, 1), X.at(N, 4, 2), X.at(N, 4, 3)};
  T dxN[4] = {dX.at(N, 4, 0), dX.at(N, 4, 1), dX.at(N, 4, 2), dX.at(N, 4, 3)};
  T r[3] = {c.t0, c.t1, c.t2};
  if (track) {
    r[0] = Xr.at(N, 3, 0);
    r[1] = Xr.at(N, 3, 1);
    r[2] = Xr.at(N, 3, 2);
    if (gxrp) {
      Gx.at(N, 3, 0) = -(T(2) * p.Qf[0]) * dxN[0];
      Gx.at(N, 3, 1) = -(T(2) * p.Qf[1]) * dxN[1];
      Gx.at(N, 3, 2) = -(T(2) * p.Qf[2]) * dxN[2];
    }
  }
  ift_terminal(xN, dxN, r, A);
  T g[DTMPC_P_COUNT];
  ift_finish(sp, p, A, track, g);
#pragma unroll
  for (int j = 0; j < DTMPC_P_COUNT; ++j) G.at(j, 1, 0) = g[j];
}

// ---------------------------------------------------------------------------------------------
// fused general step: solves + sensitivities + IFT (core/tube_mpc.py:217-584)

template <typename T>
struct GenArgs {
  int B, adapt_nominal;
  T target[3];
  T* x;
  T* b;
  T* xbar;
  T* bbar;
  T* Xnom;
  T* Unom;
  T* Xaux;
  T* Uaux;
  T* work;
  const T* theta;  // [2][12] raw
  T* partials;     // [nblocks][DTMPC_GEN_SUMS]
  T* gout;         // [25][B] or null
  int* status;
  int* iters;
  const int* sst;  // SOLVED: the solves' status per trajectory (general_solve_fast_kernel)
};

// SOLVED: the two solves already ran (the fast solver, general_solve_fast_kernel): the tapes are in
// Xnom / Unom / Xaux / Uaux and their status in a.sst; this kernel runs the rest of the step.
template <typename T, int NA, bool SOLVED>
__global__ void __launch_bounds__(kBlock) general_step_kernel(DSpec<T> s, DIlqr<T> cfn, DIlqr<T> cfa,
                                                              GenArgs<T> a) {
  __shared__ T red[kBlock / 64][DTMPC_GEN_SUMS];
  const int B = a.B;
  const int N = s.N;
  int i = blockIdx.x * kBlock + threadIdx.x;
  T acc[DTMPC_GEN_SUMS];
#pragma unroll
  for (int j = 0; j < DTMPC_GEN_SUMS; ++j) acc[j] = T(0);
  if (i < B) {
    const size_t nb = (size_t)B;
    GPar<T> pa = gpar_from(a.theta, false), pn = gpar_from(a.theta + DTMPC_P_COUNT, true);
    DSpec<T> sa = gspec(s, pa), sn = gspec(s, pn);
    DCost<T> ca = gcost(pa, DTMPC_COST_TRACK, a.target), cn = gcost(pn, DTMPC_COST_TARGET, a.target);
    Col<T> Xn = col<T>(a.Xnom, i, B), Un = col<T>(a.Unom, i, B), Xa = col<T>(a.Xaux, i, B),
           Ua = col<T>(a.Uaux, i, B);
    T* w = a.work;
    Col<T> K = col<T>(w, i, B), kf = col<T>(w + (size_t)N * 8 * nb, i, B), AB = col<T>(w + (size_t)N * 10 * nb, i, B),
           VV = col<T>(w + (size_t)N * 20 * nb, i, B),
           Gn = col<T>(w + ((size_t)N * 20 + (size_t)(N + 1) * 5) * nb, i, B);
    Col<T> none = col<T>((void*)nullptr, i, B);
    int st = 0, itn = 0, ita = 0;
    Prof pr;
    if (SOLVED) {
      st = a.sst[i];
    } else {
      // nominal MPC with theta-bar (:217-291)
      T xn0[4] = {a.xbar[i], a.xbar[nb + i], a.xbar[2 * nb + i], a.bbar[i]};
      st |= ilqr_traj<T, NA>(sn, cn, cfn, xn0, Xn, Un, GainsSoA<T>{K, kf}, none, 0, none, itn, pr, 0);
      // ancillary MPC with theta tracking the nominal plan (:296-392)
      T xa0[4] = {a.x[i], a.x[nb + i], a.x[2 * nb + i], a.b[i]};
      st |= ilqr_traj<T, NA>(sa, ca, cfa, xa0, Xa, Ua, GainsSoA<T>{K, kf}, Xn, 4, Un, ita, pr, 4);
    }
    // upper loss L = ||x* - xbar||^2 + ||b*||^2 (:403-408)
    T L1 = T(0), L2 = T(0);
    for (int k = 0; k <= N; ++k) {
      T e0 = Xa.at(k, 4, 0) - Xn.at(k, 4, 0), e1 = Xa.at(k, 4, 1) - Xn.at(k, 4, 1),
        e2 = Xa.at(k, 4, 2) - Xn.at(k, 4, 2), bb = Xa.at(k, 4, 3);
      L1 += e0 * e0 + e1 * e1 + e2 * e2;
      L2 += bb * bb;
    }
    acc[0] = L1 + L2;
    // ancillary sensitivity + IFT (theta, X_ref, U_ref) (:411-500)
    T g[DTMPC_P_COUNT];
    st |= sens_ift_traj<T, kUpperPaper, true, false, false>(sa, ca, pa, Xa, Ua, Xn, 4, Un, Xn, 4, none, none, K,
                                                            kf, AB, VV, none, Gn, none, none, none, g);
#pragma unroll
    for (int j = 0; j < 11; ++j) acc[1 + j] = g[j];
    if (a.adapt_nominal) {
      // nominal sensitivity driven by [dL/dX_ref, 0], dL/dU_ref + IFT (theta-bar) (:509-584)
      st |= sens_ift_traj<T, kUpperRef, true, false, false>(sn, cn, pn, Xn, Un, none, 4, none, none, 4, Gn, none, K,
                                                            kf, AB, VV, none, none, none, none, none, g);
#pragma unroll
      for (int j = 0; j < 12; ++j) acc[12 + j] = g[j];
    }
    // healthy-trajectory count (slot 24).  A flagged trajectory contributes nothing to the batch
    // sums -- neither L nor gradients nor the count -- so the update's mean runs over the healthy
    // ones (the paper step does the same); its gout keeps L (row 0, logged by the plant) and zero
    // gradients.
    acc[DTMPC_GEN_SUMS - 1] = st ? T(0) : T(1);
    if (a.gout) {
      a.gout[i] = acc[0];
#pragma unroll
      for (int j = 1; j < DTMPC_GEN_SUMS; ++j) a.gout[(size_t)j * nb + i] = st ? T(0) : acc[j];
    }
    if (st) {
#pragma unroll
      for (int j = 0; j < DTMPC_GEN_SUMS; ++j) acc[j] = T(0);
    }
    a.status[i] |= st;
    if (a.iters && !SOLVED) {
      a.iters[i] = itn;
      a.iters[nb + i] = ita;
    }
  }
  // fixed-order workgroup sums
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int j = 0; j < DTMPC_GEN_SUMS; ++j) {
    T v = wave_sum(acc[j]);
    if (lane == 0) red[wv][j] = v;
  }
  __syncthreads();
  if (threadIdx.x < DTMPC_GEN_SUMS) {
    T v = T(0);
#pragma unroll
    for (int q = 0; q < kBlock / 64; ++q) v += red[q][threadIdx.x];
    a.partials[(size_t)blockIdx.x * DTMPC_GEN_SUMS + threadIdx.x] = v;
  }
}

// fixed-order sum of n records of `width` (<= 32) values
template <typename T>
__global__ void __launch_bounds__(kBlock) partials_reduce_n_kernel(int64_t n, int width, const T* p, T* sums) {
  __shared__ T red[kBlock];
  for (int j = 0; j < width; ++j) {
    T v = T(0);
    for (int64_t r = threadIdx.x; r < n; r += kBlock) v += p[r * width + j];
    red[threadIdx.x] = v;
    __syncthreads();
    for (int h = kBlock / 2; h > 0; h >>= 1) {
      if ((int)threadIdx.x < h) red[threadIdx.x] += red[threadIdx.x + h];
      __syncthreads();
    }
    if (threadIdx.x == 0) sums[j] = red[0];
    __syncthreads();
  }
}

// _apply_update core/tube_mpc.py:239-255 for one parameter tensor of n elements
template <typename T>
__device__ void apply_update(T lr, T mom, double clip, int project, T ib, const T* sums, T* p, T* v, int n,
                             int proj) {
  T g[3];
  for (int j = 0; j < n; ++j) g[j] = sums[j] * ib;
  if (clip > 0) {
    T acc = T(0);
    for (int j = 0; j < n; ++j) acc += g[j] * g[j];
    double nn = sqrt((double)acc);
    if (nn > clip) {
      T sc = T(clip / (nn + 1e-12));
      for (int j = 0; j < n; ++j) g[j] = g[j] * sc;
    }
  }
  for (int j = 0; j < n; ++j) {
    T stp;
    if (mom > T(0)) {
      v[j] = v[j] * mom + g[j];
      stp = v[j];
    } else {
      stp = g[j];
    }
    T t = p[j] - lr * stp;
    if (project) {  // _project :192-237
      switch (proj) {
        case 0: t = t < T(0) ? T(0) : t; break;           // Q, Qf >= 0
        case 1: t = clampv(t, T(1e-4), T(1e4)); break;     // R
        case 2: t = clampv(t, T(0), T(1)); break;          // q_b, alpha
        case 3: t = clampv(t, T(-1), T(1)); break;         // gamma
        default: t = clampv(t, T(0), T(2)); break;         // tightening
      }
    }
    p[j] = t;
  }
}

template <typename T>
__global__ void general_update_kernel(T lr, T mom, double clip, int project, int adapt_anc, int adapt_nom,
                                      int alpha_used, T ib, const T* sums, T* theta, T* vel) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  // ib <= 0: mean over the healthy trajectories counted in the last slot
  if (!(ib > T(0))) {
    const T cnt = sums[DTMPC_GEN_SUMS - 1];
    ib = cnt > T(0) ? T(1) / cnt : T(0);
  }
  for (int set = 0; set < 2; ++set) {
    if (set == 0 && !adapt_anc) continue;
    if (set == 1 && !adapt_nom) continue;
    const T* g = sums + (set == 0 ? 1 : 12);
    T* p = theta + set * DTMPC_P_COUNT;
    T* v = vel + set * DTMPC_P_COUNT;
    apply_update(lr, mom, clip, project, ib, g + DTMPC_P_Q, p + DTMPC_P_Q, v + DTMPC_P_Q, 3, 0);
    apply_update(lr, mom, clip, project, ib, g + DTMPC_P_R, p + DTMPC_P_R, v + DTMPC_P_R, 2, 1);
    apply_update(lr, mom, clip, project, ib, g + DTMPC_P_QF, p + DTMPC_P_QF, v + DTMPC_P_QF, 3, 0);
    apply_update(lr, mom, clip, project, ib, g + DTMPC_P_QB, p + DTMPC_P_QB, v + DTMPC_P_QB, 1, 2);
    // alpha's gradient is None under the log barrier (unused in the graph): no update (:243-244)
    if (alpha_used)
      apply_update(lr, mom, clip, project, ib, g + DTMPC_P_ALPHA, p + DTMPC_P_ALPHA, v + DTMPC_P_ALPHA, 1, 2);
    apply_update(lr, mom, clip, project, ib, g + DTMPC_P_GAMMA, p + DTMPC_P_GAMMA, v + DTMPC_P_GAMMA, 1, 3);
    if (set == 1)
      apply_update(lr, mom, clip, project, ib, g + DTMPC_P_TIGHT, p + DTMPC_P_TIGHT, v + DTMPC_P_TIGHT, 1, 4);
  }
}

// plant + nominal propagation with the UPDATED parameters (:589-600), log (:602-614), shift (:616-621)
template <typename T>
struct PlantArgs {
  int B;
  int64_t goff, step;
  T* x;
  T* b;
  T* xbar;
  T* bbar;
  T* Unom;
  T* Uaux;
  const T* theta;
  const T* gout;  // row 0 = L per trajectory (logged)
  T* log;
  const T* w;
  int disturbance;
  uint64_t seed;
  T wlo[3], whi[3];
};

template <typename T>
__global__ void __launch_bounds__(kBlock) general_plant_kernel(DSpec<T> s, PlantArgs<T> a) {
  const int B = a.B;
  const int N = s.N;
  int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= B) return;
  const size_t nb = (size_t)B;
  GPar<T> pa = gpar_from(a.theta, false), pn = gpar_from(a.theta + DTMPC_P_COUNT, true);
  DSpec<T> sa = gspec(s, pa), sn = gspec(s, pn);
  Col<T> Un = col<T>(a.Unom, i, B), Ua = col<T>(a.Uaux, i, B);
  T x0 = a.x[i], x1 = a.x[nb + i], x2 = a.x[2 * nb + i], xb = a.b[i];
  T y0 = a.xbar[i], y1 = a.xbar[nb + i], y2 = a.xbar[2 * nb + i], yb = a.bbar[i];
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
  if (a.log) {
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
    lg[11 * nb + i] = a.gout ? a.gout[i] : T(0);
  }
  {
    T p0[1] = {x0}, p1[1] = {x1}, p2[1] = {x2}, pb[1] = {xb}, q0[1] = {u0}, q1[1] = {u1};
    T Bc[1] = {barrier_of_state(sa, x0, x1)};
    fhat_vec<T, 1>(sa, p0, p1, p2, pb, q0, q1, Bc);
    a.x[i] = p0[0] + w[0];
    a.x[nb + i] = p1[0] + w[1];
    a.x[2 * nb + i] = p2[0] + w[2];
    a.b[i] = pb[0];
  }
  {
    T p0[1] = {y0}, p1[1] = {y1}, p2[1] = {y2}, pb[1] = {yb}, q0[1] = {v0}, q1[1] = {v1};
    T Bc[1] = {barrier_of_state(sn, y0, y1)};
    fhat_vec<T, 1>(sn, p0, p1, p2, pb, q0, q1, Bc);
    a.xbar[i] = p0[0];
    a.xbar[nb + i] = p1[0];
    a.xbar[2 * nb + i] = p2[0];
    a.bbar[i] = pb[0];
  }
  for (int k = 0; k + 1 < N; ++k) {
    Un.at(k, 2, 0) = Un.at(k + 1, 2, 0);
    Un.at(k, 2, 1) = Un.at(k + 1, 2, 1);
    Ua.at(k, 2, 0) = Ua.at(k + 1, 2, 0);
    Ua.at(k, 2, 1) = Ua.at(k + 1, 2, 1);
  }
}

// ---------------------------------------------------------------------------------------------
// host launchers

// the workspace: the generic scratch of the step (N x 20 + (N+1) x 10 values per trajectory; the fast
// solves' records use its first bytes before the sensitivity does) and the solves' status [B] after it
static size_t general_scratch_bytes(int dtype, int32_t horizon, int64_t B) {
  const size_t el = dtype == DTMPC_F64 ? 8 : 4;
  return (el * ((size_t)horizon * 20 + (size_t)(horizon + 1) * 10) * (size_t)B + 255) / 256 * 256;
}

template <typename T>
static int launch_general(const dtmpc_spec* sp, const dtmpc_general_cfg* cf, int64_t B,
                          const dtmpc_general_state* S, hipStream_t st) {
  DSpec<T> s = make_spec<T>(*sp);
  DIlqr<T> cfn = make_ilqr<T>(cf->nom_ilqr), cfa = make_ilqr<T>(cf->aux_ilqr);
  GenArgs<T> a;
  std::memset(&a, 0, sizeof(a));
  a.B = (int)B;
  a.adapt_nominal = cf->adapt_nominal ? 1 : 0;
  for (int f = 0; f < 3; ++f) a.target[f] = T(cf->target[f]);
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
  a.gout = (T*)S->gout;
  a.status = S->status;
  a.iters = S->iters;
  const int dtype = sizeof(T) == 4 ? DTMPC_F32 : DTMPC_F64;
  const bool f32 = general_fast_eligible(dtype, sp, cf), f64 = !f32 && general_fast_eligible64(dtype, sp, cf);
  if (f32 || f64) {
    int* sst = (int*)((char*)S->work + general_scratch_bytes(dtype, sp->horizon, B));
    const int e = f32 ? launch_general_solve_fast(sp, cf, B, S, sst, st) : launch_general_solve_fast64(sp, cf, B, S, sst, st);
    if (e) return e;
    a.sst = sst;
    hipLaunchKernelGGL((general_step_kernel<T, 1, true>), grid_for(B), dim3(kBlock), 0, st, s, cfn, cfa, a);
    return check_launch("general_step_kernel");
  }
  switch (cfn.nc) {
#define CASE(n)                                                                                          \
  case n:                                                                                                \
    hipLaunchKernelGGL((general_step_kernel<T, n, false>), grid_for(B), dim3(kBlock), 0, st, s, cfn, cfa, a); \
    break;
    DTMPC_NA_CASES(CASE)
#undef CASE
    default: return set_err(DTMPC_ERR_BAD_ARG, "n_alphas out of range");
  }
  return check_launch("general_step_kernel");
}

template <typename T>
static int launch_plant(const dtmpc_spec* sp, const dtmpc_general_cfg* cf, int64_t B, int64_t goff, int64_t step,
                        const dtmpc_general_state* S, const void* w, hipStream_t st) {
  PlantArgs<T> a;
  std::memset(&a, 0, sizeof(a));
  a.B = (int)B;
  a.goff = goff;
  a.step = step;
  a.x = (T*)S->x;
  a.b = (T*)S->b;
  a.xbar = (T*)S->xbar;
  a.bbar = (T*)S->bbar;
  a.Unom = (T*)S->Unom;
  a.Uaux = (T*)S->Uaux;
  a.theta = (const T*)S->theta;
  a.gout = (const T*)S->gout;
  a.log = cf->write_log ? (T*)S->log : nullptr;
  a.w = (const T*)w;
  a.disturbance = cf->disturbance;
  a.seed = cf->seed;
  for (int f = 0; f < 3; ++f) {
    a.wlo[f] = T(cf->w_low[f]);
    a.whi[f] = T(cf->w_high[f]);
  }
  hipLaunchKernelGGL(general_plant_kernel<T>, grid_for(B), dim3(kBlock), 0, st, make_spec<T>(*sp), a);
  return check_launch("general_plant_kernel");
}

static int check_general(const dtmpc_spec* spec, const dtmpc_general_cfg* cfg, int64_t B,
                         const dtmpc_general_state* S) {
  int e = check_spec(spec, B);
  if (e) return e;
  if (!cfg || !S) return set_err(DTMPC_ERR_BAD_ARG, "NULL cfg/state");
  if ((e = check_ilqr(&cfg->nom_ilqr)) || (e = check_ilqr(&cfg->aux_ilqr))) return e;
  if (cfg->nom_ilqr.n_alphas != cfg->aux_ilqr.n_alphas)
    return set_err(DTMPC_ERR_BAD_ARG, "nominal and ancillary line searches must have the same width");
  for (int a = 0; a < cfg->nom_ilqr.n_alphas; ++a)
    if (cfg->nom_ilqr.alphas[a] != cfg->aux_ilqr.alphas[a])
      return set_err(DTMPC_ERR_BAD_ARG, "nominal and ancillary alphas must match");
  if (cfg->disturbance != 0 && cfg->disturbance != 1) return set_err(DTMPC_ERR_BAD_ARG, "bad disturbance mode");
  if (!S->x || !S->b || !S->xbar || !S->bbar || !S->Unom || !S->Uaux || !S->theta)
    return set_err(DTMPC_ERR_BAD_ARG, "NULL state array");
  return DTMPC_OK;
}

}  // namespace dtmpc

using namespace dtmpc;

extern "C" {

size_t dtmpc_sensitivity_upper_workspace_bytes(int dtype, int32_t horizon, int64_t B) {
  size_t el = dtype == DTMPC_F64 ? 8 : 4;
  return el * ((size_t)horizon * 20 + (size_t)(horizon + 1) * 25) * (size_t)B;
}

int dtmpc_ddp_sensitivity_upper(int dtype, const dtmpc_spec* spec, const dtmpc_cost* cost, int64_t B,
                                const void* X, const void* U, const void* gX, const void* gU, void* dX,
                                void* dU, void* dlam, void* work, int32_t* status, void* stream) {
  int e = check_spec(spec, B);
  if (e) return e;
  if (!cost || (cost->kind != DTMPC_COST_TARGET && cost->kind != DTMPC_COST_TRACK))
    return set_err(DTMPC_ERR_BAD_ARG, "bad cost");
  if (!X || !U || !gX || !gU || !dX || !dU || !work || !status) return set_err(DTMPC_ERR_BAD_ARG, "NULL array");
  hipStream_t st = (hipStream_t)stream;
#define LAUNCH(T)                                                                                          \
  {                                                                                                        \
    DSpec<T> s = make_spec<T>(*spec);                                                                      \
    DCost<T> c = make_cost<T>(*cost);                                                                      \
    if (dlam)                                                                                              \
      hipLaunchKernelGGL((sens_upper_kernel<T, true>), grid_for(B), dim3(kBlock), 0, st, s, c, (int)B, X, U, \
                         gX, gU, dX, dU, dlam, work, status);                                             \
    else                                                                                                   \
      hipLaunchKernelGGL((sens_upper_kernel<T, false>), grid_for(B), dim3(kBlock), 0, st, s, c, (int)B, X,  \
                         U, gX, gU, dX, dU, dlam, work, status);                                          \
  }
  if (dtype == DTMPC_F32)
    LAUNCH(float)
  else if (dtype == DTMPC_F64)
    LAUNCH(double)
  else
    return set_err(DTMPC_ERR_BAD_ARG, "bad dtype");
#undef LAUNCH
  return check_launch("sens_upper_kernel");
}

int dtmpc_ift_gradient(int dtype, const dtmpc_spec* spec, const dtmpc_cost* cost, const double* theta_raw,
                       int64_t B, const void* X, const void* U, const void* dX, const void* dU, const void* dlam,
                       const void* Xref, const void* Uref, void* g_theta, void* g_xref, void* g_uref,
                       void* stream) {
  int e = check_spec(spec, B);
  if (e) return e;
  if ((e = check_cost(cost, Xref, Uref))) return e;
  if (!theta_raw) return set_err(DTMPC_ERR_BAD_ARG, "theta_raw is NULL");
  if (!X || !U || !dX || !dU || !dlam || !g_theta) return set_err(DTMPC_ERR_BAD_ARG, "NULL array");
  hipStream_t st = (hipStream_t)stream;
#define LAUNCH(T)                                                                                          \
  {                                                                                                        \
    Raw12<T> r;                                                                                            \
    for (int j = 0; j < DTMPC_P_COUNT; ++j) r.v[j] = T(theta_raw[j]);                                      \
    hipLaunchKernelGGL(ift_kernel<T>, grid_for(B), dim3(kBlock), 0, st, make_spec<T>(*spec), make_cost<T>(*cost), \
                       r, (int)B, X, U, dX, dU, dlam, Xref, Uref, g_theta, g_xref, g_uref);               \
  }
  if (dtype == DTMPC_F32)
    LAUNCH(float)
  else if (dtype == DTMPC_F64)
    LAUNCH(double)
  else
    return set_err(DTMPC_ERR_BAD_ARG, "bad dtype");
#undef LAUNCH
  return check_launch("ift_kernel");
}

int64_t dtmpc_general_partials_count(int64_t B) { return B < 1 ? 0 : (B + kBlock - 1) / kBlock; }

size_t dtmpc_general_workspace_bytes(int dtype, int32_t horizon, int64_t B) {
  if ((dtype != DTMPC_F32 && dtype != DTMPC_F64) || horizon < 1 || B < 1) return 0;
  return general_scratch_bytes(dtype, horizon, B) + 4 * (size_t)B;
}

int dtmpc_general_step(int dtype, const dtmpc_spec* spec, const dtmpc_general_cfg* cfg, int64_t B,
                       const dtmpc_general_state* state, void* stream) {
  int e = check_general(spec, cfg, B, state);
  if (e) return e;
  const dtmpc_general_state* S = state;
  if (!S->Xnom || !S->Xaux || !S->work || !S->partials || !S->status)
    return set_err(DTMPC_ERR_BAD_ARG, "NULL state array");
  if (S->n_partials < dtmpc_general_partials_count(B))
    return set_err(DTMPC_ERR_BAD_ARG, "state->n_partials < dtmpc_general_partials_count(B)");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DTMPC_F32) return launch_general<float>(spec, cfg, B, S, st);
  if (dtype == DTMPC_F64) return launch_general<double>(spec, cfg, B, S, st);
  return set_err(DTMPC_ERR_BAD_ARG, "bad dtype");
}

int dtmpc_partials_reduce_n(int dtype, int64_t n, int32_t width, const void* partials, void* sums, void* stream) {
  if (n < 1 || width < 1 || width > 32 || !partials || !sums) return set_err(DTMPC_ERR_BAD_ARG, "bad partials");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DTMPC_F32)
    hipLaunchKernelGGL(partials_reduce_n_kernel<float>, dim3(1), dim3(kBlock), 0, st, n, (int)width,
                       (const float*)partials, (float*)sums);
  else if (dtype == DTMPC_F64)
    hipLaunchKernelGGL(partials_reduce_n_kernel<double>, dim3(1), dim3(kBlock), 0, st, n, (int)width,
                       (const double*)partials, (double*)sums);
  else
    return set_err(DTMPC_ERR_BAD_ARG, "bad dtype");
  return check_launch("partials_reduce_n_kernel");
}

int dtmpc_general_update(int dtype, const dtmpc_spec* spec, const dtmpc_general_cfg* cfg, double inv_batch,
                         const dtmpc_general_state* state, void* stream) {
  if (!spec || !cfg || !state || !state->sums || !state->theta || !state->velocity)
    return set_err(DTMPC_ERR_BAD_ARG, "NULL argument");
  int alpha_used = spec->barrier_type != DTMPC_BARRIER_LOG;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DTMPC_F32)
    hipLaunchKernelGGL(general_update_kernel<float>, dim3(1), dim3(64), 0, st, (float)cfg->lr_eta,
                       (float)cfg->momentum, cfg->clip_norm, cfg->project_params, cfg->adapt_ancillary,
                       cfg->adapt_nominal, alpha_used, (float)inv_batch, (const float*)state->sums,
                       (float*)state->theta, (float*)state->velocity);
  else if (dtype == DTMPC_F64)
    hipLaunchKernelGGL(general_update_kernel<double>, dim3(1), dim3(64), 0, st, cfg->lr_eta, cfg->momentum,
                       cfg->clip_norm, cfg->project_params, cfg->adapt_ancillary, cfg->adapt_nominal, alpha_used,
                       inv_batch, (const double*)state->sums, (double*)state->theta, (double*)state->velocity);
  else
    return set_err(DTMPC_ERR_BAD_ARG, "bad dtype");
  return check_launch("general_update_kernel");
}

int dtmpc_general_plant(int dtype, const dtmpc_spec* spec, const dtmpc_general_cfg* cfg, int64_t B,
                        int64_t global_offset, int64_t step, const dtmpc_general_state* state, const void* w,
                        void* stream) {
  int e = check_general(spec, cfg, B, state);
  if (e) return e;
  if (cfg->disturbance == 0 && !w) return set_err(DTMPC_ERR_BAD_ARG, "injected disturbance w is NULL");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DTMPC_F32) return launch_plant<float>(spec, cfg, B, global_offset, step, state, w, st);
  if (dtype == DTMPC_F64) return launch_plant<double>(spec, cfg, B, global_offset, step, state, w, st);
  return set_err(DTMPC_ERR_BAD_ARG, "bad dtype");
}

}  // extern "C"
