// dtmpc_solver.hpp — per-trajectory solver bodies (one lane = one trajectory).
//
//   ilqr_traj      core/ddp.py:102-307  ilqr_solve (typed: Dubins + DBaS + obstacles + quad cost)
//   sens_traj      core/ddp.py:317-427  ddp_sensitivity with the paper upper loss
//                  (core/tube_mpc.py:924-957) and, fused, the DOC gradient (:963-976)
#pragma once

#include "dtmpc_device.hpp"

namespace dtmpc {

template <typename T>
__device__ __forceinline__ void cost_diag(const DCost<T>& c, T* lxx, T* luu, T* pxx) {
  lxx[0] = T(2) * c.Q0;
  lxx[1] = T(2) * c.Q1;
  lxx[2] = T(2) * c.Q2;
  lxx[3] = T(2) * c.qb;
  luu[0] = T(2) * c.R0;
  luu[1] = T(2) * c.R1;
  pxx[0] = T(2) * c.Qf0;
  pxx[1] = T(2) * c.Qf1;
  pxx[2] = T(2) * c.Qf2;
  pxx[3] = T(2) * c.qb;
}

// ---------------------------------------------------------------------------------------------
// Feedback gains K [N][2x4] and k [N][2] of the last backward pass, written by the backward pass and
// read by the line search and the commit.  Two layouts:
//   GainsSoA  -- planes [N][8][B] / [N][2][B] (the ABI layout of dtmpc_ilqr_solve's K_out / k_out);
//   GainsAoS  -- per step, each lane's 8 + 2 values contiguous ([N][B][8] / [N][B][2]): two 16-B and
//                one 8-B access per step instead of ten 4-B ones, and a wave's gains of one step in
//                one 2 KB + 512 B span instead of ten planes 4*B bytes apart.  Used for the tube
//                step's internal workspace (the ten-plane stores were the costliest part of the
//                backward pass: without them the tube step ran 16 % faster).
template <typename T>
struct GainsSoA {
  Col<T> K, kf;
  __device__ __forceinline__ void store(int k, const T* Kk, const T* kk) const {
#pragma unroll
    for (int j = 0; j < 8; ++j) K.at(k, 8, j) = Kk[j];
    kf.at(k, 2, 0) = kk[0];
    kf.at(k, 2, 1) = kk[1];
  }
  __device__ __forceinline__ void load(int k, T* Kk, T& k0, T& k1) const {
#pragma unroll
    for (int j = 0; j < 8; ++j) Kk[j] = K.at(k, 8, j);
    k0 = kf.at(k, 2, 0);
    k1 = kf.at(k, 2, 1);
  }
};

template <typename T>
struct GainsAoS {
  typedef T v2 __attribute__((ext_vector_type(2)));
  typedef T v4 __attribute__((ext_vector_type(4)));
  T* Kb;  // [N][B][8]
  T* kb;  // [N][B][2]
  unsigned ld, lane;
  __device__ __forceinline__ T* kp(int k) const {
    return (T*)__builtin_assume_aligned(Kb + ((size_t)(unsigned)k * ld + lane) * 8, 16);
  }
  __device__ __forceinline__ T* fp(int k) const {
    return (T*)__builtin_assume_aligned(kb + ((size_t)(unsigned)k * ld + lane) * 2, 8);
  }
  __device__ __forceinline__ void store(int k, const T* Kk, const T* kk) const {
    T* p = kp(k);
    if constexpr (sizeof(T) == 4) {
      *(v4*)p = v4{Kk[0], Kk[1], Kk[2], Kk[3]};
      *(v4*)(p + 4) = v4{Kk[4], Kk[5], Kk[6], Kk[7]};
    } else {
#pragma unroll
      for (int j = 0; j < 8; j += 2) *(v2*)(p + j) = v2{Kk[j], Kk[j + 1]};
    }
    *(v2*)fp(k) = v2{kk[0], kk[1]};
  }
  __device__ __forceinline__ void load(int k, T* Kk, T& k0, T& k1) const {
    const T* p = kp(k);
    if constexpr (sizeof(T) == 4) {
      v4 a = *(const v4*)p, b = *(const v4*)(p + 4);
      Kk[0] = a.x; Kk[1] = a.y; Kk[2] = a.z; Kk[3] = a.w;
      Kk[4] = b.x; Kk[5] = b.y; Kk[6] = b.z; Kk[7] = b.w;
    } else {
#pragma unroll
      for (int j = 0; j < 8; j += 2) {
        v2 a = *(const v2*)(p + j);
        Kk[j] = a.x;
        Kk[j + 1] = a.y;
      }
    }
    v2 f = *(const v2*)fp(k);
    k0 = f.x;
    k1 = f.y;
  }
};

template <typename T>
__device__ __forceinline__ void load_ref(const DCost<T>& c, const Col<T>& Xr, int rf, int k, T& r0,
                                         T& r1, T& r2) {
  if (c.kind == DTMPC_COST_TRACK) {
    r0 = Xr.at(k, rf, 0);
    r1 = Xr.at(k, rf, 1);
    r2 = Xr.at(k, rf, 2);
  } else {
    r0 = r1 = r2 = T(0);
  }
}

template <typename T>
__device__ __forceinline__ void load_uref(const DCost<T>& c, const Col<T>& Ur, int k, T& q0, T& q1) {
  if (c.kind == DTMPC_COST_TRACK) {
    q0 = Ur.at(k, 2, 0);
    q1 = Ur.at(k, 2, 1);
  } else {
    q0 = q1 = T(0);
  }
}

// ---------------------------------------------------------------------------------------------
// Software prefetch depth of the step loops.  At the benchmark batch there is exactly one wave per
// SIMD, so no other wave hides HBM latency: every pass keeps the loads of the next kPrefetch steps
// in flight (stores share vmcnt with loads on gfx9-family parts, so loads are issued ahead of them).
#ifndef DTMPC_PREFETCH
#define DTMPC_PREFETCH 1
#endif
constexpr int kPrefetch = DTMPC_PREFETCH;

// The backward pass and the commit rollout load their step inputs kRing steps ahead into a RING of
// kRing register buffers that rotates by unrolling the step loop kRing times -- never by copying:
// q[j] = q[j + 1] on a buffer whose load is still in flight makes the copy wait for that load, which
// caps the shift-register form's effective distance at one step whatever its depth.  A step of
// either pass (1,500-3,000 cycles) already outlasts an HBM miss (~900 cycles idle), and deeper rings
// only add registers: the default is 1.
#ifndef DTMPC_RING
#define DTMPC_RING 1  // backward pass; measured (both passes): depth 2 / 3 / 4 = +1 / +2 / +8 % step time
#endif
#ifndef DTMPC_RING_COMMIT
#define DTMPC_RING_COMMIT 3  // commit rollout; measured depth 1 / 2 / 3 / 4 = 7.12 / 7.06 / 7.02 / 7.03 ms
#endif
constexpr int kRing = DTMPC_RING;
constexpr int kRingC = DTMPC_RING_COMMIT;

// Everything the backward pass reads at step k: tape X[k], V[k] and the tracking references.
template <typename T>
struct BackIn {
  T X0, X1, X2, X3, V0, V1, r0, r1, r2, q0, q1;
};

template <typename T>
__device__ __forceinline__ void load_back(BackIn<T>& L, const DCost<T>& c, const Col<T>& X,
                                          const Col<T>& U, const Col<T>& Xr, int rf, const Col<T>& Ur,
                                          int k) {
  L.X0 = X.at(k, 4, 0);
  L.X1 = X.at(k, 4, 1);
  L.X2 = X.at(k, 4, 2);
  L.X3 = X.at(k, 4, 3);
  L.V0 = U.at(k, 2, 0);
  L.V1 = U.at(k, 2, 1);
  load_ref(c, Xr, rf, k, L.r0, L.r1, L.r2);
  load_uref(c, Ur, k, L.q0, L.q1);
}

// ---------------------------------------------------------------------------------------------
// backward pass (core/ddp.py:172-254): linearise along (X, U) and run the Riccati recursion,
// writing K [N][8], kff [N][2].  grad h / B' at x_{k+1} are carried from step k+1 (the reference
// recomputes x_{k+1} = f(x_k, u_k) inside dubins_augmented_jacobian; it is the tape's X[k+1]).
template <typename T, typename G>
__device__ __forceinline__ bool ilqr_backward(const DSpec<T>& s, const DCost<T>& c, T reg, const Col<T>& X,
                              const Col<T>& U, const G& gains,
                              const Col<T>& Xr, int rf, const Col<T>& Ur) {
  const int N = s.N;
  T lxx[4], luu[2], pxx[4];
  cost_diag(c, lxx, luu, pxx);
  T xn0 = X.at(N, 4, 0), xn1 = X.at(N, 4, 1), xn2 = X.at(N, 4, 2), xnb = X.at(N, 4, 3);
  T r0, r1, r2;
  load_ref(c, Xr, rf, N, r0, r1, r2);
  T d0, d1, d2;
  deriv_dx(c, xn0, xn1, xn2, r0, r1, r2, d0, d1, d2);
  Riccati<T> R;
  R.Vx[0] = pxx[0] * d0;
  R.Vx[1] = pxx[1] * d1;
  R.Vx[2] = pxx[2] * d2;
  R.Vx[3] = pxx[3] * xnb;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) R.Vxx[i][j] = i == j ? pxx[i] : T(0);
  T gxn, gyn;
  T hn = h_grad(s, xn0, xn1, gxn, gyn);
  T dBn = dbarrier_relaxed(s, hn);
  bool ok = finite(R.Vx[0]) && finite(R.Vx[1]) && finite(R.Vx[2]) && finite(R.Vx[3]);
  // step inputs (x_k, u_k, references) in a kRing-deep prefetch ring
  BackIn<T> q[kRing];
#pragma unroll
  for (int j = 0; j < kRing; ++j)
    if (N - 1 - j >= 0) load_back(q[j], c, X, U, Xr, rf, Ur, N - 1 - j);
  for (int k0 = N - 1; k0 >= 0; k0 -= kRing) {
#pragma unroll
    for (int jr = 0; jr < kRing; ++jr) {
      const int k = k0 - jr;
      if (k < 0) break;
      const BackIn<T> cur = q[jr];
      if (k - kRing >= 0) load_back(q[jr], c, X, U, Xr, rf, Ur, k - kRing);
      const T x0 = cur.X0, x1 = cur.X1, x2 = cur.X2, xb = cur.X3, u0 = cur.V0, u1 = cur.V1, q0 = cur.q0,
              q1 = cur.q1;
      r0 = cur.r0;
      r1 = cur.r1;
      r2 = cur.r2;
      T sn, cs;
      m_sincos(x2, &sn, &cs);
      T gxk, gyk;
      T hk = h_grad(s, x0, x1, gxk, gyk);
      T dBk = dbarrier_relaxed(s, hk);
      Jac<T> J = make_jac(s, sn, cs, u0, gxk, gyk, dBk, gxn, gyn, dBn);
      deriv_dx(c, x0, x1, x2, r0, r1, r2, d0, d1, d2);
      T lx[4] = {lxx[0] * d0, lxx[1] * d1, lxx[2] * d2, lxx[3] * xb};
      T lu[2];
      if (c.kind == DTMPC_COST_TRACK) {
        lu[0] = luu[0] * (u0 - q0);
        lu[1] = luu[1] * (u1 - q1);
      } else {
        lu[0] = luu[0] * u0;
        lu[1] = luu[1] * u1;
      }
      T Kk[8], kk[2];
      ok = riccati_step(J, lx, lu, lxx, luu, reg, R, Kk, kk) && ok;
      gains.store(k, Kk, kk);
      gxn = gxk;
      gyn = gyk;
      dBn = dBk;
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) ok = ok && finite(R.Vx[i]);
  return ok;
}

// ---------------------------------------------------------------------------------------------
// Everything the forward passes read at step k: old tape X[k], V[k], gains K[k], k[k] and the
// tracking references.  Loaded one step ahead (software prefetch): with one wave per SIMD at the
// benchmark batch there is no other wave to hide HBM latency behind.
template <typename T>
struct StepIn {
  T X0, X1, X2, X3, V0, V1, K[8], k0, k1, r0, r1, r2, q0, q1;
};

template <typename T, typename G>
__device__ __forceinline__ void load_step(StepIn<T>& L, const DCost<T>& c, const Col<T>& X,
                                          const Col<T>& U, const G& gains,
                                          const Col<T>& Xr, int rf, const Col<T>& Ur, int k) {
  L.X0 = X.at(k, 4, 0);
  L.X1 = X.at(k, 4, 1);
  L.X2 = X.at(k, 4, 2);
  L.X3 = X.at(k, 4, 3);
  L.V0 = U.at(k, 2, 0);
  L.V1 = U.at(k, 2, 1);
  gains.load(k, L.K, L.k0, L.k1);
  load_ref(c, Xr, rf, k, L.r0, L.r1, L.r2);
  load_uref(c, Ur, k, L.q0, L.q1);
}

// ---------------------------------------------------------------------------------------------
// line search (core/ddp.py:256-301): the NC rolled-out candidates (cfg.calphas) advance together;
// the alpha = 0 candidate (cfg.zpos) has cost Jprev (the current tape).  Returns the ORIGINAL index
// of the strictly smallest cost (first wins ties), with its alpha in al_out, or -1 if any candidate is
// non-finite.
// The rollouts of NG candidates (alphas al[0..NG)) over the whole horizon, advancing together: their
// total costs into Jout.
template <typename T, int NG, typename G>
__device__ __forceinline__ void ls_rollout(const DSpec<T>& s, const DCost<T>& c, const T* al, const T* x0, T Bc0,
                                           const Col<T>& X, const Col<T>& U, const G& gains, const Col<T>& Xr,
                                           int rf, const Col<T>& Ur, T* Jout) {
  DTMPC_NOCONTRACT
  const int N = s.N;
  T a0[NG], a1[NG], a2[NG], ab[NG], Bc[NG], J[NG];
#pragma unroll
  for (int a = 0; a < NG; ++a) {
    a0[a] = x0[0];
    a1[a] = x0[1];
    a2[a] = x0[2];
    ab[a] = x0[3];
    Bc[a] = Bc0;
    J[a] = T(0);
  }
  StepIn<T> q[kPrefetch];
#pragma unroll
  for (int j = 0; j < kPrefetch; ++j)
    if (j < N) load_step(q[j], c, X, U, gains, Xr, rf, Ur, j);
  for (int k = 0; k < N; ++k) {
    const StepIn<T> cur = q[0];
#pragma unroll
    for (int j = 0; j + 1 < kPrefetch; ++j) q[j] = q[j + 1];
    if (k + kPrefetch < N) load_step(q[kPrefetch - 1], c, X, U, gains, Xr, rf, Ur, k + kPrefetch);
    T u0[NG], u1[NG];
#pragma unroll
    for (int a = 0; a < NG; ++a) {
      T e0 = a0[a] - cur.X0, e1 = a1[a] - cur.X1, e2 = a2[a] - cur.X2, e3 = ab[a] - cur.X3;
      T du0 = cur.k0 + (cur.K[0] * e0 + cur.K[1] * e1 + cur.K[2] * e2 + cur.K[3] * e3);
      T du1 = cur.k1 + (cur.K[4] * e0 + cur.K[5] * e1 + cur.K[6] * e2 + cur.K[7] * e3);
      u0[a] = clampv(cur.V0 + al[a] * du0, s.umin0, s.umax0);
      u1[a] = clampv(cur.V1 + al[a] * du1, s.umin1, s.umax1);
      J[a] = J[a] + stage_cost(c, a0[a], a1[a], a2[a], ab[a], u0[a], u1[a], cur.r0, cur.r1, cur.r2,
                               cur.q0, cur.q1);
    }
    fhat_vec<T, NG>(s, a0, a1, a2, ab, u0, u1, Bc);
  }
  T r0, r1, r2;
  load_ref(c, Xr, rf, N, r0, r1, r2);
#pragma unroll
  for (int a = 0; a < NG; ++a) Jout[a] = J[a] + term_cost(c, a0[a], a1[a], a2[a], ab[a], r0, r1, r2);
}

// candidates [C0, NC) in groups of at most GS rollouts (one pass over the step inputs per group)
template <typename T, int NC, int GS, int C0, typename G>
__device__ __forceinline__ void ls_groups(const DSpec<T>& s, const DCost<T>& c, const DIlqr<T>& cfg, const T* x0,
                                          T Bc0, const Col<T>& X, const Col<T>& U, const G& gains,
                                          const Col<T>& Xr, int rf, const Col<T>& Ur, T* J) {
  constexpr int n = NC - C0 < GS ? NC - C0 : GS;
  T al[n];
#pragma unroll
  for (int a = 0; a < n; ++a) al[a] = cfg.calphas[C0 + a];
  ls_rollout<T, n>(s, c, al, x0, Bc0, X, U, gains, Xr, rf, Ur, J + C0);
  if constexpr (C0 + n < NC) ls_groups<T, NC, GS, C0 + n>(s, c, cfg, x0, Bc0, X, U, gains, Xr, rf, Ur, J);
}

// -D DTMPC_LS_GROUPS_F64=1 rolls the f64 candidates out in two groups of three (two passes over the step
// inputs) instead of six at once.  Measured and kept off (round 3): it cuts the f64 tube kernel's spills
// from 237 VGPRs to 34 but the step goes 18.6 -> 19.7 ms at B = 65,536 -- the second pass costs more than
// the scratch traffic it saves.
#ifndef DTMPC_LS_GROUPS_F64
#define DTMPC_LS_GROUPS_F64 0
#endif

template <typename T, int NC, typename G>
__device__ __forceinline__ int line_search(const DSpec<T>& s, const DCost<T>& c, const DIlqr<T>& cfg,
                                           const T* x0, T Bc0, const Col<T>& X, const Col<T>& U,
                                           const G& gains, const Col<T>& Xr, int rf,
                                           const Col<T>& Ur, T Jprev, T& bestJ, T& al_out) {
  DTMPC_NOCONTRACT
  constexpr int GS = (DTMPC_LS_GROUPS_F64 && sizeof(T) == 8 && NC > 3) ? (NC + 1) / 2 : NC;
  T J[NC];
  ls_groups<T, NC, GS, 0>(s, c, cfg, x0, Bc0, X, U, gains, Xr, rf, Ur, J);
  bool ok = true;
#pragma unroll
  for (int a = 0; a < NC; ++a) ok = ok && finite(J[a]);
  // first strict minimum among the rolled-out candidates (their relative order is the original one)
  int bc = 0;
  bestJ = J[0];
#pragma unroll
  for (int a = 1; a < NC; ++a) {
    if (J[a] < bestJ) {
      bestJ = J[a];
      bc = a;
    }
  }
  int best = cfg.cpos[0];
  al_out = cfg.calphas[0];
#pragma unroll
  for (int a = 1; a < NC; ++a) {
    if (bc == a) {
      best = cfg.cpos[a];
      al_out = cfg.calphas[a];
    }
  }
  if (cfg.zpos >= 0) {
    // the zero candidate sits at zpos: it wins iff it is strictly below every earlier candidate and
    // not above any later one
    T mb = T(0), ma = T(0);
    bool hb = false, ha = false;
#pragma unroll
    for (int a = 0; a < NC; ++a) {
      if (cfg.cpos[a] < cfg.zpos) {
        mb = (!hb || J[a] < mb) ? J[a] : mb;
        hb = true;
      } else {
        ma = (!ha || J[a] < ma) ? J[a] : ma;
        ha = true;
      }
    }
    if ((!hb || Jprev < mb) && (!ha || Jprev <= ma)) {
      best = cfg.zpos;
      bestJ = Jprev;
      al_out = T(0);
    }
    ok = ok && finite(Jprev);
  }
  return ok ? best : -1;
}

// Paired line search: TWO lanes per trajectory (lane half h = 0, 1 of an adjacent lane pair), each
// rolling out every other candidate -- candidate c = 2j + h (the last slot of half 1 repeats candidate
// NC - 1 when NC is odd).  Both halves compute identical tapes everywhere else, so the only exchange
// is here: the per-half first strict minimum (J, candidate) is combined with the partner's by
// lexicographic (J, original position) order, which is exactly "strict <, first wins" over the
// original list; the alpha = 0 rule and the finiteness flag are combined the same way.  Both halves
// return the same decision.
template <typename T, int NC, typename G>
__device__ __forceinline__ int line_search_pair(const DSpec<T>& s, const DCost<T>& c, const DIlqr<T>& cfg,
                                                const T* x0, T Bc0, const Col<T>& X, const Col<T>& U,
                                                const G& gains, const Col<T>& Xr, int rf,
                                                const Col<T>& Ur, T Jprev, T& bestJ, T& al_out, int h) {
  DTMPC_NOCONTRACT
  constexpr int NL = (NC + 1) / 2;
  const int N = s.N;
  T a0[NL], a1[NL], a2[NL], ab[NL], Bc[NL], J[NL], al[NL];
  int ci[NL];
#pragma unroll
  for (int a = 0; a < NL; ++a) {
    const int c0 = 2 * a, c1 = 2 * a + 1 < NC ? 2 * a + 1 : NC - 1;
    ci[a] = h ? c1 : c0;
    al[a] = h ? cfg.calphas[c1] : cfg.calphas[c0];
    a0[a] = x0[0];
    a1[a] = x0[1];
    a2[a] = x0[2];
    ab[a] = x0[3];
    Bc[a] = Bc0;
    J[a] = T(0);
  }
  StepIn<T> q[kPrefetch];
#pragma unroll
  for (int j = 0; j < kPrefetch; ++j)
    if (j < N) load_step(q[j], c, X, U, gains, Xr, rf, Ur, j);
  for (int k = 0; k < N; ++k) {
    const StepIn<T> cur = q[0];
#pragma unroll
    for (int j = 0; j + 1 < kPrefetch; ++j) q[j] = q[j + 1];
    if (k + kPrefetch < N) load_step(q[kPrefetch - 1], c, X, U, gains, Xr, rf, Ur, k + kPrefetch);
    T u0[NL], u1[NL];
#pragma unroll
    for (int a = 0; a < NL; ++a) {
      T e0 = a0[a] - cur.X0, e1 = a1[a] - cur.X1, e2 = a2[a] - cur.X2, e3 = ab[a] - cur.X3;
      T du0 = cur.k0 + (cur.K[0] * e0 + cur.K[1] * e1 + cur.K[2] * e2 + cur.K[3] * e3);
      T du1 = cur.k1 + (cur.K[4] * e0 + cur.K[5] * e1 + cur.K[6] * e2 + cur.K[7] * e3);
      u0[a] = clampv(cur.V0 + al[a] * du0, s.umin0, s.umax0);
      u1[a] = clampv(cur.V1 + al[a] * du1, s.umin1, s.umax1);
      J[a] = J[a] + stage_cost(c, a0[a], a1[a], a2[a], ab[a], u0[a], u1[a], cur.r0, cur.r1, cur.r2,
                               cur.q0, cur.q1);
    }
    fhat_vec<T, NL>(s, a0, a1, a2, ab, u0, u1, Bc);
  }
  T r0, r1, r2;
  load_ref(c, Xr, rf, N, r0, r1, r2);
  bool ok = true;
#pragma unroll
  for (int a = 0; a < NL; ++a) {
    J[a] = J[a] + term_cost(c, a0[a], a1[a], a2[a], ab[a], r0, r1, r2);
    ok = ok && finite(J[a]);
  }
  // this half's first strict minimum (its candidates are in increasing original order)
  T bJ = J[0];
  int bi = ci[0];
#pragma unroll
  for (int a = 1; a < NL; ++a) {
    if (J[a] < bJ) {
      bJ = J[a];
      bi = ci[a];
    }
  }
  // the zero candidate's neighbours: min over candidates before / after position zpos
  T mb = T(0), ma = T(0);
  int hb = 0, ha = 0;
  if (cfg.zpos >= 0) {
#pragma unroll
    for (int a = 0; a < NL; ++a) {
      if (cfg.cpos[ci[a]] < cfg.zpos) {
        mb = (!hb || J[a] < mb) ? J[a] : mb;
        hb = 1;
      } else {
        ma = (!ha || J[a] < ma) ? J[a] : ma;
        ha = 1;
      }
    }
  }
  // combine with the partner lane
  const T oJ = __shfl_xor(bJ, 1, 64);
  const int oi = __shfl_xor(bi, 1, 64);
  ok = __shfl_xor((int)ok, 1, 64) && ok;
  if (oJ < bJ || (oJ == bJ && oi < bi)) {
    bJ = oJ;
    bi = oi;
  }
  bestJ = bJ;
  int best = cfg.cpos[0];
  al_out = cfg.calphas[0];
#pragma unroll
  for (int cc = 1; cc < NC; ++cc) {
    if (bi == cc) {
      best = cfg.cpos[cc];
      al_out = cfg.calphas[cc];
    }
  }
  if (cfg.zpos >= 0) {
    const T omb = __shfl_xor(mb, 1, 64), oma = __shfl_xor(ma, 1, 64);
    const int ohb = __shfl_xor(hb, 1, 64), oha = __shfl_xor(ha, 1, 64);
    if (ohb) mb = (!hb || omb < mb) ? omb : mb;
    if (oha) ma = (!ha || oma < ma) ? oma : ma;
    hb |= ohb;
    ha |= oha;
    if ((!hb || Jprev < mb) && (!ha || Jprev <= ma)) {
      best = cfg.zpos;
      bestJ = Jprev;
      al_out = T(0);
    }
    ok = ok && finite(Jprev);
  }
  return ok ? best : -1;
}

// cost of the tape (X, U) with the line search's accumulation order: the alpha = 0 candidate's cost
// before the first iteration (core/ddp.py:256-301 rolls it out; it is the initial tape)
template <typename T>
__device__ __forceinline__ T tape_cost(const DCost<T>& c, const Col<T>& X, const Col<T>& U,
                                       const Col<T>& Xr, int rf, const Col<T>& Ur, int N) {
  DTMPC_NOCONTRACT
  T J = T(0);
  for (int k = 0; k < N; ++k) {
    T r0, r1, r2, q0, q1;
    load_ref(c, Xr, rf, k, r0, r1, r2);
    load_uref(c, Ur, k, q0, q1);
    J = J + stage_cost(c, T(X.at(k, 4, 0)), T(X.at(k, 4, 1)), T(X.at(k, 4, 2)), T(X.at(k, 4, 3)),
                       T(U.at(k, 2, 0)), T(U.at(k, 2, 1)), r0, r1, r2, q0, q1);
  }
  T r0, r1, r2;
  load_ref(c, Xr, rf, N, r0, r1, r2);
  return J + term_cost(c, T(X.at(N, 4, 0)), T(X.at(N, 4, 1)), T(X.at(N, 4, 2)), T(X.at(N, 4, 3)), r0, r1, r2);
}

// iLQR start (core/ddp.py:127-131 + the alpha = 0 candidate's cost): V = clamp(V_init), X = rollout(x0, V)
// and, if want_cost, the tape's cost -- one pass with U (and the references) prefetched one step ahead,
// instead of a clamp pass, a dependent-load rollout pass and a tape_cost pass.  Same operations in the
// same order as clamp + rollout_traj + tape_cost.
template <typename T>
__device__ __forceinline__ T init_tape(const DSpec<T>& s, const DCost<T>& c, const T* x0, const Col<T>& X,
                                       const Col<T>& U, const Col<T>& Xr, int rf, const Col<T>& Ur,
                                       bool want_cost) {
  DTMPC_NOCONTRACT
  const int N = s.N;
  T s0[1] = {x0[0]}, s1[1] = {x0[1]}, s2[1] = {x0[2]}, sb[1] = {x0[3]};
  T Bc[1] = {barrier_of_state(s, x0[0], x0[1])};
  X.at(0, 4, 0) = s0[0];
  X.at(0, 4, 1) = s1[0];
  X.at(0, 4, 2) = s2[0];
  X.at(0, 4, 3) = sb[0];
  T J = T(0);
  T n0 = U.at(0, 2, 0), n1 = U.at(0, 2, 1), nr0, nr1, nr2, nq0, nq1;
  load_ref(c, Xr, rf, 0, nr0, nr1, nr2);
  load_uref(c, Ur, 0, nq0, nq1);
  for (int k = 0; k < N; ++k) {
    const T v0 = n0, v1 = n1, r0 = nr0, r1 = nr1, r2 = nr2, q0 = nq0, q1 = nq1;
    if (k + 1 < N) {
      n0 = U.at(k + 1, 2, 0);
      n1 = U.at(k + 1, 2, 1);
      load_ref(c, Xr, rf, k + 1, nr0, nr1, nr2);
      load_uref(c, Ur, k + 1, nq0, nq1);
    }
    T u0[1] = {clampv(v0, s.umin0, s.umax0)}, u1[1] = {clampv(v1, s.umin1, s.umax1)};
    U.at(k, 2, 0) = u0[0];
    U.at(k, 2, 1) = u1[0];
    if (want_cost) J = J + stage_cost(c, s0[0], s1[0], s2[0], sb[0], u0[0], u1[0], r0, r1, r2, q0, q1);
    fhat_vec<T, 1>(s, s0, s1, s2, sb, u0, u1, Bc);
    X.at(k + 1, 4, 0) = s0[0];
    X.at(k + 1, 4, 1) = s1[0];
    X.at(k + 1, 4, 2) = s2[0];
    X.at(k + 1, 4, 3) = sb[0];
  }
  if (!want_cost) return T(0);
  T r0, r1, r2;
  load_ref(c, Xr, rf, N, r0, r1, r2);
  return J + term_cost(c, s0[0], s1[0], s2[0], sb[0], r0, r1, r2);
}

// ---------------------------------------------------------------------------------------------
// Materialise the chosen candidate in place: X, U <- rollout with step alpha (same arithmetic
// as the candidate lane of line_search).  X[k+1] of the old tape is read before it is replaced.
template <typename T, typename G>
__device__ __forceinline__ void commit_candidate(const DSpec<T>& s, T al, const T* x0, T Bc0, const Col<T>& X,
                                 const Col<T>& U, const G& gains) {
  DTMPC_NOCONTRACT
  const int N = s.N;
  T s0[1] = {x0[0]}, s1[1] = {x0[1]}, s2[1] = {x0[2]}, sb[1] = {x0[3]}, Bc[1] = {Bc0};
  DCost<T> none;
  none.kind = DTMPC_COST_TARGET;  // the references are not needed here
  Col<T> nc = X;
  StepIn<T> q[kRingC];
#pragma unroll
  for (int j = 0; j < kRingC; ++j)
    if (j < N) load_step(q[j], none, X, U, gains, nc, 0, nc, j);
  for (int k0 = 0; k0 < N; k0 += kRingC) {
#pragma unroll
    for (int jr = 0; jr < kRingC; ++jr) {
      const int k = k0 + jr;
      if (k >= N) break;
      // the ring also fetches the OLD X[k+kRingC] before step k+kRingC-1 overwrites it
      const StepIn<T> cur = q[jr];
      if (k + kRingC < N) load_step(q[jr], none, X, U, gains, nc, 0, nc, k + kRingC);
      T e0 = s0[0] - cur.X0, e1 = s1[0] - cur.X1, e2 = s2[0] - cur.X2, e3 = sb[0] - cur.X3;
      T du0 = cur.k0 + (cur.K[0] * e0 + cur.K[1] * e1 + cur.K[2] * e2 + cur.K[3] * e3);
      T du1 = cur.k1 + (cur.K[4] * e0 + cur.K[5] * e1 + cur.K[6] * e2 + cur.K[7] * e3);
      T u0[1] = {clampv(cur.V0 + al * du0, s.umin0, s.umax0)};
      T u1[1] = {clampv(cur.V1 + al * du1, s.umin1, s.umax1)};
      U.at(k, 2, 0) = u0[0];
      U.at(k, 2, 1) = u1[0];
      fhat_vec<T, 1>(s, s0, s1, s2, sb, u0, u1, Bc);
      X.at(k + 1, 4, 0) = s0[0];
      X.at(k + 1, 4, 1) = s1[0];
      X.at(k + 1, 4, 2) = s2[0];
      X.at(k + 1, 4, 3) = sb[0];
    }
  }
}

// rollout core/ddp.py:89-99 (U used as stored)
template <typename T>
__device__ __forceinline__ void rollout_traj(const DSpec<T>& s, const T* x0, const Col<T>& X, const Col<T>& U) {
  DTMPC_NOCONTRACT
  const int N = s.N;
  T s0[1] = {x0[0]}, s1[1] = {x0[1]}, s2[1] = {x0[2]}, sb[1] = {x0[3]};
  T Bc[1] = {barrier_of_state(s, x0[0], x0[1])};
  X.at(0, 4, 0) = s0[0];
  X.at(0, 4, 1) = s1[0];
  X.at(0, 4, 2) = s2[0];
  X.at(0, 4, 3) = sb[0];
  for (int k = 0; k < N; ++k) {
    T u0[1] = {U.at(k, 2, 0)}, u1[1] = {U.at(k, 2, 1)};
    fhat_vec<T, 1>(s, s0, s1, s2, sb, u0, u1, Bc);
    X.at(k + 1, 4, 0) = s0[0];
    X.at(k + 1, 4, 1) = s1[0];
    X.at(k + 1, 4, 2) = s2[0];
    X.at(k + 1, 4, 3) = sb[0];
  }
}

}  // namespace dtmpc
#include "dtmpc_ls_pk.hpp"
namespace dtmpc {

// f32, even candidate count: the line search on candidate pairs (packed-f32 VALU, dtmpc_ls_pk.hpp)
#ifndef DTMPC_LS_PACKED
#define DTMPC_LS_PACKED 1
#endif
constexpr bool kPackedLS = DTMPC_LS_PACKED != 0;

// ---------------------------------------------------------------------------------------------
// iLQR for one trajectory (core/ddp.py:102-307).  U: in V_init, out V*.  X: out X*.
// K/kf: scratch + gains of the last backward pass.  Returns DTMPC_ST_* bits.
// ch (or NULL): the decision record -- the winning alpha's original position of iteration it at
// ch[it * chs], -1 for iterations not run (written by lane h == 0).
template <typename T, int NA, int LPT = 1, typename G = GainsSoA<T>>
__device__ __forceinline__ int ilqr_traj(const DSpec<T>& s, const DCost<T>& c, const DIlqr<T>& cfg, const T* x0,
                         const Col<T>& X, const Col<T>& U, const G& gains,
                         const Col<T>& Xr, int rf, const Col<T>& Ur, int& iters, Prof& pr,
                         int pb, int h = 0, signed char* ch = nullptr, size_t chs = 0) {
  if (ch && h == 0)
    for (int it = 0; it < cfg.max_iter; ++it) ch[it * chs] = -1;
  // V = clamp(V_init); X = rollout(x0, V)   (:127-131); the cost of that tape is the alpha = 0
  // candidate's cost (only needed when alpha = 0 is listed)
  T Jcur = init_tape(s, c, x0, X, U, Xr, rf, Ur, cfg.zpos >= 0 && cfg.max_iter > 0);
  T Bc0 = barrier_of_state(s, x0[0], x0[1]);
  pr.mark(pb + 0);
  bool have_prev = false;
  T prev = T(0);
  iters = 0;
  for (int it = 0; it < cfg.max_iter; ++it) {
    iters = it + 1;
    if (!ilqr_backward(s, c, cfg.reg, X, U, gains, Xr, rf, Ur)) return DTMPC_ST_NONFINITE;
#ifdef DTMPC_DIAG_BW2  // timing attribution only: the pass again (idempotent)
    __asm__ volatile("" ::: "memory");
    if (!ilqr_backward(s, c, cfg.reg, X, U, gains, Xr, rf, Ur)) return DTMPC_ST_NONFINITE;
#endif
    pr.mark(pb + 1);
    T bestJ, al;
    int best;
    if constexpr (LPT == 2)
      best = line_search_pair<T, NA>(s, c, cfg, x0, Bc0, X, U, gains, Xr, rf, Ur, Jcur, bestJ, al, h);
    else if constexpr (kPackedLS && sizeof(T) == 4 && NA % 2 == 0)
      best = line_search_pk<NA>(s, c, cfg, x0, Bc0, X, U, gains, Xr, rf, Ur, Jcur, bestJ, al);
    else
      best = line_search<T, NA>(s, c, cfg, x0, Bc0, X, U, gains, Xr, rf, Ur, Jcur, bestJ, al);
#ifdef DTMPC_DIAG_LS2  // timing attribution only: the pass again (same decision)
    __asm__ volatile("" ::: "memory");
    best = line_search<T, NA>(s, c, cfg, x0, Bc0, X, U, gains, Xr, rf, Ur, Jcur, bestJ, al);
#endif
    pr.mark(pb + 2);
    if (best < 0) return DTMPC_ST_NONFINITE;
    if (ch && h == 0) ch[it * chs] = (signed char)best;
    if (al != T(0)) commit_candidate(s, al, x0, Bc0, X, U, gains);
#ifdef DTMPC_DIAG_CM2  // timing attribution only: a second rollout (results change)
    __asm__ volatile("" ::: "memory");
    if (al != T(0)) commit_candidate(s, al, x0, Bc0, X, U, gains);
#endif
    Jcur = bestJ;
    pr.mark(pb + 3);
    // :303-305
    if (have_prev && m_abs(prev - bestJ) < cfg.tol) break;
    have_prev = true;
    prev = bestJ;
  }
  return 0;
}

// ---------------------------------------------------------------------------------------------
// Q-blocks of the sensitivity backward step (core/ddp.py:374-377) with l_ux = 0:
//   Q_xx = l_xx + A^T V_xx A, Q_xu = A^T V_xx B, Q_ux = B^T V_xx A, Q_uu = l_uu + B^T V_xx B
template <typename T>
__device__ __forceinline__ void sens_qblocks(const Jac<T>& J, const T (&V)[4][4], const T* lxx, const T* luu,
                                             T (&Qxx)[4][4], T (&Qxu)[4][2], T (&Qux)[2][4],
                                             T (&Quu)[2][2]) {
  T P[4][4];  // A^T V_xx
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    P[0][j] = V[0][j] + J.a30 * V[3][j];
    P[1][j] = V[1][j] + J.a31 * V[3][j];
    P[2][j] = J.a02 * V[0][j] + J.a12 * V[1][j] + V[2][j] + J.a32 * V[3][j];
    P[3][j] = J.g * V[3][j];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    Qxx[i][0] = P[i][0] + P[i][3] * J.a30;
    Qxx[i][1] = P[i][1] + P[i][3] * J.a31;
    Qxx[i][2] = P[i][0] * J.a02 + P[i][1] * J.a12 + P[i][2] + P[i][3] * J.a32;
    Qxx[i][3] = P[i][3] * J.g;
    Qxx[i][i] = lxx[i] + Qxx[i][i];
    // Q_xu = l_ux^T + A^T V_xx B   (:380)
    Qxu[i][0] = P[i][0] * J.b00 + P[i][1] * J.b10 + P[i][3] * J.b30;
    Qxu[i][1] = P[i][2] * J.b21 + P[i][3] * J.b31;
  }
  T S[2][4];  // B^T V_xx
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    S[0][j] = J.b00 * V[0][j] + J.b10 * V[1][j] + J.b30 * V[3][j];
    S[1][j] = J.b21 * V[2][j] + J.b31 * V[3][j];
  }
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    Qux[a][0] = S[a][0] + S[a][3] * J.a30;
    Qux[a][1] = S[a][1] + S[a][3] * J.a31;
    Qux[a][2] = S[a][0] * J.a02 + S[a][1] * J.a12 + S[a][2] + S[a][3] * J.a32;
    Qux[a][3] = S[a][3] * J.g;
    Quu[a][0] = S[a][0] * J.b00 + S[a][1] * J.b10 + S[a][3] * J.b30;
    Quu[a][1] = S[a][2] * J.b21 + S[a][3] * J.b31;
  }
  Quu[0][0] = luu[0] + Quu[0][0];
  Quu[1][1] = luu[1] + Quu[1][1];
}

// ---------------------------------------------------------------------------------------------
// DDP sensitivity (core/ddp.py:317-427) with the paper upper loss (core/tube_mpc.py:932-944):
//   g_x(k) = [2 (x_k - xbar_k), 2 b_k], g_u = 0, same at k = N.
// AB scratch [N][10]: a02 a12 a30 a31 a32 b00 b10 b30 b31 act(=act0 + 2 act1).
// VV scratch [N+1][20] (LAMBDA): V_xx (16) and tilde V_x (4) for delta_lambda.
// GRAD: accumulate the upper loss and the analytic DOC gradient (core/tube_mpc.py:915-976) into
// acc[7] = L, gQ(3), gR(2), gqb with du = U - Ur.
template <typename T, bool LAMBDA, bool OUT, bool GRAD>
__device__ __forceinline__ int sens_traj(const DSpec<T>& s, const DCost<T>& c, const Col<T>& X, const Col<T>& U,
                         const Col<T>& Xr, int rf, const Col<T>& Ur, const Col<T>& Xb, int rfb,
                         const Col<T>& K, const Col<T>& kf, const Col<T>& AB, const Col<T>& VV,
                         const Col<T>& dX, const Col<T>& dU, const Col<T>& dL, T* acc) {
  const int N = s.N;
  T lxx[4], luu[2], pxx[4];
  cost_diag(c, lxx, luu, pxx);
  const T reg = T(1e-9);
  Riccati<T> R;  // R.Vx holds tilde V_x
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) R.Vxx[i][j] = i == j ? pxx[i] : T(0);
  T xn0 = X.at(N, 4, 0), xn1 = X.at(N, 4, 1), xnb = X.at(N, 4, 3);
  R.Vx[0] = T(2) * (xn0 - Xb.at(N, rfb, 0));
  R.Vx[1] = T(2) * (xn1 - Xb.at(N, rfb, 1));
  R.Vx[2] = T(2) * (X.at(N, 4, 2) - Xb.at(N, rfb, 2));
  R.Vx[3] = T(2) * xnb;
  if (LAMBDA) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) VV.at(N, 20, 4 * i + j) = R.Vxx[i][j];
      VV.at(N, 20, 16 + i) = R.Vx[i];
    }
  }
  T gxn, gyn;
  T hn = h_grad(s, xn0, xn1, gxn, gyn);
  T dBn = dbarrier_relaxed(s, hn);
  for (int k = N - 1; k >= 0; --k) {
    T x0 = X.at(k, 4, 0), x1 = X.at(k, 4, 1), x2 = X.at(k, 4, 2), xb = X.at(k, 4, 3);
    T u0 = U.at(k, 2, 0), u1 = U.at(k, 2, 1);
    T sn, cs;
    m_sincos(x2, &sn, &cs);
    T gxk, gyk;
    T hk = h_grad(s, x0, x1, gxk, gyk);
    T dBk = dbarrier_relaxed(s, hk);
    Jac<T> J = make_jac(s, sn, cs, u0, gxk, gyk, dBk, gxn, gyn, dBn);
    gxn = gxk;
    gyn = gyk;
    dBn = dBk;
    T Qxx[4][4], Qxu[4][2], Qux[2][4], Quu[2][2];
    sens_qblocks(J, R.Vxx, lxx, luu, Qxx, Qxu, Qux, Quu);
    const T* tv = R.Vx;
    T tQu0 = J.b00 * tv[0] + J.b10 * tv[1] + J.b30 * tv[3];
    T tQu1 = J.b21 * tv[2] + J.b31 * tv[3];
    T tQx[4];
    tQx[0] = T(2) * (x0 - Xb.at(k, rfb, 0)) + (tv[0] + J.a30 * tv[3]);
    tQx[1] = T(2) * (x1 - Xb.at(k, rfb, 1)) + (tv[1] + J.a31 * tv[3]);
    tQx[2] = T(2) * (x2 - Xb.at(k, rfb, 2)) + (J.a02 * tv[0] + J.a12 * tv[1] + tv[2] + J.a32 * tv[3]);
    tQx[3] = T(2) * xb + J.g * tv[3];
    // active set (core/control.py:66-70)
    bool act0 = (u0 <= s.umin0 + s.active_tol) || (u0 >= s.umax0 - s.active_tol);
    bool act1 = (u1 <= s.umin1 + s.active_tol) || (u1 >= s.umax1 - s.active_tol);
    T m00 = Quu[0][0] + reg, m11 = Quu[1][1] + reg;
    LU2<T> f = lu2(m00, Quu[0][1], Quu[1][0], m11);
    T Kk[8], kk[2];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      T y0, y1;
      solve_reduced(f, m00, m11, act0, act1, Qux[0][j], Qux[1][j], y0, y1);
      Kk[j] = -y0;
      Kk[4 + j] = -y1;
    }
    {
      T y0, y1;
      solve_reduced(f, m00, m11, act0, act1, tQu0, tQu1, y0, y1);
      kk[0] = -y0;
      kk[1] = -y1;
    }
    // tilde V_x = tilde Q_x + Q_xu k ; V_xx = Q_xx + Q_xu K   (:403-404)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      R.Vx[i] = tQx[i] + (Qxu[i][0] * kk[0] + Qxu[i][1] * kk[1]);
#pragma unroll
      for (int j = 0; j < 4; ++j) R.Vxx[i][j] = Qxx[i][j] + (Qxu[i][0] * Kk[j] + Qxu[i][1] * Kk[4 + j]);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) K.at(k, 8, j) = Kk[j];
    kf.at(k, 2, 0) = kk[0];
    kf.at(k, 2, 1) = kk[1];
    AB.at(k, 10, 0) = J.a02;
    AB.at(k, 10, 1) = J.a12;
    AB.at(k, 10, 2) = J.a30;
    AB.at(k, 10, 3) = J.a31;
    AB.at(k, 10, 4) = J.a32;
    AB.at(k, 10, 5) = J.b00;
    AB.at(k, 10, 6) = J.b10;
    AB.at(k, 10, 7) = J.b30;
    AB.at(k, 10, 8) = J.b31;
    AB.at(k, 10, 9) = T((act0 ? 1 : 0) + (act1 ? 2 : 0));
    if (LAMBDA) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) VV.at(k, 20, 4 * i + j) = R.Vxx[i][j];
        VV.at(k, 20, 16 + i) = R.Vx[i];
      }
    }
  }
  // forward (:413-425)
  T d[4] = {T(0), T(0), T(0), T(0)};
  T L1 = T(0), L2 = T(0), gQ0 = T(0), gQ1 = T(0), gQ2 = T(0), gR0 = T(0), gR1 = T(0), gqb = T(0);
  bool ok = true;
  const T g = s.gamma, dt = s.dt;
  for (int k = 0; k < N; ++k) {
    T Kk[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) Kk[j] = K.at(k, 8, j);
    T k0 = kf.at(k, 2, 0), k1 = kf.at(k, 2, 1);
    T a02 = AB.at(k, 10, 0), a12 = AB.at(k, 10, 1), a30 = AB.at(k, 10, 2), a31 = AB.at(k, 10, 3),
      a32 = AB.at(k, 10, 4), b00 = AB.at(k, 10, 5), b10 = AB.at(k, 10, 6), b30 = AB.at(k, 10, 7),
      b31 = AB.at(k, 10, 8);
    int act = (int)AB.at(k, 10, 9);
    T v0 = (act & 1) ? T(0) : k0 + (Kk[0] * d[0] + Kk[1] * d[1] + Kk[2] * d[2] + Kk[3] * d[3]);
    T v1 = (act & 2) ? T(0) : k1 + (Kk[4] * d[0] + Kk[5] * d[1] + Kk[6] * d[2] + Kk[7] * d[3]);
    if (LAMBDA) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        T acc1 = VV.at(k, 20, 4 * i + 0) * d[0] + VV.at(k, 20, 4 * i + 1) * d[1] +
                 VV.at(k, 20, 4 * i + 2) * d[2] + VV.at(k, 20, 4 * i + 3) * d[3];
        dL.at(k, 4, i) = VV.at(k, 20, 16 + i) + acc1;
      }
    }
    if (OUT) {
#pragma unroll
      for (int i = 0; i < 4; ++i) dX.at(k, 4, i) = d[i];
      dU.at(k, 2, 0) = v0;
      dU.at(k, 2, 1) = v1;
    }
    if (GRAD) {
      T e0 = X.at(k, 4, 0) - Xb.at(k, rfb, 0);
      T e1 = X.at(k, 4, 1) - Xb.at(k, rfb, 1);
      T e2 = X.at(k, 4, 2) - Xb.at(k, rfb, 2);
      T bb = X.at(k, 4, 3);
      T w0 = U.at(k, 2, 0) - Ur.at(k, 2, 0);
      T w1 = U.at(k, 2, 1) - Ur.at(k, 2, 1);
      L1 += e0 * e0 + e1 * e1 + e2 * e2;
      L2 += bb * bb;
      gQ0 += T(2) * e0 * d[0];
      gQ1 += T(2) * e1 * d[1];
      gQ2 += T(2) * e2 * d[2];
      gR0 += T(2) * w0 * v0;
      gR1 += T(2) * w1 * v1;
      gqb += T(2) * bb * d[3];
    }
    // delta x_{k+1} = A delta x_k + B delta u_k
    T n0 = (d[0] + a02 * d[2]) + b00 * v0;
    T n1 = (d[1] + a12 * d[2]) + b10 * v0;
    T n2 = d[2] + dt * v1;
    T n3 = (a30 * d[0] + a31 * d[1] + a32 * d[2] + g * d[3]) + (b30 * v0 + b31 * v1);
    d[0] = n0;
    d[1] = n1;
    d[2] = n2;
    d[3] = n3;
  }
  if (LAMBDA) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      T acc1 = VV.at(N, 20, 4 * i + 0) * d[0] + VV.at(N, 20, 4 * i + 1) * d[1] +
               VV.at(N, 20, 4 * i + 2) * d[2] + VV.at(N, 20, 4 * i + 3) * d[3];
      dL.at(N, 4, i) = VV.at(N, 20, 16 + i) + acc1;
    }
  }
  if (OUT) {
#pragma unroll
    for (int i = 0; i < 4; ++i) dX.at(N, 4, i) = d[i];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) ok = ok && finite(d[i]);
  if (GRAD) {
    T e0 = X.at(N, 4, 0) - Xb.at(N, rfb, 0);
    T e1 = X.at(N, 4, 1) - Xb.at(N, rfb, 1);
    T e2 = X.at(N, 4, 2) - Xb.at(N, rfb, 2);
    T bb = X.at(N, 4, 3);
    L1 += e0 * e0 + e1 * e1 + e2 * e2;
    L2 += bb * bb;
    acc[0] = L1 + L2;
    acc[1] = gQ0 + T(2) * e0 * d[0];
    acc[2] = gQ1 + T(2) * e1 * d[1];
    acc[3] = gQ2 + T(2) * e2 * d[2];
    acc[4] = gR0;
    acc[5] = gR1;
    acc[6] = gqb + T(2) * bb * d[3];
    ok = ok && finite(acc[1]) && finite(acc[4]) && finite(acc[5]);
  }
  return ok ? 0 : DTMPC_ST_NONFINITE;
}

}  // namespace dtmpc
