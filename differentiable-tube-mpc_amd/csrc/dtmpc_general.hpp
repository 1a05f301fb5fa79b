// dtmpc_general.hpp — device bodies of the GENERAL IFT path (core/tube_mpc.py:40-663).
//
//   GPar / gpar_from   core/params.py:9-59  softplus / tanh parameterisation + its derivatives
//   sens_ift_traj      core/ddp.py:317-427  ddp_sensitivity with arbitrary upper gradients, fused
//                      with core/ift.py:35-92 ift_gradient in closed form (oracle/oracle_general.h
//                      derives every term) and, for the ancillary, dL/dX_ref, dL/dU_ref
//   ift_step / ift_terminal   the per-step terms of ift_gradient (also used stand-alone)
//
// Same mapping as the paper path: one lane per trajectory, SoA [step][field][B] tapes.
#pragma once

#include "dtmpc_solver.hpp"

namespace dtmpc {

__device__ __forceinline__ float m_log1p(float x) { return log1pf(x); }
__device__ __forceinline__ double m_log1p(double x) { return log1p(x); }
__device__ __forceinline__ float m_tanh(float x) { return tanhf(x); }
__device__ __forceinline__ double m_tanh(double x) { return tanh(x); }

// torch.nn.functional.softplus (beta 1, threshold 20) and its backward.  Evaluated once per launch
// per parameter, so the accurate library exp / log1p are used in f32 as well.
template <typename T>
__device__ __forceinline__ T softplus(T x) {
  return x > T(20) ? x : m_log1p(exp(x));
}
template <typename T>
__device__ __forceinline__ T softplus_d(T x) {
  if (x > T(20)) return T(1);
  T z = exp(x);
  return z / (z + T(1));
}

template <typename T>
struct GPar {
  T Q[3], R[2], Qf[3], qb, alpha, gamma, tight;
  T dQ[3], dR[2], dQf[3], dqb, dalpha, dgamma, dtight;  // d value / d raw
};

// NominalTheta / AuxiliaryTheta (core/params.py:28-35, 49-56) from the raw [12] block
template <typename T>
__device__ __forceinline__ GPar<T> gpar_from(const T* raw, bool nominal) {
  GPar<T> p;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    p.Q[i] = softplus(raw[DTMPC_P_Q + i]);
    p.dQ[i] = softplus_d(raw[DTMPC_P_Q + i]);
    p.Qf[i] = softplus(raw[DTMPC_P_QF + i]);
    p.dQf[i] = softplus_d(raw[DTMPC_P_QF + i]);
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    p.R[j] = softplus(raw[DTMPC_P_R + j]);
    p.dR[j] = softplus_d(raw[DTMPC_P_R + j]);
  }
  p.qb = softplus(raw[DTMPC_P_QB]);
  p.dqb = softplus_d(raw[DTMPC_P_QB]);
  p.alpha = softplus(raw[DTMPC_P_ALPHA]) + T(1e-6);
  p.dalpha = softplus_d(raw[DTMPC_P_ALPHA]);
  p.gamma = m_tanh(raw[DTMPC_P_GAMMA]);
  p.dgamma = T(1) - p.gamma * p.gamma;
  p.tight = nominal ? softplus(raw[DTMPC_P_TIGHT]) : T(0);
  p.dtight = nominal ? softplus_d(raw[DTMPC_P_TIGHT]) : T(0);
  return p;
}

// spec / cost of a solve with the parameterised DBaS and weights (core/tube_mpc.py:134-149,
// 230-256, 347-379).  The obstacle table stays in the kernarg segment (kspec()).
template <typename T>
__device__ __forceinline__ DSpec<T> gspec(const DSpec<T>& s, const GPar<T>& p) {
  DSpec<T> o = s;
  o.alpha = p.alpha;
  o.gamma = p.gamma;
  o.tight = p.tight;
  return o;
}

template <typename T>
__device__ __forceinline__ DCost<T> gcost(const GPar<T>& p, int kind, const T* target) {
  DCost<T> c;
  c.kind = kind;
  c.wrap = 0;
  c.Q0 = p.Q[0];
  c.Q1 = p.Q[1];
  c.Q2 = p.Q[2];
  c.R0 = p.R[0];
  c.R1 = p.R[1];
  c.Qf0 = p.Qf[0];
  c.Qf1 = p.Qf[1];
  c.Qf2 = p.Qf[2];
  c.qb = p.qb;
  c.t0 = kind == DTMPC_COST_TARGET ? target[0] : T(0);
  c.t1 = kind == DTMPC_COST_TARGET ? target[1] : T(0);
  c.t2 = kind == DTMPC_COST_TARGET ? target[2] : T(0);
  return c;
}

// dB/dz of the dynamics barrier (autograd of core/barrier.py:36-72)
template <typename T>
__device__ __forceinline__ T dbarrier_dyn(const DSpec<T>& s, T z) {
  if (s.barrier == DTMPC_BARRIER_LOG) return z >= s.eps ? T(-1) / z : T(0);
  return dbarrier_relaxed(s, z);
}

// dB_alpha / d alpha_eff of the relaxed inverse barrier: 0 on the safe branch, -3 (z-a)^2 / a^4
template <typename T>
__device__ __forceinline__ T dbarrier_da(const DSpec<T>& s, T z) {
  if (s.barrier == DTMPC_BARRIER_LOG) return T(0);
  T a = s.alpha > s.eps ? s.alpha : s.eps;
  if (z >= a) return T(0);
  T d = z - a;
  T a2 = a * a;
  return T(-3) * (d * d) / (a2 * a2);
}

template <typename T>
__device__ __forceinline__ T h_value(const DSpec<T>& s, T px, T py) {
  T h[1], x[1] = {px}, y[1] = {py};
  h_vec<T, 1>(s, x, y, h);
  return h[0];
}

// running sums of ift_gradient (before the softplus / tanh chain)
template <typename T>
struct IftAcc {
  T gQ[3], gR[2], gQf[3], gqb, ga, gg, gs;
  __device__ __forceinline__ void zero() {
    gQ[0] = gQ[1] = gQ[2] = gR[0] = gR[1] = gQf[0] = gQf[1] = gQf[2] = T(0);
    gqb = ga = gg = gs = T(0);
  }
};

// step k < N of ift_gradient: cost terms of l_x . dx_k, l_u . du_k and the DBaS dynamics term
// dlam_{k+1,b} . b'(x_k, u_k; theta), x' = f(x_k, u_k) recomputed as the reference does
// (core/ift.py:76-80).  (r, q): tracking references of step k (ancillary) or the target / 0.
template <typename T>
__device__ __forceinline__ void ift_step(const DSpec<T>& s, const T* xk, const T* uk, const T* dxk,
                                         const T* duk, T lam, const T* r, const T* q, IftAcc<T>& A) {
#pragma unroll
  for (int i = 0; i < 3; ++i) A.gQ[i] += T(2) * (xk[i] - r[i]) * dxk[i];
#pragma unroll
  for (int j = 0; j < 2; ++j) A.gR[j] += T(2) * (uk[j] - q[j]) * duk[j];
  A.gqb += T(2) * xk[3] * dxk[3];
  T sn, cs;
  m_sincos(xk[2], &sn, &cs);
  T dv = s.dt * uk[0];
  T hn = h_value(s, xk[0] + dv * cs, xk[1] + dv * sn) - s.tight;
  T hc = h_value(s, xk[0], xk[1]) - s.tight;
  T Bc = barrier_dyn(s, hc);
  A.gg += lam * (-(Bc - xk[3]));
  A.ga += lam * (dbarrier_da(s, hn) - s.gamma * dbarrier_da(s, hc));
  A.gs += lam * (-dbarrier_dyn(s, hn) + s.gamma * dbarrier_dyn(s, hc));
}

template <typename T>
__device__ __forceinline__ void ift_terminal(const T* xN, const T* dxN, const T* r, IftAcc<T>& A) {
#pragma unroll
  for (int i = 0; i < 3; ++i) A.gQf[i] += T(2) * (xN[i] - r[i]) * dxN[i];
  A.gqb += T(2) * xN[3] * dxN[3];
}

// chain through core/params.py into the raw layout DTMPC_P_* (g[12])
template <typename T>
__device__ __forceinline__ void ift_finish(const DSpec<T>& s, const GPar<T>& p, const IftAcc<T>& A, bool track,
                                           T* g) {
  T dmax = p.alpha > s.eps ? T(1) : (p.alpha == s.eps ? T(0.5) : T(0));
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    g[DTMPC_P_Q + i] = A.gQ[i] * p.dQ[i];
    g[DTMPC_P_QF + i] = A.gQf[i] * p.dQf[i];
  }
  g[DTMPC_P_R] = A.gR[0] * p.dR[0];
  g[DTMPC_P_R + 1] = A.gR[1] * p.dR[1];
  g[DTMPC_P_QB] = A.gqb * p.dqb;
  g[DTMPC_P_ALPHA] = A.ga * dmax * p.dalpha;
  g[DTMPC_P_GAMMA] = A.gg * p.dgamma;
  g[DTMPC_P_TIGHT] = track ? T(0) : A.gs * p.dtight;
}

// sources of the upper-level gradients g_x, g_u of sens_ift_traj
constexpr int kUpperPaper = 0;   // [2 (x_k - xbar_k), 2 b_k], 0 (ancillary, core/tube_mpc.py:424-439)
constexpr int kUpperArrays = 1;  // Gx [N+1][4], Gu [N][2] as given (dtmpc_ddp_sensitivity_upper)
constexpr int kUpperRef = 2;     // Gx = the ancillary's Gn [N+1][5]: [dL/dX_ref_k, 0], dL/dU_ref_k (:511-530)

// ---------------------------------------------------------------------------------------------
// ddp_sensitivity with general upper gradients (core/ddp.py:317-427), optionally fused with the IFT
// gradient of the same solve.
//   UPPER:       kUpperPaper (xbar = Xb, rfb fields per row), kUpperArrays or kUpperRef (see above).
//   IFT:         accumulate ift_gradient (cost kind c.kind; references Xr/Ur for TRACK) into g[12],
//                and for TRACK write the nominal's upper gradients [dL/dX_ref, 0], dL/dU_ref into
//                Gn [N+1][5] (fields 0-2 = -2 Q dx, 3-4 = -2 R du; row N fields 0-2 = -2 Qf dx_N).
//   OUT:         write dX [N+1][4], dU [N][2], dlam [N+1][4] (dlam when LAMBDA_OUT).
// Scratch: K [N][8], kf [N][2], AB [N][10], VV [N+1][5] (row b of V_xx and tilde V_x[b]: the IFT needs
// delta_lambda_b only), VF [N+1][20] (all of V_xx, tilde V_x) when LAMBDA_OUT writes dL [N+1][4].
template <typename T, int UPPER, bool IFT, bool OUT, bool LAMBDA_OUT>
__device__ __forceinline__ int sens_ift_traj(const DSpec<T>& s, const DCost<T>& c, const GPar<T>& p,
                                             const Col<T>& X, const Col<T>& U, const Col<T>& Xr, int rf,
                                             const Col<T>& Ur, const Col<T>& Xb, int rfb, const Col<T>& Gx,
                                             const Col<T>& Gu, const Col<T>& K, const Col<T>& kf,
                                             const Col<T>& AB, const Col<T>& VV, const Col<T>& VF,
                                             const Col<T>& Gn, const Col<T>& dX, const Col<T>& dU,
                                             const Col<T>& dL, T* g) {
  const int N = s.N;
  const bool track = c.kind == DTMPC_COST_TRACK;
  T lxx[4], luu[2], pxx[4];
  cost_diag(c, lxx, luu, pxx);
  const T reg = T(1e-9);
  Riccati<T> R;  // R.Vx holds tilde V_x
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) R.Vxx[i][j] = i == j ? pxx[i] : T(0);
  T xn0 = X.at(N, 4, 0), xn1 = X.at(N, 4, 1), xn2 = X.at(N, 4, 2), xnb = X.at(N, 4, 3);
  if (UPPER == kUpperPaper) {
    R.Vx[0] = T(2) * (xn0 - Xb.at(N, rfb, 0));
    R.Vx[1] = T(2) * (xn1 - Xb.at(N, rfb, 1));
    R.Vx[2] = T(2) * (xn2 - Xb.at(N, rfb, 2));
    R.Vx[3] = T(2) * xnb;
  } else if (UPPER == kUpperArrays) {
#pragma unroll
    for (int i = 0; i < 4; ++i) R.Vx[i] = Gx.at(N, 4, i);
  } else {
#pragma unroll
    for (int i = 0; i < 3; ++i) R.Vx[i] = Gx.at(N, 5, i);
    R.Vx[3] = T(0);
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) VV.at(N, 5, j) = R.Vxx[3][j];
  VV.at(N, 5, 4) = R.Vx[3];
  if (LAMBDA_OUT) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) VF.at(N, 20, 4 * i + j) = R.Vxx[i][j];
      VF.at(N, 20, 16 + i) = R.Vx[i];
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
    T gx[4], gu[2];
    if (UPPER == kUpperPaper) {
      gx[0] = T(2) * (x0 - Xb.at(k, rfb, 0));
      gx[1] = T(2) * (x1 - Xb.at(k, rfb, 1));
      gx[2] = T(2) * (x2 - Xb.at(k, rfb, 2));
      gx[3] = T(2) * xb;
      gu[0] = gu[1] = T(0);
    } else if (UPPER == kUpperArrays) {
#pragma unroll
      for (int i = 0; i < 4; ++i) gx[i] = Gx.at(k, 4, i);
      gu[0] = Gu.at(k, 2, 0);
      gu[1] = Gu.at(k, 2, 1);
    } else {
#pragma unroll
      for (int i = 0; i < 3; ++i) gx[i] = Gx.at(k, 5, i);
      gx[3] = T(0);
      gu[0] = Gx.at(k, 5, 3);
      gu[1] = Gx.at(k, 5, 4);
    }
    const T* tv = R.Vx;
    // tilde Q_u = g_u + B^T tilde V_x ; tilde Q_x = g_x + A^T tilde V_x   (:383-384)
    T tQu0 = gu[0] + (J.b00 * tv[0] + J.b10 * tv[1] + J.b30 * tv[3]);
    T tQu1 = gu[1] + (J.b21 * tv[2] + J.b31 * tv[3]);
    T tQx[4];
    tQx[0] = gx[0] + (tv[0] + J.a30 * tv[3]);
    tQx[1] = gx[1] + (tv[1] + J.a31 * tv[3]);
    tQx[2] = gx[2] + (J.a02 * tv[0] + J.a12 * tv[1] + tv[2] + J.a32 * tv[3]);
    tQx[3] = gx[3] + J.g * tv[3];
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
#pragma unroll
    for (int j = 0; j < 4; ++j) VV.at(k, 5, j) = R.Vxx[3][j];
    VV.at(k, 5, 4) = R.Vx[3];
    if (LAMBDA_OUT) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
#pragma unroll
        for (int j = 0; j < 4; ++j) VF.at(k, 20, 4 * i + j) = R.Vxx[i][j];
        VF.at(k, 20, 16 + i) = R.Vx[i];
      }
    }
  }
  // forward (:413-425), fused with ift_gradient
  T d[4] = {T(0), T(0), T(0), T(0)};
  IftAcc<T> A;
  A.zero();
  const T g_ = s.gamma, dt = s.dt;
  bool ok = true;
  T tgt[3] = {c.t0, c.t1, c.t2};
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
    if (OUT) {
#pragma unroll
      for (int i = 0; i < 4; ++i) dX.at(k, 4, i) = d[i];
      dU.at(k, 2, 0) = v0;
      dU.at(k, 2, 1) = v1;
    }
    T n0 = (d[0] + a02 * d[2]) + b00 * v0;
    T n1 = (d[1] + a12 * d[2]) + b10 * v0;
    T n2 = d[2] + dt * v1;
    T n3 = (a30 * d[0] + a31 * d[1] + a32 * d[2] + g_ * d[3]) + (b30 * v0 + b31 * v1);
    if (IFT) {
      // delta_lambda_{k+1, b} = tilde V_x[b] + V_xx[b, :] delta x_{k+1}   (:422, :425)
      T lam = VV.at(k + 1, 5, 4) + (VV.at(k + 1, 5, 0) * n0 + VV.at(k + 1, 5, 1) * n1 +
                                    VV.at(k + 1, 5, 2) * n2 + VV.at(k + 1, 5, 3) * n3);
      T xk[4] = {X.at(k, 4, 0), X.at(k, 4, 1), X.at(k, 4, 2), X.at(k, 4, 3)};
      T uk[2] = {U.at(k, 2, 0), U.at(k, 2, 1)};
      T r[3], q[2];
      if (track) {
        r[0] = Xr.at(k, rf, 0);
        r[1] = Xr.at(k, rf, 1);
        r[2] = Xr.at(k, rf, 2);
        q[0] = Ur.at(k, 2, 0);
        q[1] = Ur.at(k, 2, 1);
        // the nominal's upper gradients dL/dX_ref_k = -2 Q dx_k, dL/dU_ref_k = -2 R du_k
        Gn.at(k, 5, 0) = -(T(2) * p.Q[0]) * d[0];
        Gn.at(k, 5, 1) = -(T(2) * p.Q[1]) * d[1];
        Gn.at(k, 5, 2) = -(T(2) * p.Q[2]) * d[2];
        Gn.at(k, 5, 3) = -(T(2) * p.R[0]) * v0;
        Gn.at(k, 5, 4) = -(T(2) * p.R[1]) * v1;
      } else {
        r[0] = tgt[0];
        r[1] = tgt[1];
        r[2] = tgt[2];
        q[0] = q[1] = T(0);
      }
      T dxk[4] = {d[0], d[1], d[2], d[3]}, duk[2] = {v0, v1};
      ift_step(s, xk, uk, dxk, duk, lam, r, q, A);
    }
    if (LAMBDA_OUT) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        T acc1 = VF.at(k, 20, 4 * i + 0) * d[0] + VF.at(k, 20, 4 * i + 1) * d[1] +
                 VF.at(k, 20, 4 * i + 2) * d[2] + VF.at(k, 20, 4 * i + 3) * d[3];
        dL.at(k, 4, i) = VF.at(k, 20, 16 + i) + acc1;
      }
    }
    d[0] = n0;
    d[1] = n1;
    d[2] = n2;
    d[3] = n3;
  }
  if (OUT) {
#pragma unroll
    for (int i = 0; i < 4; ++i) dX.at(N, 4, i) = d[i];
  }
  if (LAMBDA_OUT) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      T acc1 = VF.at(N, 20, 4 * i + 0) * d[0] + VF.at(N, 20, 4 * i + 1) * d[1] +
               VF.at(N, 20, 4 * i + 2) * d[2] + VF.at(N, 20, 4 * i + 3) * d[3];
      dL.at(N, 4, i) = VF.at(N, 20, 16 + i) + acc1;
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) ok = ok && finite(d[i]);
  if (IFT) {
    T xN[4] = {X.at(N, 4, 0), X.at(N, 4, 1), X.at(N, 4, 2), X.at(N, 4, 3)};
    T r[3];
    if (track) {
      r[0] = Xr.at(N, rf, 0);
      r[1] = Xr.at(N, rf, 1);
      r[2] = Xr.at(N, rf, 2);
      Gn.at(N, 5, 0) = -(T(2) * p.Qf[0]) * d[0];
      Gn.at(N, 5, 1) = -(T(2) * p.Qf[1]) * d[1];
      Gn.at(N, 5, 2) = -(T(2) * p.Qf[2]) * d[2];
    } else {
      r[0] = tgt[0];
      r[1] = tgt[1];
      r[2] = tgt[2];
    }
    ift_terminal(xN, d, r, A);
    ift_finish(s, p, A, track, g);
#pragma unroll
    for (int j = 0; j < DTMPC_P_COUNT; ++j) ok = ok && finite(g[j]);
  }
  return ok ? 0 : DTMPC_ST_NONFINITE;
}

}  // namespace dtmpc
