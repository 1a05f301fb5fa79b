// dtmpc_device.hpp — CDNA4 device code for the batched DDP/IFT tube-MPC hot path.
//
// Mapping: ONE LANE PER TRAJECTORY.  A wave holds 64 independent trajectories;
// every per-step tape (states, controls, gains) lives in HBM in SoA [step][field][B] order, so each
// per-step load/store of a field is one fully coalesced 256 B (f32) line per wave.  The small
// per-step blocks (4x4 Riccati matrices, 2x2 solves) stay in VGPRs, the obstacle parameters in
// SGPRs.  The line search advances all L alphas in the same loop over k (L-wide ILP, one tape read
// per step instead of L).
//
// Every function cites the reference (lmcggg/differentiable-tube-mpc) code it restates.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dtmpc.h"

namespace dtmpc {

// Forward-pass arithmetic (rollouts, line-search candidates, commit, costs, h, barriers) is
// evaluated WITHOUT multiply-add contraction: every product and sum rounded as the reference's
// PyTorch CPU code rounds it.  This makes the scalar and the packed-pair (dtmpc_ls_pk.hpp) forms
// of a rollout bitwise identical by construction -- the committed tape is exactly the candidate the
// line search priced -- instead of depending on where the compiler happens to fuse.
#define DTMPC_NOCONTRACT _Pragma("clang fp contract(off)")

// ---------------------------------------------------------------------------------------------
// math helpers (precision-overloaded).
// f64 (parity builds) uses the OCML functions.  f32 (the benchmark precision) uses the CDNA4
// transcendental units directly for exp / log (v_exp_f32 / v_log_f32, base 2) and reciprocals
// (v_rcp_f32): 1-2 instructions each instead of 15-40.  sin/cos: sincos_cw below (the native
// v_sin_f32 / v_cos_f32 were measured (round 1) to push the f32 tube-step gradients and nominal
// plans outside the oracle-calibrated parity gates of tests/test_gpu_parity.py).
// f32 sin/cos: Cody-Waite reduction by pi/2 in three fma steps and the Cephes minimax polynomials on
// [-pi/4, pi/4] (max 1.5 ulp, mean 0.34 ulp against the exact values, measured over 1.1e5 points in
// [-1e3, 1e3]); |x| > 65536, inf and NaN take OCML sincosf.  Every step is an explicit fma / mul, so
// the packed-pair form (pk_sincos, dtmpc_ls_pk.hpp) gives bitwise the same values.
constexpr float kSinS1 = -1.6666654611e-1f, kSinS2 = 8.3321608736e-3f, kSinS3 = -1.9515295891e-4f;
constexpr float kCosK1 = 4.166664568298827e-2f, kCosK2 = -1.388731625493765e-3f, kCosK3 = 2.443315711809948e-5f;
constexpr float kPio2A = 1.57079637050628662109375f, kPio2B = -4.37113900018624283e-08f,
                kPio2C = -1.77635683940025046e-15f, k2oPi = 0.636619772367581343f;
__device__ __forceinline__ void sincos_cw(float x, float* sp, float* cp) {
  const float q = __builtin_rintf(x * k2oPi);
  float r = __builtin_fmaf(-q, kPio2A, x);
  r = __builtin_fmaf(-q, kPio2B, r);
  r = __builtin_fmaf(-q, kPio2C, r);
  const float z = r * r;
  float ps = __builtin_fmaf(z, kSinS3, kSinS2);
  ps = __builtin_fmaf(z, ps, kSinS1);
  const float sn = __builtin_fmaf(r * z, ps, r);
  float pc = __builtin_fmaf(z, kCosK3, kCosK2);
  pc = __builtin_fmaf(z, pc, kCosK1);
  const float cs = __builtin_fmaf(z * z, pc, __builtin_fmaf(-0.5f, z, 1.0f));
  const int j = (int)q & 3;
  float so = (j & 1) ? cs : sn, co = (j & 1) ? sn : cs;
  *sp = (j & 2) ? -so : so;
  *cp = ((j + 1) & 2) ? -co : co;
}
__device__ __forceinline__ void m_sincos(float x, float* s, float* c) {
#ifdef DTMPC_OCML_SINCOS
  sincosf(x, s, c);
#else
  if (__builtin_expect(!(__builtin_fabsf(x) <= 65536.0f), 0)) {
    sincosf(x, s, c);
    return;
  }
  sincos_cw(x, s, c);
#endif
}
__device__ __forceinline__ void m_sincos(double x, double* s, double* c) { sincos(x, s, c); }
__device__ __forceinline__ float m_exp(float x) { return __builtin_amdgcn_exp2f(x * 1.44269504088896341f); }
__device__ __forceinline__ double m_exp(double x) { return exp(x); }
__device__ __forceinline__ float m_log(float x) { return __builtin_amdgcn_logf(x) * 0.693147180559945309f; }
__device__ __forceinline__ double m_log(double x) { return log(x); }
__device__ __forceinline__ float m_rcp(float x) { return __builtin_amdgcn_rcpf(x); }
__device__ __forceinline__ double m_rcp(double x) { return 1.0 / x; }
__device__ __forceinline__ float m_atan2(float y, float x) { return atan2f(y, x); }
__device__ __forceinline__ double m_atan2(double y, double x) { return atan2(y, x); }
__device__ __forceinline__ float m_min(float a, float b) { return __builtin_fminf(a, b); }
__device__ __forceinline__ double m_min(double a, double b) { return __builtin_fmin(a, b); }
__device__ __forceinline__ float m_abs(float x) { return fabsf(x); }
__device__ __forceinline__ double m_abs(double x) { return fabs(x); }
template <typename T>
__device__ __forceinline__ bool finite(T x) {
  return __builtin_isfinite(x);
}
// torch.clamp semantics: NaN propagates (core/control.py:61-64)
template <typename T>
__device__ __forceinline__ T clampv(T v, T lo, T hi) {
  return v < lo ? lo : (v > hi ? hi : v);
}
template <typename T>
__device__ __forceinline__ T wrap_angle(T e) {  // run_nominal.py:32-34
  T s, c;
  m_sincos(e, &s, &c);
  return m_atan2(s, c);
}

// ---------------------------------------------------------------------------------------------
// Phase timers for profiling builds only (build.py --variant prof -D DTMPC_PROFILE): per-lane
// s_memtime deltas accumulated per phase, summed by lane 0 of every wave into g_prof.  In product
// builds Prof is empty and every call folds away.
#ifdef DTMPC_PROFILE
__device__ unsigned long long g_prof[16];
struct Prof {
  unsigned long long acc[12], last;
  __device__ __forceinline__ void start() {
#pragma unroll
    for (int i = 0; i < 12; ++i) acc[i] = 0;
    last = __builtin_readcyclecounter();
  }
  __device__ __forceinline__ void mark(int i) {
    unsigned long long t = __builtin_readcyclecounter();
    acc[i] += t - last;
    last = t;
  }
  __device__ __forceinline__ void flush() {
    if ((threadIdx.x & 63) == 0)
      for (int i = 0; i < 12; ++i) atomicAdd(&g_prof[i], acc[i]);
  }
};
#else
struct Prof {
  __device__ __forceinline__ void start() {}
  __device__ __forceinline__ void mark(int) {}
  __device__ __forceinline__ void flush() {}
};
#endif

// ---------------------------------------------------------------------------------------------
// typed problem description (built on the host from dtmpc_spec / dtmpc_cost / dtmpc_ilqr_cfg)
template <typename T>
struct DSpec {
  int N, M, agg, barrier;
  T dt, umin0, umin1, umax0, umax1, active_tol;
  T neg_beta, neg_inv_beta;  // (-beta), -(1/beta) as the reference's python floats
  T alpha, gamma, eps;
  T tight;  // h offset of the DBaS dynamics (nominal tightening s, core/tube_mpc.py:151-153); 0 else
  T cx[DTMPC_MAX_OBS], cy[DTMPC_MAX_OBS], r2[DTMPC_MAX_OBS];
};

template <typename T>
struct DCost {
  int kind, wrap;
  T Q0, Q1, Q2, R0, R1, Qf0, Qf1, Qf2, qb, t0, t1, t2;
};

template <typename T>
struct DIlqr {
  int max_iter, na;
  T tol, reg;
  T alphas[DTMPC_MAX_ALPHAS];
  // line-search candidates that need a rollout: the non-zero alphas in order (calphas, original
  // positions cpos), and zpos = position of the first alpha == 0 (-1 if none).  The alpha = 0
  // candidate is clamp(V + 0 du) = V, i.e. the current tape, whose cost is the previous iteration's
  // best J (or the initial tape's cost): it is never rolled out (core/ddp.py:256-301 semantics kept,
  // including the first-wins tie order).
  int nc, zpos;
  int cpos[DTMPC_MAX_ALPHAS];
  T calphas[DTMPC_MAX_ALPHAS];
};

// One trajectory's view of a SoA [rows][F][B] array: element (k, f) of lane `lane` lives at
// base[(k*F + f)*ld + lane].  base/ld/k are wave-uniform, so the plane address is scalar (SALU) and
// the per-lane part is a single 32-bit offset: one coalesced 256 B (f32) line per wave per access.
template <typename T>
struct Col {
  T* base;
  unsigned ld;    // B
  unsigned lane;  // trajectory index
  // (A raw-buffer-resource form of this accessor -- SGPR plane base, no VALU address add per access --
  // measured 10 % SLOWER on the tube step: the extra SGPRs per live descriptor deepen the SGPR spill.)
  __device__ __forceinline__ T& at(int k, int F, int f) const {
    return (base + (size_t)((unsigned)(k * F + f) * ld))[lane];
  }
};

// Pin the first kFastObs obstacle entries of a kernel-local spec copy in VGPRs (an empty asm the
// compiler cannot see through, so the values are neither re-loaded nor constant-folded back to
// kernarg reads).  Used with DTMPC_OBS_REGS.
template <typename T>
__device__ __forceinline__ void obs_pin(DSpec<T>& s) {
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    __asm__ volatile("" : "+v"(s.cx[j]));
    __asm__ volatile("" : "+v"(s.cy[j]));
    __asm__ volatile("" : "+v"(s.r2[j]));
  }
}

// ---------------------------------------------------------------------------------------------
// safety function h  (core/systems/dubins_obstacles.py)

// Obstacle parameters are read in place from the kernarg segment: every kernel that takes a spec
// takes it BY VALUE AS ITS FIRST PARAMETER, so it sits at offset 0 of the (read-only, wave-uniform)
// kernarg block.  Indexing the by-value copy `s.cx[i]` with a runtime i instead makes the compiler
// materialise the whole spec in scratch once the kernel also has compile-time-indexed paths.
template <typename T>
__device__ __forceinline__ const DSpec<T>& kspec() {
  return *(const DSpec<T>*)(__builtin_amdgcn_kernarg_segment_ptr());  // addrspace(4) -> generic
}

// h_circle_k: runtime obstacle index, table read from the kernarg segment.
template <typename T>
__device__ __forceinline__ T h_circle_k(int i, T px, T py) {  // :16-30
  const DSpec<T>& k = kspec<T>();
  T dx = px - k.cx[i];
  T dy = py - k.cy[i];
  return dx * dx + dy * dy - k.r2[i];
}

// Obstacle table used by the compile-time-indexed paths: the spec the caller passes (DTMPC_OBS_REGS,
// default).  The tube-step kernel passes a local spec whose first kFastObs table entries were pinned
// in VGPRs at kernel start (obs_pin), so its unrolled obstacle loops read registers instead of
// re-issuing scalar kernarg loads inside the step loops once SGPRs run short (tube step 7.51 ->
// 7.33 ms).  -DDTMPC_OBS_KERNARG reads the kernarg segment everywhere.
#ifndef DTMPC_OBS_KERNARG
#define DTMPC_OBS_REGS 1
#endif
template <typename T>
__device__ __forceinline__ const DSpec<T>& obs_tab(const DSpec<T>& s) {
  DTMPC_NOCONTRACT
#ifdef DTMPC_OBS_REGS
  return s;
#else
  (void)s;
  return kspec<T>();
#endif
}

// h_circle: compile-time obstacle index (unrolled loops only)
template <typename T>
__device__ __forceinline__ T h_circle(const DSpec<T>& s, int i, T px, T py) {  // :16-30
  const DSpec<T>& k = obs_tab(s);
  T dx = px - k.cx[i];
  T dy = py - k.cy[i];
  return dx * dx + dy * dy - k.r2[i];
}

// h_i rounded as the reference rounds it (dx*dx, dy*dy, their sum, minus r^2: no fused multiply-add).
// Used where h_i decides a discrete choice -- the exact-min argmin and the collision test: on a
// symmetric obstacle field (e.g. x = y with obstacles mirrored about the diagonal) two h_i tie up to
// an ulp and a contracted fma(dx, dx, dy*dy) picks the other obstacle than the reference does.
template <typename T>
__device__ __forceinline__ T h_circle_exact(const DSpec<T>&, int i, T px, T py) {
  DTMPC_NOCONTRACT
#pragma clang fp contract(off)
  const DSpec<T>& k = kspec<T>();
  T dx = px - k.cx[i];
  T dy = py - k.cy[i];
  return dx * dx + dy * dy - k.r2[i];
}

// h for W points at once (obstacle loop outer, points inner => W-wide ILP).
//   smoothmin: h_multi_circle_obstacles :41-69 (stable LSE, two passes)
//   min:       h_min_circle_obstacles :95-106
//   single:    h_circle_obstacle :16-30;  none: 1 (run_nominal.py:256)
// Obstacle counts up to kFastObs are specialised at compile time (a wave-uniform switch; the table is
// read in place from the kernarg segment, kspec(), so the by-value spec is never copied to scratch);
// larger counts take the runtime obstacle loop.
constexpr int kFastObs = 8;

template <typename T, int MO>
__device__ __forceinline__ T h_smoothmin1(const DSpec<T>& s, T px, T py) {
  DTMPC_NOCONTRACT
  T hm = h_circle(s, 0, px, py);
#pragma unroll
  for (int i = 1; i < MO; ++i) hm = m_min(hm, h_circle(s, i, px, py));
  const T zmax = s.neg_beta * hm;
  T se = T(0);
#pragma unroll
  for (int i = 0; i < MO; ++i) se += m_exp(s.neg_beta * h_circle(s, i, px, py) - zmax);
  return s.neg_inv_beta * (zmax + m_log(se));
}

// W points, compile-time obstacle count: the h_i of the first (max) pass are kept in registers for
// the exp pass instead of being recomputed (same values, same rounding).  Line search (W = NC):
// tube step 8.14 -> 7.48 ms at B = 65,536 (round 1, v6).
template <typename T, int W, int MO>
__device__ __forceinline__ void h_smoothmin_w(const DSpec<T>& s, const T* px, const T* py, T* h) {
  DTMPC_NOCONTRACT
  T hi[MO][W], hm[W];
#pragma unroll
  for (int w = 0; w < W; ++w) hm[w] = hi[0][w] = h_circle(s, 0, px[w], py[w]);
#pragma unroll
  for (int i = 1; i < MO; ++i)
#pragma unroll
    for (int w = 0; w < W; ++w) {
      hi[i][w] = h_circle(s, i, px[w], py[w]);
      hm[w] = m_min(hm[w], hi[i][w]);
    }
#pragma unroll
  for (int w = 0; w < W; ++w) {
    const T zmax = s.neg_beta * hm[w];
    T se = T(0);
#pragma unroll
    for (int i = 0; i < MO; ++i) se += m_exp(s.neg_beta * hi[i][w] - zmax);
    h[w] = s.neg_inv_beta * (zmax + m_log(se));
  }
}

template <typename T, int W>
__device__ __forceinline__ void h_vec(const DSpec<T>& s, const T* px, const T* py, T* h) {
  DTMPC_NOCONTRACT
#ifndef DTMPC_LS_RUNTIME_OBS
  if constexpr (W > 1) {
    if (s.agg == DTMPC_OBS_SMOOTHMIN && s.M > 0 && s.M <= kFastObs) {
      switch (s.M) {  // wave-uniform
        case 1: h_smoothmin_w<T, W, 1>(s, px, py, h); return;
        case 2: h_smoothmin_w<T, W, 2>(s, px, py, h); return;
        case 3: h_smoothmin_w<T, W, 3>(s, px, py, h); return;
        case 4: h_smoothmin_w<T, W, 4>(s, px, py, h); return;
        case 5: h_smoothmin_w<T, W, 5>(s, px, py, h); return;
        case 6: h_smoothmin_w<T, W, 6>(s, px, py, h); return;
        case 7: h_smoothmin_w<T, W, 7>(s, px, py, h); return;
        default: h_smoothmin_w<T, W, 8>(s, px, py, h); return;
      }
    }
  }
#endif
  if constexpr (W == 1) {
    // single point (commit / rollout / plant): a dependent chain, so the compile-time count matters
    if (s.agg == DTMPC_OBS_SMOOTHMIN && s.M > 0 && s.M <= kFastObs) {
      switch (s.M) {  // wave-uniform
        case 1: h[0] = h_smoothmin1<T, 1>(s, px[0], py[0]); return;
        case 2: h[0] = h_smoothmin1<T, 2>(s, px[0], py[0]); return;
        case 3: h[0] = h_smoothmin1<T, 3>(s, px[0], py[0]); return;
        case 4: h[0] = h_smoothmin1<T, 4>(s, px[0], py[0]); return;
        case 5: h[0] = h_smoothmin1<T, 5>(s, px[0], py[0]); return;
        case 6: h[0] = h_smoothmin1<T, 6>(s, px[0], py[0]); return;
        case 7: h[0] = h_smoothmin1<T, 7>(s, px[0], py[0]); return;
        default: h[0] = h_smoothmin1<T, 8>(s, px[0], py[0]); return;
      }
    }
  }
  if (s.agg == DTMPC_OBS_SMOOTHMIN && s.M > 0) {
    // max_i fl(-beta h_i) == fl(-beta min_i h_i) (rounding is monotone): one v_min per obstacle
    T zmax[W];
#pragma unroll
    for (int w = 0; w < W; ++w) zmax[w] = h_circle_k<T>(0, px[w], py[w]);
    for (int i = 1; i < s.M; ++i) {
#pragma unroll
      for (int w = 0; w < W; ++w) zmax[w] = m_min(zmax[w], h_circle_k<T>(i, px[w], py[w]));
    }
#pragma unroll
    for (int w = 0; w < W; ++w) zmax[w] = s.neg_beta * zmax[w];
    T se[W];
#pragma unroll
    for (int w = 0; w < W; ++w) se[w] = T(0);
    for (int i = 0; i < s.M; ++i) {
#pragma unroll
      for (int w = 0; w < W; ++w) se[w] += m_exp(s.neg_beta * h_circle_k<T>(i, px[w], py[w]) - zmax[w]);
    }
#pragma unroll
    for (int w = 0; w < W; ++w) h[w] = s.neg_inv_beta * (zmax[w] + m_log(se[w]));
  } else if (s.agg == DTMPC_OBS_MIN && s.M > 0) {
#pragma unroll
    for (int w = 0; w < W; ++w) h[w] = h_circle_exact(s, 0, px[w], py[w]);
    for (int i = 1; i < s.M; ++i) {
#pragma unroll
      for (int w = 0; w < W; ++w) {
        T hi = h_circle_exact(s, i, px[w], py[w]);
        h[w] = hi < h[w] ? hi : h[w];
      }
    }
  } else if (s.agg == DTMPC_OBS_SINGLE && s.M > 0) {
#pragma unroll
    for (int w = 0; w < W; ++w) h[w] = h_circle_exact(s, 0, px[w], py[w]);
  } else {
#pragma unroll
    for (int w = 0; w < W; ++w) h[w] = T(1);
  }
}

// h and dh/d(px,py) at one point (grad_h_multi_circle_obstacles :72-92,
// grad_h_min_circle_obstacles :109-117, grad_h_circle_obstacle :33-38).  The softmax weights are
// e_i * (1/sum e) instead of e_i / sum e (one reciprocal per point).
template <typename T, int MO>
__device__ __forceinline__ T h_grad_fixed(const DSpec<T>& s, T px, T py, T& gx, T& gy) {
  // no contraction: z_i = -beta h_i is rounded before z_i - zmax, as in the reference (a fused
  // fma(-beta, h_i, -zmax) shifts f32 plans measurably on knife-edge golden cases)
#ifndef DTMPC_HGRAD_CONTRACT
#pragma clang fp contract(off)
#endif
  T z[MO], zmax = T(0);
#pragma unroll
  for (int i = 0; i < MO; ++i) {
    z[i] = s.neg_beta * h_circle(s, i, px, py);
    zmax = (i == 0 || z[i] > zmax) ? z[i] : zmax;
  }
  T se = T(0), sx = T(0), sy = T(0);
#pragma unroll
  for (int i = 0; i < MO; ++i) {
    T e = m_exp(z[i] - zmax);
    se += e;
    sx += e * (T(2) * (px - obs_tab(s).cx[i]));
    sy += e * (T(2) * (py - obs_tab(s).cy[i]));
  }
  T inv = m_rcp(se);
  gx = sx * inv;
  gy = sy * inv;
  return s.neg_inv_beta * (zmax + m_log(se));
}

template <typename T>
__device__ __forceinline__ T h_grad(const DSpec<T>& s, T px, T py, T& gx, T& gy) {
  if (s.agg == DTMPC_OBS_SMOOTHMIN && s.M > 0 && s.M <= kFastObs) {
    switch (s.M) {  // wave-uniform
      case 1: return h_grad_fixed<T, 1>(s, px, py, gx, gy);
      case 2: return h_grad_fixed<T, 2>(s, px, py, gx, gy);
      case 3: return h_grad_fixed<T, 3>(s, px, py, gx, gy);
      case 4: return h_grad_fixed<T, 4>(s, px, py, gx, gy);
      case 5: return h_grad_fixed<T, 5>(s, px, py, gx, gy);
      case 6: return h_grad_fixed<T, 6>(s, px, py, gx, gy);
      case 7: return h_grad_fixed<T, 7>(s, px, py, gx, gy);
      default: return h_grad_fixed<T, 8>(s, px, py, gx, gy);
    }
  }
  if (s.agg == DTMPC_OBS_SMOOTHMIN && s.M > 0) {
    T zmax = s.neg_beta * h_circle_k<T>(0, px, py);
    for (int i = 1; i < s.M; ++i) {
      T z = s.neg_beta * h_circle_k<T>(i, px, py);
      zmax = z > zmax ? z : zmax;
    }
    T se = T(0), sx = T(0), sy = T(0);
    for (int i = 0; i < s.M; ++i) {
      T e = m_exp(s.neg_beta * h_circle_k<T>(i, px, py) - zmax);
      se += e;
      sx += e * (T(2) * (px - kspec<T>().cx[i]));
      sy += e * (T(2) * (py - kspec<T>().cy[i]));
    }
    T inv = m_rcp(se);
    gx = sx * inv;
    gy = sy * inv;
    return s.neg_inv_beta * (zmax + m_log(se));
  }
  if (s.agg == DTMPC_OBS_MIN && s.M > 0) {
    int am = 0;
    T hm = h_circle_exact(s, 0, px, py);
    for (int i = 1; i < s.M; ++i) {
      T hi = h_circle_exact(s, i, px, py);
      if (hi < hm) {
        hm = hi;
        am = i;
      }
    }
    gx = T(2) * (px - kspec<T>().cx[am]);
    gy = T(2) * (py - kspec<T>().cy[am]);
    return hm;
  }
  if (s.agg == DTMPC_OBS_SINGLE && s.M > 0) {
    gx = T(2) * (px - kspec<T>().cx[0]);
    gy = T(2) * (py - kspec<T>().cy[0]);
    return h_circle_exact(s, 0, px, py);
  }
  gx = T(0);
  gy = T(0);
  return T(1);
}

// ---------------------------------------------------------------------------------------------
// barriers (core/barrier.py, core/systems/dubins_aug_jac.py)

// relaxed_inverse_barrier_B_alpha core/barrier.py:36-59, alpha_eff = max(alpha, eps)
template <typename T>
__device__ __forceinline__ T barrier_relaxed(const DSpec<T>& s, T z) {
  DTMPC_NOCONTRACT
  T a = s.alpha > s.eps ? s.alpha : s.eps;
  if (z >= a) {
    T zc = z < s.eps ? s.eps : z;
    return m_rcp(zc);
  }
  T diff = z - a;
  T a2 = a * a;
  return (T(1) / a - diff / a2) + (diff * diff) / (a2 * a);
}

// _dB_relaxed_inv_dz core/systems/dubins_aug_jac.py:31-40
template <typename T>
__device__ __forceinline__ T dbarrier_relaxed(const DSpec<T>& s, T z) {
  T a = s.alpha > s.eps ? s.alpha : s.eps;
  if (z >= a) {
    T zc = z < s.eps ? s.eps : z;
    return -m_rcp(zc * zc);
  }
  T diff = z - a;
  T a2 = a * a;
  return -(T(1) / a2) + (T(2) * diff) / (a2 * a);
}

// barrier inside the DBaS dynamics (core/barrier.py:99-106; log: barrier_B :62-72)
template <typename T>
__device__ __forceinline__ T barrier_dyn(const DSpec<T>& s, T z) {
  DTMPC_NOCONTRACT
  if (s.barrier == DTMPC_BARRIER_LOG) {
    T zc = z < s.eps ? s.eps : z;
    return -m_log(zc);
  }
  return barrier_relaxed(s, z);
}

// ---------------------------------------------------------------------------------------------
// dynamics: W DBaS-augmented Dubins steps at once.
//   x' = dubins_step(x, u)            core/systems/dubins.py:26-45
//   b' = B(h(x')) - gamma (B(h(x)) - b) core/barrier.py:75-108
// With a tightened nominal h_nom = h - s enters the barrier (core/tube_mpc.py:235-238; s = 0 else).
// Bc[w] carries B(h(x_k)) from the previous step (the reference recomputes h(x_k) inside
// dbas_step; the value is the same function of the same state), and is updated to B(h(x_{k+1})).
template <typename T, int W>
__device__ __forceinline__ void fhat_vec(const DSpec<T>& s, T* x0, T* x1, T* x2, T* b,
                                         const T* u0, const T* u1, T* Bc) {
  DTMPC_NOCONTRACT
  T hn[W];
#pragma unroll
  for (int w = 0; w < W; ++w) {
    T sn, c;
    m_sincos(x2[w], &sn, &c);
    T dv = s.dt * u0[w];
    x0[w] = x0[w] + dv * c;
    x1[w] = x1[w] + dv * sn;
    x2[w] = x2[w] + s.dt * u1[w];
  }
  h_vec<T, W>(s, x0, x1, hn);
#pragma unroll
  for (int w = 0; w < W; ++w) {
    T Bn = barrier_dyn(s, hn[w] - s.tight);
    b[w] = Bn - s.gamma * (Bc[w] - b[w]);
    Bc[w] = Bn;
  }
}

template <typename T>
__device__ __forceinline__ T barrier_of_state(const DSpec<T>& s, T px, T py) {
  DTMPC_NOCONTRACT
  T h[1], x[1] = {px}, y[1] = {py};
  h_vec<T, 1>(s, x, y, h);
  return barrier_dyn(s, h[0] - s.tight);
}

// ---------------------------------------------------------------------------------------------
// costs (core/tube_mpc.py:823-842, 875-894; core/cost_derivs.py:58-146; run_nominal.py:297-324)

template <typename T>
__device__ __forceinline__ T stage_cost(const DCost<T>& c, T x0, T x1, T x2, T b, T u0, T u1,
                                        T r0, T r1, T r2, T ur0, T ur1) {
  DTMPC_NOCONTRACT
  T d0, d1, d2, e0, e1;
  if (c.kind == DTMPC_COST_TRACK) {
    d0 = x0 - r0;
    d1 = x1 - r1;
    d2 = x2 - r2;
    e0 = u0 - ur0;
    e1 = u1 - ur1;
  } else {
    d0 = x0 - c.t0;
    d1 = x1 - c.t1;
    d2 = x2 - c.t2;
    if (c.wrap) d2 = wrap_angle(d2);
    e0 = u0;
    e1 = u1;
  }
  T sq = c.Q0 * d0 * d0 + c.Q1 * d1 * d1 + c.Q2 * d2 * d2;
  T sr = c.R0 * e0 * e0 + c.R1 * e1 * e1;
  return sq + sr + c.qb * (b * b);
}

template <typename T>
__device__ __forceinline__ T term_cost(const DCost<T>& c, T x0, T x1, T x2, T b, T r0, T r1, T r2) {
  DTMPC_NOCONTRACT
  T d0, d1, d2;
  if (c.kind == DTMPC_COST_TRACK) {
    d0 = x0 - r0;
    d1 = x1 - r1;
    d2 = x2 - r2;
  } else {
    d0 = x0 - c.t0;
    d1 = x1 - c.t1;
    d2 = x2 - c.t2;
    if (c.wrap) d2 = wrap_angle(d2);
  }
  T sq = c.Qf0 * d0 * d0 + c.Qf1 * d1 * d1 + c.Qf2 * d2 * d2;
  return sq + c.qb * (b * b);
}

// state error used by l_x / phi_x (wrapped target of run_nominal.py:311-320)
template <typename T>
__device__ __forceinline__ void deriv_dx(const DCost<T>& c, T x0, T x1, T x2, T r0, T r1, T r2,
                                         T& d0, T& d1, T& d2) {
  if (c.kind == DTMPC_COST_TRACK) {
    d0 = x0 - r0;
    d1 = x1 - r1;
    d2 = x2 - r2;
    return;
  }
  T t2 = c.t2;
  if (c.wrap) t2 = x2 - wrap_angle(x2 - c.t2);
  d0 = x0 - c.t0;
  d1 = x1 - c.t1;
  d2 = x2 - t2;
}

// ---------------------------------------------------------------------------------------------
// sparse augmented Jacobian (core/systems/dubins_aug_jac.py:61-139)
//   A = [[1,0,a02,0],[0,1,a12,0],[0,0,1,0],[a30,a31,a32,g]],  Bm = [[b00,0],[b10,0],[0,dt],[b30,b31]]
template <typename T>
struct Jac {
  T a02, a12, a30, a31, a32, g, b00, b10, b21, b30, b31;
};

// (xk, uk): state/control at step k; (gxk, gyk, dBk): grad h and B' at x_k;
// (gxn, gyn, dBn): the same at x_{k+1} = f(x_k, u_k).
template <typename T>
__device__ __forceinline__ Jac<T> make_jac(const DSpec<T>& s, T sn, T c, T v, T gxk, T gyk, T dBk,
                                           T gxn, T gyn, T dBn) {
  Jac<T> J;
  T dt = s.dt;
  J.a02 = -dt * v * sn;
  J.a12 = dt * v * c;
  J.b00 = dt * c;
  J.b10 = dt * sn;
  J.b21 = dt;
  T r0 = dBn * gxn, r1 = dBn * gyn, r2 = dBn * T(0);
  T gd = s.gamma * dBk;
  // row_x = (dB_next dh_next)^T A3 - gamma dB_curr dh_curr   (:128-130)
  J.a30 = r0 - gd * gxk;
  J.a31 = r1 - gd * gyk;
  J.a32 = (r0 * J.a02 + r1 * J.a12 + r2) - gd * T(0);
  J.g = s.gamma;
  // row_u = (dB_next dh_next)^T B3   (:131)
  J.b30 = r0 * J.b00 + r1 * J.b10;
  J.b31 = r2 * dt;
  return J;
}

// ---------------------------------------------------------------------------------------------
// 2x2 solves.  torch.linalg.solve = LU with partial pivoting (LAPACK getrf/getrs).
template <typename T>
struct LU2 {
  bool sw;
  T a00, a01, l, inv00, inv11;
};

template <typename T>
__device__ __forceinline__ LU2<T> lu2(T m00, T m01, T m10, T m11) {
  LU2<T> f;
  f.sw = m_abs(m10) > m_abs(m00);
  T a00 = f.sw ? m10 : m00, a01 = f.sw ? m11 : m01;
  T a10 = f.sw ? m00 : m10, a11 = f.sw ? m01 : m11;
  f.inv00 = m_rcp(a00);
  f.l = a10 * f.inv00;
  T u11 = a11 - f.l * a01;
  f.inv11 = m_rcp(u11);
  f.a00 = a00;
  f.a01 = a01;
  return f;
}

template <typename T>
__device__ __forceinline__ void lu2_solve(const LU2<T>& f, T r0, T r1, T& x0, T& x1) {
  T p0 = f.sw ? r1 : r0, p1 = f.sw ? r0 : r1;
  T y1 = p1 - f.l * p0;
  x1 = y1 * f.inv11;
  x0 = (p0 - f.a01 * x1) * f.inv00;
}

// _solve_reduced core/ddp.py:23-60 for one right-hand side, given the active set.
template <typename T>
__device__ __forceinline__ void solve_reduced(const LU2<T>& f, T m00, T m11, bool act0, bool act1,
                                              T r0, T r1, T& x0, T& x1) {
  if (!act0 && !act1) {
    lu2_solve(f, r0, r1, x0, x1);
  } else {
    x0 = (!act0 && act1) ? r0 / m00 : T(0);
    x1 = (act0 && !act1) ? r1 / m11 : T(0);
  }
}

// all of K[8], k[2] finite.  f32: one NaN-propagating max of the magnitudes (v_maximum3_f32) and a
// single class test instead of ten.
__device__ __forceinline__ bool finite10(const float* K, const float* k) {
  float m = __builtin_elementwise_maximum(__builtin_fabsf(k[0]), __builtin_fabsf(k[1]));
#pragma unroll
  for (int j = 0; j < 8; ++j) m = __builtin_elementwise_maximum(m, __builtin_fabsf(K[j]));
  return finite(m);
}
__device__ __forceinline__ bool finite10(const double* K, const double* k) {
  bool ok = finite(k[0]) && finite(k[1]);
#pragma unroll
  for (int j = 0; j < 8; ++j) ok = ok && finite(K[j]);
  return ok;
}

// ---------------------------------------------------------------------------------------------
// iLQR backward step with the sparse Jacobian (core/ddp.py:213-254).
// l_xx = diag(lxx0..3), l_uu = diag(luu0,1), l_ux = 0.  Vx/Vxx are updated in place.
template <typename T>
struct Riccati {
  T Vx[4];
  T Vxx[4][4];
};

template <typename T>
__device__ __forceinline__ bool riccati_step(const Jac<T>& J, const T* lx, const T* lu,
                                             const T* lxx, const T* luu, T reg, Riccati<T>& R,
                                             T* K, T* kff) {
  const T(&V)[4][4] = R.Vxx;
  const T* vx = R.Vx;
  // Q_x = l_x + A^T V_x ; Q_u = l_u + B^T V_x
  T Qx0 = lx[0] + (vx[0] + J.a30 * vx[3]);
  T Qx1 = lx[1] + (vx[1] + J.a31 * vx[3]);
  T Qx2 = lx[2] + (J.a02 * vx[0] + J.a12 * vx[1] + vx[2] + J.a32 * vx[3]);
  T Qx3 = lx[3] + J.g * vx[3];
  T Qu0 = lu[0] + (J.b00 * vx[0] + J.b10 * vx[1] + J.b30 * vx[3]);
  T Qu1 = lu[1] + (J.b21 * vx[2] + J.b31 * vx[3]);
  // A^T V_xx
  T P[4][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    P[0][j] = V[0][j] + J.a30 * V[3][j];
    P[1][j] = V[1][j] + J.a31 * V[3][j];
    P[2][j] = J.a02 * V[0][j] + J.a12 * V[1][j] + V[2][j] + J.a32 * V[3][j];
    P[3][j] = J.g * V[3][j];
  }
  // Q_xx = l_xx + (A^T V_xx) A
  T Qxx[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    Qxx[i][0] = P[i][0] + P[i][3] * J.a30;
    Qxx[i][1] = P[i][1] + P[i][3] * J.a31;
    Qxx[i][2] = P[i][0] * J.a02 + P[i][1] * J.a12 + P[i][2] + P[i][3] * J.a32;
    Qxx[i][3] = P[i][3] * J.g;
    Qxx[i][i] = lxx[i] + Qxx[i][i];
  }
  // B^T V_xx
  T S[2][4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    S[0][j] = J.b00 * V[0][j] + J.b10 * V[1][j] + J.b30 * V[3][j];
    S[1][j] = J.b21 * V[2][j] + J.b31 * V[3][j];
  }
  // Q_ux = (B^T V_xx) A ; Q_uu = l_uu + (B^T V_xx) B
  T Qux[2][4], Quu[2][2];
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
  // gains with the regularised Q_uu (:239-249)
  LU2<T> f = lu2(Quu[0][0] + reg, Quu[0][1], Quu[1][0], Quu[1][1] + reg);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    T x0, x1;
    lu2_solve(f, Qux[0][j], Qux[1][j], x0, x1);
    K[j] = -x0;
    K[4 + j] = -x1;
  }
  {
    T x0, x1;
    lu2_solve(f, Qu0, Qu1, x0, x1);
    kff[0] = -x0;
    kff[1] = -x1;
  }
  bool ok = finite10(K, kff);
  // V_x = Q_x + K^T Q_uu k + K^T Q_u + Q_xu k  ;  V_xx = Q_xx + K^T Q_uu K + K^T Q_ux + Q_xu K
  // (unregularised Q_uu, :251-252)
  T KQ[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    KQ[i][0] = K[i] * Quu[0][0] + K[4 + i] * Quu[1][0];
    KQ[i][1] = K[i] * Quu[0][1] + K[4 + i] * Quu[1][1];
  }
  T Qx[4] = {Qx0, Qx1, Qx2, Qx3};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    T t1 = KQ[i][0] * kff[0] + KQ[i][1] * kff[1];
    T t2 = K[i] * Qu0 + K[4 + i] * Qu1;
    T t3 = Qux[0][i] * kff[0] + Qux[1][i] * kff[1];
    R.Vx[i] = Qx[i] + t1 + t2 + t3;
  }
  // K^T Q_ux and Q_xu K are transposes of each other (same products, commutative).
  T M2[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) M2[i][j] = K[i] * Qux[0][j] + K[4 + i] * Qux[1][j];
#ifdef DTMPC_VXX_SYM
  // V_xx is symmetric in exact arithmetic: the upper triangle is computed and mirrored (the reference's
  // full product differs from its transpose by rounding only); the lower half of Q_xx then goes dead.
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = i; j < 4; ++j) {
      T m1 = KQ[i][0] * K[j] + KQ[i][1] * K[4 + j];
      R.Vxx[i][j] = Qxx[i][j] + m1 + M2[i][j] + M2[j][i];
      R.Vxx[j][i] = R.Vxx[i][j];
    }
#else
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      T m1 = KQ[i][0] * K[j] + KQ[i][1] * K[4 + j];
      R.Vxx[i][j] = Qxx[i][j] + m1 + M2[i][j] + M2[j][i];
    }
#endif
  return ok;
}

// fixed-order wave64 sum (lane 0 holds the result)
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  return v;
}

// ---------------------------------------------------------------------------------------------
// Philox4x32-10 (shared with oracle/dtmpc_oracle.c) -> disturbance w ~ U[low, high)^3
__device__ __forceinline__ void philox4x32_10(uint64_t seed, uint64_t gidx, uint64_t step,
                                              uint32_t* out) {
  uint32_t c0 = (uint32_t)gidx, c1 = (uint32_t)(gidx >> 32), c2 = (uint32_t)step,
           c3 = (uint32_t)(step >> 32);
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0 = __umulhi(0xD2511F53u, c0), lo0 = 0xD2511F53u * c0;
    uint32_t hi1 = __umulhi(0xCD9E8D57u, c2), lo1 = 0xCD9E8D57u * c2;
    uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0;
    c1 = lo1;
    c2 = n2;
    c3 = lo0;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  out[0] = c0;
  out[1] = c1;
  out[2] = c2;
  out[3] = c3;
}

}  // namespace dtmpc
