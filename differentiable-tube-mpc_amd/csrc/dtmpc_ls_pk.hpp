// dtmpc_ls_pk.hpp — f32 line search on candidate PAIRS (packed-f32 VALU).
//
// Same algorithm, same expression trees and -- forward passes are contraction-free -- the same
// IEEE operations as line_search<float, NC> (dtmpc_solver.hpp, core/ddp.py:256-301) and as the commit
// rollout of the chosen candidate (measured: a bench-size nominal solve agrees bitwise with the
// scalar form on all but 4 of 65,536 trajectories, max rel 1e-3 there): the NC rolled-out candidates
// are held as NC/2 two-wide
// vectors, so every elementwise add / mul / fma of the rollout (feedback, cost, Dubins move,
// smooth-min obstacle distances, DBaS update) issues as one v_pk_add_f32 / v_pk_mul_f32 /
// v_pk_fma_f32 for two candidates.  Transcendentals, compares / selects and min stay per element
// (gfx950 has no packed form of them).  Used for f32 with an even candidate count (the bench's 6):
// tube step 7.12 -> 6.66 ms against the contraction-free scalar form.
#pragma once

#include "dtmpc_device.hpp"

namespace dtmpc {

#define PK_CONTRACT DTMPC_NOCONTRACT  // no fusion: bitwise the scalar forward pass (dtmpc_device.hpp)

typedef float pf2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ pf2 pk_clamp(pf2 v, float lo, float hi) {
  return pf2{clampv(v.x, lo, hi), clampv(v.y, lo, hi)};
}
__device__ __forceinline__ pf2 pk_min(pf2 a, pf2 b) { return pf2{m_min(a.x, b.x), m_min(a.y, b.y)}; }
__device__ __forceinline__ pf2 pk_exp(pf2 x) {  // m_exp per element, the scaling packed
  pf2 y = x * 1.44269504088896341f;
  return pf2{__builtin_amdgcn_exp2f(y.x), __builtin_amdgcn_exp2f(y.y)};
}
__device__ __forceinline__ pf2 pk_log(pf2 x) {  // m_log per element, the scaling packed
  pf2 y = pf2{__builtin_amdgcn_logf(x.x), __builtin_amdgcn_logf(x.y)};
  return y * 0.693147180559945309f;
}

// m_sincos (dtmpc_device.hpp) on a pair: sincos_cw with every fma / mul packed; the rare element
// outside |x| <= 65536 (or non-finite) sends the pair through the scalar function
__device__ __forceinline__ void pk_sincos(pf2 x, pf2& sn, pf2& cs) {
#ifndef DTMPC_OCML_SINCOS
  if (__builtin_expect(__builtin_fabsf(x.x) <= 65536.0f && __builtin_fabsf(x.y) <= 65536.0f, 1)) {
    const pf2 q = pf2{__builtin_rintf(x.x * k2oPi), __builtin_rintf(x.y * k2oPi)};
    pf2 r = __builtin_elementwise_fma(-q, pf2(kPio2A), x);
    r = __builtin_elementwise_fma(-q, pf2(kPio2B), r);
    r = __builtin_elementwise_fma(-q, pf2(kPio2C), r);
    const pf2 z = r * r;
    pf2 ps = __builtin_elementwise_fma(z, pf2(kSinS3), pf2(kSinS2));
    ps = __builtin_elementwise_fma(z, ps, pf2(kSinS1));
    const pf2 s = __builtin_elementwise_fma(r * z, ps, r);
    pf2 pc = __builtin_elementwise_fma(z, pf2(kCosK3), pf2(kCosK2));
    pc = __builtin_elementwise_fma(z, pc, pf2(kCosK1));
    const pf2 c = __builtin_elementwise_fma(z * z, pc, __builtin_elementwise_fma(pf2(-0.5f), z, pf2(1.0f)));
    const int j0 = (int)q.x & 3, j1 = (int)q.y & 3;
    const float so0 = (j0 & 1) ? c.x : s.x, co0 = (j0 & 1) ? s.x : c.x;
    const float so1 = (j1 & 1) ? c.y : s.y, co1 = (j1 & 1) ? s.y : c.y;
    sn = pf2{(j0 & 2) ? -so0 : so0, (j1 & 2) ? -so1 : so1};
    cs = pf2{((j0 + 1) & 2) ? -co0 : co0, ((j1 + 1) & 2) ? -co1 : co1};
    return;
  }
#endif
  float s0, c0, s1, c1;
  m_sincos(x.x, &s0, &c0);
  m_sincos(x.y, &s1, &c1);
  sn = pf2{s0, s1};
  cs = pf2{c0, c1};
}

// stage_cost / term_cost of dtmpc_device.hpp on two candidates (TRACK, or TARGET without wrap; the
// wrapped target goes element by element through the scalar function)
__device__ __forceinline__ pf2 pk_stage_cost(const DCost<float>& c, pf2 x0, pf2 x1, pf2 x2, pf2 b, pf2 u0, pf2 u1,
                                             float r0, float r1, float r2, float ur0, float ur1) {
  PK_CONTRACT
  if (c.kind != DTMPC_COST_TRACK && c.wrap) {
    return pf2{stage_cost(c, x0.x, x1.x, x2.x, b.x, u0.x, u1.x, r0, r1, r2, ur0, ur1),
               stage_cost(c, x0.y, x1.y, x2.y, b.y, u0.y, u1.y, r0, r1, r2, ur0, ur1)};
  }
  pf2 d0, d1, d2, e0, e1;
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
    e0 = u0;
    e1 = u1;
  }
  pf2 sq = c.Q0 * d0 * d0 + c.Q1 * d1 * d1 + c.Q2 * d2 * d2;
  pf2 sr = c.R0 * e0 * e0 + c.R1 * e1 * e1;
  return sq + sr + c.qb * (b * b);
}

__device__ __forceinline__ pf2 pk_term_cost(const DCost<float>& c, pf2 x0, pf2 x1, pf2 x2, pf2 b, float r0, float r1,
                                            float r2) {
  PK_CONTRACT
  if (c.kind != DTMPC_COST_TRACK && c.wrap) {
    return pf2{term_cost(c, x0.x, x1.x, x2.x, b.x, r0, r1, r2), term_cost(c, x0.y, x1.y, x2.y, b.y, r0, r1, r2)};
  }
  pf2 d0, d1, d2;
  if (c.kind == DTMPC_COST_TRACK) {
    d0 = x0 - r0;
    d1 = x1 - r1;
    d2 = x2 - r2;
  } else {
    d0 = x0 - c.t0;
    d1 = x1 - c.t1;
    d2 = x2 - c.t2;
  }
  pf2 sq = c.Qf0 * d0 * d0 + c.Qf1 * d1 * d1 + c.Qf2 * d2 * d2;
  return sq + c.qb * (b * b);
}

// h_smoothmin_w (dtmpc_device.hpp) on NP candidate pairs, compile-time obstacle count
template <int NP, int MO>
__device__ __forceinline__ void pk_h_smoothmin(const DSpec<float>& s, const pf2* px, const pf2* py, pf2* h) {
  PK_CONTRACT
  const DSpec<float>& k = obs_tab(s);
  pf2 hi[MO][NP], hm[NP];
#pragma unroll
  for (int i = 0; i < MO; ++i)
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      pf2 dx = px[p] - k.cx[i];
      pf2 dy = py[p] - k.cy[i];
      hi[i][p] = dx * dx + dy * dy - k.r2[i];
      hm[p] = i == 0 ? hi[0][p] : pk_min(hm[p], hi[i][p]);
    }
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const pf2 zmax = s.neg_beta * hm[p];
    pf2 se = pf2{0.f, 0.f};
#pragma unroll
    for (int i = 0; i < MO; ++i) se += pk_exp(s.neg_beta * hi[i][p] - zmax);
    h[p] = s.neg_inv_beta * (zmax + pk_log(se));
  }
}

// fhat_vec<float, 2 NP> (dtmpc_device.hpp) on NP candidate pairs
template <int NP>
__device__ __forceinline__ void pk_fhat(const DSpec<float>& s, pf2* x0, pf2* x1, pf2* x2, pf2* b, const pf2* u0,
                                        const pf2* u1, pf2* Bc) {
  PK_CONTRACT
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    pf2 sn, cs;
    pk_sincos(x2[p], sn, cs);
    pf2 dv = s.dt * u0[p];
    x0[p] = x0[p] + dv * cs;
    x1[p] = x1[p] + dv * sn;
    x2[p] = x2[p] + s.dt * u1[p];
  }
  pf2 hn[NP];
  if (s.agg == DTMPC_OBS_SMOOTHMIN && s.M > 0 && s.M <= kFastObs) {
    switch (s.M) {  // wave-uniform
      case 1: pk_h_smoothmin<NP, 1>(s, x0, x1, hn); break;
      case 2: pk_h_smoothmin<NP, 2>(s, x0, x1, hn); break;
      case 3: pk_h_smoothmin<NP, 3>(s, x0, x1, hn); break;
      case 4: pk_h_smoothmin<NP, 4>(s, x0, x1, hn); break;
      case 5: pk_h_smoothmin<NP, 5>(s, x0, x1, hn); break;
      case 6: pk_h_smoothmin<NP, 6>(s, x0, x1, hn); break;
      case 7: pk_h_smoothmin<NP, 7>(s, x0, x1, hn); break;
      default: pk_h_smoothmin<NP, 8>(s, x0, x1, hn); break;
    }
  } else {  // other aggregations: the scalar h_vec on the 2 NP points
    float qx[2 * NP], qy[2 * NP], qh[2 * NP];
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      qx[2 * p] = x0[p].x;
      qx[2 * p + 1] = x0[p].y;
      qy[2 * p] = x1[p].x;
      qy[2 * p + 1] = x1[p].y;
    }
    h_vec<float, 2 * NP>(s, qx, qy, qh);
#pragma unroll
    for (int p = 0; p < NP; ++p) hn[p] = pf2{qh[2 * p], qh[2 * p + 1]};
  }
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const pf2 z = hn[p] - s.tight;
    const pf2 Bn = pf2{barrier_dyn(s, z.x), barrier_dyn(s, z.y)};
    b[p] = Bn - s.gamma * (Bc[p] - b[p]);
    Bc[p] = Bn;
  }
}

// line_search<float, NC> (dtmpc_solver.hpp) with the candidates in pairs; NC even.
template <int NC, typename G>
__device__ __forceinline__ int line_search_pk(const DSpec<float>& s, const DCost<float>& c, const DIlqr<float>& cfg,
                                              const float* x0, float Bc0, const Col<float>& X, const Col<float>& U,
                                              const G& gains, const Col<float>& Xr, int rf, const Col<float>& Ur,
                                              float Jprev, float& bestJ, float& al_out) {
  PK_CONTRACT
  static_assert(NC % 2 == 0, "pairs");
  constexpr int NP = NC / 2;
  const int N = s.N;
  pf2 a0[NP], a1[NP], a2[NP], ab[NP], Bc[NP], J[NP], al[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    a0[p] = x0[0];
    a1[p] = x0[1];
    a2[p] = x0[2];
    ab[p] = x0[3];
    Bc[p] = Bc0;
    J[p] = 0.f;
    al[p] = pf2{cfg.calphas[2 * p], cfg.calphas[2 * p + 1]};
  }
  StepIn<float> q[kPrefetch];
#pragma unroll
  for (int j = 0; j < kPrefetch; ++j)
    if (j < N) load_step(q[j], c, X, U, gains, Xr, rf, Ur, j);
  for (int k = 0; k < N; ++k) {
    const StepIn<float> cur = q[0];
#pragma unroll
    for (int j = 0; j + 1 < kPrefetch; ++j) q[j] = q[j + 1];
    if (k + kPrefetch < N) load_step(q[kPrefetch - 1], c, X, U, gains, Xr, rf, Ur, k + kPrefetch);
    pf2 u0[NP], u1[NP];
#pragma unroll
    for (int p = 0; p < NP; ++p) {
      pf2 e0 = a0[p] - cur.X0, e1 = a1[p] - cur.X1, e2 = a2[p] - cur.X2, e3 = ab[p] - cur.X3;
      pf2 du0 = cur.k0 + (cur.K[0] * e0 + cur.K[1] * e1 + cur.K[2] * e2 + cur.K[3] * e3);
      pf2 du1 = cur.k1 + (cur.K[4] * e0 + cur.K[5] * e1 + cur.K[6] * e2 + cur.K[7] * e3);
      u0[p] = pk_clamp(cur.V0 + al[p] * du0, s.umin0, s.umax0);
      u1[p] = pk_clamp(cur.V1 + al[p] * du1, s.umin1, s.umax1);
      J[p] = J[p] + pk_stage_cost(c, a0[p], a1[p], a2[p], ab[p], u0[p], u1[p], cur.r0, cur.r1, cur.r2, cur.q0,
                                  cur.q1);
    }
    pk_fhat<NP>(s, a0, a1, a2, ab, u0, u1, Bc);
  }
  float r0, r1, r2;
  load_ref(c, Xr, rf, N, r0, r1, r2);
  float Jc[NC];
  bool ok = true;
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const pf2 Jt = J[p] + pk_term_cost(c, a0[p], a1[p], a2[p], ab[p], r0, r1, r2);
    Jc[2 * p] = Jt.x;
    Jc[2 * p + 1] = Jt.y;
    ok = ok && finite(Jt.x) && finite(Jt.y);
  }
  // selection exactly as line_search
  int bc = 0;
  bestJ = Jc[0];
#pragma unroll
  for (int a = 1; a < NC; ++a) {
    if (Jc[a] < bestJ) {
      bestJ = Jc[a];
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
    float mb = 0.f, ma = 0.f;
    bool hb = false, ha = false;
#pragma unroll
    for (int a = 0; a < NC; ++a) {
      if (cfg.cpos[a] < cfg.zpos) {
        mb = (!hb || Jc[a] < mb) ? Jc[a] : mb;
        hb = true;
      } else {
        ma = (!ha || Jc[a] < ma) ? Jc[a] : ma;
        ha = true;
      }
    }
    if ((!hb || Jprev < mb) && (!ha || Jprev <= ma)) {
      best = cfg.zpos;
      bestJ = Jprev;
      al_out = 0.f;
    }
    ok = ok && finite(Jprev);
  }
  return ok ? best : -1;
}

}  // namespace dtmpc
