/*
 * dtmpc_oracle.c — TEST INFRASTRUCTURE ONLY: CPU restatement of the reference hot path.
 *
 * Builds liboracle.so (see oracle/Makefile) with every oracle_* entry point in an f64 and an f32
 * flavour.  Used by tests/ (parity checker), __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg, and by nothing else.  The algorithm is restated in oracle_impl.h; each function there cites
 * the reference file:line it follows.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "../include/dtmpc.h"

/* Philox4x32-10 (Salmon et al., SC'11) — shared bit stream with the HIP kernels
 * (differentiable-tube-mpc_amd/csrc/dtmpc_device.hpp: philox4x32_10).  counter = (global
 * trajectory index, step), key = seed. */
static void dtmpc_philox_uniform_bits(uint64_t seed, uint64_t gidx, uint64_t step, uint32_t out[4]) {
  uint32_t c0 = (uint32_t)gidx, c1 = (uint32_t)(gidx >> 32), c2 = (uint32_t)step,
           c3 = (uint32_t)(step >> 32);
  uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  for (int r = 0; r < 10; ++r) {
    uint64_t p0 = (uint64_t)0xD2511F53u * c0;
    uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
    uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
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

void oracle_philox_bits(uint64_t seed, uint64_t gidx, uint64_t step, uint32_t* out) {
  dtmpc_philox_uniform_bits(seed, gidx, step, out);
}

int oracle_abi_version(void) { return DTMPC_ABI_VERSION; }

#ifdef ORACLE_ULP_NOISE
/* Calibration build (liboracle_ulp.so): every transcendental result is moved by one ulp up or down,
 * chosen by a hash of the argument's bits.  The spread between this build and liboracle.so measures
 * how sensitive a case is to last-bit differences between math libraries (glibc vs the GPU's). */
static uint64_t ulp_hash(uint64_t v) {
  v ^= v >> 33;
  v *= 0xff51afd7ed558ccdULL;
  v ^= v >> 33;
  v *= 0xc4ceb9fe1a85ec53ULL;
  v ^= v >> 33;
  return v;
}
static double ulpn_d(double v, double x) {
  uint64_t b;
  memcpy(&b, &x, sizeof b);
  return nextafter(v, (ulp_hash(b) & 1) ? INFINITY : -INFINITY);
}
static float ulpn_f(float v, float x) {
  uint32_t b;
  memcpy(&b, &x, sizeof b);
  return nextafterf(v, (ulp_hash(b) & 1) ? INFINITY : -INFINITY);
}
#define D_EXP(x) ulpn_d(exp(x), (x))
#define D_LOG(x) ulpn_d(log(x), (x))
#define D_SIN(x) ulpn_d(sin(x), (x))
#define D_COS(x) ulpn_d(cos(x), (x) + 1.0)
#define D_ATAN2(y, x) ulpn_d(atan2((y), (x)), (y))
#define D_LOG1P(x) ulpn_d(log1p(x), (x))
#define D_TANH(x) ulpn_d(tanh(x), (x))
#define F_EXP(x) ulpn_f(expf(x), (x))
#define F_LOG(x) ulpn_f(logf(x), (x))
#define F_SIN(x) ulpn_f(sinf(x), (x))
#define F_COS(x) ulpn_f(cosf(x), (x) + 1.0f)
#define F_ATAN2(y, x) ulpn_f(atan2f((y), (x)), (y))
#define F_LOG1P(x) ulpn_f(log1pf(x), (x))
#define F_TANH(x) ulpn_f(tanhf(x), (x))
#else
#define D_EXP exp
#define D_LOG log
#define D_SIN sin
#define D_COS cos
#define D_ATAN2 atan2
#define D_LOG1P log1p
#define D_TANH tanh
#define F_EXP expf
#define F_LOG logf
#define F_SIN sinf
#define F_COS cosf
#define F_ATAN2 atan2f
#define F_LOG1P log1pf
#define F_TANH tanhf
#endif

#define REAL double
#define SUFFIX _f64
#define M_EXP D_EXP
#define M_LOG D_LOG
#define M_SIN D_SIN
#define M_COS D_COS
#define M_ATAN2 D_ATAN2
#define M_LOG1P D_LOG1P
#define M_TANH D_TANH
#define M_FABS fabs
#include "oracle_impl.h"
#undef REAL
#undef SUFFIX
#undef M_EXP
#undef M_LOG
#undef M_SIN
#undef M_COS
#undef M_ATAN2
#undef M_LOG1P
#undef M_TANH
#undef M_FABS

#define REAL float
#define SUFFIX _f32
#define M_EXP F_EXP
#define M_LOG F_LOG
#define M_SIN F_SIN
#define M_COS F_COS
#define M_ATAN2 F_ATAN2
#define M_LOG1P F_LOG1P
#define M_TANH F_TANH
#define M_FABS fabsf
#include "oracle_impl.h"
