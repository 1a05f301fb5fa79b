// dtmpc_fast.hip — the closed-loop tube step specialised for the paper problem (gfx950, f32).
//
// Same algorithm, same operations and -- in every forward pass -- the same IEEE rounding as
// tube_step_kernel (dtmpc_kernels.hip) on the configuration the benchmark and the paper run:
// smooth-min obstacles (compile-time count M <= 8), the relaxed inverse barrier, an untightened h,
// a fixed target-tracking nominal cost without angle wrap, an ancillary tracking cost, and six
// rolled-out line-search candidates (seven alphas, one of them 0).  Everything the generic kernel
// decides at run time inside its step loops (obstacle aggregation and count, barrier kind, cost
// kind, wrapped targets, lane count) is fixed here, so its loops are straight-line code with the
// problem constants in scalar registers, and every tape access is one global load/store with a
// scalar plane base and a fixed per-lane byte offset (no per-access address arithmetic).
//
// Lanes per trajectory P (1 or 2).  P = 1: one lane runs the trajectory (all six candidates as
// three packed pairs).  P = 2: two adjacent lanes run it; each rolls out three of the six
// line-search candidates (one packed pair + one single) and the pair agrees on the winner through one
// DPP lane swap; the rest (backward pass, commit, sensitivity, plant) is computed by both lanes.
// With P = 2 a batch has twice the waves: two waves per SIMD at the benchmark batch, so one
// wave's memory waits and dependency stalls hide behind the other's issue.
//
// Reference: core/tube_mpc.py:803-1023 (loop body), core/ddp.py:102-307 (iLQR), :317-427
// (sensitivity), core/tube_mpc.py:915-984 (upper loss, DOC gradient, update).
#include <hip/hip_runtime.h>

#include "../../include/dtmpc.h"
#include "dtmpc_host.hpp"
#include "dtmpc_ls_pk.hpp"

// this file is the tube step's translation unit; dtmpc_fast_ilqr.hip / dtmpc_fast_general.hip include it
// for the standalone iLQR's and the general path's instantiations (their host parts below)
#if defined(DTMPC_FAST_ILQR_TU) || defined(DTMPC_FAST_GENERAL_TU) || defined(DTMPC_FAST_ILP_TU)
#define DTMPC_FAST_AUX_TU 1
#endif
// The one-lane tube kernels (the headline's form) and the f32 two-lane ones live in their own translation units
// (dtmpc_fast_ilp.hip, dtmpc_fast64_ilp.hip), compiled with LLVM's iterative ILP scheduler (build.py UNIT_FLAGS): at
// one or two waves per SIMD little hides a wave's own wait states, so the schedule that shortens the chains wins
// there, while the four-lane forms (and the f64 two-lane one, even) keep the default scheduler (round-6 A/B,
// profiles/r06/ab_sched.txt).  Profiling and ISA-only builds keep every form in this unit (the phase counters are
// this unit's symbols).
#if !defined(DTMPC_PROFILE) && !defined(DTMPC_FAST_ISA_ONLY) && !defined(DTMPC_FAST_ILP_INLINE)
#define DTMPC_FAST_ILP_SPLIT 1
#else
#define DTMPC_FAST_ILP_SPLIT 0
#endif
#define DTMPC_FAST_ILP_P2 (DTMPC_FAST_ILP_SPLIT && !DTMPC_FAST_F64)  // the two-lane form in the split unit too

// DTMPC_FAST_F64 = 1 (csrc/dtmpc_fast64.hip): the same kernels in f64, the reference's configured precision
// (configs/dubins.yaml:8) -- `real` is the value type of every tape, record and register, ES its size in
// 32-bit words (the record strides scale by it); the f64 instantiation lives in namespace fk64 and its host
// entry points carry the suffix 64 (FKN).  Where the f32 kernel leans on f32-only hardware (v_exp_f32 /
// v_log_f32 / v_rcp_f32, packed f32, the f32 minimax sin/cos), the f64 form evaluates what the generic
// f64 kernel evaluates (exp / log / 1/x, the f64 sin/cos of m_sincos).
#ifndef DTMPC_FAST_F64
#define DTMPC_FAST_F64 0
#endif
#if DTMPC_FAST_F64
#define FK_NS fk64
#define FKN(x) x##64
#else
#define FK_NS fk
#define FKN(x) x
#endif

namespace dtmpc {
namespace FK_NS {

#if DTMPC_FAST_F64
typedef double real;
#else
typedef float real;
#endif
constexpr unsigned ES = sizeof(real) / 4;  // 32-bit words per value: record and SoA byte strides scale by it

typedef real f2 __attribute__((ext_vector_type(2)));
typedef real f4 __attribute__((ext_vector_type(4)));
typedef real f8 __attribute__((ext_vector_type(8)));
typedef int i8v __attribute__((ext_vector_type(8)));

constexpr int NC = 6;  // rolled-out line-search candidates (alpha = 0 is the current tape)

// Uniform problem constants (kernarg).  a = max(alpha, eps) and its powers are formed on the host in
// f32 exactly as the generic kernel forms them on the device (1/a and 1/a^2 correctly rounded).
struct FP {
  int N;
  real dt, umin0, umin1, umax0, umax1, active_tol;
  real neg_beta, neg_inv_beta;
  real nbl2e;  // neg_beta * log2(e): exp(-beta h_i - zmax) = exp2(fma(h_i, nbl2e, -zmax log2(e)))
  real a, eps, gamma, inv_a, a2, a3, inv_a2;
  f8 cx, cy, r2;  // ext-vector: SSA values (a real[8] became a private array in memory)
  real tight;    // h offset of a tightened solve (Obs<M>::tight: the general path's nominal), else unused
};

// The obstacle template argument M of every h-evaluating function: the obstacle count, with kTight set
// for a solve whose barrier sees the tightened h - s (core/tube_mpc.py:235-238: the general path's
// nominal MPC; barrier_dyn(s, h - s.tight) in the generic kernels).  Instantiations without the flag are
// the tube step's and carry no extra instruction.
constexpr int kTight = 16;
// kWrap: the nominal target cost with the heading error wrapped to (-pi, pi] (run_nominal.py:297-324, the
// receding-horizon driver's stage / terminal cost and derivatives); only the receding kernel sets it.
constexpr int kWrap = 32;
// kLds (f64): the obstacle table read again at each use instead of being held in registers -- the f64
// instantiations whose table cannot be pinned in VGPRs without spilling (tab_flag below).  DTMPC_FAST64_TABSRC:
// 1 (default) a scalar load of the kernarg segment's copy (every kernel's arguments start with its FP); 0 the
// workgroup's LDS copy (obs_lds; A/B: at four lanes its even-M general-record kernels gave run-to-run
// different results).
constexpr int kLds = 64;
// kXasm (f64): the smooth-min exp's polynomial as one inline-assembly block (exp_sm<true>) -- set only where it
// fits the register file without a private segment (xasm_flag below); elsewhere the same fmas compiled normally.
constexpr int kXasm = 128;
#ifndef DTMPC_FAST64_TABSRC
#define DTMPC_FAST64_TABSRC 1
#endif
template <int M>
struct Obs {
  static constexpr int n = M & (kTight - 1);
  static constexpr bool tight = (M & kTight) != 0;
  static constexpr bool wrap = (M & kWrap) != 0;
  static constexpr bool lds = (M & kLds) != 0;
  static constexpr bool xasm = (M & kXasm) != 0;
};

#if DTMPC_FAST_F64 && DTMPC_FAST64_TABSRC == 0
// the f64 kernels' obstacle table in LDS (x, y, r^2, -) per obstacle, written once per workgroup (obs_fill)
__shared__ real obs_lds[32];
#endif
// obstacle i of the table: the registers of FP, or (kLds) loaded again at each use -- through an opaque pointer
// (a hoisted load would hold the table in registers for the whole loop, which is what kLds instantiations cannot
// afford): a scalar load from the kernarg segment (the value is wave-uniform, so it lands in an SGPR pair for the
// few instructions that use it), or the LDS copy
template <int M>
__device__ __forceinline__ real otab_at(int f, int i) {
#if DTMPC_FAST_F64 && DTMPC_FAST64_TABSRC == 0
  return ((volatile __attribute__((address_space(3))) real*)obs_lds)[4 * i + f];
#else
  // kernarg FP: cx at offsetof(FP, cx), cy, r2 follow (f8 each); the pointer made opaque per use
  typedef __attribute__((address_space(4))) const real creal;
  creal* k = (creal*)((__attribute__((address_space(4))) const char*)__builtin_amdgcn_kernarg_segment_ptr() +
                      offsetof(FP, cx) + (unsigned)f * sizeof(f8));
  __asm__ volatile("" : "+s"(k));
  return k[i];
#endif
}
template <int M>
__device__ __forceinline__ real ocx(const FP& p, int i) {
  if (DTMPC_FAST_F64 && Obs<M>::lds) return otab_at<M>(0, i);
  return p.cx[i];
}
template <int M>
__device__ __forceinline__ real ocy(const FP& p, int i) {
  if (DTMPC_FAST_F64 && Obs<M>::lds) return otab_at<M>(1, i);
  return p.cy[i];
}
template <int M>
__device__ __forceinline__ real or2(const FP& p, int i) {
  if (DTMPC_FAST_F64 && Obs<M>::lds) return otab_at<M>(2, i);
  return p.r2[i];
}
// kLds kernels: the table into LDS from the kernarg copy, before any lane returns (one barrier)
template <int M>
__device__ __forceinline__ void obs_fill(const FP& p) {
#if DTMPC_FAST_F64 && DTMPC_FAST64_TABSRC == 0
  if (Obs<M>::lds) {
    if (threadIdx.x == 0) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        obs_lds[4 * j] = p.cx[j];
        obs_lds[4 * j + 1] = p.cy[j];
        obs_lds[4 * j + 2] = p.r2[j];
        obs_lds[4 * j + 3] = 0.0;
      }
    }
    __syncthreads();
  }
#endif
}

struct FCost {  // nominal: target; ancillary: tracking (terminal weight = stage weight)
  real Q0, Q1, Q2, R0, R1, Qf0, Qf1, Qf2, qb;
  f4 tg;  // target (x, y, theta, -): ext-vector, an SSA value (three floats became a private array)
};

struct FIlqr {
  int max_iter, zpos;
  real tol, reg;
  f8 cal;   // rolled-out candidates' alphas (NC used); ext-vectors: SSA values, never a private array
  i8v cpos; // their original positions
};

struct FArgs {
  int B;       // trajectories of the batch: the stride of the ABI SoA arrays
  int i0, Bc;  // this launch's chunk of trajectories [i0, i0 + Bc): the workspace records hold Bc
  long long goff, step;
  real* x;
  real* b;
  real* xbar;
  real* bbar;
  real* Xnom;
  real* Unom;
  real* Xaux;
  real* Uaux;
  real* work;  // workspace: the per-lane records below, one buffer resource (< 2^31 bytes)
  unsigned wsz;  // bytes of it the records use
  unsigned oXn, oUn, oXa, oUa, oK, ok, oA8, oA2;  // byte offsets of the record arrays in the workspace
  unsigned oPH;  // the split step's hand-over [3][Bc] int: nominal tape's record offsets, status | iterations << 8
  int phase;     // dtmpc_tube_state.phase: 0 whole step, 1 nominal solve, 2 the rest
  const real* theta;
  real* partials;
  real* log;
  int* status;
  int* iters;
  const real* w;
  int disturbance, write_log;
  unsigned long long seed;
  real wlo[3], whi[3];
  int stagger;  // s_sleep(127) rounds before this workgroup starts (phase desynchronisation, see launch)
  signed char* choices;  // [nom max_iter + aux max_iter][B] or NULL (dtmpc_tube_state.choices)
  real gbound;          // health bound on the gradient row (dtmpc_tube_cfg.grad_bound; +inf: none)
  real* costs;          // [nom max_iter + aux max_iter][8][B] or NULL (dtmpc_tube_state.costs)
};

// ---------------------------------------------------------------------------------------------
// memory access.  Every tape access is ONE global load / store in the scalar-base form
// (global_load v, v_off, s[base:base+1]): the row base is uniform (kept in SGPRs: the empty asm
// stops the compiler from folding the per-lane offset into a 64-bit per-lane VGPR address, which
// costs a 64-bit VALU multiply-add per access), the per-lane part a 32-bit byte offset fixed for
// the whole kernel.
typedef __attribute__((address_space(1))) char gchar;
__device__ __forceinline__ real* gaddr(const char* base, size_t row_off, unsigned lane_off) {
  gchar* row = (gchar*)base + row_off;
  __asm__("" : "+s"(row));
  // the lane offset is re-materialised here (volatile: not hoisted out of the step loop), so the
  // zero-extension and the add stay in the access's block and select the scalar-base form
  __asm__ volatile("" : "+v"(lane_off));
  return (real*)(row + lane_off);
}

// a step index known to be wave-uniform (readfirstlane: free when the compiler already keeps it in an
// SGPR; it pins a clamped refill index to the scalar unit, where gaddr needs its row base)
__device__ __forceinline__ int uidx(int k) { return __builtin_amdgcn_readfirstlane(k); }

// per-lane byte offsets of field f of a SoA row: trajectory * 4 + f * B * 4 (four VGPRs shared by
// every SoA tape of the batch)
struct Lane {
  unsigned f0, f1, f2, f3;
};

// SoA [rows][F][B] f32 array (the ABI tapes): element (k, f) of this lane (f a compile-time constant)
template <int F>
struct Soa {
  char* base;
  unsigned rs;  // F * B * 4
  Lane L;
  __device__ __forceinline__ real* p(int k, int f) const {
    const unsigned o = f == 0 ? L.f0 : f == 1 ? L.f1 : f == 2 ? L.f2 : L.f3;
    return gaddr(base, (size_t)(unsigned)k * rs, o);
  }
  __device__ __forceinline__ real ld(int k, int f) const { return *p(k, f); }
  __device__ __forceinline__ void st(int k, int f, real v) const { *p(k, f) = v; }
};

// per-lane records [rows][B][W] f32 (W = 2 or 8): row k of this lane
template <int W>
struct Rec {
  char* base;
  unsigned rs;  // B * W * 4
  unsigned lo;  // trajectory * W * 4
  __device__ __forceinline__ real* p(int k) const {
    return gaddr(base, (size_t)(unsigned)k * rs, lo);
  }
};

__device__ __forceinline__ f4 ld4(const real* q) { return *(const f4*)__builtin_assume_aligned(q, 16); }
__device__ __forceinline__ f2 ld2(const real* q) { return *(const f2*)__builtin_assume_aligned(q, 8); }
__device__ __forceinline__ void st4(real* q, f4 v) { *(f4*)__builtin_assume_aligned(q, 16) = v; }
__device__ __forceinline__ void st2(real* q, f2 v) { *(f2*)__builtin_assume_aligned(q, 8) = v; }

// ---------------------------------------------------------------------------------------------
// the workspace records.  Every per-step array the solver iterates on lives in the workspace as
// per-lane records [rows][Bc][W] (AoS: one trajectory's row is W contiguous floats), addressed through
// ONE buffer resource: element (row k, field f) of this lane is at soffset = base + k * rs (SGPR, a
// running scalar add per step) + voffset = lane * W * 4 (a VGPR fixed for the kernel) + the field's
// byte offset.  A row of a record is one 16-byte (or 8-byte) access, and every array is dense (no
// padding: a padded record costs its padding in HBM reads -- measured +25 % traffic with 32-byte XU
// and 48-byte gain records).
//   X   [N+1][Bc][4]  x0 x1 x2 b        U  [N][Bc][2]  u0 u1      (nominal and ancillary tapes)
//   K   [N][Bc][8]    K00..K03 K10..K13 k  [N][Bc][2]  k0 k1      (gains)
//                     gamma = 0 (Gains<G0>): K [N][Bc][8] = K00 K01 K02 K10 K11 K12 k0 k1, k unused
//   A8  [N][Bc][8]    a02 a12 a30 a31 a32 b00 b10 b30   A2 [N][Bc][2] b31 act  (sensitivity scratch)
typedef __amdgpu_buffer_rsrc_t Rsrc;
typedef unsigned u4v __attribute__((ext_vector_type(4)));
typedef unsigned u2v __attribute__((ext_vector_type(2)));

struct RA {
  unsigned base, rs, lo;  // uniform base and row stride (bytes), per-lane offset (bytes)
  __device__ __forceinline__ unsigned so(int k) const { return base + (unsigned)k * rs; }
};
#ifndef DTMPC_FAST_STPOL
#define DTMPC_FAST_STPOL 0  // cache-policy bits of the record stores (A/B)
#endif
// 128-bit buffer stores and the gfx950 store-data hazard (round 5).  A buffer_store_dwordx4 reads its data VGPRs
// after issue; a VALU write to them in the next cycles changes what the store writes.  The compiler pads this hazard
// only for stores without an SGPR soffset, and every record store here has one (the row base): it emitted a
// dwordx4 store followed at once by a move into its data registers, and the store wrote the moved value
// (profiles/r05/store_hazard.txt: one component of one record, a reproducible wrong tape).  DTMPC_FAST_STNOP = 1
// (default): every 128-bit record store is followed by an s_nop 1 that reads its data registers, so they stay
// unwritten for its two wait states.  Stores of 64 bits and less are not affected.
#ifndef DTMPC_FAST_STNOP
#define DTMPC_FAST_STNOP 1
#endif
template <class D>
__device__ __forceinline__ void st128(D d, Rsrc r, unsigned voff, unsigned soff) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v, d), r, voff, soff, DTMPC_FAST_STPOL);
#if DTMPC_FAST_STNOP
  __asm__ volatile("s_nop 1" ::"v"(d));
#endif
}
#if DTMPC_FAST_F64
// f64: a 4-value row is 32 bytes (two 16-byte accesses), a 2-value row 16 bytes (one)
typedef double d2v __attribute__((ext_vector_type(2)));
#ifdef DTMPC_DIAG_STALE
// diagnostics builds (scripts/diag_stale.py): a workspace pre-filled with 0xff bytes holds the all-ones pattern, which
// no arithmetic produces (a computed NaN is 0x7ff8...): a record load that returns it read a slot this run never wrote
__device__ __noinline__ void stale_hit(unsigned base, unsigned so, unsigned vo, int which) {
  printf("STALE blk=%d thr=%d base=%u soff=%u voff=%u part=%d\n", (int)blockIdx.x, (int)threadIdx.x, base, so, vo, which);
}
__device__ __forceinline__ void stale_chk(d2v v, const RA& a, int k, unsigned off, int which) {
  const unsigned long long ones = ~0ull;
  if (__builtin_bit_cast(unsigned long long, v.x) == ones || __builtin_bit_cast(unsigned long long, v.y) == ones)
    stale_hit(a.base, a.so(k), a.lo + off, which);
}
#else
__device__ __forceinline__ void stale_chk(d2v, const RA&, int, unsigned, int) {}
#endif
__device__ __forceinline__ f4 rld4(Rsrc r, const RA& a, int k, unsigned off) {
  const d2v lo = __builtin_bit_cast(d2v, __builtin_amdgcn_raw_buffer_load_b128(r, a.lo + off, a.so(k), 0));
  const d2v hi = __builtin_bit_cast(d2v, __builtin_amdgcn_raw_buffer_load_b128(r, a.lo + off + 16u, a.so(k), 0));
  stale_chk(lo, a, k, off, 0);
  stale_chk(hi, a, k, off, 1);
  return f4{lo.x, lo.y, hi.x, hi.y};
}
__device__ __forceinline__ f2 rld2(Rsrc r, const RA& a, int k, unsigned off) {
  const d2v v = __builtin_bit_cast(d2v, __builtin_amdgcn_raw_buffer_load_b128(r, a.lo + off, a.so(k), 0));
  stale_chk(v, a, k, off, 2);
  return __builtin_bit_cast(f2, v);
}
__device__ __forceinline__ void rst4(Rsrc r, const RA& a, int k, unsigned off, f4 v) {
  st128(d2v{v.x, v.y}, r, a.lo + off, a.so(k));
  st128(d2v{v.z, v.w}, r, a.lo + off + 16u, a.so(k));
}
__device__ __forceinline__ void rst2(Rsrc r, const RA& a, int k, unsigned off, f2 v) { st128(v, r, a.lo + off, a.so(k)); }
#elif !defined(DTMPC_FAST_GLOBAL)
__device__ __forceinline__ f4 rld4(Rsrc r, const RA& a, int k, unsigned off) {
  return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, a.lo + off, a.so(k), 0));
}
__device__ __forceinline__ f2 rld2(Rsrc r, const RA& a, int k, unsigned off) {
  return __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(r, a.lo + off, a.so(k), 0));
}
__device__ __forceinline__ void rst4(Rsrc r, const RA& a, int k, unsigned off, f4 v) { st128(v, r, a.lo + off, a.so(k)); }
__device__ __forceinline__ void rst2(Rsrc r, const RA& a, int k, unsigned off, f2 v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, v), r, a.lo + off, a.so(k), DTMPC_FAST_STPOL);
}
#else  // A/B: the same records through global loads / stores with a scalar row base
__device__ __forceinline__ const char* kargs_ws();
__device__ __forceinline__ f4 rld4(Rsrc, const RA& a, int k, unsigned off) {
  return *(const f4*)gaddr(kargs_ws(), (size_t)a.so(k), a.lo + off);
}
__device__ __forceinline__ f2 rld2(Rsrc, const RA& a, int k, unsigned off) {
  return *(const f2*)gaddr(kargs_ws(), (size_t)a.so(k), a.lo + off);
}
__device__ __forceinline__ void rst4(Rsrc, const RA& a, int k, unsigned off, f4 v) {
  *(f4*)gaddr(kargs_ws(), (size_t)a.so(k), a.lo + off) = v;
}
__device__ __forceinline__ void rst2(Rsrc, const RA& a, int k, unsigned off, f2 v) {
  *(f2*)gaddr(kargs_ws(), (size_t)a.so(k), a.lo + off) = v;
}
#endif

// (LDS-resident gains -- the first steps' iLQR gains kept in the CU's LDS instead of the workspace -- were
// built in round 3, measured slower at every lane form (profiles/r03/ab_lds.txt) and deleted in round 4: with
// the option off, the step-index test in front of every gain access was still compiled as a runtime branch
// (the sign of a readfirstlane'd index is unknown to the compiler))

template <int P>
struct Gains {
  RA K, k;     // K and k records (the iLQR's; the sensitivity pass's full records)
  // G0 (gamma = 0): K's column for the barrier state b is exactly zero (A's column 3 is (0, 0, 0, gamma),
  // so Q_ux's is gamma * S = 0 and K = -Q_uu^-1 Q_ux keeps it), and the iLQR record is the 32 bytes
  // K00 K01 K02 K10 | K11 K12 k0 k1 -- 8 B less per step, two loads instead of three
  template <bool G0>
  __device__ __forceinline__ void store(Rsrc r, int s, const real* Kk, const real* kk) const {
    const f4 g0 = G0 ? f4{Kk[0], Kk[1], Kk[2], Kk[4]} : f4{Kk[0], Kk[1], Kk[2], Kk[3]};
    const f4 g1 = G0 ? f4{Kk[5], Kk[6], kk[0], kk[1]} : f4{Kk[4], Kk[5], Kk[6], Kk[7]};
    rst4(r, K, s, 0, g0);
    rst4(r, K, s, 16 * ES, g1);
    if (!G0) rst2(r, k, s, 0, f2{kk[0], kk[1]});
  }
  // step s's gains: K rows (Ka, Kb; G0: the zero column as 0) and k
  template <bool G0>
  __device__ __forceinline__ void load(Rsrc r, int s, f4& Ka, f4& Kb, f2& kf) const {
    const f4 g0 = rld4(r, K, s, 0), g1 = rld4(r, K, s, 16 * ES);
    if (G0) {
      Ka = f4{g0.x, g0.y, g0.z, 0.f};
      Kb = f4{g0.w, g1.x, g1.y, 0.f};
      kf = f2{g1.z, g1.w};
    } else {
      Ka = g0;
      Kb = g1;
      kf = rld2(r, k, s, 0);
    }
  }
  // the sensitivity pass's full records K (32 B) + k (8 B), always in the workspace
  __device__ __forceinline__ void store_full(Rsrc r, int s, const real* Kk, const real* kk) const {
    rst4(r, K, s, 0, f4{Kk[0], Kk[1], Kk[2], Kk[3]});
    rst4(r, K, s, 16 * ES, f4{Kk[4], Kk[5], Kk[6], Kk[7]});
    rst2(r, k, s, 0, f2{kk[0], kk[1]});
  }
};

// ---------------------------------------------------------------------------------------------
// elementwise math on V = real (one candidate) or f2 (a candidate pair, packed f32 VALU)

template <class V> struct VT;
template <> struct VT<real> { static constexpr int W = 1; };
template <> struct VT<f2> { static constexpr int W = 2; };

__device__ __forceinline__ real vmin(real a, real b) { return m_min(a, b); }
__device__ __forceinline__ f2 vmin(f2 a, f2 b) { return f2{m_min(a.x, b.x), m_min(a.y, b.y)}; }
// torch.clamp (core/control.py:61-64) as v_maximum3_f32 / v_minimum3_f32: IEEE 754-2019 maximum /
// minimum propagate NaN like the compare-select form, without a VCC write (no hazard wait states)
__device__ __forceinline__ real vclamp(real v, real lo, real hi) {
  return __builtin_elementwise_minimum(__builtin_elementwise_maximum(v, lo), hi);
}
__device__ __forceinline__ f2 vclamp(f2 v, real lo, real hi) { return f2{vclamp(v.x, lo, hi), vclamp(v.y, lo, hi)}; }
__device__ __forceinline__ real vmaxnan(real a, real b) { return __builtin_elementwise_maximum(a, b); }
// a * b + c of the forward passes (dynamics, h_i, DBaS update, costs, the commit's u): one fused
// rounding (v_fma / v_pk_fma; measured 4.66 -> 4.55 ms), the rounding of the oracle's FMA-contraction
// build; DTMPC_FAST_FWD_FMA=0 rounds twice, as the reference's separate torch ops do.  Written at the
// same places of the line search, the commit and the start rollout, so either way a committed tape is
// the candidate priced.
#ifndef DTMPC_FAST_FWD_FMA
#define DTMPC_FAST_FWD_FMA 1
#endif
template <class V>
__device__ __forceinline__ V ffma(V a, V b, V c) {
#if DTMPC_FAST_FWD_FMA
  return __builtin_elementwise_fma(a, b, c);
#else
  DTMPC_NOCONTRACT
  return a * b + c;
#endif
}
#if DTMPC_FAST_F64
// f64: exp / log as the generic f64 kernel evaluates them (OCML), the smooth-min terms as it forms them
// (smterm); sin / cos by a Cody-Waite reduction by pi/2 in three fma steps (the first exact) and the
// fdlibm kernels __kernel_sin / __kernel_cos on [-pi/4, pi/4] (< 1 ulp), the quadrant applied by exact
// products with (A, B) in {0, +-1} as in the f32 form; |x| > 2^20 and non-finite take OCML sincos, out of
// line (its Payne-Hanek branch would otherwise be inlined into every rollout step).
// DTMPC_FAST64_EXP = 1: OCML's exp_f64 operation for operation (the same reduction, coefficients and fma order,
// so bitwise the same values on [-1075, 1024]) without its two range selects -- every caller's argument is a
// smooth-min exponent in [-50, 0] or NaN -- and with the polynomial's fmas in the three-address form
// (v_fma_f64): the compiler otherwise emits each as a copy of the coefficient plus a two-address v_fmac_f64.
#ifndef DTMPC_FAST64_EXP
#define DTMPC_FAST64_EXP 3
#endif
template <bool ASM>
__device__ __forceinline__ double exp_sm(double x) {
  const double k = __builtin_rint(x * 0x1.71547652b82fep+0);
  double r = __builtin_fma(-k, 0x1.62e42fefa39efp-1, x);
  r = __builtin_fma(-k, 0x1.abc9e3b39803fp-56, r);
  double q;
  if (ASM) {
  // the nine-fma Horner chain as one block: dependent v_fma_f64 need no wait states, and one block takes the
  // compiler's conservative s_nop around inline assembly once instead of once per fma
  __asm__("v_fma_f64 %0, %1, %2, %3\n\t"
          "v_fma_f64 %0, %1, %0, %4\n\t"
          "v_fma_f64 %0, %1, %0, %5\n\t"
          "v_fma_f64 %0, %1, %0, %6\n\t"
          "v_fma_f64 %0, %1, %0, %7\n\t"
          "v_fma_f64 %0, %1, %0, %8\n\t"
          "v_fma_f64 %0, %1, %0, %9\n\t"
          "v_fma_f64 %0, %1, %0, %10\n\t"
          "v_fma_f64 %0, %1, %0, %11"
          : "=&v"(q)
          : "v"(r), "v"(0x1.ade156a5dcb37p-26), "v"(0x1.28af3fca7ab0cp-22), "v"(0x1.71dee623fde64p-19),
            "v"(0x1.a01997c89e6b0p-16), "v"(0x1.a01a014761f6ep-13), "v"(0x1.6c16c1852b7b0p-10),
            "v"(0x1.1111111122322p-7), "v"(0x1.55555555502a1p-5), "v"(0x1.5555555555511p-3),
            "v"(0x1.000000000000bp-1));
  } else {
  q = __builtin_fma(r, 0x1.ade156a5dcb37p-26, 0x1.28af3fca7ab0cp-22);
  q = __builtin_fma(r, q, 0x1.71dee623fde64p-19);
  q = __builtin_fma(r, q, 0x1.a01997c89e6b0p-16);
  q = __builtin_fma(r, q, 0x1.a01a014761f6ep-13);
  q = __builtin_fma(r, q, 0x1.6c16c1852b7b0p-10);
  q = __builtin_fma(r, q, 0x1.1111111122322p-7);
  q = __builtin_fma(r, q, 0x1.55555555502a1p-5);
  q = __builtin_fma(r, q, 0x1.5555555555511p-3);
  q = __builtin_fma(r, q, 0x1.000000000000bp-1);
  }
  q = __builtin_fma(r, q, 1.0);
  q = __builtin_fma(r, q, 1.0);
  return __builtin_ldexp(q, (int)k);
}
#ifdef DTMPC_DIAG_CHEAPEXP  // timing only (wrong results by design): exp through v_exp_f32
__device__ __forceinline__ real vexp(real x) { return (double)__builtin_amdgcn_exp2f((float)(x * 1.4426950408889634)); }
#elif DTMPC_FAST64_EXP
__device__ __forceinline__ real vexp(real x) { return exp_sm<false>(x); }
#else
__device__ __forceinline__ real vexp(real x) { return m_exp(x); }
#endif
__device__ __forceinline__ f2 vexp(f2 x) { return f2{vexp(x.x), vexp(x.y)}; }
// 1 / x and a / b for the call sites whose divisor is a finite positive normal or NaN (the barrier's max(z, eps),
// the smooth-min sum se in [1, M], the log's 2 + f in [1.4, 2.9]).  DTMPC_FAST64_RCP = 1: v_rcp_f64 (~2^-23
// relative) and two Newton steps (1 / x within an ulp); the quotient a r corrected by one residual step, i.e. 5 and
// 6 instructions against IEEE division's 11 (div_scale, div_fmas, div_fixup).  0: IEEE division.
#ifndef DTMPC_FAST64_HGLOG
#define DTMPC_FAST64_HGLOG 1
#endif
#ifndef DTMPC_FAST64_RCP
#define DTMPC_FAST64_RCP 1
#endif
__device__ __forceinline__ real frcp(real x) {
#if DTMPC_FAST64_RCP
  double r = __builtin_amdgcn_rcp(x);
  double e = __builtin_fma(-x, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-x, r, 1.0);
  return __builtin_fma(r, e, r);
#else
  return 1.0 / x;
#endif
}
__device__ __forceinline__ real fdiv(real a, real b) {
#if DTMPC_FAST64_RCP
  double r = __builtin_amdgcn_rcp(b);
  r = __builtin_fma(r, __builtin_fma(-b, r, 1.0), r);
  const double q = a * r;
  return __builtin_fma(r, __builtin_fma(-b, q, a), q);
#else
  return a / b;
#endif
}
// the smooth-min log log(se), se in [1, M] (its largest term is exp(0)): fdlibm's e_log -- frexp, s = f / (2 + f),
// a degree-14 odd polynomial in s (< 1 ulp), ~35 instructions against OCML's ~90 (a double-double evaluation);
// +inf passes through.  Measured: f64 tube step 14.72 -> 13.90 ms at B = 65,536 (profiles/r03/f64_log_experiment.txt)
__device__ __forceinline__ real vlog(real x) {
  constexpr double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
  constexpr double Lg1 = 6.666666666666735130e-01, Lg2 = 3.999999999940941908e-01, Lg3 = 2.857142874366239149e-01,
                   Lg4 = 2.222219843214978396e-01, Lg5 = 1.818357216161805012e-01, Lg6 = 1.531383769920937332e-01,
                   Lg7 = 1.479819860511658591e-01;
  double m = __builtin_amdgcn_frexp_mant(x);  // [0.5, 1)
  int e = __builtin_amdgcn_frexp_exp(x);
  if (m < 0.70710678118654752440) {
    m = m + m;
    e = e - 1;
  }
  const double k = (double)e, f = m - 1.0, s = fdiv(f, 2.0 + f), z = s * s, w = z * z;
  const double t1 = w * __builtin_fma(w, __builtin_fma(w, Lg6, Lg4), Lg2);
  const double t2 = z * __builtin_fma(w, __builtin_fma(w, __builtin_fma(w, Lg7, Lg5), Lg3), Lg1);
  const double R = t2 + t1, hfsq = 0.5 * f * f;
  const double r = k * ln2_hi - ((hfsq - (s * (hfsq + R) + k * ln2_lo)) - f);
  return x == __builtin_inf() ? x : r;
}
__device__ __forceinline__ f2 vlog(f2 x) { return f2{vlog(x.x), vlog(x.y)}; }
// A smooth-min term exp(-beta h_i - zmax) below exp(-kSmSkip) = exp(-50) = 1.9e-22 is taken as 0: se >= 1 (its
// largest term is exp(0)), so at most eight such terms move se by < 1.6e-21, i.e. < 1e-5 ulp -- the f64 sum is
// unchanged except on a one-in-10^5 rounding tie.  The rule is per value (the same candidate state gives the
// same se in the line search, the commit and the start rollout); smsum skips the exp for an obstacle no lane
// of the wave needs (a uniform branch: far obstacles -- h_i > h_min + 2.5 at beta = 20 -- are most of them).
// f64 only: the f32 term is one v_exp_f32.
constexpr double kSmSkip = 50.0;
template <class V>
__device__ __forceinline__ V smarg(const FP& p, V hi, V zmax) {
  DTMPC_NOCONTRACT
  return p.neg_beta * hi - zmax;
}
#if DTMPC_FAST64_EXP
// branch-free: the caller's wave-uniform branch already decided that some lane needs this term; exp_sm of an
// argument below -50 (down to -inf) is a finite number, 0 or NaN and is replaced by 0
template <int M = 0>
__device__ __forceinline__ real smexp(real x) {
  const real e = exp_sm<Obs<M>::xasm && DTMPC_FAST64_EXP == 3>(x);
  return x < -kSmSkip ? 0.0 : e;
}
#else
template <int M = 0>
__device__ __forceinline__ real smexp(real x) { return x < -kSmSkip ? 0.0 : vexp(x); }
#endif
template <int M = 0>
__device__ __forceinline__ f2 smexp(f2 x) { return f2{smexp<M>(x.x), smexp<M>(x.y)}; }
__device__ __forceinline__ bool smneed(real x) { return !(x < -kSmSkip); }  // NaN: needed (it propagates)
__device__ __forceinline__ bool smneed(f2 x) { return smneed(x.x) || smneed(x.y); }
template <int M = 0, class V>
__device__ __forceinline__ V smterm(const FP& p, V hi, V zmax, V) {
  const V x = smarg(p, hi, zmax);
  V e = V(0.0);
  if (__builtin_amdgcn_ballot_w64(smneed(x))) e = smexp<M>(x);  // wave-uniform
  return e;
}
#ifndef DTMPC_FAST_SINCOS_AB
#define DTMPC_FAST_SINCOS_AB 1
#endif
constexpr double kDPio2A = 1.5707963267948966, kDPio2B = 6.123233995736766e-17, kDPio2C = -1.4973849048591698e-33,
                 kD2oPi = 0.6366197723675814;
constexpr double kDS1 = -1.66666666666666324348e-01, kDS2 = 8.33333333332248946124e-03,
                 kDS3 = -1.98412698298579493134e-04, kDS4 = 2.75573137070700676789e-06,
                 kDS5 = -2.50507602534068634195e-08, kDS6 = 1.58969099521155010221e-10;
constexpr double kDC1 = 4.16666666666666019037e-02, kDC2 = -1.38888888888741095749e-03,
                 kDC3 = 2.48015872894767294178e-05, kDC4 = -2.75573143513906633035e-07,
                 kDC5 = 2.08757232129817482790e-09, kDC6 = -1.13596475577881948265e-11;
// 1: OCML sincos out of line (the default); 0: inline in the cold branch; 2: none (ISA experiments only).
// Round 3 measured wrong results with 0 on the one-lane f64 kernel (test_tube_step_fast64_vs_generic[1]);
// on the round-4 source 0 and 1 are bitwise equal over two closed-loop steps (default contraction and
// -ffp-contract=off alike) and 0 passes that test (profiles/r04/f64_far_sincos.txt).  The two sources differ
// in the inline form's SGPR spilling (482 -> 403 spills to VGPR lanes in the cold-branch kernel), which is
// where a compiler defect would sit; the round-3 build is not reproducible, so 1 stays the default.
#ifndef DTMPC_FAST64_FAR
#define DTMPC_FAST64_FAR 1
#endif
#ifndef DTMPC_FAST64_FARRET
#define DTMPC_FAST64_FARRET 1
#endif
struct SinCos {
  double s, c;
};
#if DTMPC_FAST64_FARRET
// returned by value (v0..v3): no out-parameter, so no local of the caller ever has its address taken
#if DTMPC_FAST64_FAR == 1
__device__ __attribute__((noinline)) SinCos sincos_far(double x) {
#else
__device__ __forceinline__ SinCos sincos_far(double x) {
#endif
  SinCos r;
  sincos(x, &r.s, &r.c);
  return r;
}
#elif DTMPC_FAST64_FAR == 1
__device__ __attribute__((noinline)) void sincos_far(double x, double* s, double* c) {
#ifdef DTMPC_FAST_DIAG_FARPRINT
  printf("DIAG far x=%.17g\n", x);
#endif
  sincos(x, s, c);
#ifdef DTMPC_FAST_DIAG_FARWAIT
  __builtin_amdgcn_s_waitcnt(0);
#endif
}
#else
__device__ __forceinline__ void sincos_far(double x, double* s, double* c) { sincos(x, s, c); }
#endif
__device__ __forceinline__ void vsincos(real x, real& sn, real& cs) {
#if DTMPC_FAST64_FAR != 2
  if (__builtin_expect(!(__builtin_fabs(x) <= 1048576.0), 0)) {
#if DTMPC_FAST64_FARRET
    const SinCos r = sincos_far(x);
    sn = r.s;
    cs = r.c;
#else
    sincos_far(x, &sn, &cs);
#endif
    return;
  }
#endif
  const double q = __builtin_rint(x * kD2oPi);
  double r = __builtin_fma(-q, kDPio2A, x);
  r = __builtin_fma(-q, kDPio2B, r);
  r = __builtin_fma(-q, kDPio2C, r);
  const double z = r * r;
  double ps = __builtin_fma(z, kDS6, kDS5);
  ps = __builtin_fma(z, ps, kDS4);
  ps = __builtin_fma(z, ps, kDS3);
  ps = __builtin_fma(z, ps, kDS2);
  const double s = __builtin_fma(z * r, __builtin_fma(z, ps, kDS1), r);
  double pc = __builtin_fma(z, kDC6, kDC5);
  pc = __builtin_fma(z, pc, kDC4);
  pc = __builtin_fma(z, pc, kDC3);
  pc = __builtin_fma(z, pc, kDC2);
  pc = __builtin_fma(z, pc, kDC1);
  const double hz = 0.5 * z, w = 1.0 - hz;
  const double c = w + (((1.0 - w) - hz) + (z * z) * pc);
  const double m = __builtin_fma(-4.0, __builtin_floor(__builtin_fma(q, 0.25, 0.25)), q);
  const double A = 1.0 - __builtin_fabs(m), Bq = __builtin_fmin(m, 2.0 - m);
  sn = __builtin_fma(s, A, c * Bq);
  cs = __builtin_fma(c, A, -(s * Bq));
}
__device__ __forceinline__ void vsincos(f2 x, f2& s, f2& c) {
  real s0, c0, s1, c1;
  vsincos(x.x, s0, c0);
  vsincos(x.y, s1, c1);
  s = f2{s0, s1};
  c = f2{c0, c1};
}
#else
__device__ __forceinline__ real vexp(real x) { return m_exp(x); }
__device__ __forceinline__ real vexp2(real x) { return __builtin_amdgcn_exp2f(x); }
__device__ __forceinline__ f2 vexp2(f2 x) { return f2{__builtin_amdgcn_exp2f(x.x), __builtin_amdgcn_exp2f(x.y)}; }
__device__ __forceinline__ f2 vexp(f2 x) { return pk_exp(x); }
__device__ __forceinline__ real vlog(real x) { return m_log(x); }
__device__ __forceinline__ f2 vlog(f2 x) { return pk_log(x); }
__device__ __forceinline__ real frcp(real x) { return m_rcp(x); }
// the smooth-min term exp(-beta h_i - zmax) = exp2(fma(h_i, -beta log2(e), -zmax log2(e))) (zl = zmax log2 e)
template <int M = 0, class V>
__device__ __forceinline__ V smterm(const FP& p, V hi, V, V zl) {
  return vexp2(__builtin_elementwise_fma(hi, V(p.nbl2e), -zl));
}
// sin / cos for the forward passes: sincos_cw's Cody-Waite reduction x = r + j pi/2 and minimax
// polynomials, with the quadrant applied WITHOUT selects: sin x = A s + B c, cos x = A c - B s with
// (A, B) = (cos j pi/2, sin j pi/2) in {0, +-1} -- m = j - 4 floor((j + 1) / 4) in {-1, 0, 1, 2},
// A = 1 - |m|, B = min(m, 2 - m).  Every product is by 0 or +-1, so the values are exactly the
// quadrant-selected ones (the sign of a zero result aside); |x| > 65536 and non-finite take OCML.
// Same operations element by element in the scalar (commit, start rollout, plant) and the pair (line
// search) form: a committed tape is bitwise the candidate priced.
#ifndef DTMPC_FAST_SINCOS_AB
#define DTMPC_FAST_SINCOS_AB 1
#endif
__device__ __forceinline__ void sincos_poly(real r, real& s, real& c) {
  const real z = r * r;
  real ps = __builtin_fmaf(z, kSinS3, kSinS2);
  ps = __builtin_fmaf(z, ps, kSinS1);
  s = __builtin_fmaf(r * z, ps, r);
  real pc = __builtin_fmaf(z, kCosK3, kCosK2);
  pc = __builtin_fmaf(z, pc, kCosK1);
  c = __builtin_fmaf(z * z, pc, __builtin_fmaf(-0.5f, z, 1.0f));
}
__device__ __forceinline__ void vsincos(real x, real& sn, real& cs) {
#if DTMPC_FAST_SINCOS_AB
  if (__builtin_expect(!(__builtin_fabsf(x) <= 65536.0f), 0)) {
    sincosf(x, &sn, &cs);
    return;
  }
  const real q = __builtin_rintf(x * k2oPi);
  real r = __builtin_fmaf(-q, kPio2A, x);
  r = __builtin_fmaf(-q, kPio2B, r);
  r = __builtin_fmaf(-q, kPio2C, r);
  real s, c;
  sincos_poly(r, s, c);
  const real m = __builtin_fmaf(-4.f, __builtin_floorf(__builtin_fmaf(q, 0.25f, 0.25f)), q);
  const real A = 1.f - __builtin_fabsf(m), Bq = __builtin_fminf(m, 2.f - m);
  sn = __builtin_fmaf(s, A, c * Bq);
  cs = __builtin_fmaf(c, A, -(s * Bq));
#else
  m_sincos(x, &sn, &cs);
#endif
}
__device__ __forceinline__ void vsincos(f2 x, f2& s, f2& c) { pk_sincos(x, s, c); }
#endif
__device__ __forceinline__ bool vfinite(real x) { return finite(x); }
__device__ __forceinline__ bool vfinite(f2 x) { return finite(x.x) && finite(x.y); }

// relaxed inverse barrier B_alpha (core/barrier.py:36-59) as barrier_relaxed (dtmpc_device.hpp):
// 1 / max(z, eps) for z >= a; the quadratic extension below a (rare: a trajectory inside an
// obstacle's margin) is a divergent branch the wave skips when no lane needs it
__device__ __forceinline__ real bar_relaxed(const FP& p, real z) {
  DTMPC_NOCONTRACT
  const real diff = z - p.a;
  return (p.inv_a - diff / p.a2) + (diff * diff) / p.a3;
}
// 1 / max(z, eps) with max NaN-propagating (= the reference's torch.clamp_min then reciprocal)
__device__ __forceinline__ real vbarrier(const FP& p, real z) {
  DTMPC_NOCONTRACT
  real r = frcp(vmaxnan(z, p.eps));
  if (!(z >= p.a)) r = bar_relaxed(p, z);
  return r;
}
__device__ __forceinline__ f2 vbarrier(const FP& p, f2 z) {
  DTMPC_NOCONTRACT
  f2 r = f2{frcp(vmaxnan(z.x, p.eps)), frcp(vmaxnan(z.y, p.eps))};
  if (!(z.x >= p.a) || !(z.y >= p.a)) {
    if (!(z.x >= p.a)) r.x = bar_relaxed(p, z.x);
    if (!(z.y >= p.a)) r.y = bar_relaxed(p, z.y);
  }
  return r;
}
// _dB_relaxed_inv_dz core/systems/dubins_aug_jac.py:31-40 (dbarrier_relaxed)
// f64: without a divergent branch -- one IEEE division of a selected numerator and denominator, the same values bit
// for bit (-(1 / zc^2) = -1 / zc^2 exactly; the relaxed branch's (2 diff) / a3 - 1 / a^2 as written).  The branch
// form's if / else gave the register allocator a flow block that runs with the then-lanes' exec mask only, and it
// placed live-range-split copies of long-lived values there: the else-lanes never received them (ROCm 7.2, the
// round-5 "stale workspace" defect, profiles/r06/flow_copy_root_cause.txt; build.py flow_copies scans for it).
__device__ __forceinline__ real dbarrier(const FP& p, real z) {
#if DTMPC_FAST_F64
  DTMPC_NOCONTRACT
  const bool inv = z >= p.a;
  const real zc = z < p.eps ? p.eps : z;
  const real diff = z - p.a;
  const real q = (inv ? -1.0 : 2.0 * diff) / (inv ? zc * zc : p.a3);
  return inv ? q : -p.inv_a2 + q;
#else
  if (z >= p.a) {
    const real zc = z < p.eps ? p.eps : z;
    return -m_rcp(zc * zc);
  }
  const real diff = z - p.a;
  return -p.inv_a2 + (2.f * diff) / p.a3;
#endif
}

// smooth-min h (dubins_obstacles.py:41-69), two passes, the h_i of the first kept (h_smoothmin_w)
template <int M, class V>
__device__ __forceinline__ V h_sm(const FP& p, V px, V py) {
  DTMPC_NOCONTRACT
  constexpr int MO = Obs<M>::n;
  V hi[MO], hm;
#pragma unroll
  for (int i = 0; i < MO; ++i) {
    const V dx = px - ocx<M>(p, i);
    const V dy = py - ocy<M>(p, i);
    hi[i] = ffma(dx, dx, dy * dy) - or2<M>(p, i);
    hm = i == 0 ? hi[0] : vmin(hm, hi[i]);
  }
  const V zmax = p.neg_beta * hm;
  const V zl = zmax * real(1.44269504088896341);
  V se = 0.f;
#pragma unroll
  for (int i = 0; i < MO; ++i) se += smterm<M>(p, hi[i], zmax, zl);
  const V hv = p.neg_inv_beta * (zmax + vlog(se));
  return Obs<M>::tight ? hv - p.tight : hv;  // kTight: the tightened h the barrier sees
}

// h and grad h at one point (h_grad_fixed, grad_h_multi_circle_obstacles :72-92)
template <int M>
__device__ __forceinline__ real h_grad(const FP& p, real px, real py, real& gx, real& gy) {
#pragma clang fp contract(off)
  constexpr int MO = Obs<M>::n;
  // kLds (f64): the per-obstacle values are evaluated again in the sum pass instead of kept (bitwise the same)
  constexpr bool TWO = Obs<M>::lds;
  constexpr int MK = TWO ? 1 : MO;
  real z[MK], hh[MK], dxs[MK], dys[MK], zmax = 0.f;
#pragma unroll
  for (int i = 0; i < MO; ++i) {
    const real dx = px - ocx<M>(p, i);
    const real dy = py - ocy<M>(p, i);
    const real h = dx * dx + dy * dy - or2<M>(p, i);
    const real zi = p.neg_beta * h;
    if (!TWO) {
      dxs[i] = dx;
      dys[i] = dy;
      hh[i] = h;
      z[i] = zi;
    }
    zmax = (i == 0 || zi > zmax) ? zi : zmax;
  }
#if !DTMPC_FAST_F64
  const real zl = zmax * real(1.44269504088896341);
#endif
  real se = 0.f, sx = 0.f, sy = 0.f;
#pragma unroll
  for (int i = 0; i < MO; ++i) {
    real dx, dy, zi;
    if (TWO) {
      dx = px - ocx<M>(p, i);
      dy = py - ocy<M>(p, i);
      zi = p.neg_beta * (dx * dx + dy * dy - or2<M>(p, i));
    } else {
      dx = dxs[i];
      dy = dys[i];
      zi = z[i];
    }
#if DTMPC_FAST_F64
    // the generic kernel's h_grad (dtmpc_device.hpp), with the smooth-min's rule for negligible terms (smterm)
    const real x = zi - zmax;
    real e = 0.0;
    if (__builtin_amdgcn_ballot_w64(smneed(x))) e = smexp<M>(x);
#else
    (void)zi;
    const real e = __builtin_amdgcn_exp2f(__builtin_fmaf(hh[TWO ? 0 : i], p.nbl2e, -zl));
#endif
    se += e;
    sx += e * (2.f * dx);  // = 2 (px - cx_i), the first loop's difference
    sy += e * (2.f * dy);
  }
  const real inv = frcp(se);
  gx = sx * inv;
  gy = sy * inv;
  // untightened also under kTight: the reference linearises the nominal with dubins_augmented_jacobian of
  // the plain h (core/tube_mpc.py:315-320) while its dynamics see h - s (:273-276); dtmpc_solver.hpp alike
#if DTMPC_FAST_F64 && DTMPC_FAST64_HGLOG
  return p.neg_inv_beta * (zmax + vlog(se));  // the line search's log (fdlibm, < 1 ulp) instead of OCML's
#else
  return p.neg_inv_beta * (zmax + m_log(se));
#endif
}

// DBaS-augmented Dubins step (fhat_vec): x' = dubins_step(x, u) (core/systems/dubins.py:26-45),
// b' = B(h(x')) - gamma (B(h(x)) - b) (core/barrier.py:75-108); Bc carries B(h(x))
// G0 (gamma = 0): b' = B(h(x')) -- the general form adds (-0) * (B(h(x)) - b), which changes nothing
// for finite values
// the Dubins part alone (fhat's first half, operation for operation)
template <class V>
__device__ __forceinline__ void dubins(const FP& p, V& x0, V& x1, V& x2, V u0, V u1) {
  DTMPC_NOCONTRACT
  V sn, cs;
  vsincos(x2, sn, cs);
  const V dv = p.dt * u0;
  x0 = ffma(dv, cs, x0);
  x1 = ffma(dv, sn, x1);
  x2 = ffma(V(p.dt), u1, x2);
}
template <int M, bool G0 = false, class V>
__device__ __forceinline__ void fhat(const FP& p, V& x0, V& x1, V& x2, V& b, V u0, V u1, V& Bc) {
  DTMPC_NOCONTRACT
  dubins(p, x0, x1, x2, u0, u1);
  const V Bn = vbarrier(p, h_sm<M>(p, x0, x1));
  b = G0 ? Bn : ffma(V(-p.gamma), Bc - b, Bn);
  Bc = Bn;
}

template <int M>
__device__ __forceinline__ real barrier_at(const FP& p, real px, real py) {
  return vbarrier(p, h_sm<M>(p, px, py));
}

// _wrap_angle (run_nominal.py:32-34): atan2(sin e, cos e) maps e to (-pi, pi].  The fused solver evaluates that
// map directly, e - 2 pi rint(e / 2 pi) with 2 pi in two parts (the first product exact in the fma): < 1 ulp
// from the exact wrap, where the reference's sin -> cos -> atan2 chain carries 2-3 ulp of its own, in 5
// instructions instead of OCML's sin, cos and atan2 (~7 of them per step and iteration in the receding
// solver).  The generic kernels keep atan2(sin, cos) (wrap_angle, dtmpc_device.hpp).  The one point where the
// two maps part is e = +-pi itself (the reference's sign there is that of the rounded sin(pi)); the costs
// square the wrapped error, so only a derivative at that exact point sees it.
#if DTMPC_FAST_F64
constexpr double k2PiA = 6.283185307179586, k2PiB = 2.4492935982947064e-16, k1o2Pi = 0.15915494309189535;
#else
constexpr float k2PiA = 6.28318548f, k2PiB = -1.74845553e-7f, k1o2Pi = 0.159154937f;
#endif
__device__ __forceinline__ real vrint(real x) {
#if DTMPC_FAST_F64
  return __builtin_rint(x);
#else
  return __builtin_rintf(x);
#endif
}
__device__ __forceinline__ real vwrap(real e) {
  DTMPC_NOCONTRACT
  const real k = vrint(e * k1o2Pi);
  return __builtin_elementwise_fma(-k, real(k2PiB), __builtin_elementwise_fma(-k, real(k2PiA), e));
}
__device__ __forceinline__ f2 vwrap(f2 e) {
  DTMPC_NOCONTRACT
  const f2 k = f2{vrint(e.x * k1o2Pi), vrint(e.y * k1o2Pi)};
  return __builtin_elementwise_fma(-k, f2(k2PiB), __builtin_elementwise_fma(-k, f2(k2PiA), e));
}

// stage / terminal cost (stage_cost / term_cost, core/tube_mpc.py:823-842, 875-894): TRACK takes the
// references r (state) and q (control), the nominal its fixed target (WRAP: heading error wrapped,
// run_nominal.py:297-309)
template <bool TRACK, bool WRAP = false, class V>
__device__ __forceinline__ V stage(const FCost& c, V x0, V x1, V x2, V b, V u0, V u1, real r0, real r1, real r2,
                                   real q0, real q1) {
  DTMPC_NOCONTRACT
  V d0, d1, d2, e0, e1;
  if (TRACK) {
    d0 = x0 - r0;
    d1 = x1 - r1;
    d2 = x2 - r2;
    e0 = u0 - q0;
    e1 = u1 - q1;
  } else {
    d0 = x0 - c.tg.x;
    d1 = x1 - c.tg.y;
    d2 = x2 - c.tg.z;
    if (WRAP) d2 = vwrap(d2);
    e0 = u0;
    e1 = u1;
  }
  const V sq = ffma(c.Q2 * d2, d2, ffma(c.Q1 * d1, d1, (c.Q0 * d0) * d0));
  const V sr = ffma(c.R1 * e1, e1, (c.R0 * e0) * e0);
  return ffma(V(c.qb), b * b, sq + sr);
}
template <bool TRACK, bool WRAP = false, class V>
__device__ __forceinline__ V term(const FCost& c, V x0, V x1, V x2, V b, real r0, real r1, real r2) {
  DTMPC_NOCONTRACT
  V d0, d1, d2;
  if (TRACK) {
    d0 = x0 - r0;
    d1 = x1 - r1;
    d2 = x2 - r2;
  } else {
    d0 = x0 - c.tg.x;
    d1 = x1 - c.tg.y;
    d2 = x2 - c.tg.z;
    if (WRAP) d2 = vwrap(d2);
  }
  const V sq = ffma(c.Qf2 * d2, d2, ffma(c.Qf1 * d1, d1, (c.Qf0 * d0) * d0));
  return ffma(V(c.qb), b * b, sq);
}

// K_row . e of the feedback du = k + K (x - X_k) (core/ddp.py:267-268), as an fma chain: the
// reference's K @ dx is a BLAS/ATen matrix-vector product whose summation and fusion are its own; the
// line search and the commit use this same chain, so a committed tape is the candidate priced.
#ifndef DTMPC_FAST_KFMA
#define DTMPC_FAST_KFMA 1
#endif
template <bool G0, class V>
__device__ __forceinline__ V kdot(const f4& K, V e0, V e1, V e2, V e3) {
  V t = K.x * e0;
  t = __builtin_elementwise_fma(V(K.y), e1, t);
  t = __builtin_elementwise_fma(V(K.z), e2, t);
  return G0 ? t : __builtin_elementwise_fma(V(K.w), e3, t);  // G0: K.w = 0 (Gains)
}

// ---------------------------------------------------------------------------------------------
// the tapes one iLQR solve works on
// RROLL (TRACK): the references are an exact rollout of their controls from X_ref[0] by this kernel's own
// arithmetic -- the tube step's and the general path's ancillary solves, whose references are the nominal solve's
// tape -- so the f32 line search may re-roll them instead of reading them (LS_RECOMP).  The standalone iLQR takes
// any caller references (X_ref need not be a rollout of U_ref): RROLL = false, every reference row is read.
template <bool TRACK, bool G0, bool RG0, int P, int NCV = NC, bool RROLL = true>
struct Solve {
  static_assert(NCV == NC || (NCV == 4 && P != 4), "four lanes split six candidates");
  static constexpr bool rroll = RROLL;
  static constexpr bool g0 = G0;    // gamma = 0: the compact gain records (Gains)
  static constexpr bool ric0 = RG0; // gamma = 0: the Riccati step without the barrier state's zero column
  static constexpr int lanes = P;   // lanes per trajectory
  static constexpr int nc = NCV;    // rolled-out line-search candidates (6; the general path's 4 alphas: 4)
  Rsrc r;         // the workspace
  RA XA, UA;      // this solve's tape records (states + barrier state, controls); P = 4: the current slot
  RA XRA, URA;    // TRACK: the nominal plan's records
  Gains<P> G;
  Soa<4> X;       // ABI [N+1][4][B] tape (written at the end of the solve)
  Soa<2> U;       // ABI [N][2][B] controls (in: warm start, out: plan)
  __device__ __forceinline__ f4 x(int k) const { return rld4(r, XA, k, 0); }
  __device__ __forceinline__ f2 u(int k) const { return rld2(r, UA, k, 0); }
  __device__ __forceinline__ void stx(int k, f4 v) const { rst4(r, XA, k, 0, v); }
  __device__ __forceinline__ void stu(int k, f2 v) const { rst2(r, UA, k, 0, v); }
  __device__ __forceinline__ f4 xr(int k) const { return rld4(r, XRA, k, 0); }
  __device__ __forceinline__ f2 ur(int k) const { return rld2(r, URA, k, 0); }
};

struct StepIn {
  real X0, X1, X2, X3, V0, V1, r0, r1, r2, q0, q1;
  f4 Ka, Kb;
  f2 kk;
};

template <bool TRACK, bool LOADX = true, class SV, bool LOADR = true>
__device__ __forceinline__ void load_step(StepIn& L, const SV& S, int k) {
  if (LOADX) {
    const f4 X = S.x(k);
    L.X0 = X.x;
    L.X1 = X.y;
    L.X2 = X.z;
    L.X3 = X.w;
  } else {
    L.X0 = L.X1 = L.X2 = L.X3 = 0.f;
  }
  const f2 V = S.u(k);
  L.V0 = V.x;
  L.V1 = V.y;
  S.G.template load<SV::g0>(S.r, k, L.Ka, L.Kb, L.kk);
  if (TRACK) {
    if (LOADR) {
      const f4 R = S.xr(k);
      L.r0 = R.x;
      L.r1 = R.y;
      L.r2 = R.z;
    } else {
      L.r0 = L.r1 = L.r2 = 0.f;
    }
    const f2 Q = S.ur(k);
    L.q0 = Q.x;
    L.q1 = Q.y;
  } else {
    L.r0 = L.r1 = L.r2 = L.q0 = L.q1 = 0.f;
  }
}

// the solved tape out to the ABI SoA arrays, once per solve: X as solved, U as the next step's warm
// start -- the tube step's shift V <- [V[1:], V[-1]] (core/tube_mpc.py:1015-1020) applied on the way
// out (the step's plant and log read the plan's first controls from the records)
// Rows are read two ahead of their stores (a load waited for right before its own stores would leave
// one memory latency per row exposed).
// SHIFT = false (the standalone solve, dtmpc_ilqr_solve_ws): U out as solved.
template <bool SHIFT = true>
__device__ __forceinline__ void copy_out(int N, const Rsrc& r, const RA& XA, const RA& UA, const Soa<4>& X,
                                         const Soa<2>& U) {
  const int N1 = N - 1;
  auto iu = [&](int j) { return uidx(j < N1 ? j : N1); };
  auto ix = [&](int j) { return uidx(j < N ? j : N); };
  f4 xq[3];
  f2 uq[3];
  xq[0] = rld4(r, XA, 0, 0);
  uq[0] = rld2(r, UA, 0, 0);
  xq[1] = rld4(r, XA, ix(1), 0);
  uq[1] = rld2(r, UA, iu(1), 0);
  for (int k = 0; k <= N; k += 3) {
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int kk = k + j;
      xq[(j + 2) % 3] = rld4(r, XA, ix(kk + 2), 0);
      uq[(j + 2) % 3] = rld2(r, UA, iu(kk + 2), 0);
      if (kk > N) break;
      const f4 x = xq[j];
      X.st(kk, 0, x.x);
      X.st(kk, 1, x.y);
      X.st(kk, 2, x.z);
      X.st(kk, 3, x.w);
      if (kk < N) {
        const f2 u = uq[j];
        if (!SHIFT) {
          U.st(kk, 0, u.x);
          U.st(kk, 1, u.y);
        } else {
          if (kk > 0) {
            U.st(kk - 1, 0, u.x);
            U.st(kk - 1, 1, u.y);
          }
          if (kk == N1) {
            U.st(kk, 0, u.x);
            U.st(kk, 1, u.y);
          }
        }
      }
    }
  }
}

// iLQR start (init_tape): V = clamp(V_init) (the warm start, ABI SoA), X = rollout(x0, V) into this
// solve's records, and the alpha = 0 candidate's cost
template <bool TRACK, int M, class SV>
__device__ __forceinline__ real init_tape(const FP& p, const FCost& c, const real* x0, const SV& S,
                                           bool want_cost) {
  DTMPC_NOCONTRACT
  const int N = p.N;
  real s0 = x0[0], s1 = x0[1], s2 = x0[2], sb = x0[3];
  real Bc = barrier_at<M>(p, x0[0], x0[1]);
  S.stx(0, f4{s0, s1, s2, sb});
  real J = 0.f;
  real n0 = S.U.ld(0, 0), n1 = S.U.ld(0, 1);
  f4 nR = f4{0.f, 0.f, 0.f, 0.f};
  f2 nQ = f2{0.f, 0.f};
  if (TRACK) {
    nR = S.xr(0);
    nQ = S.ur(0);
  }
  for (int k = 0; k < N; ++k) {
    const real v0 = n0, v1 = n1;
    const f4 R = nR;
    const f2 Q = nQ;
    if (k + 1 < N) {
      n0 = S.U.ld(k + 1, 0);
      n1 = S.U.ld(k + 1, 1);
      if (TRACK) {
        nR = S.xr(k + 1);
        nQ = S.ur(k + 1);
      }
    }
    const real u0 = vclamp(v0, p.umin0, p.umax0), u1 = vclamp(v1, p.umin1, p.umax1);
    S.stu(k, f2{u0, u1});
    if (want_cost) J = J + stage<TRACK, Obs<M>::wrap>(c, s0, s1, s2, sb, u0, u1, R.x, R.y, R.z, Q.x, Q.y);
    fhat<M, SV::g0>(p, s0, s1, s2, sb, u0, u1, Bc);
    S.stx(k + 1, f4{s0, s1, s2, sb});
  }
  if (!want_cost) return 0.f;
  f4 R = f4{0.f, 0.f, 0.f, 0.f};
  if (TRACK) R = S.xr(N);
  return J + term<TRACK, Obs<M>::wrap>(c, s0, s1, s2, sb, R.x, R.y, R.z);
}

// DTMPC_FAST_RIC_FMA = 1 (round 6): the backward step -- this Jacobian and the Riccati step (riccati_pk) -- compiled
// without implicit contraction, its multiply-adds as explicit fmas at fixed places (rfm / fma2): every rounding of the
// recursion is written in the source, so the lane forms, the record forms and every code placement get the same bits
// (with implicit contraction the compiler re-rounded it per call site: DESIGN.md section 3 "Four lanes").
#ifndef DTMPC_FAST_RIC_FMA
#define DTMPC_FAST_RIC_FMA 1
#endif
// a * b + c as one rounding (RIC_FMA) or two
__device__ __forceinline__ real rfm(real a, real b, real c) {
#if DTMPC_FAST_RIC_FMA
  return __builtin_elementwise_fma(a, b, c);  // the value type's own fma (__builtin_fma is the double one)
#else
  DTMPC_NOCONTRACT
  return a * b + c;
#endif
}
__device__ __forceinline__ f2 rfm2(f2 a, f2 b, f2 c) {
#if DTMPC_FAST_RIC_FMA
  return __builtin_elementwise_fma(a, b, c);
#else
  DTMPC_NOCONTRACT
  return a * b + c;
#endif
}
// (a0 b0 + a1 b1 + c) + a3 b3 in the reference's left-to-right order: the P A / S A row sums (and Q_x's) of the step
__device__ __forceinline__ real rdot3c(real a0, real b0, real a1, real b1, real c, real a3, real b3) {
  DTMPC_NOCONTRACT
  return rfm(a3, b3, rfm(a1, b1, a0 * b0) + c);
}
// sparse augmented Jacobian (make_jac, core/systems/dubins_aug_jac.py:61-139)
__device__ __forceinline__ Jac<real> jac(const FP& p, real sn, real cs, real v, real gxk, real gyk, real dBk,
                                          real gxn, real gyn, real dBn) {
#if DTMPC_FAST_RIC_FMA
  DTMPC_NOCONTRACT
#endif
  Jac<real> J;
  const real dt = p.dt;
  J.a02 = -dt * v * sn;
  J.a12 = dt * v * cs;
  J.b00 = dt * cs;
  J.b10 = dt * sn;
  J.b21 = dt;
  const real r0 = dBn * gxn, r1 = dBn * gyn, r2 = dBn * 0.f;
  const real gd = p.gamma * dBk;
#if DTMPC_FAST_RIC_FMA
  J.a30 = rfm(-gd, gxk, r0);
  J.a31 = rfm(-gd, gyk, r1);
  J.a32 = (rfm(r1, J.a12, r0 * J.a02) + r2) - gd * 0.f;
  J.g = p.gamma;
  J.b30 = rfm(r1, J.b10, r0 * J.b00);
#else
  J.a30 = r0 - gd * gxk;
  J.a31 = r1 - gd * gyk;
  J.a32 = (r0 * J.a02 + r1 * J.a12 + r2) - gd * 0.f;
  J.g = p.gamma;
  J.b30 = r0 * J.b00 + r1 * J.b10;
#endif
  J.b31 = r2 * dt;
  return J;
}

// iLQR backward step (core/ddp.py:213-254) on the sparse Jacobian with the 4 x 4 blocks held as rows of
// column PAIRS, so that most of the recursion issues as packed f32 (two columns per instruction):
// P = A^T V, Q_xx = P A, S = B^T V, Q_ux = S A row by row; the 2 x 2 LU solve (partial pivoting, as
// torch.linalg.solve) on pairs of right-hand-side columns; V_x and V_xx updates as fma chains.  The
// same products as riccati_step (the reference's dense update restricted to the nonzeros of A, B),
// contracted and grouped for pairs: V_xx' = Q_xx + K^T Q_uu K + K^T Q_ux + Q_xu K accumulated term by
// term in one fma chain per pair.
#ifndef DTMPC_FAST_RICPK
#define DTMPC_FAST_RICPK 1
#endif
struct RicP {
  f2 V[4][2];  // V_xx: row i, columns (0, 1) and (2, 3)
  f2 Vx[2];    // (V_x0, V_x1), (V_x2, V_x3)
};
__device__ __forceinline__ f2 fma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
__device__ __forceinline__ f2 bc(real v) { return f2{v, v}; }

// G0 (gamma = 0): A's column for the barrier state is exactly zero, so the recursion keeps V_xx's row /
// column 3 at (0, 0, 0, 2 q_b) and V_x[3] at l_x[3] = 2 q_b b (the terms it would add are products with
// exact zeros): row 3 of P, Q_xx and V_xx, the g * (.) products and B's zero entry b31 = dB(h') * 0 * dt
// are dropped (-31 instructions per step).  The same sums, but with the zero terms gone the compiler
// contracts two of them differently (l_u1 + b21 V_x2 and l_uu1 + s2 b21 become one fma each): an FMA
// rounding of the same recursion, checked against the oracle builds like the rest of the kernel.
template <bool G0>
__device__ __forceinline__ bool riccati_pk(const Jac<real>& J, const real* lx, const real* lu, const real* lxx,
                                           const real* luu, real reg, RicP& R, real* K, real* kff) {
#if DTMPC_FAST_RIC_FMA
  DTMPC_NOCONTRACT  // every rounding of the step is written below (rfm / fma2): the same bits at every call site
#endif
  const real a02 = J.a02, a12 = J.a12, a30 = J.a30, a31 = J.a31, a32 = J.a32, g = J.g;
  const real b00 = J.b00, b10 = J.b10, b21 = J.b21, b30 = J.b30, b31 = J.b31;
  const f2 A3 = f2{a30, a31};
  const real vx0 = R.Vx[0].x, vx1 = R.Vx[0].y, vx2 = R.Vx[1].x, vx3 = R.Vx[1].y;
  // G0: V_xx row 3 = (0, 0 | 0, 2 q_b)
  const f2 V30 = G0 ? f2{0.f, 0.f} : R.V[3][0];
  const f2 V31 = G0 ? f2{0.f, lxx[3]} : R.V[3][1];
  // Q_x = l_x + A^T V_x ; Q_u = l_u + B^T V_x
  const f2 Qx01 = f2{lx[0], lx[1]} + fma2(A3, bc(vx3), R.Vx[0]);
#if DTMPC_FAST_RIC_FMA
  const real Qx2 = lx[2] + rdot3c(a02, vx0, a12, vx1, vx2, a32, vx3);
  const real Qx3 = G0 ? lx[3] : rfm(g, vx3, lx[3]);
  const real Qu0 = lu[0] + rfm(b30, vx3, rfm(b10, vx1, b00 * vx0));
  const real Qu1 = G0 ? rfm(b21, vx2, lu[1]) : lu[1] + rfm(b31, vx3, b21 * vx2);
#else
  const real Qx2 = lx[2] + (a02 * vx0 + a12 * vx1 + vx2 + a32 * vx3);
  const real Qx3 = G0 ? lx[3] : lx[3] + g * vx3;
  const real Qu0 = lu[0] + (b00 * vx0 + b10 * vx1 + b30 * vx3);
  const real Qu1 = G0 ? lu[1] + b21 * vx2 : lu[1] + (b21 * vx2 + b31 * vx3);
#endif
  // P = A^T V_xx
  f2 P[4][2];
  if (G0) {
    P[0][0] = R.V[0][0];
    P[1][0] = R.V[1][0];
    P[2][0] = fma2(bc(a12), R.V[1][0], fma2(bc(a02), R.V[0][0], R.V[2][0]));
    P[0][1] = fma2(bc(a30), V31, R.V[0][1]);
    P[1][1] = fma2(bc(a31), V31, R.V[1][1]);
    P[2][1] = fma2(bc(a32), V31, fma2(bc(a12), R.V[1][1], fma2(bc(a02), R.V[0][1], R.V[2][1])));
  } else {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const f2 V3c = c ? V31 : V30;
      P[0][c] = fma2(bc(a30), V3c, R.V[0][c]);
      P[1][c] = fma2(bc(a31), V3c, R.V[1][c]);
      P[2][c] = fma2(bc(a32), V3c, fma2(bc(a12), R.V[1][c], fma2(bc(a02), R.V[0][c], R.V[2][c])));
      P[3][c] = bc(g) * V3c;
    }
  }
  // Q_xx = P A + l_xx
  constexpr int NR = G0 ? 3 : 4;  // G0: Q_xx row 3 = (0, 0, 0, 2 q_b)
  f2 Q[4][2];
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const real p0 = P[i][0].x, p1 = P[i][0].y, p2 = P[i][1].x, p3 = P[i][1].y;
    Q[i][0] = fma2(A3, bc(p3), P[i][0]);
#if DTMPC_FAST_RIC_FMA
    Q[i][1] = f2{rdot3c(a02, p0, a12, p1, p2, a32, p3), G0 ? 0.f : g * p3};
#else
    Q[i][1] = f2{a02 * p0 + a12 * p1 + p2 + a32 * p3, G0 ? 0.f : g * p3};
#endif
  }
  Q[0][0].x = lxx[0] + Q[0][0].x;
  Q[1][0].y = lxx[1] + Q[1][0].y;
  Q[2][1].x = lxx[2] + Q[2][1].x;
  if (G0) {
    Q[3][0] = f2{0.f, 0.f};
    Q[3][1] = f2{0.f, lxx[3]};
  } else {
    Q[3][1].y = lxx[3] + Q[3][1].y;
  }
  // S = B^T V_xx ; Q_ux = S A ; Q_uu = l_uu + S B
  f2 S[2][2];
  if (G0) {
    S[0][0] = fma2(bc(b10), R.V[1][0], bc(b00) * R.V[0][0]);
    S[0][1] = fma2(bc(b30), V31, fma2(bc(b10), R.V[1][1], bc(b00) * R.V[0][1]));
    S[1][0] = bc(b21) * R.V[2][0];
    S[1][1] = bc(b21) * R.V[2][1];
  } else {
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const f2 V3c = c ? V31 : V30;
      S[0][c] = fma2(bc(b30), V3c, fma2(bc(b10), R.V[1][c], bc(b00) * R.V[0][c]));
      S[1][c] = fma2(bc(b31), V3c, bc(b21) * R.V[2][c]);
    }
  }
  f2 Qux[2][2];
  real Quu[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const real s0 = S[a][0].x, s1 = S[a][0].y, s2 = S[a][1].x, s3 = S[a][1].y;
    Qux[a][0] = fma2(A3, bc(s3), S[a][0]);
#if DTMPC_FAST_RIC_FMA
    Qux[a][1] = f2{rdot3c(a02, s0, a12, s1, s2, a32, s3), G0 ? 0.f : g * s3};
    Quu[a][0] = rfm(s3, b30, rfm(s1, b10, s0 * b00));
    Quu[a][1] = G0 ? s2 * b21 : rfm(s3, b31, s2 * b21);
#else
    Qux[a][1] = f2{a02 * s0 + a12 * s1 + s2 + a32 * s3, G0 ? 0.f : g * s3};
    Quu[a][0] = s0 * b00 + s1 * b10 + s3 * b30;
    Quu[a][1] = G0 ? s2 * b21 : s2 * b21 + s3 * b31;
#endif
  }
  Quu[0][0] = luu[0] + Quu[0][0];
  Quu[1][1] = luu[1] + Quu[1][1];
  // gains with the regularised Q_uu (:239-249): LU with partial pivoting, K = -x, k = -x
#if DTMPC_FAST_RIC_FMA
  // lu2 (dtmpc_device.hpp) with its one multiply-add fused: u11 = a11 - l a01
  LU2<real> f;
  {
    const real m00 = Quu[0][0] + reg, m01 = Quu[0][1], m10 = Quu[1][0], m11 = Quu[1][1] + reg;
    f.sw = m_abs(m10) > m_abs(m00);
    const real a00 = f.sw ? m10 : m00, a01 = f.sw ? m11 : m01, a10 = f.sw ? m00 : m10, a11 = f.sw ? m01 : m11;
    f.inv00 = m_rcp(a00);
    f.l = a10 * f.inv00;
    f.inv11 = m_rcp(rfm(-f.l, a01, a11));
    f.a00 = a00;
    f.a01 = a01;
  }
#else
  const LU2<real> f = lu2(Quu[0][0] + reg, Quu[0][1], Quu[1][0], Quu[1][1] + reg);
#endif
  f2 Kp[2][2];  // K row a, columns (0, 1) and (2, 3)
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const f2 r0 = Qux[0][c], r1 = Qux[1][c];
    const f2 p0 = f2{f.sw ? r1.x : r0.x, f.sw ? r1.y : r0.y}, p1 = f2{f.sw ? r0.x : r1.x, f.sw ? r0.y : r1.y};
#if DTMPC_FAST_RIC_FMA
    Kp[1][c] = rfm2(bc(-f.l), p0, p1) * bc(-f.inv11);
    Kp[0][c] = rfm2(bc(f.a01), Kp[1][c], p0) * bc(-f.inv00);
#else
    const f2 y1 = p1 - bc(f.l) * p0;
    Kp[1][c] = y1 * bc(-f.inv11);
    Kp[0][c] = (p0 + bc(f.a01) * Kp[1][c]) * bc(-f.inv00);
#endif
  }
  {
    const real p0 = f.sw ? Qu1 : Qu0, p1 = f.sw ? Qu0 : Qu1;
#if DTMPC_FAST_RIC_FMA
    kff[1] = rfm(-f.l, p0, p1) * -f.inv11;
    kff[0] = rfm(f.a01, kff[1], p0) * -f.inv00;
#else
    const real y1 = p1 - f.l * p0;
    kff[1] = y1 * -f.inv11;
    kff[0] = (p0 + f.a01 * kff[1]) * -f.inv00;
#endif
  }
  K[0] = Kp[0][0].x;
  K[1] = Kp[0][0].y;
  K[2] = Kp[0][1].x;
  K[3] = Kp[0][1].y;
  K[4] = Kp[1][0].x;
  K[5] = Kp[1][0].y;
  K[6] = Kp[1][1].x;
  K[7] = Kp[1][1].y;
  const bool ok = finite10(K, kff);
  // KQ = K^T Q_uu (unregularised, :251-252), pairs over i: KQa[c] = (KQ[2c][a], KQ[2c+1][a])
  f2 KQ0[2], KQ1[2];
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    KQ0[c] = fma2(bc(Quu[1][0]), Kp[1][c], bc(Quu[0][0]) * Kp[0][c]);
    KQ1[c] = fma2(bc(Quu[1][1]), Kp[1][c], bc(Quu[0][1]) * Kp[0][c]);
  }
  // V_x = Q_x + K^T Q_uu k + K^T Q_u + Q_xu k
  const f2 Qxp[2] = {Qx01, f2{Qx2, Qx3}};
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const f2 t1 = fma2(KQ1[c], bc(kff[1]), KQ0[c] * bc(kff[0]));
    const f2 t2 = fma2(Kp[1][c], bc(Qu1), Kp[0][c] * bc(Qu0));
    const f2 t3 = fma2(Qux[1][c], bc(kff[1]), Qux[0][c] * bc(kff[0]));
    R.Vx[c] = ((Qxp[c] + t1) + t2) + t3;
  }
  if (G0) R.Vx[1].y = Qx3;  // V_x[3] = l_x[3]: its K-terms are products with K's zero column
  // V_xx = Q_xx + K^T Q_uu K + K^T Q_ux + Q_xu K: row i, column pair c, one fma chain
#pragma unroll
  for (int i = 0; i < NR; ++i) {
    const int ci = i >> 1;
    const real kq0 = (i & 1) ? KQ0[ci].y : KQ0[ci].x, kq1 = (i & 1) ? KQ1[ci].y : KQ1[ci].x;
    const real k0i = (i & 1) ? Kp[0][ci].y : Kp[0][ci].x, k1i = (i & 1) ? Kp[1][ci].y : Kp[1][ci].x;
    const real q0i = (i & 1) ? Qux[0][ci].y : Qux[0][ci].x, q1i = (i & 1) ? Qux[1][ci].y : Qux[1][ci].x;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      f2 acc = fma2(bc(kq0), Kp[0][c], Q[i][c]);
      acc = fma2(bc(kq1), Kp[1][c], acc);
      acc = fma2(bc(k0i), Qux[0][c], acc);
      acc = fma2(bc(k1i), Qux[1][c], acc);
      acc = fma2(bc(q0i), Kp[0][c], acc);
      R.V[i][c] = fma2(bc(q1i), Kp[1][c], acc);
    }
  }
  return ok;
}

// one DPP move of a real (f64: both 32-bit halves with the same control)
template <int C>
__device__ __forceinline__ real dpp_mov(real v) {
#if DTMPC_FAST_F64
  typedef int i2v __attribute__((ext_vector_type(2)));
  const i2v w = __builtin_bit_cast(i2v, v);
  return __builtin_bit_cast(real, i2v{__builtin_amdgcn_mov_dpp(w.x, C, 0xF, 0xF, false),
                                      __builtin_amdgcn_mov_dpp(w.y, C, 0xF, 0xF, false)});
#else
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), C, 0xF, 0xF, false));
#endif
}

// broadcast of lane J of each group of P lanes (P = 2: quad_perm [J, J, J+2, J+2]; P = 4: [J, J, J, J]),
// one DPP move; j is a constant after unrolling
template <int P, int J>
__device__ __forceinline__ real gbc(real v) {
  constexpr int ctrl = P == 4 ? J * 0x55 : (J == 0 ? 0xA0 : 0xF5);
  return dpp_mov<ctrl>(v);
}
template <int P>
__device__ __forceinline__ real gbcast(real v, int j) {
  switch (j) {
    case 0: return gbc<P, 0>(v);
    case 1: return gbc<P, 1 % P>(v);
    case 2: return gbc<P, 2 % P>(v);
    default: return gbc<P, 3 % P>(v);
  }
}

// the per-point part of the linearisation: sin / cos of the heading, grad h and B'(h) at X
struct Lin {
  real sn, cs, gx, gy, dB;
};
template <int M>
__device__ __forceinline__ Lin lin_point(const FP& p, const f4& X) {
  Lin L;
  vsincos(X.z, L.sn, L.cs);
  L.dB = dbarrier(p, h_grad<M>(p, X.x, X.y, L.gx, L.gy));
  return L;
}

// backward pass (ilqr_backward, core/ddp.py:172-254).  P > 1: the per-point linearisation (sin / cos,
// grad h, B' -- about a third of a step) is computed for P steps at once, one step per lane of the
// trajectory, and handed to every lane by DPP broadcasts; the Riccati recursion itself is sequential
// and runs on every lane (each needs the gains).  Same operations on the same values as P = 1: the
// gains are bitwise those of the one-lane form.
// DTMPC_FAST_BW_BCAST (DESIGN.md section 3 "Small batches: the four-lane step's latency"): at P > 1 the step inputs
// come from the group's per-lane rows by DPP instead of being loaded one step ahead -- 2 (default since round 6): in the
// step itself, lane j of the group owning row k; 1: handed on one step ahead.  The same values; round 5 left both off
// because the compiler contracted the Riccati step differently in each form.  Since round 6 the step's rounding is
// written in the source (DTMPC_FAST_RIC_FMA), so every form gives the same bits (tests/test_gpu_lanes.py) and the
// in-step form is taken for its latency: B = 4,096 tube step 1.94 -> 1.85 ms, config-2 DDP 0.656 -> 0.630 ms,
// f64 B = 8,192 4.65 -> 4.29 ms (profiles/r06/ab_ric.txt).
#ifndef DTMPC_FAST_BW_BCAST
#define DTMPC_FAST_BW_BCAST 2
#endif
template <bool TRACK, int M, class SV>
__device__ __forceinline__ bool backward(const FP& p, const FCost& c, real reg, const SV& S, int h) {
  constexpr int P = SV::lanes;
  const int N = p.N;
  const real lxx[4] = {2.f * c.Q0, 2.f * c.Q1, 2.f * c.Q2, 2.f * c.qb};
  const real luu[2] = {2.f * c.R0, 2.f * c.R1};
  const real pxx[4] = {2.f * c.Qf0, 2.f * c.Qf1, 2.f * c.Qf2, 2.f * c.qb};
  const f4 XN = S.x(N);
  const real xn0 = XN.x, xn1 = XN.y, xn2 = XN.z, xnb = XN.w;
  real d0, d1, d2;
  if (TRACK) {
    const f4 RN = S.xr(N);
    d0 = xn0 - RN.x;
    d1 = xn1 - RN.y;
    d2 = xn2 - RN.z;
  } else {
    d0 = xn0 - c.tg.x;
    d1 = xn1 - c.tg.y;
    // WRAP: phi_x against the wrapped target x - wrap(x - t) (run_nominal.py:318-324, deriv_dx)
    d2 = Obs<M>::wrap ? xn2 - (xn2 - vwrap(xn2 - c.tg.z)) : xn2 - c.tg.z;
  }
#if DTMPC_FAST_RICPK
  RicP R;
  R.V[0][0] = f2{pxx[0], 0.f};
  R.V[0][1] = f2{0.f, 0.f};
  R.V[1][0] = f2{0.f, pxx[1]};
  R.V[1][1] = f2{0.f, 0.f};
  R.V[2][0] = f2{0.f, 0.f};
  R.V[2][1] = f2{pxx[2], 0.f};
  R.V[3][0] = f2{0.f, 0.f};
  R.V[3][1] = f2{0.f, pxx[3]};
  R.Vx[0] = f2{pxx[0] * d0, pxx[1] * d1};
  R.Vx[1] = f2{pxx[2] * d2, pxx[3] * xnb};
#define RVX(i) ((i) == 0 ? R.Vx[0].x : (i) == 1 ? R.Vx[0].y : (i) == 2 ? R.Vx[1].x : R.Vx[1].y)
#else
  Riccati<real> R;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) R.Vxx[i][j] = i == j ? pxx[i] : 0.f;
  R.Vx[0] = pxx[0] * d0;
  R.Vx[1] = pxx[1] * d1;
  R.Vx[2] = pxx[2] * d2;
  R.Vx[3] = pxx[3] * xnb;
#define RVX(i) (R.Vx[i])
#endif
  real gxn, gyn;
  real dBn = dbarrier(p, h_grad<M>(p, xn0, xn1, gxn, gyn));
  bool ok = finite(RVX(0)) && finite(RVX(1)) && finite(RVX(2)) && finite(RVX(3));
  // step inputs one step ahead (P > 1 with BW_BCAST 1: after the first, from the group's per-lane rows; 2: none, every
  // step takes its inputs from the group's rows by broadcast)
  constexpr bool BCI = P > 1 && DTMPC_FAST_BW_BCAST == 2;
  f4 nX = BCI ? f4{0.f, 0.f, 0.f, 0.f} : S.x(N - 1), nR = f4{0.f, 0.f, 0.f, 0.f};
  f2 nV = BCI ? f2{0.f, 0.f} : S.u(N - 1), nQ = f2{0.f, 0.f};
  if (TRACK && !BCI) {
    nR = S.xr(N - 1);
    nQ = S.ur(N - 1);
  }
  auto step = [&](const f4& X, const f2& V, const f4& Rr, const f2& Q, int k, const Lin& Lk) {
    const real x0 = X.x, x1 = X.y, x2 = X.z, xb = X.w, u0 = V.x, u1 = V.y;
    const Jac<real> J = jac(p, Lk.sn, Lk.cs, u0, Lk.gx, Lk.gy, Lk.dB, gxn, gyn, dBn);
    if (TRACK) {
      d0 = x0 - Rr.x;
      d1 = x1 - Rr.y;
      d2 = x2 - Rr.z;
    } else {
      d0 = x0 - c.tg.x;
      d1 = x1 - c.tg.y;
      d2 = Obs<M>::wrap ? x2 - (x2 - vwrap(x2 - c.tg.z)) : x2 - c.tg.z;  // run_nominal.py:311-317
    }
    const real lx[4] = {lxx[0] * d0, lxx[1] * d1, lxx[2] * d2, lxx[3] * xb};
    real lu[2];
    if (TRACK) {
      lu[0] = luu[0] * (u0 - Q.x);
      lu[1] = luu[1] * (u1 - Q.y);
    } else {
      lu[0] = luu[0] * u0;
      lu[1] = luu[1] * u1;
    }
    real Kk[8], kk[2];
#if DTMPC_FAST_RICPK
    ok = riccati_pk<SV::ric0>(J, lx, lu, lxx, luu, reg, R, Kk, kk) && ok;
#else
    ok = riccati_step(J, lx, lu, lxx, luu, reg, R, Kk, kk) && ok;
#endif
#ifdef DTMPC_FAST_DIAG_LANES
    // diagnostics builds: the lanes of a trajectory must hold the same gains (they store the same record)
    if (P > 1) {
      int bad = -1;
      real mine = 0, ref = 0;
#pragma unroll
      for (int j = 0; j < 10; ++j) {
        const real v = j < 8 ? Kk[j] : kk[j - 8];
        const real r0 = gbc<P, 0>(v);
        if (__builtin_bit_cast(unsigned long long, (double)v) != __builtin_bit_cast(unsigned long long, (double)r0)) {
          bad = j;
          mine = v;
          ref = r0;
        }
      }
      const real in[9] = {X.x, X.y, X.z, X.w, V.x, V.y, Lk.sn, Lk.gx, Lk.dB};
      int badin = -1;
#pragma unroll
      for (int j = 0; j < 9; ++j)
        if (__builtin_bit_cast(unsigned long long, (double)in[j]) !=
            __builtin_bit_cast(unsigned long long, (double)gbc<P, 0>(in[j])))
          badin = j;
      if (bad >= 0 || badin >= 0)
        printf("DIAG lanes blk=%d thr=%d h=%d k=%d gain=%d mine=%.17g lane0=%.17g input=%d\n", (int)blockIdx.x,
               (int)threadIdx.x, h, k, bad, (double)mine, (double)ref, badin);
    }
#endif
    S.G.template store<SV::g0>(S.r, k, Kk, kk);
    gxn = Lk.gx;
    gyn = Lk.gy;
    dBn = Lk.dB;
  };
  auto next_inputs = [&](int k) {  // the inputs of step k - 1
    if (k > 0) {
      nX = S.x(k - 1);
      nV = S.u(k - 1);
      if (TRACK) {
        nR = S.xr(k - 1);
        nQ = S.ur(k - 1);
      }
    }
  };
  if (P == 1) {
    for (int k = N - 1; k >= 0; --k) {
      const f4 X = nX, Rr = nR;
      const f2 V = nV, Q = nQ;
      next_inputs(k);
      step(X, V, Rr, Q, k, lin_point<M>(p, X));
    }
  } else {
    // lane h of the trajectory linearises row kt - h of each group of P steps kt, kt - 1, ...; the
    // group's rows are read one group ahead (per-lane row: the group's lowest row as the uniform base)
    auto prow = [&](int kt) {
      const int rb = kt - (P - 1) > 0 ? kt - (P - 1) : 0;
      const int r = kt - h > 0 ? kt - h : 0;
      return rld4(S.r, S.XA, uidx(rb), (unsigned)(r - rb) * S.XA.rs);
    };
    // BW_BCAST: the step inputs too -- lane h reads the controls (and the ancillary's reference rows) of row kt - h
    // one group ahead, and every step takes row k's values from lane kt - k by the same DPP broadcasts instead of
    // reading them one step ahead (a group of P steps of load latency covered instead of one)
    auto prow2 = [&](const RA& A, int kt) {
      const int rb = kt - (P - 1) > 0 ? kt - (P - 1) : 0;
      const int r = kt - h > 0 ? kt - h : 0;
      return rld2(S.r, A, uidx(rb), (unsigned)(r - rb) * A.rs);
    };
    auto prow4 = [&](const RA& A, int kt) {
      const int rb = kt - (P - 1) > 0 ? kt - (P - 1) : 0;
      const int r = kt - h > 0 ? kt - h : 0;
      return rld4(S.r, A, uidx(rb), (unsigned)(r - rb) * A.rs);
    };
    constexpr bool BC = DTMPC_FAST_BW_BCAST != 0;
    f4 PX = prow(N - 1), PR = f4{0.f, 0.f, 0.f, 0.f};
    f2 PV = f2{0.f, 0.f}, PQ = f2{0.f, 0.f};
    if (BC) {
      PV = prow2(S.UA, N - 1);
      if (TRACK) {
        PR = prow4(S.XRA, N - 1);
        PQ = prow2(S.URA, N - 1);
      }
    }
    for (int kt = N - 1; kt >= 0; kt -= P) {
      const f4 PXc = PX, PRc = PR;
      const f2 PVc = PV, PQc = PQ;
      if (kt - P >= 0) {
        PX = prow(kt - P);
        if (BC) {
          PV = prow2(S.UA, kt - P);
          if (TRACK) {
            PR = prow4(S.XRA, kt - P);
            PQ = prow2(S.URA, kt - P);
          }
        }
      }
      const Lin Lh = lin_point<M>(p, PXc);
#pragma unroll
      for (int j = 0; j < P; ++j) {
        const int k = kt - j;
        if (k < 0) break;
        f4 X = nX, Rr = nR;
        f2 V = nV, Q = nQ;
        if (BCI) {
          // BW_BCAST 2 (in-step): step k's inputs from lane j of this group (row kt - j = k), broadcast in the step
          X = f4{gbcast<P>(PXc.x, j), gbcast<P>(PXc.y, j), gbcast<P>(PXc.z, j), gbcast<P>(PXc.w, j)};
          V = f2{gbcast<P>(PVc.x, j), gbcast<P>(PVc.y, j)};
          if (TRACK) {
            Rr = f4{gbcast<P>(PRc.x, j), gbcast<P>(PRc.y, j), gbcast<P>(PRc.z, j), 0.f};
            Q = f2{gbcast<P>(PQc.x, j), gbcast<P>(PQc.y, j)};
          }
        } else if (BC) {
          // the inputs of step k - 1, handed on to the next step as next_inputs hands on its loads (the step
          // itself then reads loop-carried values in both forms): row k - 1 from lane j + 1 of this group, or from
          // lane 0 of the next group's rows
          if (k > 0) {
            const int jn = j + 1 < P ? j + 1 : 0;
            const f4 XS = j + 1 < P ? PXc : PX, RS = j + 1 < P ? PRc : PR;
            const f2 VS = j + 1 < P ? PVc : PV, QS = j + 1 < P ? PQc : PQ;
            nX = f4{gbcast<P>(XS.x, jn), gbcast<P>(XS.y, jn), gbcast<P>(XS.z, jn), gbcast<P>(XS.w, jn)};
            nV = f2{gbcast<P>(VS.x, jn), gbcast<P>(VS.y, jn)};
            if (TRACK) {
              nR = f4{gbcast<P>(RS.x, jn), gbcast<P>(RS.y, jn), gbcast<P>(RS.z, jn), 0.f};
              nQ = f2{gbcast<P>(QS.x, jn), gbcast<P>(QS.y, jn)};
            }
          }
        } else {
          next_inputs(k);
        }
        Lin Lk;
        Lk.sn = gbcast<P>(Lh.sn, j);
        Lk.cs = gbcast<P>(Lh.cs, j);
        Lk.gx = gbcast<P>(Lh.gx, j);
        Lk.gy = gbcast<P>(Lh.gy, j);
        Lk.dB = gbcast<P>(Lh.dB, j);
        step(X, V, Rr, Q, k, Lk);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) ok = ok && finite(RVX(i));
#undef RVX
  return ok;
}

// ---------------------------------------------------------------------------------------------
// line search (core/ddp.py:256-301) over this lane's NL candidates, held as NPR two-wide pairs (an odd
// NL repeats its last candidate in the second slot of the last pair: a packed op costs one issue slot
// for one element or two).  One step of the rollout is written operation by operation ACROSS the
// pairs, so the instruction stream interleaves NPR independent chains: no dependent pair of packed
// ops / compare-select sits back to back (each such pair costs an s_nop wait state on gfx950).
// Arithmetic per candidate is the scalar forward pass (fhat, stage) operation for operation.
#ifndef DTMPC_FAST_LS_DEPTH2
// two steps of prefetch lead (f32, one lane per trajectory: measured -1.5 %).  f64: one -- the four step
// buffers of 21 doubles would not fit beside the candidates (at one lane: 380 scratch spill / reload
// instructions in the kernel, 23 with two buffers)
#define DTMPC_FAST_LS_DEPTH2 (DTMPC_FAST_F64 ? 0 : 1)
#endif
#ifndef DTMPC_FAST_LS_RECOMP
// 1 (default): the line search re-rolls the tape's states (and the ancillary's reference states) from their
// controls at gamma = 0 in f32 instead of reading them: -16 (nominal) / -32 (ancillary) B of reads per step,
// bitwise the same tapes; same-box A/B (profiles/r04/ab_recompute.txt) time +-0, HBM traffic -15 %
#define DTMPC_FAST_LS_RECOMP 1
#endif
#ifndef DTMPC_FAST64_RECOMP
// f64: the same re-roll in the f64 line search and commit (the f64 step reads 43.1 GB per launch
// against 35.96 GB algorithmic because its passes read the tape states the f32 kernel re-rolls)
#define DTMPC_FAST64_RECOMP 0
#endif
template <int NPR>
struct Cand {
  f2 a0[NPR], a1[NPR], a2[NPR], ab[NPR], Bp[NPR], J[NPR], al[NPR];
};

#if !DTMPC_FAST_F64 && !defined(DTMPC_OCML_SINCOS)
// sin / cos of NPR pairs whose elements are all in [-65536, 65536] (no range test, no branch)
template <int NPR>
__device__ __forceinline__ void sincos_pairs_fast(const f2* x, f2* sn, f2* cs) {
    f2 qq[NPR], r[NPR], z[NPR], s[NPR], c[NPR];
#pragma unroll
    for (int q = 0; q < NPR; ++q) qq[q] = f2{__builtin_rintf(x[q].x * k2oPi), __builtin_rintf(x[q].y * k2oPi)};
#pragma unroll
    for (int q = 0; q < NPR; ++q) r[q] = __builtin_elementwise_fma(-qq[q], f2(kPio2A), x[q]);
#pragma unroll
    for (int q = 0; q < NPR; ++q) r[q] = __builtin_elementwise_fma(-qq[q], f2(kPio2B), r[q]);
#pragma unroll
    for (int q = 0; q < NPR; ++q) r[q] = __builtin_elementwise_fma(-qq[q], f2(kPio2C), r[q]);
#pragma unroll
    for (int q = 0; q < NPR; ++q) z[q] = r[q] * r[q];
#pragma unroll
    for (int q = 0; q < NPR; ++q) {
      f2 ps = __builtin_elementwise_fma(z[q], f2(kSinS3), f2(kSinS2));
      f2 pc = __builtin_elementwise_fma(z[q], f2(kCosK3), f2(kCosK2));
      ps = __builtin_elementwise_fma(z[q], ps, f2(kSinS1));
      pc = __builtin_elementwise_fma(z[q], pc, f2(kCosK1));
      s[q] = __builtin_elementwise_fma(r[q] * z[q], ps, r[q]);
      c[q] = __builtin_elementwise_fma(z[q] * z[q], pc, __builtin_elementwise_fma(f2(-0.5f), z[q], f2(1.0f)));
    }
#if DTMPC_FAST_SINCOS_AB
    f2 A[NPR], Bq[NPR];
#pragma unroll
    for (int q = 0; q < NPR; ++q) {
      const f2 t = __builtin_elementwise_fma(qq[q], f2(0.25f), f2(0.25f));
      const f2 m = __builtin_elementwise_fma(f2(-4.f), f2{__builtin_floorf(t.x), __builtin_floorf(t.y)}, qq[q]);
      A[q] = f2{1.f - __builtin_fabsf(m.x), 1.f - __builtin_fabsf(m.y)};
      const f2 w = f2(2.f) - m;
      Bq[q] = f2{__builtin_fminf(m.x, w.x), __builtin_fminf(m.y, w.y)};
    }
#pragma unroll
    for (int q = 0; q < NPR; ++q) {
      sn[q] = __builtin_elementwise_fma(s[q], A[q], c[q] * Bq[q]);
      cs[q] = __builtin_elementwise_fma(c[q], A[q], -(s[q] * Bq[q]));
    }
#else
#pragma unroll
    for (int q = 0; q < NPR; ++q) {
      const int j0 = (int)qq[q].x & 3, j1 = (int)qq[q].y & 3;
      const real so0 = (j0 & 1) ? c[q].x : s[q].x, co0 = (j0 & 1) ? s[q].x : c[q].x;
      const real so1 = (j1 & 1) ? c[q].y : s[q].y, co1 = (j1 & 1) ? s[q].y : c[q].y;
      sn[q] = f2{(j0 & 2) ? -so0 : so0, (j1 & 2) ? -so1 : so1};
      cs[q] = f2{((j0 + 1) & 2) ? -co0 : co0, ((j1 + 1) & 2) ? -co1 : co1};
    }
#endif
}
#endif
// sin / cos of NPR pairs (pk_sincos per pair); one range test for all of them
template <int NPR>
__device__ __forceinline__ void sincos_pairs(const f2* x, f2* sn, f2* cs) {
#if DTMPC_FAST_F64
#pragma unroll
  for (int q = 0; q < NPR; ++q) vsincos(x[q], sn[q], cs[q]);
}
#else
  real m = __builtin_fabsf(x[0].x);
#pragma unroll
  for (int q = 0; q < NPR; ++q) m = __builtin_fmaxf(m, __builtin_fmaxf(__builtin_fabsf(x[q].x), __builtin_fabsf(x[q].y)));
#ifndef DTMPC_OCML_SINCOS
  if (__builtin_expect(m <= 65536.0f, 1)) {
    sincos_pairs_fast<NPR>(x, sn, cs);
    return;
  }
#endif
#pragma unroll
  for (int q = 0; q < NPR; ++q) {  // some element out of range: each element as the scalar form
    real s0, c0, s1, c1;
    vsincos(x[q].x, s0, c0);
    vsincos(x[q].y, s1, c1);
    sn[q] = f2{s0, s1};
    cs[q] = f2{c0, c1};
  }
}
#endif

// B(h(x)) of NPR pairs of positions (the line search's DBaS barrier; relaxed inverse barrier of the smooth-min h)
template <int M, int NPR>
__device__ __forceinline__ void ls_bar(const FP& p, const f2* px, const f2* py, f2* Bn) {
  DTMPC_NOCONTRACT
  // smooth-min h over the M obstacles (h_sm), all pairs together.  TWO (kLds, f64): the h_i are not kept between
  // the min and the exp pass but evaluated again (the same operations, so bitwise the same values) -- at M = 8
  // the kept 8 x NPR pairs of doubles were what made the general-record kernels spill (build.py check_resources)
  constexpr int MO = Obs<M>::n;
  constexpr bool TWO = Obs<M>::lds;
  f2 hi[TWO ? 1 : MO][NPR], hm[NPR];
  auto hval = [&](int i, int q) {
    const f2 dx = px[q] - ocx<M>(p, i);
    const f2 dy = py[q] - ocy<M>(p, i);
    return ffma(dx, dx, dy * dy) - or2<M>(p, i);
  };
  (void)hval;  // f32 keeps the h_i (only the f64 exp pass below evaluates them again)
#pragma unroll
  for (int i = 0; i < MO; ++i) {
    const real cxi = ocx<M>(p, i), cyi = ocy<M>(p, i), r2i = or2<M>(p, i);  // one read per obstacle (kLds)
#pragma unroll
    for (int q = 0; q < NPR; ++q) {
      const f2 dx = px[q] - cxi;
      const f2 dy = py[q] - cyi;
      const f2 h = ffma(dx, dx, dy * dy) - r2i;
      if (!TWO) hi[i][q] = h;
      hm[q] = i == 0 ? h : vmin(hm[q], h);
    }
  }
  f2 zmax[NPR], zl[NPR], se[NPR], z[NPR];
#pragma unroll
  for (int q = 0; q < NPR; ++q) {
    zmax[q] = p.neg_beta * hm[q];
    zl[q] = zmax[q] * real(1.44269504088896341);
  }
#pragma unroll
  for (int i = 0; i < MO; ++i) {
#if DTMPC_FAST_F64
    // one wave-uniform branch per obstacle for all the lane's candidates (smterm)
    f2 x[NPR], e[NPR];
    bool need = false;
#pragma unroll
    for (int q = 0; q < NPR; ++q) {
      x[q] = smarg(p, TWO ? hval(i, q) : hi[TWO ? 0 : i][q], zmax[q]);
      need = need || smneed(x[q]);
      e[q] = f2(0.0);
    }
    if (__builtin_amdgcn_ballot_w64(need))
#pragma unroll
      for (int q = 0; q < NPR; ++q) e[q] = smexp<M>(x[q]);
#pragma unroll
    for (int q = 0; q < NPR; ++q) se[q] = i == 0 ? e[q] : se[q] + e[q];
#else
#pragma unroll
    for (int q = 0; q < NPR; ++q) {
      const f2 e = smterm<M>(p, hi[TWO ? 0 : i][q], zmax[q], zl[q]);
      se[q] = i == 0 ? e : se[q] + e;  // = 0 + e_0 + ...: e_0 >= 0, so 0 + e_0 == e_0 bitwise
    }
#endif
  }
#pragma unroll
  for (int q = 0; q < NPR; ++q) {
    z[q] = p.neg_inv_beta * (zmax[q] + vlog(se[q]));
    if (Obs<M>::tight) z[q] = z[q] - p.tight;
  }
  // relaxed inverse barrier: the reciprocal for every element, the quadratic branch (z < a) once
  // per step for whichever elements need it
  real zmin = z[0].x;
#pragma unroll
  for (int q = 0; q < NPR; ++q) {
    Bn[q] = f2{frcp(vmaxnan(z[q].x, p.eps)), frcp(vmaxnan(z[q].y, p.eps))};
    zmin = m_min(zmin, m_min(z[q].x, z[q].y));
  }
  if (!(zmin >= p.a)) {
#pragma unroll
    for (int q = 0; q < NPR; ++q) {
      if (!(z[q].x >= p.a)) Bn[q].x = bar_relaxed(p, z[q].x);
      if (!(z[q].y >= p.a)) Bn[q].y = bar_relaxed(p, z[q].y);
    }
  }
}

// one step of the NPR pairs' rollouts: feedback + clamp, stage cost, DBaS-augmented Dubins move
template <bool TRACK, int M, int NPR, bool G0>
__device__ __forceinline__ void ls_step(const FP& p, const FCost& c, const StepIn& s, Cand<NPR>& C, f2* u0, f2* u1) {
  DTMPC_NOCONTRACT
#pragma unroll
  for (int q = 0; q < NPR; ++q) {
    const f2 e0 = C.a0[q] - s.X0, e1 = C.a1[q] - s.X1, e2 = C.a2[q] - s.X2, e3 = C.ab[q] - s.X3;
#if DTMPC_FAST_KFMA
    const f2 du0 = s.kk.x + kdot<G0>(s.Ka, e0, e1, e2, e3);
    const f2 du1 = s.kk.y + kdot<G0>(s.Kb, e0, e1, e2, e3);
#else
    const f2 du0 = s.kk.x + (s.Ka.x * e0 + s.Ka.y * e1 + s.Ka.z * e2 + s.Ka.w * e3);
    const f2 du1 = s.kk.y + (s.Kb.x * e0 + s.Kb.y * e1 + s.Kb.z * e2 + s.Kb.w * e3);
#endif
    u0[q] = ffma(C.al[q], du0, f2(s.V0));
    u1[q] = ffma(C.al[q], du1, f2(s.V1));
  }
#pragma unroll
  for (int q = 0; q < NPR; ++q) {
    u0[q] = vclamp(u0[q], p.umin0, p.umax0);
    u1[q] = vclamp(u1[q], p.umin1, p.umax1);
  }
#pragma unroll
  for (int q = 0; q < NPR; ++q)
    C.J[q] = C.J[q] + stage<TRACK, Obs<M>::wrap>(c, C.a0[q], C.a1[q], C.a2[q], C.ab[q], u0[q], u1[q], s.r0, s.r1,
                                                  s.r2, s.q0, s.q1);
  f2 sn[NPR], cs[NPR];
  sincos_pairs<NPR>(C.a2, sn, cs);
#pragma unroll
  for (int q = 0; q < NPR; ++q) {
    const f2 dv = p.dt * u0[q];
    C.a0[q] = ffma(dv, cs[q], C.a0[q]);
    C.a1[q] = ffma(dv, sn[q], C.a1[q]);
    C.a2[q] = ffma(f2(p.dt), u1[q], C.a2[q]);
  }
  f2 Bn[NPR];
  ls_bar<M, NPR>(p, C.a0, C.a1, Bn);
#pragma unroll
  for (int q = 0; q < NPR; ++q) {
    if (G0) {  // b' = B(h(x')) (fhat<M, true>)
      C.ab[q] = Bn[q];
    } else {
      C.ab[q] = ffma(f2(-p.gamma), C.Bp[q] - C.ab[q], Bn[q]);
      C.Bp[q] = Bn[q];
    }
  }
}

// The same step software-pipelined (f32, gamma = 0, four lanes: one candidate pair per lane, i.e. one dependent
// chain per step).  At gamma = 0 the controls do not read b (K's b column is zero), so b_k = B(h(x_k)) -- which
// ls_step evaluates at the end of step k - 1, right after the move that produced x_k -- is evaluated here, in
// step k, beside the move x_k -> x_{k+1}: two independent chains in one basic block, so the smooth-min's exp /
// log / rcp latencies fill the move's sin / cos chain.  The out-of-range sin / cos case is redone after them
// (one uniform branch).  Step 0 takes b_0 from the start state (`first`).  The same operations on the same
// values as ls_step: bitwise the same candidates.  x_k comes back in xk* for the slot stores (row k = x_k, b_k).
#ifndef DTMPC_FAST_LS_PIPE
#define DTMPC_FAST_LS_PIPE 0  // A/B: bitwise the same tapes, same time (B = 4,096: 1.91 ms both ways), so off
#endif
#if !DTMPC_FAST_F64 && !defined(DTMPC_OCML_SINCOS)
template <bool TRACK, int M, int NPR>
__device__ __forceinline__ void ls_step_pipe(const FP& p, const FCost& c, const StepIn& s, Cand<NPR>& C, f2* u0,
                                             f2* u1, f2* xk0, f2* xk1, f2* xk2, bool first) {
  DTMPC_NOCONTRACT
  static_assert(DTMPC_FAST_KFMA, "the pipelined step is written for the fma feedback");
#pragma unroll
  for (int q = 0; q < NPR; ++q) {
    xk0[q] = C.a0[q];
    xk1[q] = C.a1[q];
    xk2[q] = C.a2[q];
    const f2 e0 = C.a0[q] - s.X0, e1 = C.a1[q] - s.X1, e2 = C.a2[q] - s.X2;
    const f2 du0 = s.kk.x + kdot<true>(s.Ka, e0, e1, e2, e2);
    const f2 du1 = s.kk.y + kdot<true>(s.Kb, e0, e1, e2, e2);
    u0[q] = ffma(C.al[q], du0, f2(s.V0));
    u1[q] = ffma(C.al[q], du1, f2(s.V1));
  }
#pragma unroll
  for (int q = 0; q < NPR; ++q) {
    u0[q] = vclamp(u0[q], p.umin0, p.umax0);
    u1[q] = vclamp(u1[q], p.umin1, p.umax1);
  }
  real m = __builtin_fabsf(xk2[0].x);
#pragma unroll
  for (int q = 0; q < NPR; ++q) m = __builtin_fmaxf(m, __builtin_fmaxf(__builtin_fabsf(xk2[q].x), __builtin_fabsf(xk2[q].y)));
  f2 sn[NPR], cs[NPR];
  sincos_pairs_fast<NPR>(xk2, sn, cs);
  auto move = [&]() {
#pragma unroll
    for (int q = 0; q < NPR; ++q) {
      const f2 dv = p.dt * u0[q];
      C.a0[q] = ffma(dv, cs[q], xk0[q]);
      C.a1[q] = ffma(dv, sn[q], xk1[q]);
      C.a2[q] = ffma(f2(p.dt), u1[q], xk2[q]);
    }
  };
  move();
  f2 Bn[NPR];
  ls_bar<M, NPR>(p, xk0, xk1, Bn);
#pragma unroll
  for (int q = 0; q < NPR; ++q) {
    const f2 bk = first ? C.ab[q] : Bn[q];
    C.J[q] = C.J[q] + stage<TRACK, Obs<M>::wrap>(c, xk0[q], xk1[q], xk2[q], bk, u0[q], u1[q], s.r0, s.r1, s.r2,
                                                  s.q0, s.q1);
    C.ab[q] = bk;
  }
  if (__builtin_expect(!(m <= 65536.0f), 0)) {
    sincos_pairs<NPR>(xk2, sn, cs);
    move();
  }
}
#endif

#ifndef DTMPC_FAST_LS_LEAD4
#define DTMPC_FAST_LS_LEAD4 4  // P = 4: step inputs in a ring of LEAD + 1 buffers refilled LEAD steps ahead (0: two buffers, as P = 1; B = 4,096: 2.13 ms at 0, 2.03 at 3, 2.01 at 4)
#endif
// P = 4: the candidate tapes.  Every lane writes the rollouts of its two candidates into their own
// slots of the solve's tape records (instead of the winner being re-rolled by a commit pass): slot
// bank * 6 + candidate, in the bank the current tape is not in; the winner's slot then becomes the
// current tape (Slots::cur).  X row 0 of a slot is x0, row k + 1 the state after control row k.
struct Slots {
  RA X0, X1, U0, U1;  // this lane's two candidate slots (X and U records)
};

// per-lane choice among the three candidate pairs of a trajectory (lanes 0, 1, 2; lane 3 repeats lane 2)
template <class T>
__device__ __forceinline__ T pick3(int h, T a, T b, T c) { return h == 0 ? a : h == 1 ? b : c; }

// the partner of this lane in a lane group at distance 1 (quad_perm [1, 0, 3, 2]) or 2 ([2, 3, 0, 1])
template <int D>
__device__ __forceinline__ real gswap(real v) {
  return dpp_mov<D == 1 ? 0xB1 : 0x4E>(v);
}
template <int D>
__device__ __forceinline__ int gswap(int v) { return __builtin_amdgcn_mov_dpp(v, D == 1 ? 0xB1 : 0x4E, 0xF, 0xF, false); }

// Returns the chosen original position (or -1 if any candidate or Jprev is non-finite), its cost
// and alpha, and (bc) the chosen rolled-out candidate (-1: the zero candidate, i.e. the current tape).
// P = 1: the six candidates as three pairs; P = 2: three per lane (two pairs, the last one doubled);
// P = 4: one pair per lane (lane 3 repeats lane 2's), each lane storing its pair's tapes (Slots).  The
// lanes of a trajectory combine their minima by DPP swaps.
template <bool TRACK, int M, int P, class SV>
__device__ __forceinline__ int line_search(const FP& p, const FCost& c, const FIlqr& cf, const real* x0, real Bc0,
                                           const SV& S, real Jprev, int h, real& bestJ, real& al_out, int& bc,
                                           const Slots& Z, real* crec, size_t cst) {
  DTMPC_NOCONTRACT
  constexpr int NL = P == 4 ? 2 : SV::nc / P;  // candidates of this lane
  constexpr int NPR = (NL + 1) / 2;        // pairs
  const int N = p.N;
  const int hc = P == 4 ? (h < 2 ? h : 2) : h;  // this lane's candidate group
  const int c0 = hc * NL;                        // its first candidate (index into cf.cal / cf.cpos)
  Cand<NPR> C;
#pragma unroll
  for (int q = 0; q < NPR; ++q) {
    C.a0[q] = x0[0];
    C.a1[q] = x0[1];
    C.a2[q] = x0[2];
    C.ab[q] = x0[3];
    C.Bp[q] = Bc0;
    C.J[q] = 0.f;
    const int i0 = 2 * q, i1 = 2 * q + 1 < NL ? 2 * q + 1 : NL - 1;
    if (P == 1)
      C.al[q] = f2{cf.cal[i0], cf.cal[i1]};
    else if (P == 2)
      C.al[q] = h ? f2{cf.cal[NL + i0], cf.cal[NL + i1]} : f2{cf.cal[i0], cf.cal[i1]};
    else
      C.al[q] = f2{pick3(hc, cf.cal[0], cf.cal[2], cf.cal[4]), pick3(hc, cf.cal[1], cf.cal[3], cf.cal[5])};
  }
#if !DTMPC_FAST_F64 && !defined(DTMPC_OCML_SINCOS)
  constexpr bool PIPE = DTMPC_FAST_LS_PIPE && SV::g0 && P == 4 && DTMPC_FAST_LS_LEAD4 > 0;
#else
  constexpr bool PIPE = false;
#endif
  if (P == 4 && !PIPE) {  // the candidates' row 0 (PIPE: stored by the first step, row k = (x_k, b_k))
    const f4 X0v = f4{x0[0], x0[1], x0[2], x0[3]};
    rst4(S.r, Z.X0, 0, 0, X0v);
    rst4(S.r, Z.X1, 0, 0, X0v);
  }
  // P = 4: the pair's controls of step k and states of step k + 1 into its slots
  auto keep = [&](int k, const f2* u0, const f2* u1) {
    if (P == 4) {
      rst2(S.r, Z.U0, k, 0, f2{u0[0].x, u1[0].x});
      rst2(S.r, Z.U1, k, 0, f2{u0[0].y, u1[0].y});
      rst4(S.r, Z.X0, k + 1, 0, f4{C.a0[0].x, C.a1[0].x, C.a2[0].x, C.ab[0].x});
      rst4(S.r, Z.X1, k + 1, 0, f4{C.a0[0].y, C.a1[0].y, C.a2[0].y, C.ab[0].y});
    }
  };
  f2 u0[NPR], u1[NPR];
  const int N1 = N - 1;
  if (P == 4 && DTMPC_FAST_LS_LEAD4 > 0) {
    constexpr int LEAD = DTMPC_FAST_LS_LEAD4 > 0 ? DTMPC_FAST_LS_LEAD4 : 1, R = LEAD + 1;
    auto ix = [&](int j) { return uidx(j < N1 ? j : N1); };
    StepIn Bf[R];
#pragma unroll
    for (int j = 0; j < LEAD; ++j) load_step<TRACK>(Bf[j], S, ix(j));
    for (int k = 0; k < N; k += R) {
#pragma unroll
      for (int j = 0; j < R; ++j) {
        load_step<TRACK>(Bf[(j + LEAD) % R], S, ix(k + j + LEAD));
        if (k + j >= N) break;
#if !DTMPC_FAST_F64 && !defined(DTMPC_OCML_SINCOS)
        if (PIPE) {
          f2 xk0[NPR], xk1[NPR], xk2[NPR];
          ls_step_pipe<TRACK, M, NPR>(p, c, Bf[j], C, u0, u1, xk0, xk1, xk2, k + j == 0);
          rst2(S.r, Z.U0, k + j, 0, f2{u0[0].x, u1[0].x});
          rst2(S.r, Z.U1, k + j, 0, f2{u0[0].y, u1[0].y});
          rst4(S.r, Z.X0, k + j, 0, f4{xk0[0].x, xk1[0].x, xk2[0].x, C.ab[0].x});
          rst4(S.r, Z.X1, k + j, 0, f4{xk0[0].y, xk1[0].y, xk2[0].y, C.ab[0].y});
          continue;
        }
#endif
        ls_step<TRACK, M, NPR, SV::g0>(p, c, Bf[j], C, u0, u1);
        keep(k + j, u0, u1);
      }
    }
#if !DTMPC_FAST_F64 && !defined(DTMPC_OCML_SINCOS)
    if (PIPE) {  // b_N of the final states (the terminal cost's) and the slots' row N
      f2 Bn[NPR];
      ls_bar<M, NPR>(p, C.a0, C.a1, Bn);
#pragma unroll
      for (int q = 0; q < NPR; ++q) C.ab[q] = Bn[q];
      rst4(S.r, Z.X0, N, 0, f4{C.a0[0].x, C.a1[0].x, C.a2[0].x, C.ab[0].x});
      rst4(S.r, Z.X1, N, 0, f4{C.a0[0].y, C.a1[0].y, C.a2[0].y, C.ab[0].y});
    }
#endif
  } else {
  // RC (gamma = 0; f32, and f64 with DTMPC_FAST64_RECOMP): the current tape's states X_k -- and the ancillary's
  // reference states -- are not read but re-rolled from their controls by the same Dubins arithmetic that produced
  // them (init_tape / commit / the nominal's solve: rollout(x0, U)), so they are bit for bit the stored rows; their
  // b is never needed (K's b column is zero at gamma = 0)
  constexpr bool RC = DTMPC_FAST_LS_RECOMP && SV::g0 && (!DTMPC_FAST_F64 || DTMPC_FAST64_RECOMP);
  constexpr bool RCR = RC && SV::rroll;  // the references re-rolled too (only when they are a device rollout)
  real o0 = x0[0], o1 = x0[1], o2 = x0[2], q0 = 0.f, q1 = 0.f, q2 = 0.f;
  if (RCR && TRACK) {
    const f4 R0 = S.xr(0);
    q0 = R0.x;
    q1 = R0.y;
    q2 = R0.z;
  }
  auto roll = [&](StepIn& L) {  // the tape's (and reference's) state of this step, then advance them
    if (RC) {
      L.X0 = o0;
      L.X1 = o1;
      L.X2 = o2;
      dubins(p, o0, o1, o2, L.V0, L.V1);
      if (TRACK && RCR) {
        L.r0 = q0;
        L.r1 = q1;
        L.r2 = q2;
        dubins(p, q0, q1, q2, L.q0, L.q1);
      }
    }
  };
  if (DTMPC_FAST_LS_DEPTH2) {
  // four buffers in rotation, each refilled two steps before use
  auto ix = [&](int j) { return uidx(j < N1 ? j : N1); };
  StepIn A, Bs, Cs, Ds;
  load_step<TRACK, !RC, SV, !RCR>(A, S, 0);
  load_step<TRACK, !RC, SV, !RCR>(Bs, S, ix(1));
  for (int k = 0; k < N; k += 4) {
    load_step<TRACK, !RC, SV, !RCR>(Cs, S, ix(k + 2));
    roll(A);
    ls_step<TRACK, M, NPR, SV::g0>(p, c, A, C, u0, u1);
    keep(k, u0, u1);
    if (k + 1 >= N) break;
    load_step<TRACK, !RC, SV, !RCR>(Ds, S, ix(k + 3));
    roll(Bs);
    ls_step<TRACK, M, NPR, SV::g0>(p, c, Bs, C, u0, u1);
    keep(k + 1, u0, u1);
    if (k + 2 >= N) break;
    load_step<TRACK, !RC, SV, !RCR>(A, S, ix(k + 4));
    roll(Cs);
    ls_step<TRACK, M, NPR, SV::g0>(p, c, Cs, C, u0, u1);
    keep(k + 2, u0, u1);
    if (k + 3 >= N) break;
    load_step<TRACK, !RC, SV, !RCR>(Bs, S, ix(k + 5));
    roll(Ds);
    ls_step<TRACK, M, NPR, SV::g0>(p, c, Ds, C, u0, u1);
    keep(k + 3, u0, u1);
  }
  } else {
  // two step buffers in turn (no copies), each refilled two steps ahead; the refill index is clamped
  // (a redundant load of the last row instead of a branch)
  StepIn A, Bs;
  load_step<TRACK, !RC, SV, !RCR>(A, S, 0);
  load_step<TRACK, !RC, SV, !RCR>(Bs, S, N1 < 1 ? N1 : 1);
  for (int k = 0; k < N; k += 2) {
    roll(A);
    ls_step<TRACK, M, NPR, SV::g0>(p, c, A, C, u0, u1);
    keep(k, u0, u1);
    load_step<TRACK, !RC, SV, !RCR>(A, S, uidx(k + 2 < N1 ? k + 2 : N1));
    if (k + 1 < N) {
      roll(Bs);
      ls_step<TRACK, M, NPR, SV::g0>(p, c, Bs, C, u0, u1);
      keep(k + 1, u0, u1);
      load_step<TRACK, !RC, SV, !RCR>(Bs, S, uidx(k + 3 < N1 ? k + 3 : N1));
    }
  }
  }
  }
  real r0 = 0.f, r1 = 0.f, r2 = 0.f;
  if (TRACK) {
    const f4 RN = S.xr(N);
    r0 = RN.x;
    r1 = RN.y;
    r2 = RN.z;
  }
  real Jc[2 * NPR];
  bool ok = true;
#pragma unroll
  for (int q = 0; q < NPR; ++q) {
    const f2 Jt = C.J[q] + term<TRACK, Obs<M>::wrap>(c, C.a0[q], C.a1[q], C.a2[q], C.ab[q], r0, r1, r2);
    Jc[2 * q] = Jt.x;
    Jc[2 * q + 1] = Jt.y;
    ok = ok && vfinite(Jt);
  }
  // the candidate-cost record (diagnostics: the costs behind the decision; P = 4: lane 3 repeats lane 2)
  if (crec) {
#pragma unroll
    for (int a = 0; a < NL; ++a) {
      const int pos = P == 1 ? cf.cpos[a]
                    : P == 2 ? (h ? cf.cpos[NL + a] : cf.cpos[a])
                             : pick3(hc, cf.cpos[a], cf.cpos[2 + a], cf.cpos[4 + a]);
      if (P != 4 || h < 3) crec[(size_t)pos * cst] = Jc[a];
    }
    if (cf.zpos >= 0 && h == 0) crec[(size_t)cf.zpos * cst] = Jprev;
  }
  // this lane's first strict minimum (its candidates are in increasing original order)
  real bJ = Jc[0];
  int bl = 0;
#pragma unroll
  for (int a = 1; a < NL; ++a)
    if (Jc[a] < bJ) {
      bJ = Jc[a];
      bl = a;
    }
  int bi = c0 + bl;  // index into the candidate list (its order is the original one)
  // the zero candidate's neighbours: min over candidates before / after its position
  real mb = 0.f, ma = 0.f;
  int hb = 0, ha = 0;
  if (cf.zpos >= 0) {
#pragma unroll
    for (int a = 0; a < NL; ++a) {
      const int pos = P == 1 ? cf.cpos[a]
                    : P == 2 ? (h ? cf.cpos[NL + a] : cf.cpos[a])
                             : pick3(hc, cf.cpos[a], cf.cpos[2 + a], cf.cpos[4 + a]);
      if (pos < cf.zpos) {
        mb = (!hb || Jc[a] < mb) ? Jc[a] : mb;
        hb = 1;
      } else {
        ma = (!ha || Jc[a] < ma) ? Jc[a] : ma;
        ha = 1;
      }
    }
  }
  // combine with the trajectory's other lanes: lexicographic (J, position) = strict <, first wins
  auto combine = [&](auto sw) {
    const real oJ = sw(bJ);
    const int oi = sw(bi);
    ok = sw((int)ok) && ok;
    if (oJ < bJ || (oJ == bJ && oi < bi)) {
      bJ = oJ;
      bi = oi;
    }
    if (cf.zpos >= 0) {
      const real omb = sw(mb), oma = sw(ma);
      const int ohb = sw(hb), oha = sw(ha);
      if (ohb) mb = (!hb || omb < mb) ? omb : mb;
      if (oha) ma = (!ha || oma < ma) ? oma : ma;
      hb |= ohb;
      ha |= oha;
    }
  };
  if (P >= 2) combine([](auto v) { return gswap<1>(v); });
  if (P == 4) combine([](auto v) { return gswap<2>(v); });
  bestJ = bJ;
  bc = bi;
  int best = cf.cpos[0];
  al_out = cf.cal[0];
#pragma unroll
  for (int a = 1; a < SV::nc; ++a)
    if (bi == a) {
      best = cf.cpos[a];
      al_out = cf.cal[a];
    }
  if (cf.zpos >= 0) {
    if ((!hb || Jprev < mb) && (!ha || Jprev <= ma)) {
      best = cf.zpos;
      bestJ = Jprev;
      al_out = 0.f;
      bc = -1;
    }
    ok = ok && finite(Jprev);
  }
  return ok ? best : -1;
}

#ifndef DTMPC_FAST_CM_DEPTH2
#define DTMPC_FAST_CM_DEPTH2 1  // 0: one step of prefetch lead (measured 3 % slower)
#endif
#ifndef DTMPC_FAST_CM_LEAD
#define DTMPC_FAST_CM_LEAD 2
#endif
#ifndef DTMPC_FAST_CM_RECOMP
#define DTMPC_FAST_CM_RECOMP 1  // 1: the old tape's states are re-rolled from its controls, not read (CMR below)
#endif
// materialise the chosen candidate in place (commit_candidate): same arithmetic as its lane of the
// line search; the old X[k+1] is read (prefetched) before it is overwritten
template <bool TRACK, int M, class SV>
__device__ __forceinline__ void commit(const FP& p, real al, const real* x0, real Bc0, const SV& S) {
  DTMPC_NOCONTRACT
  const int N = p.N;
  real s0 = x0[0], s1 = x0[1], s2 = x0[2], sb = x0[3], Bc = Bc0;
  // CMR (gamma = 0, f32): the tape's X is rollout(x0, U) by this same scalar fhat (init_tape, commit), so
  // re-rolling the old controls by its Dubins part reproduces the old x, y, theta bit for bit (b is never
  // used: K's b column is zero) and saves 16 B per step of HBM reads.  (With gamma != 0 the re-roll would need
  // the barrier too, measured slower in round 2; f64 is instruction-bound: both read the old states.)
  constexpr bool CMR = DTMPC_FAST_CM_RECOMP && SV::g0 && (!DTMPC_FAST_F64 || DTMPC_FAST64_RECOMP);
  real o0 = s0, o1 = s1, o2 = s2;
  constexpr bool LX = !CMR;
  Solve<false, SV::g0, SV::ric0, SV::lanes> T0;  // no references needed
  T0.r = S.r;
  T0.XA = S.XA;
  T0.UA = S.UA;
  T0.G = S.G;
  auto step = [&](const StepIn& cur, int k) {
    const real e0 = s0 - (CMR ? o0 : cur.X0), e1 = s1 - (CMR ? o1 : cur.X1), e2 = s2 - (CMR ? o2 : cur.X2);
    const real e3 = sb - cur.X3;  // CMR: unused (kdot<g0> drops the b column)
    if (CMR) dubins(p, o0, o1, o2, cur.V0, cur.V1);
#if DTMPC_FAST_KFMA
    const real du0 = cur.kk.x + kdot<SV::g0>(cur.Ka, e0, e1, e2, e3);
    const real du1 = cur.kk.y + kdot<SV::g0>(cur.Kb, e0, e1, e2, e3);
#else
    const real du0 = cur.kk.x + (cur.Ka.x * e0 + cur.Ka.y * e1 + cur.Ka.z * e2 + cur.Ka.w * e3);
    const real du1 = cur.kk.y + (cur.Kb.x * e0 + cur.Kb.y * e1 + cur.Kb.z * e2 + cur.Kb.w * e3);
#endif
    const real u0 = vclamp(ffma(al, du0, cur.V0), p.umin0, p.umax0);
    const real u1 = vclamp(ffma(al, du1, cur.V1), p.umin1, p.umax1);
#ifdef DTMPC_FAST_DIAG_NOSTORE  // timing attribution only: the commit computes but stores nothing
    fhat<M>(p, s0, s1, s2, sb, u0, u1, Bc);
    if (__builtin_isnan(s0 + u0 + u1)) S.stx(k + 1, f4{s0, s1, s2, sb});
#else
    S.stu(k, f2{u0, u1});
    fhat<M, SV::g0>(p, s0, s1, s2, sb, u0, u1, Bc);
    S.stx(k + 1, f4{s0, s1, s2, sb});
#endif
  };
#if DTMPC_FAST_CM_DEPTH2
  // R = LEAD + 1 step buffers in rotation: each refilled LEAD steps before it is used (the commit's step
  // is short, ~190 instructions, and a loaded chip stretches an HBM read past one or two of them).
  // A refill of step j reads the OLD X[j] before step j-1 overwrites it (issued earlier in program
  // order).  The loop is entered with the same outstanding vector-memory operations as its back edge
  // carries (a refill and two stores per step): X row 0 is rewritten with x0 -- the value it holds --
  // twice after each preload, so the wait-count state at the loop header is the same on both paths.
  constexpr int LEAD = DTMPC_FAST_CM_LEAD, R = LEAD + 1;
  const int N1 = N - 1;
  auto ix = [&](int j) { return uidx(j < N1 ? j : N1); };
  const f4 X0v = f4{x0[0], x0[1], x0[2], x0[3]};
  StepIn Bf[R];
#pragma unroll
  for (int j = 0; j < LEAD; ++j) {
    load_step<false, LX>(Bf[j], T0, ix(j));
    rst2(S.r, S.XA, 0, 0, f2{X0v.x, X0v.y});
    S.stx(0, X0v);
  }
  for (int k = 0; k < N; k += R) {
#pragma unroll
    for (int j = 0; j < R; ++j) {
      load_step<false, LX>(Bf[(j + LEAD) % R], T0, ix(k + j + LEAD));
      if (k + j >= N) break;
      step(Bf[j], k + j);
    }
  }
#else
  StepIn cur, nxt;
  load_step<false, LX>(nxt, T0, 0);
  for (int k = 0; k < N; ++k) {
    cur = nxt;
    if (k + 1 < N) load_step<false, LX>(nxt, T0, k + 1);
    step(cur, k);
  }
#endif
}

#ifdef DTMPC_PROFILE
// profiling builds: line-search outcome statistics per solve (TRACK = 0 nominal, 1 ancillary), 32 slots
// each: [0..7] winners by original alpha position (lanes), [8] wave-iterations, [9] waves where every
// lane keeps its tape (alpha = 0), [10] every lane takes the first alpha, [11] every lane one of the two
__device__ unsigned long long g_lsstat[64];
__device__ __forceinline__ void ls_stat(int trk, int best, real al, const FIlqr& cf) {
  unsigned long long* g = g_lsstat + 32 * trk;
  const bool lead = (threadIdx.x & 63) == (__builtin_ctzll(__ballot(1)));
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const unsigned long long b = __ballot(best == q);
    if (lead && b) atomicAdd(g + q, (unsigned long long)__builtin_popcountll(b));
  }
  const bool z = al == 0.f, f = al == cf.cal[0] && best == cf.cpos[0];
  const unsigned long long act = __ballot(1);
  if (lead) {
    atomicAdd(g + 8, 1ull);
    if (__ballot(z) == act) atomicAdd(g + 9, 1ull);
    if (__ballot(f) == act) atomicAdd(g + 10, 1ull);
    if (__ballot(z || f) == act) atomicAdd(g + 11, 1ull);
  }
}
#endif

#ifdef DTMPC_FAST_DIAG
// diagnostics builds (scripts/diag_f64.sh, not the product): every kernel's kernarg segment starts with its FP, so
// the problem constants the solver holds in registers (the pinned obstacle table, the scalars) can be compared
// with the segment's copy at every phase boundary; the first lanes that disagree, or whose solve goes
// non-finite, print where.  The general path forms its DBaS constants on the device, so only the table and the
// dynamics constants are compared there.
template <int MM>
__device__ __forceinline__ void diag_p(const FP& p, int where, int it) {
  const FP* q = (const FP*)__builtin_amdgcn_kernarg_segment_ptr();
  int bad = -1;
  real v = 0, w = 0;
#pragma unroll
  for (int j = 0; j < Obs<MM>::n; ++j) {  // kLds: the LDS copy against the kernarg table
    if (ocx<MM>(p, j) != q->cx[j]) { bad = 40 + j; v = ocx<MM>(p, j); w = q->cx[j]; }
    if (ocy<MM>(p, j) != q->cy[j]) { bad = 50 + j; v = ocy<MM>(p, j); w = q->cy[j]; }
    if (or2<MM>(p, j) != q->r2[j]) { bad = 60 + j; v = or2<MM>(p, j); w = q->r2[j]; }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    if (__builtin_bit_cast(unsigned long long, (double)p.cx[j]) != __builtin_bit_cast(unsigned long long, (double)q->cx[j])) { bad = j; v = p.cx[j]; w = q->cx[j]; }
    if (__builtin_bit_cast(unsigned long long, (double)p.cy[j]) != __builtin_bit_cast(unsigned long long, (double)q->cy[j])) { bad = 10 + j; v = p.cy[j]; w = q->cy[j]; }
    if (__builtin_bit_cast(unsigned long long, (double)p.r2[j]) != __builtin_bit_cast(unsigned long long, (double)q->r2[j])) { bad = 20 + j; v = p.r2[j]; w = q->r2[j]; }
  }
  if (p.dt != q->dt) { bad = 30; v = p.dt; w = q->dt; }
  if (p.umax0 != q->umax0 || p.umin0 != q->umin0 || p.umax1 != q->umax1 || p.umin1 != q->umin1) { bad = 31; v = p.umax0; w = q->umax0; }
  if (p.neg_beta != q->neg_beta || p.neg_inv_beta != q->neg_inv_beta) { bad = 32; v = p.neg_beta; w = q->neg_beta; }
  if (p.eps != q->eps) { bad = 33; v = p.eps; w = q->eps; }
  if (p.N != q->N) { bad = 34; v = p.N; w = q->N; }
  if (bad >= 0)
    printf("DIAG const blk=%d thr=%d where=%d it=%d field=%d have=%.17g want=%.17g\n", (int)blockIdx.x,
           (int)threadIdx.x, where, it, bad, (double)v, (double)w);
}
#define DIAG_P(MM, p, where, it) diag_p<MM>(p, where, it)
#else
#define DIAG_P(MM, p, where, it) ((void)0)
#endif

// P = 4 tape slots: slot q of the solve's X / U records at lane offset base + q * stride
struct SlotMap {
  unsigned bx, sx, bu, su;  // X: base (trajectory * 16), slot stride (Bc * 16); U: (trajectory * 8), (Bc * 8)
};
constexpr int kSlots = 12;     // two banks of the six rolled-out candidates
constexpr int kSlotInit = 6;   // the initial rollout: bank 1, so the first line search writes bank 0

// the decision record of one solve (dtmpc_tube_state.choices / .costs, dtmpc_ilqr_solve_ws): this
// trajectory's column of the winning-alpha record ch [max_iter][B] and of the candidate-cost record
// cr [max_iter][8][B] (every line-search candidate's cost by original alpha position; the caller pre-fills
// it, NaN: not run),
// s = B (the column stride); either pointer may be null
struct DecRec {
  signed char* ch;
  real* cr;
  size_t s;
};

// iLQR for one trajectory (ilqr_traj, core/ddp.py:102-307).  P = 4: no commit pass -- the line search
// kept every candidate's tape (Slots) and the winner's slot becomes the current tape (S.XA / S.UA).
template <bool TRACK, int M, int P, bool SHIFT = true, class SV>
__device__ __forceinline__ int ilqr(const FP& p, const FCost& c, const FIlqr& cf, const real* x0,
                                    SV& S, int h, const SlotMap& sm, int& iters, Prof& pf, const DecRec& dr) {
  constexpr int ph = TRACK ? 4 : 0;  // phase-timer slots (profiling builds)
  signed char* const ch = dr.ch;
  const size_t chs = dr.s;
  if (ch && h == 0)  // the decision record: -1 for iterations not run (dtmpc_tube_state.choices)
    for (int it = 0; it < cf.max_iter; ++it) ch[it * chs] = -1;
  // (the candidate-cost record is written only where a candidate ran: the caller pre-fills it -- a fill loop
  // here made the f64 M = 3 tube kernel hit an AMDGPU back-end error, "Illegal instruction detected:
  // V_CMP_NE_U32 0, src_private_base", ROCm 7.2 hipcc)
  real Jcur = init_tape<TRACK, M>(p, c, x0, S, cf.zpos >= 0 && cf.max_iter > 0);
  const real Bc0 = barrier_at<M>(p, x0[0], x0[1]);
  bool have_prev = false;
  real prev = 0.f;
  iters = 0;
  int st = 0;
  int cur = kSlotInit;  // P = 4: the current tape's slot
  pf.mark(ph);
  DIAG_P(M, p, TRACK ? 100 : 0, -1);
  for (int it = 0; it < cf.max_iter; ++it) {
    iters = it + 1;
    if (!backward<TRACK, M>(p, c, cf.reg, S, h)) {
      st = DTMPC_ST_NONFINITE;
#ifdef DTMPC_FAST_DIAG
      printf("DIAG backward non-finite blk=%d thr=%d h=%d trk=%d it=%d x0=(%.17g %.17g %.17g %.17g)\n", (int)blockIdx.x,
             (int)threadIdx.x, h, (int)TRACK, it, (double)x0[0], (double)x0[1], (double)x0[2], (double)x0[3]);
      DIAG_P(M, p, TRACK ? 101 : 1, it);
#endif
      break;
    }
    DIAG_P(M, p, TRACK ? 102 : 2, it);
    pf.mark(ph + 1);
    real bestJ, al;
    int bc;
    Slots Z;
    const int nb = cur < 6 ? 6 : 0;  // first slot of the bank the current tape is not in
    if (P == 4) {
      const unsigned q0 = (unsigned)(nb + 2 * (h < 2 ? h : 2));
      Z.X0 = RA{S.XA.base, S.XA.rs, sm.bx + q0 * sm.sx};
      Z.X1 = RA{S.XA.base, S.XA.rs, sm.bx + (q0 + 1) * sm.sx};
      Z.U0 = RA{S.UA.base, S.UA.rs, sm.bu + q0 * sm.su};
      Z.U1 = RA{S.UA.base, S.UA.rs, sm.bu + (q0 + 1) * sm.su};
    }
    const int best = line_search<TRACK, M, P>(p, c, cf, x0, Bc0, S, Jcur, h, bestJ, al, bc, Z,
                                              dr.cr ? dr.cr + (size_t)it * 8 * chs : nullptr, chs);
    pf.mark(ph + 2);
#ifdef DTMPC_PROFILE
    ls_stat(TRACK ? 1 : 0, best, al, cf);
#endif
    if (best < 0) {
      st = DTMPC_ST_NONFINITE;
#ifdef DTMPC_FAST_DIAG
      printf("DIAG line search non-finite blk=%d thr=%d h=%d trk=%d it=%d Jprev=%.17g bestJ=%.17g x0=(%.17g %.17g %.17g %.17g)\n",
             (int)blockIdx.x, (int)threadIdx.x, h, (int)TRACK, it, (double)Jcur, (double)bestJ, (double)x0[0],
             (double)x0[1], (double)x0[2], (double)x0[3]);
      DIAG_P(M, p, TRACK ? 103 : 3, it);
#endif
      break;
    }
    DIAG_P(M, p, TRACK ? 104 : 4, it);
    if (ch && h == 0) ch[it * chs] = (signed char)best;
    if (al != 0.f) {
      if (P == 4) {
        cur = nb + bc;
        S.XA.lo = sm.bx + (unsigned)cur * sm.sx;
        S.UA.lo = sm.bu + (unsigned)cur * sm.su;
      } else {
        commit<TRACK, M>(p, al, x0, Bc0, S);
      }
    }
    pf.mark(ph + 3);
    Jcur = bestJ;
    if (have_prev && m_abs(prev - bestJ) < cf.tol) break;
    have_prev = true;
    prev = bestJ;
  }
  copy_out<SHIFT>(p.N, S.r, S.XA, S.UA, S.X, S.U);  // the tape as it stands (a failed solve's too)
  return st;
}

// ---------------------------------------------------------------------------------------------
// DDP sensitivity with the paper upper loss + DOC gradient (sens_traj<real, false, false, true>,
// core/ddp.py:317-427, core/tube_mpc.py:915-976): acc = L, gQ(3), gR(2), gqb
template <int M, class SV>
__device__ __forceinline__ int sensitivity(const FP& p, const FCost& c, const SV& S, const RA& A8, const RA& A2,
                                           real* acc) {
  const int N = p.N;
  const real lxx[4] = {2.f * c.Q0, 2.f * c.Q1, 2.f * c.Q2, 2.f * c.qb};
  const real luu[2] = {2.f * c.R0, 2.f * c.R1};
  const real pxx[4] = {2.f * c.Qf0, 2.f * c.Qf1, 2.f * c.Qf2, 2.f * c.qb};
  const real reg = 1e-9f;
  Riccati<real> R;  // R.Vx holds tilde V_x
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) R.Vxx[i][j] = i == j ? pxx[i] : 0.f;
  {
    const f4 XN = S.x(N), RN = S.xr(N);
    R.Vx[0] = 2.f * (XN.x - RN.x);
    R.Vx[1] = 2.f * (XN.y - RN.y);
    R.Vx[2] = 2.f * (XN.z - RN.z);
    R.Vx[3] = 2.f * XN.w;
  }
  real gxn, gyn;
  real dBn;
  {
    const f4 XN = S.x(N);
    dBn = dbarrier(p, h_grad<M>(p, XN.x, XN.y, gxn, gyn));
  }
  // step inputs read one step ahead (the loop's record stores would otherwise sit between a step's
  // loads and their use, exposing one memory latency per step)
  f4 nX = S.x(N - 1), nR = S.xr(N - 1);
  f2 nV = S.u(N - 1);
  for (int k = N - 1; k >= 0; --k) {
    const f4 X = nX, Rr = nR;
    const f2 V = nV;
    if (k > 0) {
      nX = S.x(k - 1);
      nR = S.xr(k - 1);
      nV = S.u(k - 1);
    }
    const real x0 = X.x, x1 = X.y, x2 = X.z, xb = X.w;
    const real u0 = V.x, u1 = V.y;
    real sn, cs;
    vsincos(x2, sn, cs);
    real gxk, gyk;
    const real dBk = dbarrier(p, h_grad<M>(p, x0, x1, gxk, gyk));
    const Jac<real> J = jac(p, sn, cs, u0, gxk, gyk, dBk, gxn, gyn, dBn);
    gxn = gxk;
    gyn = gyk;
    dBn = dBk;
    real Qxx[4][4], Qxu[4][2], Qux[2][4], Quu[2][2];
    sens_qblocks(J, R.Vxx, lxx, luu, Qxx, Qxu, Qux, Quu);
    const real* tv = R.Vx;
    const real tQu0 = J.b00 * tv[0] + J.b10 * tv[1] + J.b30 * tv[3];
    const real tQu1 = J.b21 * tv[2] + J.b31 * tv[3];
    real tQx[4];
    tQx[0] = 2.f * (x0 - Rr.x) + (tv[0] + J.a30 * tv[3]);
    tQx[1] = 2.f * (x1 - Rr.y) + (tv[1] + J.a31 * tv[3]);
    tQx[2] = 2.f * (x2 - Rr.z) + (J.a02 * tv[0] + J.a12 * tv[1] + tv[2] + J.a32 * tv[3]);
    tQx[3] = 2.f * xb + J.g * tv[3];
    const bool act0 = (u0 <= p.umin0 + p.active_tol) || (u0 >= p.umax0 - p.active_tol);
    const bool act1 = (u1 <= p.umin1 + p.active_tol) || (u1 >= p.umax1 - p.active_tol);
    const real m00 = Quu[0][0] + reg, m11 = Quu[1][1] + reg;
    const LU2<real> f = lu2(m00, Quu[0][1], Quu[1][0], m11);
    real Kk[8], kk[2];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      real y0, y1;
      solve_reduced(f, m00, m11, act0, act1, Qux[0][j], Qux[1][j], y0, y1);
      Kk[j] = -y0;
      Kk[4 + j] = -y1;
    }
    {
      real y0, y1;
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
    S.G.store_full(S.r, k, Kk, kk);  // full records in the workspace: its own K and k
    rst4(S.r, A8, k, 0, f4{J.a02, J.a12, J.a30, J.a31});
    rst4(S.r, A8, k, 16 * ES, f4{J.a32, J.b00, J.b10, J.b30});
    rst2(S.r, A2, k, 0, f2{J.b31, real((act0 ? 1 : 0) + (act1 ? 2 : 0))});
  }
  // forward (:413-425) fused with the upper loss and the DOC gradient
  real d[4] = {0.f, 0.f, 0.f, 0.f};
  real L1 = 0.f, L2 = 0.f, gQ0 = 0.f, gQ1 = 0.f, gQ2 = 0.f, gR0 = 0.f, gR1 = 0.f, gqb = 0.f;
  const real g = p.gamma, dt = p.dt;
  struct FwdIn {
    f4 Ka, Kb, A0, A1, X, Rr;
    f2 kf, A2r, V, Q;
  };
  auto fload = [&](FwdIn& F, int k) {
    F.Ka = rld4(S.r, S.G.K, k, 0);
    F.Kb = rld4(S.r, S.G.K, k, 16 * ES);
    F.kf = rld2(S.r, S.G.k, k, 0);
    F.A0 = rld4(S.r, A8, k, 0);
    F.A1 = rld4(S.r, A8, k, 16 * ES);
    F.A2r = rld2(S.r, A2, k, 0);
    F.X = S.x(k);
    F.Rr = S.xr(k);
    F.V = S.u(k);
    F.Q = S.ur(k);
  };
  FwdIn Fn;
  fload(Fn, 0);
  for (int k = 0; k < N; ++k) {
    const FwdIn F = Fn;
    if (k + 1 < N) fload(Fn, k + 1);
    const f4 Ka = F.Ka, Kb = F.Kb, A0 = F.A0, A1 = F.A1;
    const f2 kf = F.kf, A2r = F.A2r;
    const real a02 = A0.x, a12 = A0.y, a30 = A0.z, a31 = A0.w, a32 = A1.x, b00 = A1.y, b10 = A1.z, b30 = A1.w,
                b31 = A2r.x;
    const int act = (int)A2r.y;
    const real v0 = (act & 1) ? 0.f : kf.x + (Ka.x * d[0] + Ka.y * d[1] + Ka.z * d[2] + Ka.w * d[3]);
    const real v1 = (act & 2) ? 0.f : kf.y + (Kb.x * d[0] + Kb.y * d[1] + Kb.z * d[2] + Kb.w * d[3]);
    const f4 X = F.X, Rr = F.Rr;
    const f2 V = F.V, Q = F.Q;
    const real e0 = X.x - Rr.x;
    const real e1 = X.y - Rr.y;
    const real e2 = X.z - Rr.z;
    const real bb = X.w;
    const real w0 = V.x - Q.x;
    const real w1 = V.y - Q.y;
    L1 += e0 * e0 + e1 * e1 + e2 * e2;
    L2 += bb * bb;
    gQ0 += 2.f * e0 * d[0];
    gQ1 += 2.f * e1 * d[1];
    gQ2 += 2.f * e2 * d[2];
    gR0 += 2.f * w0 * v0;
    gR1 += 2.f * w1 * v1;
    gqb += 2.f * bb * d[3];
    const real n0 = (d[0] + a02 * d[2]) + b00 * v0;
    const real n1 = (d[1] + a12 * d[2]) + b10 * v0;
    const real n2 = d[2] + dt * v1;
    const real n3 = (a30 * d[0] + a31 * d[1] + a32 * d[2] + g * d[3]) + (b30 * v0 + b31 * v1);
    d[0] = n0;
    d[1] = n1;
    d[2] = n2;
    d[3] = n3;
  }
  bool ok = true;
#pragma unroll
  for (int i = 0; i < 4; ++i) ok = ok && finite(d[i]);
  const f4 XN = S.x(N), RN = S.xr(N);
  const real e0 = XN.x - RN.x;
  const real e1 = XN.y - RN.y;
  const real e2 = XN.z - RN.z;
  const real bb = XN.w;
  L1 += e0 * e0 + e1 * e1 + e2 * e2;
  L2 += bb * bb;
  acc[0] = L1 + L2;
  acc[1] = gQ0 + 2.f * e0 * d[0];
  acc[2] = gQ1 + 2.f * e1 * d[1];
  acc[3] = gQ2 + 2.f * e2 * d[2];
  acc[4] = gR0;
  acc[5] = gR1;
  acc[6] = gqb + 2.f * bb * d[3];
  ok = ok && finite(acc[1]) && finite(acc[4]) && finite(acc[5]);
  return ok ? 0 : DTMPC_ST_NONFINITE;
}

// ---------------------------------------------------------------------------------------------
// the fused closed-loop step (tube_step_kernel's body on the fast configuration)
// All kernel arguments in one struct, passed by value: it sits at offset 0 of the kernarg segment.
struct FK {
  FP p;
  FCost cn;
  FIlqr cfn, cfa;
  FArgs a;
};
typedef const FK KArg;
typedef __attribute__((address_space(4))) const FK KArg4;

// The kernel reads its arguments PHASE BY PHASE through this pointer (each call an opaque copy, so
// the compiler cannot merge the loads of two phases): the constants of one phase -- the nominal
// solve, the ancillary solve, the sensitivity, the plant -- are loaded into scalar registers when
// that phase starts and die with it, instead of all of them being loaded at kernel entry and kept
// live (and spilled) through the whole step.
__device__ __forceinline__ KArg* kargs() {
  KArg4* k = (KArg4*)__builtin_amdgcn_kernarg_segment_ptr();
  __asm__ volatile("" : "+s"(k));
  return (KArg*)k;  // generic; the compiler infers the constant address space back (scalar loads)
}

#ifdef DTMPC_FAST_GLOBAL
__device__ __forceinline__ const char* kargs_ws() { return (const char*)kargs()->a.work; }
#endif

#ifndef DTMPC_FAST_PIN
#define DTMPC_FAST_PIN 1
#endif
#ifndef DTMPC_FAST_PIN64_MAX
#define DTMPC_FAST_PIN64_MAX 5
#endif
// the problem constants of one phase; the obstacle table pinned in VGPRs (every candidate of every
// step reads it; in scalar registers it is what the compiler would spill first).  f64 pins at most five
// obstacles (30 VGPRs; the paper's M = 5): the f64 receding kernel at M = 8 with its 48-VGPR table spilled
// into scratch inside its per-lane divergent loops and returned run-to-run different results (NaN on one
// box, 55 % of the runs off on another; unchanged by -ftrivial-auto-var-init, gone with the table
// unpinned -- DESIGN.md section 9, profiles/r04/m8_receding.txt); f64 at M = 5 runs 13.6 ms pinned, 15.6 unpinned.
template <int M>
__device__ __forceinline__ FP pin_p(FP p) {
#if DTMPC_FAST_PIN
  if (Obs<M>::lds || (DTMPC_FAST_F64 && Obs<M>::n > DTMPC_FAST_PIN64_MAX)) return p;
#pragma unroll
  for (int j = 0; j < Obs<M>::n; ++j) {
    real vx = p.cx[j], vy = p.cy[j], vr = p.r2[j];
    __asm__ volatile("" : "+v"(vx));
    __asm__ volatile("" : "+v"(vy));
    __asm__ volatile("" : "+v"(vr));
    p.cx[j] = vx;
    p.cy[j] = vy;
    p.r2[j] = vr;
  }
#endif
  return p;
}
template <int M>
__device__ __forceinline__ FP phase_p() {
  return pin_p<M>(kargs()->p);
}

// Where an f64 instantiation keeps its obstacle table (round 5).  Every f64 fused kernel must run without a
// private segment (build.py check_resources: the f64 defects of rounds 3-4 all came from f64 kernels that kept
// values in scratch inside per-lane divergent loops).  The table pinned in VGPRs (pin_p) fits
// beside the compact gamma = 0 records up to DTMPC_FAST_PIN64_MAX obstacles; the general records (GM = 0, and the
// general path's solves, which hold both record forms) and larger tables read it again at each use (kLds) -- by a
// scalar load of the kernarg segment's copy (DTMPC_FAST64_TABSRC = 1, the default; 0 is the LDS copy, A/B only).
// DTMPC_FAST64_TAB: 1 that rule (default), 2 kLds in every f64 kernel, 0 never kLds (the round-4 forms, A/B).
#ifndef DTMPC_FAST64_TAB
#define DTMPC_FAST64_TAB 1
#endif
template <int M, int GM>
constexpr int tab_flag();
// the exp form of an f64 instantiation: the one-block asm polynomial holds its ten coefficients in VGPRs, which the
// table-in-kernarg (kLds) kernels and the four-lane kernels cannot afford without a private segment (build.py check:
// 48 B of scratch in fk64::tube_fast_kernel<5, 4, 2> beside the in-step broadcast of the backward inputs, in <5, 4, 1>
// without it), so it runs at one and two lanes.  Round 5 kept it at one lane after the two-lane
// form read stale values on one trajectory of 700; round 6 found the cause (profiles/r06/flow_copy_root_cause.txt): the
// register allocator's live-range-split copies in the flow block of dbarrier's divergent if / else, which ran with the
// then-lanes' exec mask only -- the asm form's extra VGPRs only made the allocator split there.  dbarrier is branchless
// in f64 now, build.py fails a build with any such copy (scan_flow_copies), and the two-lane asm form (and the
// four-lane one, where it fits) passes tests/test_gpu_reuse.py (profiles/r06/logs).
#ifndef DTMPC_FAST64_XASM_MAXP
#define DTMPC_FAST64_XASM_MAXP 2
#endif
template <int M, int GM, int P>
constexpr int xasm_flag() {
#if DTMPC_FAST_F64
  return (DTMPC_FAST64_EXP == 3 && P <= DTMPC_FAST64_XASM_MAXP && (P <= 2 || GM == 2) && tab_flag<M, GM>() == 0)
             ? kXasm
             : 0;
#else
  return 0;
#endif
}
template <int M, int GM>
constexpr int tab_flag() {
  return (DTMPC_FAST_F64 && (DTMPC_FAST64_TAB == 2 ||
                             (DTMPC_FAST64_TAB == 1 && (GM == 0 || Obs<M>::n > DTMPC_FAST_PIN64_MAX))))
             ? kLds
             : 0;
}

// GM: 0 general, 1 gamma = 0 gain records, 2 gamma = 0 gain records + Riccati step (the default at gamma = 0)
// One wave per SIMD at every lane count (amdgpu_waves_per_eu(1, 1)): the whole 512-register budget.
template <int M, int P, int GM>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(1, 1)))
tube_fast_kernel(FK kk) {
  constexpr bool G0 = GM > 0, RG0 = GM > 1;
  constexpr int ML = M | tab_flag<M, GM>() | xasm_flag<M, GM, P>();  // M with the table placement and exp form (f64)
  (void)kk;  // read through kargs()
  __shared__ f4 lds[kBlock / 64 * DTMPC_TUBE_SUMS / 4];  // the workgroup sums at the end
  const int B = kargs()->a.B, Bc = kargs()->a.Bc, i0 = kargs()->a.i0;
  const int gl = blockIdx.x * blockDim.x + threadIdx.x;  // blockDim: tube_block (64 or 256)
  const int t = gl / P, h = gl % P;  // t: index in the chunk, h: lane of the trajectory
  const int i = i0 + t;              // index in the batch
  real acc[DTMPC_TUBE_SUMS] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  {
    // desynchronise the workgroups' phases: every wave runs the same sequence of passes, so without an
    // offset the whole chip is in the same pass at once -- and the commit (the pass with the most
    // bytes per instruction) then asks for about twice the HBM bandwidth while the line search leaves
    // it idle.  Workgroup g starts (g mod 8) / 8 of `stagger` sleep rounds late.
    const int n = kargs()->a.stagger * (int)(blockIdx.x & 7) / 8;
    for (int r = 0; r < n; ++r) __builtin_amdgcn_s_sleep(127);
  }
  obs_fill<ML>(kargs()->p);
  Prof pf;
  pf.start();
  if (t < Bc) {
    const size_t nb = (size_t)B;
    const unsigned lo = (unsigned)i * (4u * ES), bb = (unsigned)B * (4u * ES);
    const Lane L{lo, lo + bb, lo + 2u * bb, lo + 3u * bb};
    // record strides: P = 4 keeps kSlots tapes per solve (slot-major inside a row), else one
    constexpr unsigned NS = P == 4 ? kSlots : 1;
    const unsigned cb = (unsigned)Bc, l8 = (unsigned)t * (8u * ES), l16 = (unsigned)t * (16u * ES), l32 = (unsigned)t * (32u * ES);
    const SlotMap sm{l16, cb * (16u * ES), l8, cb * (8u * ES)};
    const unsigned x0lo = P == 4 ? l16 + kSlotInit * cb * (16u * ES) : l16, u0lo = P == 4 ? l8 + kSlotInit * cb * (8u * ES) : l8;
    Gains<P> G;

    int st = 0, itn = 0, ita = 0;
    real x0, x1, x2, xb, y0, y1, y2, yb;
    {
      KArg* K = kargs();
      x0 = K->a.x[i];
      x1 = K->a.x[nb + i];
      x2 = K->a.x[2 * nb + i];
      xb = K->a.b[i];
      y0 = K->a.xbar[i];
      y1 = K->a.xbar[nb + i];
      y2 = K->a.xbar[2 * nb + i];
      yb = K->a.bbar[i];
    }
    const int phase = kargs()->a.phase;  // uniform: which part of the step this launch runs
    // the split step's hand-over (phase 1 -> 2): the nominal tape's final record offsets (P = 4: its slot) and
    // the nominal solve's status and iterations, [3][Bc] ints after the records
    int* const hand = (int*)((char*)kargs()->a.work + kargs()->a.oPH) + t;
    Solve<false, G0, RG0, P> Sn;
    if (phase == 2) {  // the nominal was solved by this step's phase-1 launch
      KArg* K = kargs();
      Sn.r = __builtin_amdgcn_make_buffer_rsrc(K->a.work, 0, (int)K->a.wsz, 0x00020000);
      Sn.XA = RA{K->a.oXn, NS * cb * (16u * ES), (unsigned)hand[0]};
      Sn.UA = RA{K->a.oUn, NS * cb * (8u * ES), (unsigned)hand[Bc]};
      const int w2 = hand[2 * Bc];
      st = w2 & 0xff;
      itn = w2 >> 8;
    } else {  // nominal MPC (fixed weights, :813-857)
      KArg* K = kargs();
      Sn.r = __builtin_amdgcn_make_buffer_rsrc(K->a.work, 0, (int)K->a.wsz, 0x00020000);
      Sn.XA = RA{K->a.oXn, NS * cb * (16u * ES), x0lo};
      Sn.UA = RA{K->a.oUn, NS * cb * (8u * ES), u0lo};
      Sn.XRA = Sn.XA;
      Sn.URA = Sn.UA;
      Sn.G = G;
      Sn.G.K = RA{K->a.oK, cb * (32u * ES), l32};
      Sn.G.k = RA{K->a.ok, cb * (8u * ES), l8};
      Sn.X = Soa<4>{(char*)K->a.Xnom, 4u * bb, L};
      Sn.U = Soa<2>{(char*)K->a.Unom, 2u * bb, L};
      const FP p = phase_p<ML>();
      const FCost cn = K->cn;
      const FIlqr cfn = K->cfn;
      const real xn0[4] = {y0, y1, y2, yb};
      const DecRec dr{K->a.choices ? K->a.choices + i : nullptr, K->a.costs ? K->a.costs + i : nullptr, nb};
      st |= ilqr<false, ML, P>(p, cn, cfn, xn0, Sn, h, sm, itn, pf, dr);
    }
    if (phase == 1) {  // hand over to the phase-2 launch; the plant state and theta are untouched
      if (h == 0) {
        hand[0] = (int)Sn.XA.lo;
        hand[Bc] = (int)Sn.UA.lo;
        hand[2 * Bc] = st | (itn << 8);
      }
    } else {
    FCost ca;  // ancillary weights theta (shared by the batch), terminal weight Qa (:885, :891)
    {
      const real* th = kargs()->a.theta;
      ca.Q0 = ca.Qf0 = th[0];
      ca.Q1 = ca.Qf1 = th[1];
      ca.Q2 = ca.Qf2 = th[2];
      ca.R0 = th[3];
      ca.R1 = th[4];
      ca.qb = th[5];
      ca.tg = f4{0.f, 0.f, 0.f, 0.f};
    }
    Solve<true, G0, RG0, P> Sa;
    {  // ancillary MPC tracking the nominal plan (:863-909)
      KArg* K = kargs();
      Sa.r = __builtin_amdgcn_make_buffer_rsrc(K->a.work, 0, (int)K->a.wsz, 0x00020000);
      Sa.XA = RA{K->a.oXa, NS * cb * (16u * ES), x0lo};
      Sa.UA = RA{K->a.oUa, NS * cb * (8u * ES), u0lo};
      Sa.XRA = Sn.XA;  // the nominal plan as solved (P = 4: its final slot)
      Sa.URA = Sn.UA;
      Sa.G = G;
      Sa.G.K = RA{K->a.oK, cb * (32u * ES), l32};
      Sa.G.k = RA{K->a.ok, cb * (8u * ES), l8};
      Sa.X = Soa<4>{(char*)K->a.Xaux, 4u * bb, L};
      Sa.U = Soa<2>{(char*)K->a.Uaux, 2u * bb, L};
      const FP p = phase_p<ML>();
      const FIlqr cfa = K->cfa;
      const real xa0[4] = {x0, x1, x2, xb};
      const size_t o = (size_t)K->cfn.max_iter * nb + i;
      const DecRec dr{K->a.choices ? K->a.choices + o : nullptr, K->a.costs ? K->a.costs + 8 * (o - i) + i : nullptr, nb};
      st |= ilqr<true, ML, P>(p, ca, cfa, xa0, Sa, h, sm, ita, pf, dr);
    }
    pf.mark(8);
    {  // upper loss, DOC sensitivity and gradient (:915-976)
      KArg* K = kargs();
      const RA A8{K->a.oA8, cb * (32u * ES), l32}, A2{K->a.oA2, cb * (8u * ES), l8};
      const FP p = phase_p<ML>();
      st |= sensitivity<ML>(p, ca, Sa, A8, A2, acc);
      DIAG_P(ML, p, 200, st);
    }
    pf.mark(9);
    {  // plant step with disturbance, nominal propagation (:990-1001), log, warm-start shift
      KArg* K = kargs();
      const FArgs& a = K->a;
      const FP p = phase_p<ML>();
      // the plans' first controls, from the records (the ABI tapes already hold the shifted warm starts)
      const f2 ua = rld2(Sa.r, Sa.UA, 0, 0), un = rld2(Sa.r, Sn.UA, 0, 0);
      const real u0 = ua.x, u1 = ua.y;
      const real v0 = un.x, v1 = un.y;
      real w[3];
      if (a.disturbance == 0) {
        w[0] = a.w[i];
        w[1] = a.w[nb + i];
        w[2] = a.w[2 * nb + i];
      } else {
        uint32_t r[4];
        philox4x32_10(a.seed, (uint64_t)(a.goff + i), (uint64_t)a.step, r);
#pragma unroll
        for (int f = 0; f < 3; ++f) {
          const real u = real(r[f] >> 8) * real(1.0 / 16777216.0);
          w[f] = a.wlo[f] + (a.whi[f] - a.wlo[f]) * u;
        }
      }
      if (a.write_log && h == 0) {
        real* lg = a.log;
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
        real q0 = x0, q1 = x1, q2 = x2, qb = xb, Bc = barrier_at<ML>(p, x0, x1);
        fhat<ML>(p, q0, q1, q2, qb, u0, u1, Bc);
        a.x[i] = q0 + w[0];
        a.x[nb + i] = q1 + w[1];
        a.x[2 * nb + i] = q2 + w[2];
        a.b[i] = qb;
      }
      {
        real q0 = y0, q1 = y1, q2 = y2, qb = yb, Bc = barrier_at<ML>(p, y0, y1);
        fhat<ML>(p, q0, q1, q2, qb, v0, v1, Bc);
        a.xbar[i] = q0;
        a.xbar[nb + i] = q1;
        a.xbar[2 * nb + i] = q2;
        a.bbar[i] = qb;
      }
      acc[7] = 1.f;
      DIAG_P(ML, p, 300, st);
#ifdef DTMPC_FAST_DIAG
      if (st && h == 0) printf("DIAG status traj=%d st=%d itn=%d ita=%d\n", i, st, itn, ita);
#endif
      // healthy trajectories only (status 0 and every gradient component within the bound, NaN failing
      // the test); a trajectory's lanes count once
      real gm = m_abs(acc[1]);
#pragma unroll
      for (int j = 2; j < 7; ++j) gm = vmaxnan(gm, m_abs(acc[j]));
      if (st || h != 0 || !(gm <= a.gbound)) {
#pragma unroll
        for (int j = 0; j < DTMPC_TUBE_SUMS; ++j) acc[j] = 0.f;
      }
      if (h == 0) {
        a.status[i] |= st;
        if (a.iters) {
          a.iters[i] = itn;
          a.iters[nb + i] = ita;
        }
      }
    }
    pf.mark(10);
    }  // phase != 1
  }
  pf.flush();
  if (kargs()->a.phase == 1) return;  // the step's sums come from its phase-2 launch (uniform)
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  real ws[DTMPC_TUBE_SUMS];
#pragma unroll
  for (int j = 0; j < DTMPC_TUBE_SUMS; ++j) ws[j] = wave_sum(acc[j]);
  __syncthreads();
  real* red = (real*)lds;
  if (lane == 0)
#pragma unroll
    for (int j = 0; j < DTMPC_TUBE_SUMS; ++j) red[wv * DTMPC_TUBE_SUMS + j] = ws[j];
  __syncthreads();
  if (threadIdx.x < DTMPC_TUBE_SUMS) {
    real v = 0.f;
#pragma unroll
    for (int q = 0; q < (int)(blockDim.x / 64); ++q) v += red[q * DTMPC_TUBE_SUMS + threadIdx.x];
    kargs()->a.partials[((size_t)blockIdx.x + (size_t)i0 * P / blockDim.x) * DTMPC_TUBE_SUMS + threadIdx.x] = v;
  }
}

#if !defined(DTMPC_FAST_AUX_TU) && !DTMPC_FAST_F64
// Known-byte calibration launch for the HBM counters (scripts/pmc_calib.py, rocprofv3 --pmc FETCH_SIZE /
// WRITE_SIZE): the fast kernel's own access pattern -- per-lane 16-byte X records and 8-byte U records
// [rows][B][W] through one buffer resource, loaded and stored row by row -- copied from src to dst, so
// the counters' ratio to the known bytes corrects the tube step's figures (MI355X_MICROARCH.md §HBM:
// "calibrate on a known byte count in your own access pattern").
__global__ void __launch_bounds__(kBlock) record_stream_kernel(const real* src, real* dst, int B, int N,
                                                               unsigned bytes) {
  const int t = blockIdx.x * kBlock + threadIdx.x;
  if (t >= B) return;
  const Rsrc rs = __builtin_amdgcn_make_buffer_rsrc((void*)src, 0, (int)bytes, 0x00020000);
  const Rsrc rd = __builtin_amdgcn_make_buffer_rsrc(dst, 0, (int)bytes, 0x00020000);
  const unsigned cb = (unsigned)B, X = cb * (N + 1) * (16u * ES);
  const RA XA{0, cb * (16u * ES), (unsigned)t * (16u * ES)}, UA{X, cb * (8u * ES), (unsigned)t * (8u * ES)};
  for (int k = 0; k <= N; ++k) {
    rst4(rd, XA, k, 0, rld4(rs, XA, k, 0));
    if (k < N) rst2(rd, UA, k, 0, rld2(rs, UA, k, 0));
  }
}

// The headline kernel's record stream on its own (what HBM delivers to THIS access pattern at THIS
// occupancy, not to a float4 copy at full occupancy): one lane per trajectory, per pass and step one 16-B X row and
// one 8-B U row of the current bank and one 32-B gain record read, the other bank's X and U rows written -- 56 B
// read : 24 B written (70 % read, the step's measured mix is 69 %), every access a buffer access with the row base
// in soffset and the lane's record in voffset, as the tube kernel addresses them; loads issued D steps ahead (a ring
// of D + 1 rows).  Records: bank 0 X [N][B][4] U [N][B][2], bank 1 the same, K [N][B][8] (80 B per trajectory-step).
template <int D>
__global__ void __launch_bounds__(kBlock) stream_probe_kernel(real* base, int B, int N, int passes, unsigned bytes) {
  const int t = blockIdx.x * kBlock + threadIdx.x;
  if (t >= B) return;
  const Rsrc r = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, (int)bytes, 0x00020000);
  const unsigned cb = (unsigned)B, X = cb * N * 16u, U = cb * N * 8u;
  const RA XA[2] = {{0, cb * 16u, (unsigned)t * 16u}, {X + U, cb * 16u, (unsigned)t * 16u}};
  const RA UA[2] = {{X, cb * 8u, (unsigned)t * 8u}, {2 * X + U, cb * 8u, (unsigned)t * 8u}};
  const RA KA{2 * (X + U), cb * 32u, (unsigned)t * 32u};
  for (int p = 0; p < passes; ++p) {
    const int s = p & 1;
    f4 xq[D + 1], ka[D + 1], kb[D + 1];
    f2 uq[D + 1];
#pragma unroll
    for (int j = 0; j < D; ++j) {
      xq[j] = rld4(r, XA[s], j, 0);
      uq[j] = rld2(r, UA[s], j, 0);
      ka[j] = rld4(r, KA, j, 0);
      kb[j] = rld4(r, KA, j, 16);
    }
    for (int k = 0; k < N; k += D + 1) {
#pragma unroll
      for (int j = 0; j <= D; ++j) {
        const int kk = k + j, kn = uidx(kk + D < N ? kk + D : N - 1);
        const int q = (j + D) % (D + 1);
        xq[q] = rld4(r, XA[s], kn, 0);
        uq[q] = rld2(r, UA[s], kn, 0);
        ka[q] = rld4(r, KA, kn, 0);
        kb[q] = rld4(r, KA, kn, 16);
        if (kk >= N) break;
        rst4(r, XA[1 - s], kk, 0, xq[j] + ka[j]);
        rst2(r, UA[1 - s], kk, 0, uq[j] + f2{kb[j].x, kb[j].y});
      }
    }
  }
}
#endif

// ---------------------------------------------------------------------------------------------
// the standalone batched iLQR (dtmpc_ilqr_solve_ws; core/ddp.py:102-307 ilqr_solve) on the fast
// configuration: the tube step's solver -- the same ilqr() with its lane forms, tape slots and records --
// run once over a batch of (x0, V_init[, X_ref, U_ref]).  The ABI arrays are the generic kernel's:
// x0 [4][B], Xref [N+1][3][B], Uref [N][2][B], X [N+1][4][B], U [N][2][B] (in: V_init, out: V*),
// K [N][8][B] / kff [N][2][B] out (the last backward pass's gains), iters / status [B], choices.
// Workspace records of one chunk (Bc trajectories): X [N+1][NS][Bc][4], U [N][NS][Bc][2],
// gains K [N][Bc][8] + k [N][Bc][2], the tracking references XR [N+1][Bc][4] / UR [N][Bc][2].
struct IArgs {
  int B, i0, Bc;
  const real* x0;
  const real* Xref;
  const real* Uref;
  real* X;
  real* U;
  real* K;
  real* kff;
  int* iters;
  int* status;
  signed char* choices;
  real* costs;
  real* work;
  unsigned wsz, oX, oU, oK, ok, oXR, oUR;
};
struct IK {
  FP p;
  FCost c;
  FIlqr cf;
  IArgs a;
};
__device__ __forceinline__ const IK* ikargs() {
  __attribute__((address_space(4))) const IK* k =
      (__attribute__((address_space(4))) const IK*)__builtin_amdgcn_kernarg_segment_ptr();
  __asm__ volatile("" : "+s"(k));
  return (const IK*)k;
}

template <int M, int P, bool TRACK, int GM>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(1, 1)))
ilqr_fast_kernel(IK kk) {
  constexpr bool G0 = GM > 0, RG0 = GM > 1;
  (void)kk;  // read through ikargs()
  const IArgs& a = ikargs()->a;
  constexpr int ML = M | tab_flag<M, GM>() | xasm_flag<M, GM, P>();
  obs_fill<ML>(ikargs()->p);
  const int B = a.B, Bc = a.Bc, i0 = a.i0;
  const int gl = blockIdx.x * blockDim.x + threadIdx.x;
  const int t = gl / P, h = gl % P;
  const int i = i0 + t;
  if (t >= Bc) return;
  const size_t nb = (size_t)B;
  const unsigned lo = (unsigned)i * (4u * ES), bb = (unsigned)B * (4u * ES);
  const Lane L{lo, lo + bb, lo + 2u * bb, lo + 3u * bb};
  constexpr unsigned NS = P == 4 ? kSlots : 1;
  const unsigned cb = (unsigned)Bc, l8 = (unsigned)t * (8u * ES), l16 = (unsigned)t * (16u * ES), l32 = (unsigned)t * (32u * ES);
  const SlotMap sm{l16, cb * (16u * ES), l8, cb * (8u * ES)};
  const unsigned x0lo = P == 4 ? l16 + kSlotInit * cb * (16u * ES) : l16, u0lo = P == 4 ? l8 + kSlotInit * cb * (8u * ES) : l8;
  Solve<TRACK, G0, RG0, P, NC, false> S;  // caller references: read, never re-rolled (RROLL)
  S.r = __builtin_amdgcn_make_buffer_rsrc(a.work, 0, (int)a.wsz, 0x00020000);
  S.XA = RA{a.oX, NS * cb * (16u * ES), x0lo};
  S.UA = RA{a.oU, NS * cb * (8u * ES), u0lo};
  S.XRA = RA{a.oXR, cb * (16u * ES), l16};
  S.URA = RA{a.oUR, cb * (8u * ES), l8};
  S.G.K = RA{a.oK, cb * (32u * ES), l32};
  S.G.k = RA{a.ok, cb * (8u * ES), l8};
  S.X = Soa<4>{(char*)a.X, 4u * bb, L};
  S.U = Soa<2>{(char*)a.U, 2u * bb, L};
  const FP p = pin_p<ML>(ikargs()->p);
  const int N = p.N;
  if (TRACK) {  // the references into records (the lanes of a trajectory split the rows; one wave: in order)
    for (int k = h; k <= N; k += P) {
      const real* q = a.Xref + (size_t)k * 3 * nb + i;
      rst4(S.r, S.XRA, k, 0, f4{q[0], q[nb], q[2 * nb], 0.f});
      if (k < N) {
        const real* w = a.Uref + (size_t)k * 2 * nb + i;
        rst2(S.r, S.URA, k, 0, f2{w[0], w[nb]});
      }
    }
  }
  const real x0[4] = {a.x0[i], a.x0[nb + i], a.x0[2 * nb + i], a.x0[3 * nb + i]};
  const FCost c = ikargs()->c;
  const FIlqr cf = ikargs()->cf;
  const DecRec dr{a.choices ? a.choices + i : nullptr, a.costs ? a.costs + i : nullptr, nb};
  int it = 0;
  Prof pf;
  pf.start();
  const int st = ilqr<TRACK, ML, P, false>(p, c, cf, x0, S, h, sm, it, pf, dr);
  // the last backward pass's gains out to the ABI arrays (G0 records: K's barrier column is exactly 0);
  // max_iter = 0: no backward pass ran and the records were never written -- zeros, as the generic kernel
  // leaves the zeroed arrays
  const bool have_gains = cf.max_iter > 0;
  for (int k = h; k < N; k += P) {
    f4 Ka = f4{0.f, 0.f, 0.f, 0.f}, Kb = f4{0.f, 0.f, 0.f, 0.f};
    f2 kf = f2{0.f, 0.f};
    if (have_gains) S.G.template load<G0>(S.r, k, Ka, Kb, kf);
    real* Kq = a.K + (size_t)k * 8 * nb + i;
    Kq[0] = Ka.x;
    Kq[nb] = Ka.y;
    Kq[2 * nb] = Ka.z;
    Kq[3 * nb] = Ka.w;
    Kq[4 * nb] = Kb.x;
    Kq[5 * nb] = Kb.y;
    Kq[6 * nb] = Kb.z;
    Kq[7 * nb] = Kb.w;
    real* kq = a.kff + (size_t)k * 2 * nb + i;
    kq[0] = kf.x;
    kq[nb] = kf.y;
  }
  if (h == 0) {
    if (a.iters) a.iters[i] = it;
    a.status[i] |= st;
  }
}

// ---------------------------------------------------------------------------------------------
// the receding-horizon nominal MPC (dtmpc_nominal_receding; run_nominal.py:204-415) on the fused solver: per
// lane one trajectory's whole task horizon -- iLQR with the angle-wrapped target cost (kWrap) -> log x, u0, b
// -> the run's exits (non-finite solve, collision: the TRUE min_i h_i <= 0, success: ||p - target|| <= r)
// -> plant step x <- f_hat(x, u0) -> warm-start shift U <- [U[1:], U[-1]] -- as receding_kernel
// (dtmpc_receding.hip) does with the generic solver.  One lane per trajectory: the solves of different
// lanes stop at their own tol exits and the runs at their own exits.
// Workspace records of one chunk: X [N+1][Bc][4], U [N][Bc][2], gains K [N][Bc][8] + k [N][Bc][2]; the
// ABI-layout plan Xs [N+1][4][B] (copy_out's target) follows the records.
struct RArgs {
  int B, i0, Bc, H;
  real success_r;
  const real* x0;  // [3][B]
  real* U;         // [N][2][B] warm start in, the last shifted plan out
  real* Xs;        // [N+1][4][B] the plan in the ABI layout (scratch)
  real* log;       // [H][6][B]
  int* h_ran;
  int* success_t;
  int* collided;
  int* status;
  int* iters;  // [B] the run's total iLQR iterations (the receding leg's algorithmic bytes), or NULL
  real* work;
  unsigned wsz, oX, oU, oK, ok;
};
struct RK {
  FP p;
  FCost c;
  FIlqr cf;
  RArgs a;
};
__device__ __forceinline__ const RK* rkargs() {
  __attribute__((address_space(4))) const RK* k =
      (__attribute__((address_space(4))) const RK*)__builtin_amdgcn_kernarg_segment_ptr();
  __asm__ volatile("" : "+s"(k));
  return (const RK*)k;
}

// the true min_i h_i over the circles (run_nominal.py:388-397), rounded as h_circle_exact (no contraction)
template <int M>
__device__ __forceinline__ real h_true_min(const FP& p, real px, real py) {
#pragma clang fp contract(off)
  real m = 0.f;
#pragma unroll
  for (int i = 0; i < Obs<M>::n; ++i) {
    const real dx = px - ocx<M>(p, i), dy = py - ocy<M>(p, i);
    const real hi = dx * dx + dy * dy - or2<M>(p, i);
    m = i == 0 ? hi : m_min(m, hi);
  }
  return m;
}

template <int M, int GM>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(1, 1)))
receding_fast_kernel(RK kk) {
  constexpr bool G0 = GM > 0, RG0 = GM > 1;
  constexpr int ML = M | tab_flag<M, GM>() | xasm_flag<M, GM, 1>();
  constexpr int MW = ML | kWrap;
  (void)kk;  // read through rkargs()
  obs_fill<ML>(rkargs()->p);
  const RArgs& a = rkargs()->a;
  const int B = a.B, Bc = a.Bc, i0 = a.i0;
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int i = i0 + t;
  if (t >= Bc) return;
  const size_t nb = (size_t)B;
  const unsigned lo = (unsigned)i * (4u * ES), bb = (unsigned)B * (4u * ES);
  const Lane L{lo, lo + bb, lo + 2u * bb, lo + 3u * bb};
  const unsigned cb = (unsigned)Bc, l8 = (unsigned)t * (8u * ES), l16 = (unsigned)t * (16u * ES), l32 = (unsigned)t * (32u * ES);
  const SlotMap sm{l16, cb * (16u * ES), l8, cb * (8u * ES)};
  Solve<false, G0, RG0, 1> S;
  S.r = __builtin_amdgcn_make_buffer_rsrc(a.work, 0, (int)a.wsz, 0x00020000);
  S.XA = RA{a.oX, cb * (16u * ES), l16};
  S.UA = RA{a.oU, cb * (8u * ES), l8};
  S.XRA = S.XA;
  S.URA = S.UA;
  S.G.K = RA{a.oK, cb * (32u * ES), l32};
  S.G.k = RA{a.ok, cb * (8u * ES), l8};
  S.X = Soa<4>{(char*)a.Xs, 4u * bb, L};
  S.U = Soa<2>{(char*)a.U, 2u * bb, L};
  const FP p = pin_p<ML>(rkargs()->p);
  const FCost c = rkargs()->c;
  const FIlqr cf = rkargs()->cf;
  const int N = p.N, H = a.H;
  real x[4] = {a.x0[i], a.x0[nb + i], a.x0[2 * nb + i], 0.f};
  x[3] = barrier_at<ML>(p, x[0], x[1]);  // dbas_init_b0 (run_nominal.py:279)
  int st = 0, ran = H, sidx = -1, coll = 0, itot = 0;
  for (int ts = 0; ts < H; ++ts) {
    int it = 0;
    Prof pf;
    st |= ilqr<false, MW, 1, false>(p, c, cf, x, S, 0, sm, it, pf, DecRec{nullptr, nullptr, 0});
    itot += it;
    const f2 u = rld2(S.r, S.UA, 0, 0);  // the plan's first control (the records hold the solved plan)
    real* lg = a.log + (size_t)ts * 6 * nb + i;
    lg[0] = x[0];
    lg[nb] = x[1];
    lg[2 * nb] = x[2];
    lg[3 * nb] = u.x;
    lg[4 * nb] = u.y;
    lg[5 * nb] = x[3];
    if (st) {
      ran = ts + 1;
      break;
    }
    if (h_true_min<ML>(p, x[0], x[1]) <= real(0)) {  // collision (run_nominal.py:388-397)
      coll = 1;
      ran = ts + 1;
      break;
    }
    {
      DTMPC_NOCONTRACT
      const real ex = x[0] - c.tg.x, ey = x[1] - c.tg.y;
      if (sqrt(ex * ex + ey * ey) <= a.success_r) {  // success (run_nominal.py:399-403)
        sidx = ts;
        ran = ts + 1;
        break;
      }
    }
    // x <- f_hat(x, u0) (run_nominal.py:377-378)
    real Bc = barrier_at<ML>(p, x[0], x[1]);
    fhat<ML, G0>(p, x[0], x[1], x[2], x[3], u.x, u.y, Bc);
    // U <- [U[1:], U[-1]] (run_nominal.py:405-406) on the ABI warm start the next solve starts from
    for (int k = 0; k + 1 < N; ++k) {
      S.U.st(k, 0, S.U.ld(k + 1, 0));
      S.U.st(k, 1, S.U.ld(k + 1, 1));
    }
  }
  a.h_ran[i] = ran;
  a.success_t[i] = sidx;
  a.collided[i] = coll;
  a.status[i] |= st;
  if (a.iters) a.iters[i] = itot;
}

// ---------------------------------------------------------------------------------------------
// the general path's two solves (dtmpc_general_step; core/tube_mpc.py:217-392): the nominal MPC with
// theta-bar (softplus weights, DBaS alpha / gamma from tanh / softplus, the tightened h - s) and the
// ancillary MPC with theta tracking it, both on the fast solver (general gain records: gamma is a
// parameter).  The solved tapes go out to the ABI arrays unshifted (dtmpc_general_plant shifts them) and
// each trajectory's solve status to `sst`; dtmpc_general_step's sensitivity / IFT kernel follows.
struct GSArgs {
  int B, i0, Bc;
  const real* theta;  // [2][12] raw: row 0 ancillary theta, row 1 nominal theta-bar
  f4 tgt;
  const real* x;
  const real* b;
  const real* xbar;
  const real* bbar;
  real* Xnom;
  real* Unom;
  real* Xaux;
  real* Uaux;
  int* iters;
  int* sst;
  real* work;
  unsigned wsz, oXn, oUn, oXa, oUa, oK, ok;
};
struct GSK {
  FP p;
  FIlqr cfn, cfa;
  GSArgs a;
};
__device__ __forceinline__ const GSK* gskargs() {
  __attribute__((address_space(4))) const GSK* k =
      (__attribute__((address_space(4))) const GSK*)__builtin_amdgcn_kernarg_segment_ptr();
  __asm__ volatile("" : "+s"(k));
  return (const GSK*)k;
}

// the DBaS constants of a parameterised solve, formed in f32 on the device as the generic kernels form
// them (barrier_relaxed: a = max(alpha, eps), 1 / a and 1 / a^2 correctly rounded)
__device__ __forceinline__ FP general_fp(FP p, const GPar<real>& g) {
  DTMPC_NOCONTRACT
  p.gamma = g.gamma;
  p.tight = g.tight;
  p.a = g.alpha > p.eps ? g.alpha : p.eps;
  p.a2 = p.a * p.a;
  p.a3 = p.a2 * p.a;
  p.inv_a = 1.f / p.a;
  p.inv_a2 = 1.f / p.a2;
  return p;
}

// one solve of the general path on its records: G0 when the solve's gamma is exactly 0 (the compact gain
// records and the Riccati step without the barrier column, as the tube step's default; gamma comes from
// theta on the device, so the kernel branches -- uniformly -- between the two instantiations).  XA / UA
// come back as the solved tape's records (P = 4: its final slot).
template <bool TRACK, int M, int P, int NCV, bool G0>
__device__ __forceinline__ int general_solve(const FP& p, const FCost& c, const FIlqr& cf, const real* x0, Rsrc r,
                                             RA& XA, RA& UA, const RA& XRA, const RA& URA, const Gains<P>& G,
                                             const Soa<4>& X, const Soa<2>& U, int h, const SlotMap& sm, int& it,
                                             Prof& pf) {
  Solve<TRACK, G0, G0, P, NCV> S;
  S.r = r;
  S.XA = XA;
  S.UA = UA;
  S.XRA = XRA;
  S.URA = URA;
  S.G = G;
  S.X = X;
  S.U = U;
  const int st = ilqr<TRACK, M, P, false>(p, c, cf, x0, S, h, sm, it, pf, DecRec{nullptr, nullptr, 0});
  XA = S.XA;
  UA = S.UA;
  return st;
}

template <int M, int P, int NCV>
__global__ void __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(1, 1)))
general_solve_fast_kernel(GSK kk) {
  (void)kk;  // read through gskargs()
  constexpr int ML = M | tab_flag<M, 0>();  // both record forms in one kernel: placed as the general records
  obs_fill<ML>(gskargs()->p);
  const GSArgs& a = gskargs()->a;
  const int B = a.B, Bc = a.Bc, i0 = a.i0;
  const int gl = blockIdx.x * blockDim.x + threadIdx.x;
  const int t = gl / P, h = gl % P;
  const int i = i0 + t;
  if (t >= Bc) return;
  const size_t nb = (size_t)B;
  const unsigned lo = (unsigned)i * (4u * ES), bb = (unsigned)B * (4u * ES);
  const Lane L{lo, lo + bb, lo + 2u * bb, lo + 3u * bb};
  constexpr unsigned NS = P == 4 ? kSlots : 1;
  const unsigned cb = (unsigned)Bc, l8 = (unsigned)t * (8u * ES), l16 = (unsigned)t * (16u * ES), l32 = (unsigned)t * (32u * ES);
  const SlotMap sm{l16, cb * (16u * ES), l8, cb * (8u * ES)};
  const unsigned x0lo = P == 4 ? l16 + kSlotInit * cb * (16u * ES) : l16, u0lo = P == 4 ? l8 + kSlotInit * cb * (8u * ES) : l8;
  Gains<P> G;
  G.K = RA{a.oK, cb * (32u * ES), l32};
  G.k = RA{a.ok, cb * (8u * ES), l8};
  const Rsrc r = __builtin_amdgcn_make_buffer_rsrc(a.work, 0, (int)a.wsz, 0x00020000);
  int st = 0, itn = 0, ita = 0;
  Prof pf;
  pf.start();
  RA XN{a.oXn, NS * cb * (16u * ES), x0lo}, UN{a.oUn, NS * cb * (8u * ES), u0lo};
  {  // nominal MPC with theta-bar (:217-291)
    const GPar<real> pn = gpar_from<real>(a.theta + DTMPC_P_COUNT, true);
    const FP p = pin_p<ML | kTight>(general_fp(gskargs()->p, pn));
    const FCost cn{pn.Q[0], pn.Q[1], pn.Q[2], pn.R[0], pn.R[1], pn.Qf[0], pn.Qf[1], pn.Qf[2], pn.qb, a.tgt};
    const FIlqr cfn = gskargs()->cfn;
    const real xn0[4] = {a.xbar[i], a.xbar[nb + i], a.xbar[2 * nb + i], a.bbar[i]};
    const Soa<4> X{(char*)a.Xnom, 4u * bb, L};
    const Soa<2> U{(char*)a.Unom, 2u * bb, L};
    if (pn.gamma == 0.f)
      st |= general_solve<false, ML | kTight, P, NCV, true>(p, cn, cfn, xn0, r, XN, UN, XN, UN, G, X, U, h, sm, itn, pf);
    else
      st |= general_solve<false, ML | kTight, P, NCV, false>(p, cn, cfn, xn0, r, XN, UN, XN, UN, G, X, U, h, sm, itn, pf);
  }
  {  // ancillary MPC with theta tracking the nominal plan as solved (:296-392)
    RA XA{a.oXa, NS * cb * (16u * ES), x0lo}, UA{a.oUa, NS * cb * (8u * ES), u0lo};
    const GPar<real> pa = gpar_from<real>(a.theta, false);
    const FP p = pin_p<ML>(general_fp(gskargs()->p, pa));
    const FCost ca{pa.Q[0], pa.Q[1], pa.Q[2], pa.R[0], pa.R[1], pa.Qf[0], pa.Qf[1], pa.Qf[2], pa.qb,
                   f4{0.f, 0.f, 0.f, 0.f}};
    const FIlqr cfa = gskargs()->cfa;
    const real xa0[4] = {a.x[i], a.x[nb + i], a.x[2 * nb + i], a.b[i]};
    const Soa<4> X{(char*)a.Xaux, 4u * bb, L};
    const Soa<2> U{(char*)a.Uaux, 2u * bb, L};
    if (pa.gamma == 0.f)
      st |= general_solve<true, ML, P, NCV, true>(p, ca, cfa, xa0, r, XA, UA, XN, UN, G, X, U, h, sm, ita, pf);
    else
      st |= general_solve<true, ML, P, NCV, false>(p, ca, cfa, xa0, r, XA, UA, XN, UN, G, X, U, h, sm, ita, pf);
  }
  if (h == 0) {
    a.sst[i] = st;
    if (a.iters) {
      a.iters[i] = itn;
      a.iters[nb + i] = ita;
    }
  }
}


}  // namespace FK_NS

// ---------------------------------------------------------------------------------------------
// host side
using FK_NS::ES;
using FK_NS::real;
constexpr int kFastDtype = DTMPC_FAST_F64 ? DTMPC_F64 : DTMPC_F32;  // the precision this unit instantiates

static bool fast_spec_ok(const dtmpc_spec* sp) {
  return sp->obs_aggregation == DTMPC_OBS_SMOOTHMIN && sp->n_obstacles >= 1 && sp->n_obstacles <= 8 &&
         sp->barrier_type == DTMPC_BARRIER_INVERSE && sp->h_offset == 0.0;
}

static FK_NS::FIlqr fast_ilqr(const dtmpc_ilqr_cfg& c) {
  const DIlqr<real> d = make_ilqr<real>(c);
  FK_NS::FIlqr o;
  o.max_iter = d.max_iter;
  o.zpos = d.zpos;
  o.tol = d.tol;
  o.reg = d.reg;
  for (int q = 0; q < FK_NS::NC; ++q) {
    o.cal[q] = d.calphas[q];
    o.cpos[q] = d.cpos[q];
  }
  return o;
}

static void fast_p(const dtmpc_spec* sp, FK_NS::FP& p) {
  const DSpec<real> s = make_spec<real>(*sp);
  p.N = s.N;
  p.dt = s.dt;
  p.umin0 = s.umin0;
  p.umin1 = s.umin1;
  p.umax0 = s.umax0;
  p.umax1 = s.umax1;
  p.active_tol = s.active_tol;
  p.neg_beta = s.neg_beta;
  p.neg_inv_beta = s.neg_inv_beta;
  p.nbl2e = s.neg_beta * 1.44269504088896341f;
  p.eps = s.eps;
  p.gamma = s.gamma;
  // alpha_eff = max(alpha, eps) and the constants of the relaxed branch, in f32 as the device forms them
  p.a = s.alpha > s.eps ? s.alpha : s.eps;
  p.a2 = p.a * p.a;
  p.a3 = p.a2 * p.a;
  volatile real one = 1.0f;  // f32 division on the host: correctly rounded, as the device's
  p.inv_a = one / p.a;
  p.inv_a2 = one / p.a2;
  for (int i = 0; i < 8; ++i) {
    p.cx[i] = i < s.M ? s.cx[i] : 0.f;
    p.cy[i] = i < s.M ? s.cy[i] : 0.f;
    p.r2[i] = i < s.M ? s.r2[i] : 0.f;
  }
}

#if DTMPC_FAST_ILP_SPLIT
// the tube step's launches of the split units (dtmpc_fast_ilp.hip / dtmpc_fast64_ilp.hip): M obstacles, lanes 1 (or
// 2 where DTMPC_FAST_ILP_P2), record form g0
int FKN(launch_tube_fast_ilp)(int M, int lanes, int g0, dim3 grid, unsigned bs, hipStream_t st, const FK_NS::FK& kk);
#endif

#ifndef DTMPC_FAST_AUX_TU  // the tube step (this file's own translation unit)

// The fast kernel's configuration: f32, smooth-min over 1..8 obstacles, relaxed inverse barrier,
// untightened h, nominal target cost without wrap, and six rolled-out candidates in both solves.
// DTMPC_FAST=0 (environment, read at the call) forces the generic kernel (parity tests compare both).
//
// Workspace records of one launch chunk of Bc trajectories (NS = 12 tape slots per solve at four lanes,
// else 1): nominal and ancillary X [N+1][NS][Bc][4], U [N][NS][Bc][2]; gains K [N][Bc][8], k [N][Bc][2];
// sensitivity scratch A8 [N][Bc][8], A2 [N][Bc][2].  All of it addressed through one buffer resource, so a
// chunk's records stay below 2^31 bytes (tube_fast_chunk_max); larger batches run in chunks.
struct FastLayout {
  unsigned oXn, oXa, oUn, oUa, oK, ok, oA8, oA2, oPH, wsz;
};
static int64_t fast_bytes_per_traj(int N, int lanes) {
  const int64_t ns = lanes == 4 ? FK_NS::kSlots : 1;
  return ns * ((int64_t)(N + 1) * 32 * ES + (int64_t)N * 16 * ES) + (int64_t)N * 80 * ES + 12;  // + hand-over
}
static FastLayout fast_layout(int N, int64_t Bc, int lanes) {
  const int64_t ns = lanes == 4 ? FK_NS::kSlots : 1;
  const unsigned X = (unsigned)(ns * Bc * (N + 1) * 16 * ES), U = (unsigned)(ns * Bc * N * 8 * ES);
  const unsigned K = (unsigned)(Bc * N * 32 * ES), k = (unsigned)(Bc * N * 8 * ES);
  FastLayout f;
  f.oXn = 0;
  f.oXa = X;
  f.oUn = 2 * X;
  f.oUa = 2 * X + U;
  f.oK = 2 * X + 2 * U;
  f.ok = f.oK + K;
  f.oA8 = f.ok + k;
  f.oA2 = f.oA8 + K;
  f.oPH = f.oA2 + k;
  f.wsz = f.oPH + (unsigned)(Bc * 12);
  return f;
}
int64_t FKN(tube_fast_chunk_max)(int N, int lanes) {
  const int64_t c = ((int64_t)0x7fffffff / fast_bytes_per_traj(N, lanes)) / kBlock * kBlock;
  return c < kBlock ? kBlock : c;
}
size_t FKN(tube_fast_workspace_bytes)(int N, int64_t B, int lanes, int64_t chunk) {
  const int64_t b = B < chunk ? B : chunk;
  return (size_t)b * (size_t)fast_bytes_per_traj(N, lanes);
}

bool FKN(tube_fast_eligible)(int dtype, const dtmpc_spec* sp, const dtmpc_tube_cfg* cf) {
  const char* e = getenv(DTMPC_FAST_F64 ? "DTMPC_FAST64" : "DTMPC_FAST");  // "0": the generic kernel (A/B, tests)
  if (e && e[0] == '0' && e[1] == 0) return false;
  if (DTMPC_FAST_F64 && (e = getenv("DTMPC_FAST")) && e[0] == '0' && e[1] == 0) return false;
  if (dtype != kFastDtype || !fast_spec_ok(sp)) return false;
  if (cf->nominal.kind != DTMPC_COST_TARGET || cf->nominal.wrap_angle) return false;
  const DIlqr<real> n = make_ilqr<real>(cf->nom_ilqr), a = make_ilqr<real>(cf->aux_ilqr);
  return n.nc == FK_NS::NC && a.nc == FK_NS::NC;
}

// the record form a launch takes: 2 the compact gamma = 0 records and recursion (the default at gamma = 0), 1 the
// compact records with the general recursion, 0 the general records; DTMPC_FAST_G0 = 0 / 1 (environment, read at
// each call) lowers it for the A/B tests
static int fast_g0(const dtmpc_spec* sp) {
  int g0 = sp->dbas_gamma == 0.0 ? 2 : 0;
  if (const char* e = getenv("DTMPC_FAST_G0"))
    if ((e[0] == '0' || e[0] == '1') && e[1] == 0) g0 = g0 < e[0] - '0' ? g0 : e[0] - '0';
  return g0;
}

#if DTMPC_FAST_F64
// f64 general gain records at four lanes.  Round 5 v2 ran them on the generic f64 kernel: the fused form gave
// run-to-run different results at some obstacle counts and not at others, moving with every change of the kernel.
// The cause was the store-data hazard of the 128-bit record stores (st128; every f64 record store is 128-bit):
// since v3 the family runs fused (scripts/diag_records.py: every M = 1-8 at four lanes within 1e-8 of the generic
// kernel, twice bitwise equal; profiles/r05/diag_records_v3.txt).  DTMPC_FAST64_L4G=0 routes it to the generic
// kernel again (A/B only).
bool tube_fast_lanes_ok64(const dtmpc_spec* sp, int lanes) {
  static const bool generic = [] {
    const char* e = getenv("DTMPC_FAST64_L4G");
    return e && e[0] == '0';
  }();
  return !(generic && lanes == 4 && fast_g0(sp) == 0);
}
#endif

int FKN(launch_tube_fast)(const dtmpc_spec* sp, const dtmpc_tube_cfg* cf, int64_t B, int64_t goff, int64_t step,
                     const dtmpc_tube_state* S, const void* w, hipStream_t st) {
  FK_NS::FK kk;
  std::memset(&kk, 0, sizeof(kk));
  fast_p(sp, kk.p);
  const DCost<real> c = make_cost<real>(cf->nominal);
  kk.cn = FK_NS::FCost{c.Q0, c.Q1, c.Q2, c.R0, c.R1, c.Qf0, c.Qf1, c.Qf2, c.qb, FK_NS::f4{c.t0, c.t1, c.t2, 0.f}};
  kk.cfn = fast_ilqr(cf->nom_ilqr);
  kk.cfa = fast_ilqr(cf->aux_ilqr);
  FK_NS::FArgs& a = kk.a;
  const int N = sp->horizon;
  a.B = (int)B;
  a.goff = goff;
  a.step = step;
  a.x = (real*)S->x;
  a.b = (real*)S->b;
  a.xbar = (real*)S->xbar;
  a.bbar = (real*)S->bbar;
  a.Xnom = (real*)S->Xnom;
  a.Unom = (real*)S->Unom;
  a.Xaux = (real*)S->Xaux;
  a.Uaux = (real*)S->Uaux;
  a.work = (real*)S->work;
  a.theta = (const real*)S->theta;
  a.partials = (real*)S->partials;
  a.log = (real*)S->log;
  a.status = S->status;
  a.iters = S->iters;
  a.w = (const real*)w;
  a.choices = (signed char*)S->choices;
  a.costs = (real*)S->costs;
  a.gbound = cf->grad_bound > 0 ? real(cf->grad_bound) : real(__builtin_inf());
  a.disturbance = cf->disturbance;
  a.write_log = (cf->write_log && S->log) ? 1 : 0;
  a.seed = cf->seed;
  for (int f = 0; f < 3; ++f) {
    a.wlo[f] = real(cf->w_low[f]);
    a.whi[f] = real(cf->w_high[f]);
  }
  const int lanes = S->lanes;
  a.phase = S->phase;
  // gamma = 0 (the paper's DBaS): the compact gain records (FK_NS::Gains) and the Riccati step without the
  // barrier state's zero column (riccati_pk<true>).  DTMPC_FAST_G0 (environment, read at each call) = 0
  // keeps the general records and recursion, = 1 the compact records with the general recursion: the
  // tests compare 1 with 0 for exact equality (records) and the default with the oracle builds.
  const int g0 = fast_g0(sp);
#if DTMPC_FAST_F64
  if (!tube_fast_lanes_ok64(sp, lanes)) return set_err(DTMPC_ERR_BAD_ARG, "f64 general records at four lanes run the generic kernel");
#endif
  {
    const char* e = getenv("DTMPC_FAST_STAGGER");  // sleep rounds of ~8.1k cycles (A/B; default 0)
    a.stagger = e ? atoi(e) : 0;
  }
  // the batch in chunks whose workspace records fit one buffer resource (< 2^31 bytes), each chunk a
  // multiple of the workgroup size (its partial-sum rows follow the previous chunk's); the chunk comes
  // from the state (dtmpc_tube_chunk, validated against the workspace by dtmpc_tube_step)
  // (f64 records are twice as large: its chunk is at most half the f32 one, dtmpc_tube_workspace_bytes)
  const int64_t cmax = FKN(tube_fast_chunk_max)(N, lanes), chunk = S->chunk < cmax ? S->chunk : cmax;
  // a split step keeps the nominal solve's records between its two launches: one chunk's worth of workspace
  if (S->phase != 0 && B > chunk) return set_err(DTMPC_ERR_BAD_ARG, "a split step (state->phase 1 / 2) needs B <= chunk");
  for (int64_t c0 = 0; c0 < B; c0 += chunk) {
    const int64_t Bc = B - c0 < chunk ? B - c0 : chunk;
    a.i0 = (int)c0;
    a.Bc = (int)Bc;
    const FastLayout f = fast_layout(N, Bc, lanes);
    a.oXn = f.oXn;
    a.oXa = f.oXa;
    a.oUn = f.oUn;
    a.oUa = f.oUa;
    a.oK = f.oK;
    a.ok = f.ok;
    a.oA8 = f.oA8;
    a.oA2 = f.oA2;
    a.oPH = f.oPH;
    a.wsz = f.wsz;
    const int bs = tube_block(B, lanes);  // 64 while the batch leaves SIMDs idle: one wave per workgroup
    const dim3 grid = dim3((unsigned)((Bc * lanes + bs - 1) / bs));
#define FAST_LAUNCH(m, l, g) hipLaunchKernelGGL((FK_NS::tube_fast_kernel<m, l, g>), grid, dim3(bs), 0, st, kk)
#define FAST_LANES(m, l) \
  if (g0 == 2) FAST_LAUNCH(m, l, 2); else if (g0) FAST_LAUNCH(m, l, 1); else FAST_LAUNCH(m, l, 0);
#ifdef DTMPC_FAST_ISA_ONLY  // ISA inspection builds: one instantiation (lanes 1, gamma = 0 records + Riccati)
#define FAST_CASE(m) \
  case m:            \
    FAST_LAUNCH(m, DTMPC_FAST_ISA_ONLY, 2); break;
#else
#define FAST_CASE(m)                                                                                       \
  case m:                                                                                                  \
    if (lanes == 4) {                                                                                      \
      FAST_LANES(m, 4)                                                                                     \
    } else if (lanes == 2) {                                                                               \
      FAST_LANES_P2(m)                                                                                     \
    } else {                                                                                               \
      FAST_LANES_P1(m)                                                                                     \
    }                                                                                                      \
    break;
#endif
#if DTMPC_FAST_ILP_SPLIT
#define FAST_LANES_P1(m) \
  if (int r = FKN(launch_tube_fast_ilp)(m, 1, g0, grid, bs, st, kk)) return r;
#else
#define FAST_LANES_P1(m) FAST_LANES(m, 1)
#endif
#if DTMPC_FAST_ILP_P2
#define FAST_LANES_P2(m) \
  if (int r = FKN(launch_tube_fast_ilp)(m, 2, g0, grid, bs, st, kk)) return r;
#else
#define FAST_LANES_P2(m) FAST_LANES(m, 2)
#endif
    switch (sp->n_obstacles) {
#ifdef DTMPC_FAST_M_ONLY
      FAST_CASE(DTMPC_FAST_M_ONLY)
#else
      FAST_CASE(1) FAST_CASE(2) FAST_CASE(3) FAST_CASE(4) FAST_CASE(5) FAST_CASE(6) FAST_CASE(7) FAST_CASE(8)
#endif
      default: return set_err(DTMPC_ERR_BAD_ARG, "fast tube step: obstacle count not instantiated");
    }
#undef FAST_CASE
#undef FAST_LANES_P2
#undef FAST_LANES_P1
#undef FAST_LANES
#undef FAST_LAUNCH
  }
  return check_launch("tube_fast_kernel");
}

#elif defined(DTMPC_FAST_ILP_TU)  // the split units' tube kernels (csrc/dtmpc_fast_ilp.hip, dtmpc_fast64_ilp.hip)

#if DTMPC_FAST_ILP_SPLIT
int FKN(launch_tube_fast_ilp)(int M, int lanes, int g0, dim3 grid, unsigned bs, hipStream_t st, const FK_NS::FK& kk) {
#define ILP_LAUNCH(m, l, g) hipLaunchKernelGGL((FK_NS::tube_fast_kernel<m, l, g>), grid, dim3(bs), 0, st, kk)
#define ILP_LANES(m, l) \
  if (g0 == 2) ILP_LAUNCH(m, l, 2); else if (g0) ILP_LAUNCH(m, l, 1); else ILP_LAUNCH(m, l, 0);
#if DTMPC_FAST_ILP_P2
#define ILP_CASE(m)         \
  case m:                   \
    if (lanes == 2) {       \
      ILP_LANES(m, 2)       \
    } else {                \
      ILP_LANES(m, 1)       \
    }                       \
    return 0;
#else
#define ILP_CASE(m) \
  case m:           \
    ILP_LANES(m, 1) \
    return 0;
#endif
  if (lanes != 1 && !(DTMPC_FAST_ILP_P2 && lanes == 2)) return set_err(DTMPC_ERR_BAD_ARG, "split tube unit: lanes");
  switch (M) {
#ifdef DTMPC_FAST_M_ONLY
    ILP_CASE(DTMPC_FAST_M_ONLY)
#else
    ILP_CASE(1) ILP_CASE(2) ILP_CASE(3) ILP_CASE(4) ILP_CASE(5) ILP_CASE(6) ILP_CASE(7) ILP_CASE(8)
#endif
    default: return set_err(DTMPC_ERR_BAD_ARG, "fast tube step: obstacle count not instantiated");
  }
#undef ILP_CASE
#undef ILP_LANES
#undef ILP_LAUNCH
}
#endif

#elif defined(DTMPC_FAST_ILQR_TU)  // the standalone iLQR (csrc/dtmpc_fast_ilqr.hip)

// the standalone solve's records per trajectory: X / U slots, gains K + k, tracking references
static int64_t ilqr_fast_bytes_per_traj(int N, int lanes) {
  const int64_t ns = lanes == 4 ? FK_NS::kSlots : 1;
  return ns * ((int64_t)(N + 1) * 16 * ES + (int64_t)N * 8 * ES) + (int64_t)N * 40 * ES + (int64_t)(N + 1) * 16 * ES + (int64_t)N * 8 * ES;
}
int64_t FKN(ilqr_fast_chunk_max)(int N, int lanes) {
  const int64_t c = ((int64_t)0x7fffffff / ilqr_fast_bytes_per_traj(N, lanes)) / kBlock * kBlock;
  return c < kBlock ? kBlock : c;
}
size_t FKN(ilqr_fast_workspace_bytes)(int N, int64_t B, int lanes) {
  const int64_t ch = FKN(ilqr_fast_chunk_max)(N, lanes), b = B < ch ? B : ch;
  return (size_t)b * (size_t)ilqr_fast_bytes_per_traj(N, lanes);
}

bool FKN(ilqr_fast_eligible)(int dtype, const dtmpc_spec* sp, const dtmpc_cost* c, const dtmpc_ilqr_cfg* cf) {
  const char* e = getenv("DTMPC_FAST");
  if (e && e[0] == '0' && e[1] == 0) return false;
  if (DTMPC_FAST_F64 && (e = getenv("DTMPC_FAST64")) && e[0] == '0' && e[1] == 0) return false;
  if (dtype != kFastDtype || !fast_spec_ok(sp) || c->wrap_angle) return false;
  return make_ilqr<real>(*cf).nc == FK_NS::NC;
}

int FKN(launch_ilqr_fast)(const dtmpc_spec* sp, const dtmpc_cost* cp, const dtmpc_ilqr_cfg* cf, int64_t B, const void* x0,
                     const void* Xref, const void* Uref, void* X, void* U, void* K, void* kff, int* iters, int* status,
                     signed char* choices, void* costs, int lanes, void* work, size_t work_bytes, hipStream_t st) {
  const int N = sp->horizon;
  if (lanes != 1 && lanes != 2 && lanes != 4) return set_err(DTMPC_ERR_BAD_ARG, "lanes must be 1, 2 or 4");
  if (!work || work_bytes < FKN(ilqr_fast_workspace_bytes)(N, B, lanes))
    return set_err(DTMPC_ERR_BAD_ARG, "work_bytes < dtmpc_ilqr_workspace_bytes(...)");
  FK_NS::IK kk;
  std::memset(&kk, 0, sizeof(kk));
  fast_p(sp, kk.p);
  const DCost<real> c = make_cost<real>(*cp);
  const bool track = cp->kind == DTMPC_COST_TRACK;
  kk.c = FK_NS::FCost{c.Q0, c.Q1, c.Q2, c.R0, c.R1, c.Qf0, c.Qf1, c.Qf2, c.qb,
                   track ? FK_NS::f4{0.f, 0.f, 0.f, 0.f} : FK_NS::f4{c.t0, c.t1, c.t2, 0.f}};
  kk.cf = fast_ilqr(*cf);
  FK_NS::IArgs& a = kk.a;
  a.B = (int)B;
  a.x0 = (const real*)x0;
  a.Xref = (const real*)Xref;
  a.Uref = (const real*)Uref;
  a.X = (real*)X;
  a.U = (real*)U;
  a.K = (real*)K;
  a.kff = (real*)kff;
  a.iters = iters;
  a.status = status;
  a.choices = choices;
  a.costs = (real*)costs;
  a.work = (real*)work;
  // gamma = 0: the compact gain records and the Riccati step without the barrier state's column
  const int g0 = kk.p.gamma == 0.f ? 2 : 0;
  const int64_t chunk = FKN(ilqr_fast_chunk_max)(N, lanes);
  for (int64_t c0 = 0; c0 < B; c0 += chunk) {
    const int64_t Bc = B - c0 < chunk ? B - c0 : chunk;
    const int64_t ns = lanes == 4 ? FK_NS::kSlots : 1;
    a.i0 = (int)c0;
    a.Bc = (int)Bc;
    a.oX = 0;
    a.oU = (unsigned)(ns * Bc * (N + 1) * 16 * ES);
    a.oK = a.oU + (unsigned)(ns * Bc * N * 8 * ES);
    a.ok = a.oK + (unsigned)(Bc * N * 32 * ES);
    a.oXR = a.ok + (unsigned)(Bc * N * 8 * ES);
    a.oUR = a.oXR + (unsigned)(Bc * (N + 1) * 16 * ES);
    a.wsz = a.oUR + (unsigned)(Bc * N * 8 * ES);
    const int bs = tube_block(B, lanes);
    const dim3 grid = dim3((unsigned)((Bc * lanes + bs - 1) / bs));
#define IL_LAUNCH(m, l, t, g) hipLaunchKernelGGL((FK_NS::ilqr_fast_kernel<m, l, t, g>), grid, dim3(bs), 0, st, kk)
#define IL_G(m, l, t) \
  if (g0 == 2) IL_LAUNCH(m, l, t, 2); else IL_LAUNCH(m, l, t, 0);
#define IL_T(m, l) \
  if (track) { IL_G(m, l, true) } else { IL_G(m, l, false) }
#define IL_CASE(m) \
  case m:          \
    if (lanes == 4) { IL_T(m, 4) } else if (lanes == 2) { IL_T(m, 2) } else { IL_T(m, 1) } break;
    switch (sp->n_obstacles) {
#if defined(DTMPC_FAST_M_ONLY)
      IL_CASE(DTMPC_FAST_M_ONLY)
#elif defined(DTMPC_FAST_ISA_ONLY)
      IL_CASE(5)
#else
      IL_CASE(1) IL_CASE(2) IL_CASE(3) IL_CASE(4) IL_CASE(5) IL_CASE(6) IL_CASE(7) IL_CASE(8)
#endif
      default: return set_err(DTMPC_ERR_BAD_ARG, "fast iLQR: obstacle count not instantiated");
    }
#undef IL_CASE
#undef IL_T
#undef IL_G
#undef IL_LAUNCH
  }
  return check_launch("ilqr_fast_kernel");
}

// the receding-horizon driver on the same solver (dtmpc_nominal_receding): the fast configuration with the
// nominal target cost and its heading error wrapped (run_nominal.py:297-324; receding_fast_kernel compiles the
// wrapped cost in, M | kWrap), one lane per trajectory.  An unwrapped target cost runs the generic receding_kernel.
bool FKN(receding_fast_eligible)(int dtype, const dtmpc_spec* sp, const dtmpc_cost* c, const dtmpc_ilqr_cfg* cf) {
  const char* e = getenv("DTMPC_FAST");
  if (e && e[0] == '0' && e[1] == 0) return false;
  if (DTMPC_FAST_F64 && (e = getenv("DTMPC_FAST64")) && e[0] == '0' && e[1] == 0) return false;
  if (dtype != kFastDtype || !fast_spec_ok(sp) || c->kind != DTMPC_COST_TARGET || !c->wrap_angle) return false;
  return make_ilqr<real>(*cf).nc == FK_NS::NC;
}
static int64_t receding_fast_bytes_per_traj(int N) {  // records X, U, K, k + the ABI-layout plan
  return (int64_t)(N + 1) * 16 * ES + (int64_t)N * 8 * ES + (int64_t)N * 40 * ES + (int64_t)(N + 1) * 16 * ES;
}
size_t FKN(receding_fast_workspace_bytes)(int N, int64_t B) { return (size_t)B * (size_t)receding_fast_bytes_per_traj(N); }

int FKN(launch_receding_fast)(const dtmpc_spec* sp, const dtmpc_cost* cp, const dtmpc_ilqr_cfg* cf, int64_t B, int H,
                              double success_r, const void* x0, void* U, void* log, int* h_ran, int* success_t,
                              int* collided, int* status, int* iters, void* work, hipStream_t st) {
  const int N = sp->horizon;
  FK_NS::RK kk;
  std::memset(&kk, 0, sizeof(kk));
  fast_p(sp, kk.p);
  const DCost<real> c = make_cost<real>(*cp);
  kk.c = FK_NS::FCost{c.Q0, c.Q1, c.Q2, c.R0, c.R1, c.Qf0, c.Qf1, c.Qf2, c.qb, FK_NS::f4{c.t0, c.t1, c.t2, 0.f}};
  kk.cf = fast_ilqr(*cf);
  FK_NS::RArgs& a = kk.a;
  a.B = (int)B;
  a.H = H;
  a.success_r = real(success_r);
  a.x0 = (const real*)x0;
  a.U = (real*)U;
  a.log = (real*)log;
  a.h_ran = h_ran;
  a.success_t = success_t;
  a.collided = collided;
  a.status = status;
  a.iters = iters;
  // the ABI-layout plan after every chunk's records (the records of one chunk below 2^31 bytes)
  const int64_t rec = receding_fast_bytes_per_traj(N) - (int64_t)(N + 1) * 16 * ES;
  const int64_t chunk = ((int64_t)0x7fffffff / rec) / kBlock * kBlock;
  a.Xs = (real*)((char*)work + (size_t)B * (size_t)rec);
  a.work = (real*)work;
  const int g0 = kk.p.gamma == 0.f ? 2 : 0;
  for (int64_t c0 = 0; c0 < B; c0 += chunk) {
    const int64_t Bc = B - c0 < chunk ? B - c0 : chunk;
    a.i0 = (int)c0;
    a.Bc = (int)Bc;
    a.work = (real*)((char*)work + (size_t)c0 * (size_t)rec);
    a.oX = 0;
    a.oU = (unsigned)(Bc * (N + 1) * 16 * ES);
    a.oK = a.oU + (unsigned)(Bc * N * 8 * ES);
    a.ok = a.oK + (unsigned)(Bc * N * 32 * ES);
    a.wsz = a.ok + (unsigned)(Bc * N * 8 * ES);
    const int bs = tube_block(B, 1);
    const dim3 grid = dim3((unsigned)((Bc + bs - 1) / bs));
#define RC_LAUNCH(m, g) hipLaunchKernelGGL((FK_NS::receding_fast_kernel<m, g>), grid, dim3(bs), 0, st, kk)
#define RC_CASE(m) \
  case m:          \
    if (g0 == 2) RC_LAUNCH(m, 2); else RC_LAUNCH(m, 0); break;
    switch (sp->n_obstacles) {
#if defined(DTMPC_FAST_M_ONLY)
      RC_CASE(DTMPC_FAST_M_ONLY)
#elif defined(DTMPC_FAST_ISA_ONLY)
      RC_CASE(5)
#else
      RC_CASE(1) RC_CASE(2) RC_CASE(3) RC_CASE(4) RC_CASE(5) RC_CASE(6) RC_CASE(7) RC_CASE(8)
#endif
      default: return set_err(DTMPC_ERR_BAD_ARG, "fast receding: obstacle count not instantiated");
    }
#undef RC_CASE
#undef RC_LAUNCH
  }
  return check_launch("receding_fast_kernel");
}

#else  // the general path's solves (csrc/dtmpc_fast_general.hip)

// one lane per trajectory: the records of both solves (two tapes of (N+1) x 16 + N x 8 bytes and the
// gains' N x 40) fit in the generic scratch of dtmpc_general_workspace_bytes (N x 80 + (N+1) x 40)
static int64_t general_fast_bytes_per_traj(int N) {
  return 2 * ((int64_t)(N + 1) * 16 * ES + (int64_t)N * 8 * ES) + (int64_t)N * 40 * ES;
}

bool FKN(general_fast_eligible)(int dtype, const dtmpc_spec* sp, const dtmpc_general_cfg* cf) {
  const char* e = getenv("DTMPC_FAST");
  if (e && e[0] == '0' && e[1] == 0) return false;
  if (DTMPC_FAST_F64 && (e = getenv("DTMPC_FAST64")) && e[0] == '0' && e[1] == 0) return false;
  // the tightening s comes from theta-bar (spec.h_offset is not used by the general path)
  if (dtype != kFastDtype || sp->obs_aggregation != DTMPC_OBS_SMOOTHMIN || sp->n_obstacles < 1 ||
      sp->n_obstacles > 8 || sp->barrier_type != DTMPC_BARRIER_INVERSE)
    return false;
  // six rolled-out candidates (the paper's seven alphas) or four (ILQRConfig's default alphas), the
  // same list in both solves (check_general)
  const int nc = make_ilqr<real>(cf->nom_ilqr).nc;
  return (nc == FK_NS::NC || nc == 4) && make_ilqr<real>(cf->aux_ilqr).nc == nc;
}

int FKN(launch_general_solve_fast)(const dtmpc_spec* sp, const dtmpc_general_cfg* cf, int64_t B,
                              const dtmpc_general_state* S, int* sst, hipStream_t st) {
  const int N = sp->horizon;
  FK_NS::GSK kk;
  std::memset(&kk, 0, sizeof(kk));
  fast_p(sp, kk.p);
  kk.cfn = fast_ilqr(cf->nom_ilqr);
  kk.cfa = fast_ilqr(cf->aux_ilqr);
  FK_NS::GSArgs& a = kk.a;
  a.B = (int)B;
  a.theta = (const real*)S->theta;
  a.tgt = FK_NS::f4{real(cf->target[0]), real(cf->target[1]), real(cf->target[2]), 0.f};
  a.x = (const real*)S->x;
  a.b = (const real*)S->b;
  a.xbar = (const real*)S->xbar;
  a.bbar = (const real*)S->bbar;
  a.Xnom = (real*)S->Xnom;
  a.Unom = (real*)S->Unom;
  a.Xaux = (real*)S->Xaux;
  a.Uaux = (real*)S->Uaux;
  a.iters = S->iters;
  a.sst = sst;
  a.work = (real*)S->work;
  const int nc = make_ilqr<real>(cf->nom_ilqr).nc;
  const int bs = tube_block(B, 1);
  const int64_t chunk = ((int64_t)0x7fffffff / general_fast_bytes_per_traj(N)) / kBlock * kBlock;
  for (int64_t c0 = 0; c0 < B; c0 += chunk) {
    const int64_t Bc = B - c0 < chunk ? B - c0 : chunk;
    a.i0 = (int)c0;
    a.Bc = (int)Bc;
    const unsigned X = (unsigned)(Bc * (N + 1) * 16 * ES), U = (unsigned)(Bc * N * 8 * ES);
    a.oXn = 0;
    a.oXa = X;
    a.oUn = 2 * X;
    a.oUa = 2 * X + U;
    a.oK = 2 * X + 2 * U;
    a.ok = a.oK + (unsigned)(Bc * N * 32 * ES);
    a.wsz = a.ok + (unsigned)(Bc * N * 8 * ES);
#define GS_LAUNCH(m, n)                                                                                   \
  hipLaunchKernelGGL((FK_NS::general_solve_fast_kernel<m, 1, n>), dim3((unsigned)((Bc + bs - 1) / bs)), dim3(bs), 0, \
                     st, kk)
#define GS_CASE(m)                 \
  case m:                          \
    if (nc == 4) GS_LAUNCH(m, 4);  \
    else GS_LAUNCH(m, FK_NS::NC);     \
    break;
    switch (sp->n_obstacles) {
#if defined(DTMPC_FAST_M_ONLY)
      GS_CASE(DTMPC_FAST_M_ONLY)
#elif defined(DTMPC_FAST_ISA_ONLY)
      GS_CASE(5)
#else
      GS_CASE(1) GS_CASE(2) GS_CASE(3) GS_CASE(4) GS_CASE(5) GS_CASE(6) GS_CASE(7) GS_CASE(8)
#endif
      default: return set_err(DTMPC_ERR_BAD_ARG, "fast general solve: obstacle count not instantiated");
    }
#undef GS_CASE
#undef GS_LAUNCH
  }
  return check_launch("general_solve_fast_kernel");
}

#endif

}  // namespace dtmpc

#if !defined(DTMPC_FAST_AUX_TU) && !DTMPC_FAST_F64
extern "C" {
// diagnostics (not part of include/dtmpc.h): the counter-calibration copy of record_stream_kernel over
// src / dst buffers of (N+1) x 16 + N x 8 bytes per trajectory (< 2^31 bytes)
int dtmpc_diag_record_stream(int64_t B, int32_t N, const void* src, void* dst, void* stream) {
  const int64_t bytes = B * ((int64_t)(N + 1) * 16 + (int64_t)N * 8);
  if (B < 1 || N < 1 || bytes >= 0x7fffffff || !src || !dst) return dtmpc::set_err(DTMPC_ERR_BAD_ARG, "bad sizes");
  hipLaunchKernelGGL(dtmpc::FK_NS::record_stream_kernel, dtmpc::grid_for(B), dim3(dtmpc::kBlock), 0, (hipStream_t)stream,
                     (const float*)src, (float*)dst, (int)B, (int)N, (unsigned)bytes);
  return dtmpc::check_launch("record_stream_kernel");
}
// diagnostics: stream_probe_kernel<depth> (depth 0, 1, 2 or 4) over one buffer of B x N x 80 bytes (< 2^31)
int dtmpc_diag_stream_probe(int64_t B, int32_t N, int32_t passes, int32_t depth, void* buf, void* stream) {
  const int64_t bytes = B * (int64_t)N * 80;
  if (B < 1 || N < 8 || passes < 1 || bytes >= 0x7fffffff || !buf) return dtmpc::set_err(DTMPC_ERR_BAD_ARG, "bad sizes");
  const dim3 g = dtmpc::grid_for(B), b = dim3(dtmpc::kBlock);
  hipStream_t st = (hipStream_t)stream;
  float* p = (float*)buf;
  switch (depth) {
    case 0: hipLaunchKernelGGL(dtmpc::FK_NS::stream_probe_kernel<0>, g, b, 0, st, p, (int)B, (int)N, (int)passes, (unsigned)bytes); break;
    case 1: hipLaunchKernelGGL(dtmpc::FK_NS::stream_probe_kernel<1>, g, b, 0, st, p, (int)B, (int)N, (int)passes, (unsigned)bytes); break;
    case 2: hipLaunchKernelGGL(dtmpc::FK_NS::stream_probe_kernel<2>, g, b, 0, st, p, (int)B, (int)N, (int)passes, (unsigned)bytes); break;
    case 4: hipLaunchKernelGGL(dtmpc::FK_NS::stream_probe_kernel<4>, g, b, 0, st, p, (int)B, (int)N, (int)passes, (unsigned)bytes); break;
    default: return dtmpc::set_err(DTMPC_ERR_BAD_ARG, "depth must be 0, 1, 2 or 4");
  }
  return dtmpc::check_launch("stream_probe_kernel");
}
}

#ifdef DTMPC_PROFILE
extern "C" {
// profiling builds only (not part of include/dtmpc.h): this translation unit's phase-cycle accumulators
int dtmpc_prof_read_fast(void* host16) {
  return hipMemcpyFromSymbol(host16, HIP_SYMBOL(dtmpc::g_prof), 16 * sizeof(unsigned long long)) == hipSuccess ? 0 : 1;
}
int dtmpc_prof_reset_fast(void) {
  unsigned long long z[64] = {0};
  if (hipMemcpyToSymbol(HIP_SYMBOL(dtmpc::FK_NS::g_lsstat), z, sizeof(z)) != hipSuccess) return 1;
  return hipMemcpyToSymbol(HIP_SYMBOL(dtmpc::g_prof), z, 16 * sizeof(unsigned long long)) == hipSuccess ? 0 : 1;
}
int dtmpc_prof_lsstat_fast(void* host64) {
  return hipMemcpyFromSymbol(host64, HIP_SYMBOL(dtmpc::FK_NS::g_lsstat), 64 * sizeof(unsigned long long)) == hipSuccess ? 0 : 1;
}
}
#endif
#endif  // DTMPC_FAST_AUX_TU
