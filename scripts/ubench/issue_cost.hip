// Issue-cost microbenchmark (gfx950): cycles per wave-instruction of the instruction classes the tube
// step is made of, at one and two waves per SIMD.  Each lane runs R iterations of a block of 16
// instructions of one class (independent unless the class says "dep"); the kernel time (HIP events)
// divided by R*16 gives cycles per instruction at the measured clock.  VALU / SALU / s_nop only: no
// memory instruction in the timed loops.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define R 4096

#define REP16(x) x x x x x x x x x x x x x x x x

template <int K>
__global__ void __launch_bounds__(256) kern(float* out, float seed) {
  float a0 = seed + threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  float b0 = a0 * 0.5f, b1 = a1 * 0.5f, b2 = a2 * 0.5f, b3 = a3 * 0.5f, b4 = a4 * .5f, b5 = a5 * .5f, b6 = a6 * .5f, b7 = a7 * .5f;
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 p0 = {a0, b0}, p1 = {a1, b1}, p2 = {a2, b2}, p3 = {a3, b3}, p4 = {a4, b4}, p5 = {a5, b5}, p6 = {a6, b6}, p7 = {a7, b7};
  f2 q = {1.0001f, 0.9999f};
  for (int r = 0; r < R; ++r) {
    if (K == 0) {  // v_fma_f32, 8 independent chains
      __asm__ volatile(REP16("v_fma_f32 %0, %0, %8, %9\n v_fma_f32 %1, %1, %8, %9\n v_fma_f32 %2, %2, %8, %9\n v_fma_f32 %3, %3, %8, %9\n"
                             "v_fma_f32 %4, %4, %8, %9\n v_fma_f32 %5, %5, %8, %9\n v_fma_f32 %6, %6, %8, %9\n v_fma_f32 %7, %7, %8, %9\n")
                       : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                       : "v"(b0), "v"(b1));
    } else if (K == 1) {  // v_pk_fma_f32, 8 independent chains
      __asm__ volatile(REP16("v_pk_fma_f32 %0, %0, %8, %8\n v_pk_fma_f32 %1, %1, %8, %8\n v_pk_fma_f32 %2, %2, %8, %8\n v_pk_fma_f32 %3, %3, %8, %8\n"
                             "v_pk_fma_f32 %4, %4, %8, %8\n v_pk_fma_f32 %5, %5, %8, %8\n v_pk_fma_f32 %6, %6, %8, %8\n v_pk_fma_f32 %7, %7, %8, %8\n")
                       : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3), "+v"(p4), "+v"(p5), "+v"(p6), "+v"(p7)
                       : "v"(q));
    } else if (K == 2) {  // v_exp_f32 independent
      __asm__ volatile(REP16("v_exp_f32 %0, %0\n v_exp_f32 %1, %1\n v_exp_f32 %2, %2\n v_exp_f32 %3, %3\n"
                             "v_exp_f32 %4, %4\n v_exp_f32 %5, %5\n v_exp_f32 %6, %6\n v_exp_f32 %7, %7\n")
                       : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
    } else if (K == 3) {  // v_mov_b32 independent
      __asm__ volatile(REP16("v_mov_b32 %0, %8\n v_mov_b32 %1, %8\n v_mov_b32 %2, %8\n v_mov_b32 %3, %8\n"
                             "v_mov_b32 %4, %9\n v_mov_b32 %5, %9\n v_mov_b32 %6, %9\n v_mov_b32 %7, %9\n")
                       : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                       : "v"(b0), "v"(b1));
    } else if (K == 4) {  // v_cmp -> s_nop 1 -> v_cndmask (the compiler's clamp pattern), 4 pairs
      __asm__ volatile(REP16("v_cmp_lt_f32 vcc, %0, %8\n s_nop 1\n v_cndmask_b32 %0, %0, %8, vcc\n"
                             "v_cmp_lt_f32 vcc, %1, %8\n s_nop 1\n v_cndmask_b32 %1, %1, %8, vcc\n")
                       : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                       : "v"(b0), "v"(b1)
                       : "vcc");
    } else if (K == 5) {  // s_nop 0
      __asm__ volatile(REP16("s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n s_nop 0\n"));
    } else if (K == 6) {  // v_fma_f32 dependent chain (one accumulator)
      __asm__ volatile(REP16("v_fma_f32 %0, %0, %8, %9\n v_fma_f32 %0, %0, %8, %9\n v_fma_f32 %0, %0, %8, %9\n v_fma_f32 %0, %0, %8, %9\n"
                             "v_fma_f32 %0, %0, %8, %9\n v_fma_f32 %0, %0, %8, %9\n v_fma_f32 %0, %0, %8, %9\n v_fma_f32 %0, %0, %8, %9\n")
                       : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                       : "v"(b0), "v"(b1));
    } else if (K == 7) {  // v_pk_fma_f32 dependent chain
      __asm__ volatile(REP16("v_pk_fma_f32 %0, %0, %8, %8\n v_pk_fma_f32 %0, %0, %8, %8\n v_pk_fma_f32 %0, %0, %8, %8\n v_pk_fma_f32 %0, %0, %8, %8\n"
                             "v_pk_fma_f32 %0, %0, %8, %8\n v_pk_fma_f32 %0, %0, %8, %8\n v_pk_fma_f32 %0, %0, %8, %8\n v_pk_fma_f32 %0, %0, %8, %8\n")
                       : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3), "+v"(p4), "+v"(p5), "+v"(p6), "+v"(p7)
                       : "v"(q));
    } else if (K == 8) {  // VALU fma interleaved 1:1 with SALU adds (8 + 8 per block of 16)
      int s0 = r, s1 = r + 1;
      __asm__ volatile(REP16("v_fma_f32 %0, %0, %10, %11\n s_add_u32 %8, %8, 3\n v_fma_f32 %1, %1, %10, %11\n s_add_u32 %9, %9, 5\n"
                             "v_fma_f32 %2, %2, %10, %11\n s_add_u32 %8, %8, 3\n v_fma_f32 %3, %3, %10, %11\n s_add_u32 %9, %9, 5\n")
                       : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7), "+s"(s0), "+s"(s1)
                       : "v"(b0), "v"(b1)
                       : "scc");
      a4 += (float)s0 + (float)s1;
    } else if (K == 9) {  // v_exp_f32 dependent chain
      __asm__ volatile(REP16("v_exp_f32 %0, %0\n v_exp_f32 %0, %0\n v_exp_f32 %0, %0\n v_exp_f32 %0, %0\n"
                             "v_exp_f32 %0, %0\n v_exp_f32 %0, %0\n v_exp_f32 %0, %0\n v_exp_f32 %0, %0\n")
                       : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7));
    } else if (K == 10) {  // v_fma with a trans result consumed right away (exp -> fma), 4 pairs
      __asm__ volatile(REP16("v_exp_f32 %0, %0\n v_fma_f32 %1, %0, %8, %9\n v_exp_f32 %2, %2\n v_fma_f32 %3, %2, %8, %9\n"
                             "v_exp_f32 %4, %4\n v_fma_f32 %5, %4, %8, %9\n v_exp_f32 %6, %6\n v_fma_f32 %7, %6, %8, %9\n")
                       : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                       : "v"(b0), "v"(b1));
    } else if (K == 11) {  // v_med3_f32 independent
      __asm__ volatile(REP16("v_med3_f32 %0, %0, %8, %9\n v_med3_f32 %1, %1, %8, %9\n v_med3_f32 %2, %2, %8, %9\n v_med3_f32 %3, %3, %8, %9\n"
                             "v_med3_f32 %4, %4, %8, %9\n v_med3_f32 %5, %5, %8, %9\n v_med3_f32 %6, %6, %8, %9\n v_med3_f32 %7, %7, %8, %9\n")
                       : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
                       : "v"(b0), "v"(b1));
    }
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + p0.x + p1.x + p2.x + p3.x + p4.x + p5.x + p6.x + p7.x + p0.y;
}

static const char* names[] = {"v_fma_f32 indep", "v_pk_fma_f32 indep", "v_exp_f32 indep", "v_mov_b32", "cmp+nop1+cndmask (per instr of 3)",
                              "s_nop 0", "v_fma_f32 dep", "v_pk_fma_f32 dep", "fma+s_add 1:1 (per instr)", "v_exp_f32 dep",
                              "exp->fma pairs", "v_med3_f32"};
typedef void (*KF)(float*, float);

template <int K>
static double run(int wps, float* d) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int blocks = 256 * wps;  // 256 CUs x 4 waves per block -> wps waves per SIMD
  hipLaunchKernelGGL(kern<K>, dim3(blocks), dim3(256), 0, 0, d, 1.0f);
  hipEventRecord(e0);
  hipLaunchKernelGGL(kern<K>, dim3(blocks), dim3(256), 0, 0, d, 1.0f);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  return ms;
}

int main() {
  float* d;
  hipMalloc(&d, 256 * 8 * 256 * sizeof(float));
  int clk = 0;
  hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
  const double ghz = clk / 1e6;
  printf("clock attr %.3f GHz\n", ghz);
  double (*fns[])(int, float*) = {run<0>, run<1>, run<2>, run<3>, run<4>, run<5>, run<6>, run<7>, run<8>, run<9>, run<10>, run<11>};
  const double ninstr[] = {128, 128, 128, 128, 96, 128, 128, 128, 128, 128, 128, 128};
  for (int k = 0; k < 12; ++k) {
    for (int w = 1; w <= 2; ++w) {
      const double ms = fns[k](w, d);
      // cycles per wave-instruction per wave = time * clk / (R * n_instr) ; per SIMD: divide by waves
      const double cyc = ms * 1e-3 * ghz * 1e9 / ((double)R * ninstr[k]);
      printf("%-36s waves/SIMD=%d  %.3f ms  %.2f cyc per instr per wave  (%.2f per SIMD)\n", names[k], w, ms, cyc, cyc / w);
    }
  }
  hipFree(d);
  return 0;
}
