// dtmpc_control.hip — the tanh-box control parameterisation (core/control.py:10-35 BoxTanhControl) and
// the stage-cost derivatives in its unconstrained decision variable v (core/cost_derivs.py:16-107
// nominal_cost_derivs / auxiliary_cost_derivs), along a batch of tapes.
//
// Elementwise and HBM-bound: one lane per (trajectory, step), a 2-D grid (x: trajectories in blocks of
// 256, y: steps), so every field of every step is one coalesced 256 B (f32) line per wave in and out.
// Per element: 16 B (f32) of X + 8 B of v (+ 12 + 8 B of references when tracking) read, 40 B written.
// Each product is rounded in the order torch evaluates the reference's expression (no contraction).
#include <hip/hip_runtime.h>

#include "../../include/dtmpc_control.h"
#include "dtmpc_host.hpp"

namespace dtmpc {

template <typename T>
struct TanhArgs {
  int B, N, track;
  T umin0, umin1, umax0, umax1;
  T Q0, Q1, Q2, R0, R1, qb, t0, t1, t2;
  const T *X, *Vd, *Xr, *Ur;
  T *U, *dU, *lx, *lv, *lvv;
};

__device__ __forceinline__ float c_tanh(float x) { return tanhf(x); }
__device__ __forceinline__ double c_tanh(double x) { return tanh(x); }

template <typename T>
__global__ void __launch_bounds__(kBlock) tanh_cost_derivs_kernel(TanhArgs<T> a) {
#pragma clang fp contract(off)
  const int i = blockIdx.x * kBlock + threadIdx.x;
  const int k = blockIdx.y;
  if (i >= a.B) return;
  const size_t B = (size_t)a.B;
  auto at = [&](int rows_f, int f) { return ((size_t)k * rows_f + f) * B + i; };
  if (a.lx) {  // l_x = [2 Q dx, 2 qb b] (core/cost_derivs.py:48, 100)
    const T x0 = a.X[at(4, 0)], x1 = a.X[at(4, 1)], x2 = a.X[at(4, 2)], xb = a.X[at(4, 3)];
    T d0, d1, d2;
    if (a.track) {  // dx = x - x_ref (core/cost_derivs.py:93)
      d0 = x0 - a.Xr[at(3, 0)];
      d1 = x1 - a.Xr[at(3, 1)];
      d2 = x2 - a.Xr[at(3, 2)];
    } else {        // dx = x - target (core/cost_derivs.py:41)
      d0 = x0 - a.t0;
      d1 = x1 - a.t1;
      d2 = x2 - a.t2;
    }
    a.lx[at(4, 0)] = (T(2) * a.Q0) * d0;
    a.lx[at(4, 1)] = (T(2) * a.Q1) * d1;
    a.lx[at(4, 2)] = (T(2) * a.Q2) * d2;
    a.lx[at(4, 3)] = (T(2) * a.qb) * xb;
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const size_t o = at(2, j);
    const T v = a.Vd[o];
    const T lo = j ? a.umin1 : a.umin0, hi = j ? a.umax1 : a.umax0, r = j ? a.R1 : a.R0;
    const T th = c_tanh(v);
    const T w = hi - lo;
    const T u = lo + (w * (th + T(1))) * T(0.5);        // core/control.py:27
    const T scale = w * T(0.5);                         // core/control.py:33
    const T sech2 = T(1) - th * th;                     // core/control.py:34
    const T du_dv = scale * sech2;                      // core/control.py:35
    const T d2u = scale * ((T(-2) * th) * sech2);       // core/cost_derivs.py:24
    const T e = a.track ? u - a.Ur[o] : u;              // core/cost_derivs.py:96 (aux) / u (nominal)
    const T r2 = T(2) * r;
    if (a.U) a.U[o] = u;
    if (a.dU) a.dU[o] = du_dv;
    if (a.lv) a.lv[o] = (r2 * e) * du_dv;               // core/cost_derivs.py:49, 101
    if (a.lvv) a.lvv[o] = r2 * (du_dv * du_dv + e * d2u);  // core/cost_derivs.py:52, 104
  }
}

template <typename T>
static int launch_tanh(const dtmpc_spec& s, const dtmpc_cost& c, int64_t B, const void* X, const void* Vd,
                       const void* Xref, const void* Uref, void* U, void* dU, void* lx, void* lv, void* lvv,
                       hipStream_t st) {
  TanhArgs<T> a;
  a.B = (int)B;
  a.N = s.horizon;
  a.track = c.kind == DTMPC_COST_TRACK;
  a.umin0 = (T)s.u_min[0];
  a.umin1 = (T)s.u_min[1];
  a.umax0 = (T)s.u_max[0];
  a.umax1 = (T)s.u_max[1];
  a.Q0 = (T)c.Q[0];
  a.Q1 = (T)c.Q[1];
  a.Q2 = (T)c.Q[2];
  a.R0 = (T)c.R[0];
  a.R1 = (T)c.R[1];
  a.qb = (T)c.qb;
  a.t0 = (T)c.target[0];
  a.t1 = (T)c.target[1];
  a.t2 = (T)c.target[2];
  a.X = (const T*)X;
  a.Vd = (const T*)Vd;
  a.Xr = (const T*)Xref;
  a.Ur = (const T*)Uref;
  a.U = (T*)U;
  a.dU = (T*)dU;
  a.lx = (T*)lx;
  a.lv = (T*)lv;
  a.lvv = (T*)lvv;
  const dim3 grid((unsigned)((B + kBlock - 1) / kBlock), (unsigned)s.horizon);
  hipLaunchKernelGGL(tanh_cost_derivs_kernel<T>, grid, dim3(kBlock), 0, st, a);
  return check_launch("tanh_cost_derivs_kernel");
}

}  // namespace dtmpc

using namespace dtmpc;

int dtmpc_tanh_cost_derivs(int dtype, const dtmpc_spec* spec, const dtmpc_cost* cost, int64_t B, const void* X,
                           const void* Vdec, const void* Xref, const void* Uref, void* U, void* dU, void* lx,
                           void* lv, void* lvv, void* stream) {
  int e = check_spec(spec, B);
  if (e) return e;
  if ((e = check_cost(cost, Xref, Uref))) return e;
  if (cost->wrap_angle) return set_err(DTMPC_ERR_BAD_ARG, "tanh-box cost derivatives take the unwrapped cost");
  if (!Vdec || (lx && !X)) return set_err(DTMPC_ERR_BAD_ARG, "NULL array");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DTMPC_F32) return launch_tanh<float>(*spec, *cost, B, X, Vdec, Xref, Uref, U, dU, lx, lv, lvv, st);
  if (dtype == DTMPC_F64) return launch_tanh<double>(*spec, *cost, B, X, Vdec, Xref, Uref, U, dU, lx, lv, lvv, st);
  return set_err(DTMPC_ERR_BAD_ARG, "bad dtype");
}
