// dtmpc_systems.hip — per-point kernels behind the reference's per-function API (include/dtmpc_systems.h):
// core/systems/dubins.py, core/systems/dubins_obstacles.py, core/systems/dubins_aug_jac.py,
// core/barrier.py, core/control.py (BoxClampControl), core/cost_derivs.py (*_cost_derivs_u,
// *_terminal_derivs).
//
// One lane = one point of a batch of B independent points; arrays are POINT-MAJOR [B][F] (row i is one
// point, the reference's [B, F] torch layout), x rows with a caller-given stride so that the first three
// fields of an [B, 4] augmented state can be read in place.  The arithmetic is the tube kernels' own
// device code (dtmpc_device.hpp), so these entry points are also per-function probes of the hot path.
#include <hip/hip_runtime.h>

#include "../../include/dtmpc.h"
#include "../../include/dtmpc_systems.h"
#include "dtmpc_host.hpp"

namespace dtmpc {
namespace sys {

enum { OP_DUBINS, OP_H, OP_FHAT, OP_AUGJAC, OP_CLAMP };

// the point ops sharing one kernel shape: x rows (stride xs), u rows [B][2]
template <typename T, int OP>
__global__ void __launch_bounds__(kBlock) point_kernel(DSpec<T> s, int B, int xs, const T* x, const T* u,
                                                       void* o0, void* o1) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= B) return;
  const T* xi = x ? x + (size_t)i * xs : nullptr;
  const T* ui = u ? u + (size_t)i * 2 : nullptr;
  if (OP == OP_DUBINS) {  // dubins_step core/systems/dubins.py:24-43
    DTMPC_NOCONTRACT
    T sn, c;
    m_sincos(xi[2], &sn, &c);
    const T dv = s.dt * ui[0];
    T* o = (T*)o0 + (size_t)i * 3;
    o[0] = xi[0] + dv * c;
    o[1] = xi[1] + dv * sn;
    o[2] = xi[2] + s.dt * ui[1];
  } else if (OP == OP_H) {  // h_* / grad_h_* core/systems/dubins_obstacles.py:16-117
    T h[1], px[1] = {xi[0]}, py[1] = {xi[1]};
    h_vec<T, 1>(s, px, py, h);
    ((T*)o0)[i] = h[0];
    if (o1) {
      T gx, gy;
      (void)h_grad(s, xi[0], xi[1], gx, gy);
      T* g = (T*)o1 + (size_t)i * 3;
      g[0] = gx;
      g[1] = gy;
      g[2] = T(0);
    }
  } else if (OP == OP_FHAT) {  // dbas_step core/barrier.py:75-108 over dubins_step
    T x0[1] = {xi[0]}, x1[1] = {xi[1]}, x2[1] = {xi[2]}, b[1] = {xi[3]}, u0[1] = {ui[0]}, u1[1] = {ui[1]};
    T Bc[1] = {barrier_of_state(s, xi[0], xi[1])};
    fhat_vec<T, 1>(s, x0, x1, x2, b, u0, u1, Bc);
    T* o = (T*)o0 + (size_t)i * 4;
    o[0] = x0[0];
    o[1] = x1[0];
    o[2] = x2[0];
    o[3] = b[0];
  } else if (OP == OP_AUGJAC) {  // dubins_augmented_jacobian core/systems/dubins_aug_jac.py:61-139
    const T v = ui[0];
    T sn, cs;
    m_sincos(xi[2], &sn, &cs);
    T gxk, gyk, gxn, gyn;
    const T hk = h_grad(s, xi[0], xi[1], gxk, gyk);
    T n0, n1;
    {
      DTMPC_NOCONTRACT
      const T dv = s.dt * v;
      n0 = xi[0] + dv * cs;
      n1 = xi[1] + dv * sn;
    }
    const T hn = h_grad(s, n0, n1, gxn, gyn);
    const Jac<T> J = make_jac(s, sn, cs, v, gxk, gyk, dbarrier_relaxed(s, hk), gxn, gyn, dbarrier_relaxed(s, hn));
    const T Ad[16] = {T(1), T(0), J.a02, T(0), T(0), T(1), J.a12, T(0), T(0), T(0), T(1), T(0), J.a30, J.a31, J.a32, J.g};
    const T Bd[8] = {J.b00, T(0), J.b10, T(0), T(0), J.b21, J.b30, J.b31};
    T* A = (T*)o0 + (size_t)i * 16;
    T* Bm = (T*)o1 + (size_t)i * 8;
#pragma unroll
    for (int j = 0; j < 16; ++j) A[j] = Ad[j];
#pragma unroll
    for (int j = 0; j < 8; ++j) Bm[j] = Bd[j];
  } else if (OP == OP_CLAMP) {  // BoxClampControl.clamp / active_mask core/control.py:61-70
    const T lo[2] = {s.umin0, s.umin1}, hi[2] = {s.umax0, s.umax1};
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const T v = ui[j];
      if (o0) ((T*)o0)[(size_t)i * 2 + j] = v < lo[j] ? lo[j] : (v > hi[j] ? hi[j] : v);  // NaN stays NaN
      if (o1) ((unsigned char*)o1)[(size_t)i * 2 + j] = (v <= lo[j] + s.active_tol) || (v >= hi[j] - s.active_tol);
    }
  }
}

// B(z) and B'(z) (core/barrier.py:36-72, core/systems/dubins_aug_jac.py:22-40); kind: relaxed inverse,
// log, or the plain inverse 1 / max(z, eps) of barrier_B
template <typename T>
__global__ void __launch_bounds__(kBlock) barrier_kernel(DSpec<T> s, int kind, int B, const T* z, T* Bz, T* dBz) {
  DTMPC_NOCONTRACT
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= B) return;
  const T v = z[i];
  const T vc = v < s.eps ? s.eps : v;  // torch.clamp(min=eps): NaN propagates
  T b, d;
  if (kind == DTMPC_BARRIER_LOG) {
    b = -m_log(vc);
    d = v > s.eps ? -(T(1) / v) : T(0);
  } else if (kind == DTMPC_BARRIER_INVERSE_PLAIN) {
    b = T(1) / vc;
    d = -(T(1) / (vc * vc));
  } else {
    b = barrier_relaxed(s, v);
    d = dbarrier_relaxed(s, v);
  }
  if (Bz) Bz[i] = b;
  if (dBz) dBz[i] = d;
}

// stage (u-form) and terminal cost derivatives (core/cost_derivs.py:58-76, 110-146): l_x = [2Q dx, 2qb b],
// l_u = 2R (u - u_ref); terminal phi_x = [2Qf dx_N, 0]
template <typename T>
__global__ void __launch_bounds__(kBlock) cost_derivs_kernel(DCost<T> c, int terminal, int B, const T* xh, const T* u,
                                                             const T* xr, const T* ur, T* lx, T* lu) {
  DTMPC_NOCONTRACT
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= B) return;
  const T* x = xh + (size_t)i * 4;
  const bool track = c.kind == DTMPC_COST_TRACK;
  const T r0 = track ? xr[(size_t)i * 3] : c.t0, r1 = track ? xr[(size_t)i * 3 + 1] : c.t1,
          r2 = track ? xr[(size_t)i * 3 + 2] : c.t2;
  const T d0 = x[0] - r0, d1 = x[1] - r1, d2 = x[2] - r2;
  T* o = lx + (size_t)i * 4;
  if (terminal) {
    o[0] = (T(2) * c.Qf0) * d0;
    o[1] = (T(2) * c.Qf1) * d1;
    o[2] = (T(2) * c.Qf2) * d2;
    o[3] = T(0);
    return;
  }
  o[0] = (T(2) * c.Q0) * d0;
  o[1] = (T(2) * c.Q1) * d1;
  o[2] = (T(2) * c.Q2) * d2;
  o[3] = (T(2) * c.qb) * x[3];
  const T e0 = track ? u[(size_t)i * 2] - ur[(size_t)i * 2] : u[(size_t)i * 2];
  const T e1 = track ? u[(size_t)i * 2 + 1] - ur[(size_t)i * 2 + 1] : u[(size_t)i * 2 + 1];
  lu[(size_t)i * 2] = (T(2) * c.R0) * e0;
  lu[(size_t)i * 2 + 1] = (T(2) * c.R1) * e1;
}

template <int OP>
static int launch_point(int dtype, const dtmpc_spec* spec, int64_t B, int xs, const void* x, const void* u, void* o0,
                        void* o1, void* stream, const char* name) {
  int e = check_spec(spec, B);
  if (e) return e;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DTMPC_F32)
    hipLaunchKernelGGL((point_kernel<float, OP>), grid_for(B), dim3(kBlock), 0, st, make_spec<float>(*spec), (int)B, xs,
                       (const float*)x, (const float*)u, o0, o1);
  else if (dtype == DTMPC_F64)
    hipLaunchKernelGGL((point_kernel<double, OP>), grid_for(B), dim3(kBlock), 0, st, make_spec<double>(*spec), (int)B, xs,
                       (const double*)x, (const double*)u, o0, o1);
  else
    return set_err(DTMPC_ERR_BAD_ARG, "bad dtype");
  return check_launch(name);
}

}  // namespace sys
}  // namespace dtmpc

using namespace dtmpc;
using namespace dtmpc::sys;

extern "C" {

int dtmpc_dubins_step(int dtype, const dtmpc_spec* spec, int64_t B, int32_t x_stride, const void* x, const void* u,
                      void* x_next, void* stream) {
  if (!x || !u || !x_next || x_stride < 3) return set_err(DTMPC_ERR_BAD_ARG, "dubins_step: NULL array or x_stride < 3");
  return launch_point<OP_DUBINS>(dtype, spec, B, x_stride, x, u, x_next, nullptr, stream, "dubins_step");
}

int dtmpc_h_eval(int dtype, const dtmpc_spec* spec, int64_t B, int32_t x_stride, const void* x, void* h, void* grad,
                 void* stream) {
  if (!x || !h || x_stride < 2) return set_err(DTMPC_ERR_BAD_ARG, "h_eval: NULL array or x_stride < 2");
  return launch_point<OP_H>(dtype, spec, B, x_stride, x, nullptr, h, grad, stream, "h_eval");
}

int dtmpc_fhat(int dtype, const dtmpc_spec* spec, int64_t B, const void* x_hat, const void* u, void* x_hat_next,
               void* stream) {
  if (!x_hat || !u || !x_hat_next) return set_err(DTMPC_ERR_BAD_ARG, "fhat: NULL array");
  return launch_point<OP_FHAT>(dtype, spec, B, 4, x_hat, u, x_hat_next, nullptr, stream, "fhat");
}

int dtmpc_aug_jac(int dtype, const dtmpc_spec* spec, int64_t B, const void* x_hat, const void* u, void* A, void* Bm,
                  void* stream) {
  if (!x_hat || !u || !A || !Bm) return set_err(DTMPC_ERR_BAD_ARG, "aug_jac: NULL array");
  return launch_point<OP_AUGJAC>(dtype, spec, B, 4, x_hat, u, A, Bm, stream, "aug_jac");
}

int dtmpc_box_clamp(int dtype, const dtmpc_spec* spec, int64_t B, const void* u, void* u_out, void* active,
                    void* stream) {
  if (!u || (!u_out && !active)) return set_err(DTMPC_ERR_BAD_ARG, "box_clamp: NULL array");
  return launch_point<OP_CLAMP>(dtype, spec, B, 0, nullptr, u, u_out, active, stream, "box_clamp");
}

int dtmpc_barrier_eval(int dtype, int32_t kind, double alpha, double eps, int64_t B, const void* z, void* Bz,
                       void* dBz, void* stream) {
  if (B < 1) return set_err(DTMPC_ERR_BAD_ARG, "batch must be >= 1");
  if (!z || (!Bz && !dBz)) return set_err(DTMPC_ERR_BAD_ARG, "barrier_eval: NULL array");
  if (kind != DTMPC_BARRIER_INVERSE && kind != DTMPC_BARRIER_LOG && kind != DTMPC_BARRIER_INVERSE_PLAIN)
    return set_err(DTMPC_ERR_BAD_ARG, "Unknown barrier_type");
  if (alpha < 0) return set_err(DTMPC_ERR_BAD_ARG, "alpha must be >= 0");
  dtmpc_spec sp;
  std::memset(&sp, 0, sizeof(sp));
  sp.horizon = 1;
  sp.dbas_alpha = alpha;
  sp.dbas_eps = eps;
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DTMPC_F32)
    hipLaunchKernelGGL(barrier_kernel<float>, grid_for(B), dim3(kBlock), 0, st, make_spec<float>(sp), kind, (int)B,
                       (const float*)z, (float*)Bz, (float*)dBz);
  else if (dtype == DTMPC_F64)
    hipLaunchKernelGGL(barrier_kernel<double>, grid_for(B), dim3(kBlock), 0, st, make_spec<double>(sp), kind, (int)B,
                       (const double*)z, (double*)Bz, (double*)dBz);
  else
    return set_err(DTMPC_ERR_BAD_ARG, "bad dtype");
  return check_launch("barrier_kernel");
}

int dtmpc_cost_derivs(int dtype, const dtmpc_cost* cost, int32_t terminal, int64_t B, const void* x_hat,
                      const void* u, const void* x_ref, const void* u_ref, void* l_x, void* l_u, void* stream) {
  if (B < 1) return set_err(DTMPC_ERR_BAD_ARG, "batch must be >= 1");
  int e = check_cost(cost, x_ref, terminal ? (const void*)1 : u_ref);
  if (e) return e;
  if (!x_hat || !l_x || (!terminal && (!u || !l_u))) return set_err(DTMPC_ERR_BAD_ARG, "cost_derivs: NULL array");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == DTMPC_F32)
    hipLaunchKernelGGL(cost_derivs_kernel<float>, grid_for(B), dim3(kBlock), 0, st, make_cost<float>(*cost), terminal,
                       (int)B, (const float*)x_hat, (const float*)u, (const float*)x_ref, (const float*)u_ref,
                       (float*)l_x, (float*)l_u);
  else if (dtype == DTMPC_F64)
    hipLaunchKernelGGL(cost_derivs_kernel<double>, grid_for(B), dim3(kBlock), 0, st, make_cost<double>(*cost), terminal,
                       (int)B, (const double*)x_hat, (const double*)u, (const double*)x_ref, (const double*)u_ref,
                       (double*)l_x, (double*)l_u);
  else
    return set_err(DTMPC_ERR_BAD_ARG, "bad dtype");
  return check_launch("cost_derivs_kernel");
}

}  // extern "C"
