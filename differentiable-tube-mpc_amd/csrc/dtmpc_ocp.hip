// dtmpc_ocp.hip — the tape cost of core/ocp.py:63-85 `total_cost` for the typed costs: J = sum_k l(x_k, u_k)
// + phi(x_N) per trajectory, with the stage / terminal cost expressions the solvers price candidates
// with (dtmpc_device.hpp stage_cost / term_cost: core/tube_mpc.py:823-832, 875-885, run_nominal.py:297-324).
//
// One lane per trajectory, SoA tapes: each step's field is one coalesced 256 B (f32) line per wave.
// HBM-bound: (N+1)·16 + N·8 B read per trajectory (+ (N+1)·12 + N·8 B of references when tracking).
#include <hip/hip_runtime.h>

#include "../../include/dtmpc_control.h"
#include "dtmpc_host.hpp"

namespace dtmpc {

template <typename T>
__global__ void __launch_bounds__(kBlock) tape_cost_kernel(DCost<T> c, int N, int B, const T* X, const T* U,
                                                           const T* Xr, const T* Ur, T* J) {
  const int i = blockIdx.x * kBlock + threadIdx.x;
  if (i >= B) return;
  const size_t b = (size_t)B;
  const bool trk = c.kind == DTMPC_COST_TRACK;
  T acc = T(0);  // J = zeros; J = J + l_k ... (core/ocp.py:79-82)
  for (int k = 0; k < N; ++k) {
    const T* x = X + (size_t)k * 4 * b + i;
    const T* u = U + (size_t)k * 2 * b + i;
    T r0 = T(0), r1 = T(0), r2 = T(0), q0 = T(0), q1 = T(0);
    if (trk) {
      const T* r = Xr + (size_t)k * 3 * b + i;
      r0 = r[0];
      r1 = r[b];
      r2 = r[2 * b];
      q0 = Ur[(size_t)k * 2 * b + i];
      q1 = Ur[((size_t)k * 2 + 1) * b + i];
    }
    acc = acc + stage_cost(c, x[0], x[b], x[2 * b], x[3 * b], u[0], u[b], r0, r1, r2, q0, q1);
  }
  const T* x = X + (size_t)N * 4 * b + i;
  T r0 = T(0), r1 = T(0), r2 = T(0);
  if (trk) {
    const T* r = Xr + (size_t)N * 3 * b + i;
    r0 = r[0];
    r1 = r[b];
    r2 = r[2 * b];
  }
  J[i] = acc + term_cost(c, x[0], x[b], x[2 * b], x[3 * b], r0, r1, r2);  // + phi_N (core/ocp.py:83)
}

}  // namespace dtmpc

using namespace dtmpc;

int dtmpc_tape_cost(int dtype, const dtmpc_spec* spec, const dtmpc_cost* cost, int64_t B, const void* X,
                    const void* U, const void* Xref, const void* Uref, void* J, void* stream) {
  int e = check_spec(spec, B);
  if (e) return e;
  if ((e = check_cost(cost, Xref, Uref))) return e;
  if (!X || !U || !J) return set_err(DTMPC_ERR_BAD_ARG, "NULL array");
  hipStream_t st = (hipStream_t)stream;
  const int N = spec->horizon;
  if (dtype == DTMPC_F32)
    hipLaunchKernelGGL(tape_cost_kernel<float>, grid_for(B), dim3(kBlock), 0, st, make_cost<float>(*cost), N, (int)B,
                       (const float*)X, (const float*)U, (const float*)Xref, (const float*)Uref, (float*)J);
  else if (dtype == DTMPC_F64)
    hipLaunchKernelGGL(tape_cost_kernel<double>, grid_for(B), dim3(kBlock), 0, st, make_cost<double>(*cost), N, (int)B,
                       (const double*)X, (const double*)U, (const double*)Xref, (const double*)Uref, (double*)J);
  else
    return set_err(DTMPC_ERR_BAD_ARG, "bad dtype");
  return check_launch("tape_cost_kernel");
}
