/*
 * dtmpc_control.h — C ABI of libdtmpc.so, tanh-box control parameterisation and the tape cost of
 * core/ocp.py (companion of dtmpc.h:
 * same conventions -- caller-owned device buffers in SoA [rows][fields][B] layout, an explicit
 * hipStream_t, no allocation, DTMPC_ERR_BAD_ARG for invalid arguments before any device call).
 */
#ifndef DTMPC_CONTROL_H
#define DTMPC_CONTROL_H

#include "dtmpc.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Tanh-box control map and stage-cost derivatives in the unconstrained decision variable v, along
 * a batch of tapes:
 *   replaces core/control.py:10-35 `BoxTanhControl.u` / `du_dv_diag`, core/cost_derivs.py:16-24
 *   `_d2u_dv2_diag`, core/cost_derivs.py:27-55 `nominal_cost_derivs` (cost->kind TARGET) and
 *   core/cost_derivs.py:79-107 `auxiliary_cost_derivs` (cost->kind TRACK).
 *   Box bounds: spec->u_min / u_max (any values, as the reference's map takes them).  cost->wrap_angle
 *   must be 0.
 *   X [N+1][4][B] (rows 0..N-1 read; may be NULL when lx is NULL), Vdec [N][2][B]; Xref [N+1][3][B] / Uref [N][2][B] read only
 *   for TRACK.  Outputs (each may be NULL): U [N][2][B] = u(v), dU [N][2][B] = du/dv,
 *   lx [N][4][B] = l_x, lv [N][2][B] = l_v, lvv [N][2][B] = diag(l_vv).  l_xx = diag(2Q, 2qb) and
 *   l_vx = 0 are constants of the cost and not written. */
int dtmpc_tanh_cost_derivs(int dtype, const dtmpc_spec* spec, const dtmpc_cost* cost, int64_t B,
                           const void* X, const void* Vdec, const void* Xref, const void* Uref,
                           void* U, void* dU, void* lx, void* lv, void* lvv, void* stream);

/* Tape cost J = sum_{k<N} l(x_k, u_k) + phi(x_N) per trajectory:
 *   replaces core/ocp.py:63-85 `total_cost` for the typed stage / terminal costs of dtmpc_cost (the
 *   closures of core/tube_mpc.py:823-832 (TARGET), 875-885 (TRACK), run_nominal.py:297-324 (wrapped)).
 *   X [N+1][4][B], U [N][2][B]; Xref [N+1][3][B] / Uref [N][2][B] read only for TRACK; J [B] out. */
int dtmpc_tape_cost(int dtype, const dtmpc_spec* spec, const dtmpc_cost* cost, int64_t B, const void* X,
                    const void* U, const void* Xref, const void* Uref, void* J, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* DTMPC_CONTROL_H */
