/*
 * dtmpc_systems.h — C ABI of libdtmpc.so, the per-function entry points behind the reference's
 * per-point API (companion of dtmpc.h: caller-owned device buffers, an explicit hipStream_t, no
 * allocation, DTMPC_ERR_BAD_ARG for invalid arguments before any device call).
 *
 * Layout: unlike the SoA tapes of dtmpc.h these take POINT-MAJOR arrays [B][F] -- row i is one point,
 * the layout of the reference's batched torch tensors ([B, 3] states, [B, 2] controls) -- so the Python
 * mirror (diff_tube_mpc_strict_pt.core.barrier / .systems.* / .control / .cost_derivs) hands its
 * tensors over without a transpose.  Each kernel is one lane per point and runs the same device code
 * as the tube-step kernels.
 */
#ifndef DTMPC_SYSTEMS_H
#define DTMPC_SYSTEMS_H

#include "dtmpc.h"

#ifdef __cplusplus
extern "C" {
#endif

/* dtmpc_barrier_eval kind: besides DTMPC_BARRIER_INVERSE (the RELAXED inverse barrier B_alpha) and
 * DTMPC_BARRIER_LOG, the plain inverse barrier 1 / max(z, eps) of barrier_B (core/barrier.py:62-72). */
enum { DTMPC_BARRIER_INVERSE_PLAIN = 2 };

/* x_next = dubins_step(x, u): replaces core/systems/dubins.py:24-43 (dt = spec->dt).
 *   x [B][x_stride] (fields 0..2 read, x_stride >= 3), u [B][2], x_next [B][3]. */
int dtmpc_dubins_step(int dtype, const dtmpc_spec* spec, int64_t B, int32_t x_stride, const void* x,
                      const void* u, void* x_next, void* stream);

/* Safety function h(x) and its gradient for the spec's obstacle aggregation:
 *   replaces core/systems/dubins_obstacles.py:16-30 `h_circle_obstacle` (DTMPC_OBS_SINGLE),
 *   :41-69 `h_multi_circle_obstacles` (SMOOTHMIN), :95-106 `h_min_circle_obstacles` (MIN; NONE: h = 1)
 *   and :33-38, :72-92, :109-117 `grad_h_*` (argmin subgradient for MIN).
 *   x [B][x_stride] (fields 0..1 read), h [B], grad [B][3] (theta component 0) or NULL. */
int dtmpc_h_eval(int dtype, const dtmpc_spec* spec, int64_t B, int32_t x_stride, const void* x, void* h,
                 void* grad, void* stream);

/* B(z) and dB/dz per point: replaces core/barrier.py:36-59 `relaxed_inverse_barrier_B_alpha` and
 * core/systems/dubins_aug_jac.py:31-40 `_dB_relaxed_inv_dz` (kind DTMPC_BARRIER_INVERSE, alpha_eff =
 * max(alpha, eps)), core/barrier.py:62-72 `barrier_B` with barrier_type "log" (DTMPC_BARRIER_LOG; dB =
 * -1/z above eps, else 0) and "inverse" (DTMPC_BARRIER_INVERSE_PLAIN) with
 * core/systems/dubins_aug_jac.py:22-28 `_B_inv` / `_dB_inv_dz`.
 *   z [B]; Bz [B] and dBz [B] out (either may be NULL, not both). */
int dtmpc_barrier_eval(int dtype, int32_t kind, double alpha, double eps, int64_t B, const void* z,
                       void* Bz, void* dBz, void* stream);

/* One DBaS-augmented step x_hat' = [dubins_step(x, u), B(h(x')) - gamma (B(h(x)) - b)] with the spec's
 * obstacles and barrier: replaces core/barrier.py:75-108 `dbas_step` with f = dubins_step and h the
 * spec's aggregation.  x_hat [B][4], u [B][2], x_hat_next [B][4]. */
int dtmpc_fhat(int dtype, const dtmpc_spec* spec, int64_t B, const void* x_hat, const void* u,
               void* x_hat_next, void* stream);

/* Augmented Jacobians A = d x_hat'/d x_hat [B][4][4], Bm = d x_hat'/d u [B][4][2] (row-major):
 * replaces core/systems/dubins_aug_jac.py:61-139 `dubins_augmented_jacobian` (the barrier row always
 * differentiates the relaxed inverse barrier, as the reference does) and, in the top-left 3 x 3 / 3 x 2
 * blocks, :42-58 `dubins_f_jac`.  x_hat [B][4], u [B][2]. */
int dtmpc_aug_jac(int dtype, const dtmpc_spec* spec, int64_t B, const void* x_hat, const void* u, void* A,
                  void* Bm, void* stream);

/* Box clamp and active set: replaces core/control.py:61-64 `BoxClampControl.clamp` (torch.clamp to
 * [spec->u_min, spec->u_max], NaN propagating) and :66-70 `active_mask` (u within spec->active_tol of
 * a bound, evaluated on the given u).  u [B][2]; u_out [B][2] and active [B][2] (bytes 0/1) out, either
 * may be NULL, not both.  Also core/systems/dubins.py:46-54 `clamp_control`. */
int dtmpc_box_clamp(int dtype, const dtmpc_spec* spec, int64_t B, const void* u, void* u_out, void* active,
                    void* stream);

/* Quadratic cost derivatives per point, u-form: replaces core/cost_derivs.py:58-76
 * `nominal_cost_derivs_u` (cost->kind TARGET: l_x = [2Q (x - target), 2 qb b], l_u = 2R u) and
 * :110-130 `auxiliary_cost_derivs_u` (TRACK: x_ref, u_ref), or with terminal != 0 :133-146
 * `nominal_terminal_derivs` / `auxiliary_terminal_derivs` (phi_x = [2 Qf (x_N - r), 0]).
 *   x_hat [B][4], u [B][2] (stage only), x_ref [B][3] / u_ref [B][2] (TRACK); l_x [B][4], l_u [B][2]
 *   (stage only).  The Hessians diag(2Q, 2qb), diag(2R), 0 (terminal diag(2Qf, 0)) are constants of the
 *   cost and not written. */
int dtmpc_cost_derivs(int dtype, const dtmpc_cost* cost, int32_t terminal, int64_t B, const void* x_hat,
                      const void* u, const void* x_ref, const void* u_ref, void* l_x, void* l_u,
                      void* stream);

#ifdef __cplusplus
}
#endif

#endif /* DTMPC_SYSTEMS_H */
