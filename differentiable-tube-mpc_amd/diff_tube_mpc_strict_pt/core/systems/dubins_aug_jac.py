"""Analytic Jacobians of the DBaS-augmented Dubins step (counterpart of the reference's
core/systems/dubins_aug_jac.py, same names and keywords), from the HIP kernel ``dtmpc_aug_jac`` --
the linearisation the fused backward pass runs -- and the barrier derivatives of
``dtmpc_barrier_eval``.  x_hat [..., 4] and u [..., 2] on a HIP device; unbatched inputs give the
reference's [4, 4] / [4, 2] (``dubins_f_jac``: [3, 3] / [3, 2])."""
from __future__ import annotations

from typing import Union

import torch
from torch import Tensor

from ... import _abi
from .. import _points as P
from ..barrier import DBaSConfig, barrier_and_derivative
from ..problem import CircleObstacle
from .dubins import DubinsConfig

__all__ = ["dubins_f_jac", "dubins_augmented_jacobian"]


def _B_inv(z: Tensor, eps: float) -> Tensor:
    """core/systems/dubins_aug_jac.py:22-23: 1 / max(z, eps)."""
    return barrier_and_derivative(z, kind=_abi.BARRIER_INVERSE_PLAIN, eps=eps)[0]


def _dB_inv_dz(z: Tensor, eps: float) -> Tensor:
    """:26-28: -1 / max(z, eps)^2."""
    return barrier_and_derivative(z, kind=_abi.BARRIER_INVERSE_PLAIN, eps=eps, want_B=False, want_dB=True)[1]


def _dB_relaxed_inv_dz(z: Tensor, *, alpha, eps: float) -> Tensor:
    """:31-40: derivative of the relaxed inverse barrier B_alpha, alpha_eff = max(alpha, eps)."""
    return barrier_and_derivative(z, kind=_abi.BARRIER_INVERSE, alpha=P.scalar(alpha), eps=eps, want_B=False,
                                  want_dB=True)[1]


def _jac(x_hat: Tensor, u: Tensor, sp):
    P.require_device(x_hat, u)
    unbatched = x_hat.ndim == 1
    xs = x_hat.unsqueeze(0) if unbatched else x_hat
    us = u.unsqueeze(0) if u.ndim == 1 else u
    xr, lead = P.rows(xs, 4, xs)
    ur, _ = P.rows(us.expand(*lead, 2), 2, xs)
    n = xr.shape[0]
    A = torch.empty(n, 4, 4, dtype=xr.dtype, device=xr.device)
    Bm = torch.empty(n, 4, 2, dtype=xr.dtype, device=xr.device)
    if n > 0:
        P.launch("dtmpc_aug_jac", P.dtype_code(xr), P.byref(sp), n, xr.data_ptr(), ur.data_ptr(), A.data_ptr(),
                 Bm.data_ptr(), P.stream(xr))
    A, Bm = A.reshape(*lead, 4, 4), Bm.reshape(*lead, 4, 2)
    return (A.squeeze(0), Bm.squeeze(0)) if unbatched else (A, Bm)


def dubins_f_jac(x: Tensor, u: Tensor, *, cfg: DubinsConfig) -> tuple[Tensor, Tensor]:
    """core/systems/dubins_aug_jac.py:42-58: A3 = I + dt v [-sin, cos] in column theta, B3."""
    xs = x[..., :3]
    xh = torch.cat([xs, torch.zeros_like(xs[..., :1])], -1)
    A, Bm = _jac(xh, u, P.spec(dt=cfg.dt))
    return A[..., :3, :3].contiguous(), Bm[..., :3, :].contiguous()


def dubins_augmented_jacobian(x_hat: Tensor, u: Tensor, *, cfg: DubinsConfig,
                              obs: Union[CircleObstacle, list[CircleObstacle]], db_cfg: DBaSConfig,
                              obs_beta: float = 20.0, obs_agg: str = "min") -> tuple[Tensor, Tensor]:
    """core/systems/dubins_aug_jac.py:61-139: A [4, 4], B [4, 2] of x_hat' = [f(x, u), b'] with the barrier
    row dB(h') grad h(x')^T A3 - gamma dB(h) grad h(x)^T, A[3, 3] = gamma, B[3, :] = dB(h') grad h(x')^T B3
    (relaxed inverse barrier, whatever db_cfg.barrier_type, as the reference)."""
    if isinstance(obs, list):
        obstacles, agg = tuple(obs), ("smoothmin" if obs_agg == "smoothmin" else "min")
        if not obstacles:
            agg = "none"
    else:
        obstacles, agg = (obs,), "single"
    sp = P.spec(dt=cfg.dt, obstacles=obstacles, aggregation=agg, beta=obs_beta, barrier_type="inverse",
                alpha=db_cfg.alpha, gamma=db_cfg.gamma, eps=db_cfg.eps)
    return _jac(x_hat, u, sp)
