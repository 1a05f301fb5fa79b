"""Discrete Dubins vehicle (counterpart of the reference's core/systems/dubins.py, same names).

``dubins_step`` and ``clamp_control`` run in HIP kernels (``dtmpc_dubins_step``, ``dtmpc_box_clamp``)
over any batch of device tensors; unbatched [3] / [2] inputs give unbatched outputs, as in the
reference.  ``sample_disturbance`` draws from torch's generator on the tensor's device exactly as the
reference does (core/systems/dubins.py:57-65), so a seeded run consumes the same random stream.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Tuple

import torch
from torch import Tensor

from .. import _points as P

__all__ = ["DubinsConfig", "dubins_step", "clamp_control", "sample_disturbance", "default_safe_h_no_obstacles"]


@dataclass(frozen=True)
class DubinsConfig:
    """core/systems/dubins.py:10-21 (same fields and defaults)."""

    dt: float = 0.01
    v_max: float = 10.0
    omega_max: float = float(torch.pi)
    w_low: Tuple[float, float, float] = (-0.05, -0.05, -0.05)
    w_high: Tuple[float, float, float] = (0.05, 0.05, 0.05)
    x_target: Tuple[float, float, float] = (10.0, 10.0, float(torch.pi / 4))


def _dubins_launch(x3: Tensor, u: Tensor, dt: float) -> Tensor:
    xr, lead = P.rows(x3, 3, x3)
    ur, _ = P.rows(u, 2, x3)
    out = torch.empty_like(xr)
    if xr.shape[0] > 0:
        P.launch("dtmpc_dubins_step", P.dtype_code(xr), P.byref(P.spec(dt=dt)), xr.shape[0], 3, xr.data_ptr(),
                 ur.data_ptr(), out.data_ptr(), P.stream(xr))
    return out.reshape(*lead, 3)


class _DubinsStep(torch.autograd.Function):
    """dubins_step as an autograd node: forward in the HIP kernel, backward the Dubins Jacobian
    (core/systems/dubins_aug_jac.py:42-58, A3 = I + dt v [-sin, cos] in column theta, B3 = dt [[cos, 0],
    [sin, 0], [0, 1]]) written in torch ops on the saved device inputs, so it is differentiable again (the
    reference's autograd Hessians, core/autodiff.py:9-42)."""

    @staticmethod
    def forward(ctx, x3: Tensor, u: Tensor, dt: float) -> Tensor:
        P.require_device(x3, u)
        ctx.save_for_backward(x3, u)
        ctx.dt = dt
        return _dubins_launch(x3, u, dt)

    @staticmethod
    def backward(ctx, g: Tensor):
        x3, u = ctx.saved_tensors
        dt = ctx.dt
        s, c = torch.sin(x3[..., 2]), torch.cos(x3[..., 2])
        g0, g1, g2 = g[..., 0], g[..., 1], g[..., 2]
        gx = torch.stack([g0, g1, g2 + (dt * u[..., 0]) * (c * g1 - s * g0)], -1)
        gu = torch.stack([dt * (c * g0 + s * g1), dt * g2], -1)
        return gx, gu, None


def dubins_step(x: Tensor, u: Tensor, *, cfg: DubinsConfig) -> Tensor:
    """core/systems/dubins.py:24-43: [px + dt v cos(th), py + dt v sin(th), th + dt omega].
    Differentiable (autograd) in x and u (_DubinsStep)."""
    unbatched = x.ndim == 1
    xs = x.unsqueeze(0) if unbatched else x
    us = u.unsqueeze(0) if u.ndim == 1 else u
    if xs.shape[-1] < 3:
        raise ValueError("x must be [..., 3] (px, py, theta)")
    x3 = xs[..., :3]
    ue = us.expand(*x3.shape[:-1], 2)
    if torch.is_grad_enabled() and (x3.requires_grad or ue.requires_grad):
        out = _DubinsStep.apply(x3, ue, float(cfg.dt))
    else:
        P.require_device(x3, ue)
        out = _dubins_launch(x3, ue, float(cfg.dt))
    return out.squeeze(0) if unbatched else out


def clamp_control(u: Tensor, *, cfg: DubinsConfig) -> Tensor:
    """core/systems/dubins.py:46-54: v in [-v_max, v_max], omega in [-omega_max, omega_max]."""
    from ..control import BoxClampControl

    box = BoxClampControl(u_min=(-cfg.v_max, -cfg.omega_max), u_max=(cfg.v_max, cfg.omega_max))
    return box.clamp(u)


def sample_disturbance(x: Tensor, *, cfg: DubinsConfig) -> Tensor:
    """core/systems/dubins.py:57-65: w ~ U[w_low, w_high] from torch's generator (the reference's stream)."""
    unbatched = x.ndim == 1
    xs = x.unsqueeze(0) if unbatched else x
    low = torch.tensor(cfg.w_low, device=xs.device, dtype=xs.dtype)
    high = torch.tensor(cfg.w_high, device=xs.device, dtype=xs.dtype)
    w = low + (high - low) * torch.rand_like(xs)
    return w.squeeze(0) if unbatched else w


def default_safe_h_no_obstacles(x: Tensor) -> Tensor:
    """core/systems/dubins.py:68-76: h = 1 (always safe)."""
    if x.ndim == 1:
        return torch.ones((), device=x.device, dtype=x.dtype)
    return torch.ones(x.shape[0], device=x.device, dtype=x.dtype)
