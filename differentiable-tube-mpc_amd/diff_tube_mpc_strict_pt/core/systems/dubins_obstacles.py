"""Circle-obstacle safety functions (counterpart of the reference's core/systems/dubins_obstacles.py,
same names and keywords).

h_i(x) = ||p - c_i||^2 - r_i^2 aggregated as one circle, a smooth-min -(1/beta) LSE(-beta h_i), or the
exact min, and their (sub)gradients, from the HIP kernel ``dtmpc_h_eval`` -- the device code the fused
solver kernels use.  x is [..., >=2] on a HIP device (unbatched [3] gives a scalar h and a [3]
gradient); the gradients also accept a batch (the reference's analytic gradients take one point).
The h values are differentiable (autograd, first order) through the kernel's own gradient.
"""
from __future__ import annotations

from typing import Sequence

import torch
from torch import Tensor

from .. import _points as P
from ..problem import CircleObstacle

__all__ = ["CircleObstacle", "h_circle_obstacle", "grad_h_circle_obstacle", "h_multi_circle_obstacles",
           "grad_h_multi_circle_obstacles", "h_min_circle_obstacles", "grad_h_min_circle_obstacles"]


def _h_launch(xs: Tensor, sp, want_grad: bool):
    """h [n] (and grad h [n, 3]) of the points xs [..., F >= 2] from dtmpc_h_eval, shaped like xs's batch."""
    F = xs.shape[-1]
    xr, lead = P.rows(xs, F, xs)
    n = xr.shape[0]
    h = torch.empty(n, dtype=xr.dtype, device=xr.device)
    g = torch.empty(n, 3, dtype=xr.dtype, device=xr.device) if want_grad else None
    if n > 0:
        P.launch("dtmpc_h_eval", P.dtype_code(xr), P.byref(sp), n, F, xr.data_ptr(), h.data_ptr(), P.ptr(g),
                 P.stream(xr))
    return h.reshape(lead), (g.reshape(*lead, 3) if want_grad else None)


class _HValue(torch.autograd.Function):
    """h(x) as an autograd node: backward dL/dx = dL/dh grad h(x), grad h from the same kernel launch
    (the reference's analytic gradients, core/systems/dubins_obstacles.py:33-38, 72-92, 109-117; the
    exact min's argmin subgradient as torch.min's).  First order only (once_differentiable: a second
    derivative of h raises)."""

    @staticmethod
    def forward(ctx, xs: Tensor, sp):
        P.require_device(xs)
        h, g = _h_launch(xs, sp, True)
        F = xs.shape[-1]
        gx = g[..., :F] if F <= 3 else torch.cat([g, g.new_zeros(*g.shape[:-1], F - 3)], -1)
        ctx.save_for_backward(gx)
        return h

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, gh: Tensor):
        (gx,) = ctx.saved_tensors
        return gh.unsqueeze(-1) * gx, None


def _h(x: Tensor, sp, want_grad: bool):
    unbatched = x.ndim == 1
    xs = x.unsqueeze(0) if unbatched else x
    if xs.shape[-1] < 2:
        raise ValueError("x must hold (px, py, ...)")
    if not want_grad and torch.is_grad_enabled() and xs.requires_grad:
        h = _HValue.apply(xs, sp)
        return h.squeeze(0) if unbatched else h
    P.require_device(xs)
    h, g = _h_launch(xs, sp, want_grad)
    out = g if want_grad else h
    return out.squeeze(0) if unbatched else out


def _agg_spec(obstacles: Sequence[CircleObstacle], agg: str, beta: float = 20.0):
    return P.spec(obstacles=tuple(obstacles), aggregation=agg if len(obstacles) else "none", beta=beta)


def h_circle_obstacle(x: Tensor, *, obs: CircleObstacle) -> Tensor:
    """core/systems/dubins_obstacles.py:16-30: ||p - c||^2 - r^2."""
    return _h(x, _agg_spec((obs,), "single"), False)


def grad_h_circle_obstacle(x: Tensor, *, obs: CircleObstacle) -> Tensor:
    """core/systems/dubins_obstacles.py:33-38: [2 (px - cx), 2 (py - cy), 0]."""
    return _h(x, _agg_spec((obs,), "single"), True)


def h_multi_circle_obstacles(x: Tensor, *, obstacles: list[CircleObstacle], beta: float = 20.0) -> Tensor:
    """core/systems/dubins_obstacles.py:41-69: smooth-min -(1/beta) log sum exp(-beta h_i) (stable LSE);
    no obstacles: h = 1."""
    return _h(x, _agg_spec(obstacles, "smoothmin", beta), False)


def grad_h_multi_circle_obstacles(x: Tensor, *, obstacles: list[CircleObstacle], beta: float = 20.0) -> Tensor:
    """core/systems/dubins_obstacles.py:72-92: sum_i softmax(-beta h)_i grad h_i."""
    return _h(x, _agg_spec(obstacles, "smoothmin", beta), True)


def h_min_circle_obstacles(x: Tensor, *, obstacles: list[CircleObstacle]) -> Tensor:
    """core/systems/dubins_obstacles.py:95-106: min_i h_i; no obstacles: h = 1."""
    return _h(x, _agg_spec(obstacles, "min"), False)


def grad_h_min_circle_obstacles(x: Tensor, *, obstacles: list[CircleObstacle]) -> Tensor:
    """core/systems/dubins_obstacles.py:109-117: grad h of the argmin obstacle."""
    return _h(x, _agg_spec(obstacles, "min"), True)
