"""Discrete barrier states (counterpart of the reference's core/barrier.py, same names and keywords).

The barrier functions evaluate in the HIP kernel of ``dtmpc_barrier_eval`` (include/dtmpc_systems.h),
elementwise over tensors of any shape on a HIP device; ``dbas_step`` / ``dbas_init_b0`` take the
reference's callables f and h (evaluated as given -- the package's own ``systems.dubins.dubins_step``
and ``systems.dubins_obstacles.h_*`` are device kernels) and combine them with the device barrier.
There is no CPU fallback.  B is differentiable (autograd, first order, through the kernel's dB), so
``dbas_step`` composed with the package's differentiable ``dubins_step`` and ``h_*`` is too.  The fused solver kernels use the same device barrier code
(``dtmpc_device.hpp`` barrier_relaxed / barrier_dyn).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Callable, Literal, Union

import torch
from torch import Tensor

from .. import _abi
from . import _points as P

__all__ = ["BarrierType", "DBaSConfig", "relaxed_inverse_barrier_B_alpha", "barrier_B", "dbas_step", "dbas_init_b0",
           "barrier_and_derivative"]

BarrierType = Literal["inverse", "log"]
ScalarLike = Union[float, Tensor]


@dataclass(frozen=True)
class DBaSConfig:
    """core/barrier.py:16-33 (same fields and defaults)."""

    barrier_type: BarrierType = "inverse"
    alpha: ScalarLike = 0.1
    gamma: ScalarLike = 0.0
    eps: float = 1e-6


def _barrier_launch(z: Tensor, kind: int, alpha: float, eps: float, want_B: bool, want_dB: bool):
    n = z.numel()
    Bz = torch.empty_like(z) if want_B else None
    dBz = torch.empty_like(z) if want_dB else None
    if n > 0:
        P.launch("dtmpc_barrier_eval", P.dtype_code(z), int(kind), float(alpha), float(eps), n, z.data_ptr(),
                 P.ptr(Bz), P.ptr(dBz), P.stream(z))
    return Bz, dBz


class _Barrier(torch.autograd.Function):
    """B(zeta) as an autograd node: backward dL/dzeta = dL/dB dB/dzeta with dB from the same launch (the
    reference's barriers are torch expressions, core/barrier.py:36-72).  First order only."""

    @staticmethod
    def forward(ctx, zeta: Tensor, kind: int, alpha: float, eps: float):
        P.require_device(zeta)
        Bz, dBz = _barrier_launch(zeta.contiguous(), kind, alpha, eps, True, True)
        ctx.save_for_backward(dBz)
        return Bz

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, g: Tensor):
        (dBz,) = ctx.saved_tensors
        return g * dBz, None, None, None


def barrier_and_derivative(zeta: Tensor, *, kind: int, alpha: float = 0.0, eps: float = 1e-12, want_B: bool = True,
                           want_dB: bool = False):
    """(B(zeta), dB/dzeta) of one barrier kind of ``dtmpc_barrier_eval`` (either may be skipped: None).
    B alone of an input that requires grad is an autograd node (_Barrier); dB is not differentiable."""
    if want_B and not want_dB and torch.is_grad_enabled() and zeta.requires_grad:
        return _Barrier.apply(zeta, int(kind), float(alpha), float(eps)), None
    P.require_device(zeta)
    return _barrier_launch(zeta.contiguous(), kind, alpha, eps, want_B, want_dB)


def relaxed_inverse_barrier_B_alpha(zeta: Tensor, *, alpha: ScalarLike, eps: float = 1e-12) -> Tensor:
    """core/barrier.py:36-59: 1/zeta for zeta >= alpha_eff, else the quadratic extension
    1/a - (zeta - a)/a^2 + (zeta - a)^2/a^3, with alpha_eff = max(alpha, eps)."""
    a = P.scalar(alpha)
    if a < 0:
        raise ValueError("alpha must be >= 0")
    return barrier_and_derivative(zeta, kind=_abi.BARRIER_INVERSE, alpha=a, eps=eps)[0]


def barrier_B(zeta: Tensor, *, barrier_type: BarrierType, eps: float = 1e-12) -> Tensor:
    """core/barrier.py:62-72: inverse 1 / max(zeta, eps), log -log(max(zeta, eps))."""
    if barrier_type == "inverse":
        return barrier_and_derivative(zeta, kind=_abi.BARRIER_INVERSE_PLAIN, eps=eps)[0]
    if barrier_type == "log":
        return barrier_and_derivative(zeta, kind=_abi.BARRIER_LOG, eps=eps)[0]
    raise ValueError(f"Unknown barrier_type: {barrier_type}")


def _B(h: Tensor, cfg: DBaSConfig) -> Tensor:
    if cfg.barrier_type == "inverse":
        return relaxed_inverse_barrier_B_alpha(h, alpha=cfg.alpha, eps=cfg.eps)
    return barrier_B(h, barrier_type="log", eps=cfg.eps)


def dbas_step(*, x_k: Tensor, u_k: Tensor, b_k: Tensor, f: Callable[[Tensor, Tensor], Tensor],
              h: Callable[[Tensor], Tensor], cfg: DBaSConfig) -> tuple[Tensor, Tensor]:
    """core/barrier.py:75-108: x_{k+1} = f(x_k, u_k), b_{k+1} = B(h(x_{k+1})) - gamma (B(h(x_k)) - b_k)
    (relaxed inverse B_alpha, or the exact log barrier)."""
    if isinstance(cfg.gamma, (float, int)) and not (-1.0 <= cfg.gamma <= 1.0):
        raise ValueError("gamma must be in [-1, 1]")
    x_next = f(x_k, u_k)
    B_next = _B(h(x_next), cfg)
    B_curr = _B(h(x_k), cfg)
    gamma = cfg.gamma if isinstance(cfg.gamma, Tensor) else torch.tensor(cfg.gamma, device=B_next.device,
                                                                           dtype=B_next.dtype)
    return x_next, B_next - gamma * (B_curr - b_k)


def dbas_init_b0(x0: Tensor, *, h: Callable[[Tensor], Tensor], cfg: DBaSConfig) -> Tensor:
    """core/barrier.py:111-120: b_0 = B_alpha(h(x_0)) (inverse) or -log(h(x_0)) (log)."""
    return _B(h(x0), cfg)
