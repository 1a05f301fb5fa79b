"""Optimal-control-problem utilities (counterpart of the reference's core/ocp.py:35-85).

The reference's ``rollout_dynamics(x0, U, *, f)`` and ``total_cost(*, X, U, stage_cost, terminal_cost,
stage_kwargs, terminal_kwargs)`` take Python closures; here the closure is the typed problem / cost
(``f``: :class:`DubinsDBaSProblem`, the DBaS-augmented Dubins step f_hat; ``cost``:
:class:`QuadraticCost`, the stage / terminal expressions of core/tube_mpc.py:823-832 / 875-885 and
run_nominal.py:297-324), evaluated by the HIP kernels behind ``dtmpc_dbas_rollout`` and
``dtmpc_tape_cost``.  Both accept the reference's batched ([B, ...]) and unbatched layouts.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional

import torch
from torch import Tensor

from .. import _lib
from .ddp import _dtype_code, _ptr, _require_device, rollout, to_soa
from .problem import DubinsDBaSProblem, QuadraticCost

__all__ = ["OCPConfig", "rollout_dynamics", "total_cost"]


@dataclass(frozen=True)
class OCPConfig:
    """core/ocp.py:28-32"""

    horizon: int
    nx: int
    nu: int


def rollout_dynamics(x0: Tensor, U: Tensor, *, f: DubinsDBaSProblem) -> Tensor:
    """X[k+1] = f_hat(X[k], U[k]) (core/ocp.py:35-60).  x0 [B, 4] or [4] (x, y, theta, b); U [B, N, 2] or
    [N, 2]; returns X [B, N+1, 4] or [N+1, 4], matching the batch mode of the inputs."""
    batched = x0.ndim == 2
    x0b, Ub = (x0, U) if batched else (x0.unsqueeze(0), U.unsqueeze(0))
    if Ub.shape[1] != f.horizon:
        raise ValueError(f"U has {Ub.shape[1]} steps, the problem's horizon is {f.horizon}")
    X = rollout(f, x0b, Ub)
    return X if batched else X.squeeze(0)


def total_cost(*, X: Tensor, U: Tensor, cost: QuadraticCost, X_ref: Optional[Tensor] = None,
               U_ref: Optional[Tensor] = None) -> Tensor:
    """J = sum_{k<N} l_k + phi_N per trajectory (core/ocp.py:63-85).  X [B, N+1, 4] or [N+1, 4], U [B, N, 2]
    or [N, 2]; X_ref [.., N+1, >=3] / U_ref [.., N, 2] for a tracking cost.  Returns J [B] or a scalar."""
    batched = X.ndim == 3
    up = (lambda t: t) if batched else (lambda t: None if t is None else t.unsqueeze(0))
    Xb, Ub, Xr, Ur = up(X), up(U), up(X_ref), up(U_ref)
    _require_device(Xb, Ub, Xr, Ur)
    if Ub.ndim != 3 or Ub.shape[-1] != 2:
        raise ValueError("U must be [B, N, 2] (or [N, 2])")
    B, N = Ub.shape[0], Ub.shape[1]
    if Xb.shape != (B, N + 1, 4):
        raise ValueError(f"X must be [{B}, {N + 1}, 4]")
    if cost.kind == "track":
        if Xr is None or Ur is None:
            raise ValueError("a tracking cost needs X_ref and U_ref")
        # the kernel reads [N+1][3][B] / [N][2][B] references: an unbatched one is broadcast, anything
        # else must match the batch exactly (never read past a short reference on the device)
        if Xr.ndim == 3 and Xr.shape[0] == 1 and B > 1:
            Xr = Xr.expand(B, *Xr.shape[1:])
        if Ur.ndim == 3 and Ur.shape[0] == 1 and B > 1:
            Ur = Ur.expand(B, *Ur.shape[1:])
        if Xr.ndim != 3 or Xr.shape[:2] != (B, N + 1) or Xr.shape[-1] < 3:
            raise ValueError(f"X_ref must be [{B}, {N + 1}, >=3]")
        if Ur.shape != (B, N, 2):
            raise ValueError(f"U_ref must be [{B}, {N}, 2]")
    spec = DubinsDBaSProblem(horizon=N).to_c()
    cc = cost.to_c()
    Xs, Us = to_soa(Xb), to_soa(Ub.to(Xb.dtype))
    Xrs = to_soa(Xr[..., :3].to(Xb.dtype)) if cost.kind == "track" else None
    Urs = to_soa(Ur.to(Xb.dtype)) if cost.kind == "track" else None
    J = torch.empty(B, dtype=Xb.dtype, device=Xb.device)
    lib = _lib.load()
    _lib.check(lib.dtmpc_tape_cost(_dtype_code(Xb), C.byref(spec), C.byref(cc), B, Xs.data_ptr(), Us.data_ptr(),
                                   _ptr(Xrs), _ptr(Urs), J.data_ptr(), _lib.stream_of(Xb)), "dtmpc_tape_cost")
    return J if batched else J.squeeze(0)
