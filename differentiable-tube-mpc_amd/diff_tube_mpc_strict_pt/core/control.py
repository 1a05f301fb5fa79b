"""Control parameterisations (counterpart of the reference's core/control.py).

* :class:`BoxClampControl` (core/control.py:38-70) -- the box the solvers clamp to.  Every solver
  entry point takes its bounds from the problem (``DubinsDBaSProblem.u_min / u_max / active_tol``);
  :meth:`BoxClampControl.problem_bounds` gives those fields, so a caller that builds the reference's
  object keeps doing so.  ``clamp`` and ``active_mask`` evaluate in the HIP kernel of
  ``dtmpc_box_clamp`` (include/dtmpc_systems.h) over u [..., 2] on a HIP device.
* :class:`BoxTanhControl` (core/control.py:10-35) -- u = u_min + (u_max - u_min)(tanh(v) + 1)/2 over an
  unconstrained decision variable v.  ``u`` and ``du_dv_diag`` evaluate in the HIP kernel of
  ``dtmpc_tanh_cost_derivs`` (include/dtmpc_control.h); v must be a device tensor of shape [..., 2].
  There is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass
from typing import Dict, Optional, Sequence, Tuple

import torch
from torch import Tensor

from .. import _lib
from .problem import DubinsDBaSProblem, QuadraticCost

__all__ = ["BoxClampControl", "BoxTanhControl", "tanh_box_eval"]


def _pair(v) -> Tuple[float, float]:
    vals = [float(x) for x in (v.tolist() if isinstance(v, Tensor) else v)]
    if len(vals) != 2:
        raise ValueError("the Dubins control box has two bounds per side")
    return vals[0], vals[1]


@dataclass(frozen=True)
class BoxClampControl:
    """Hard box u in [u_min, u_max] with the active-set tolerance (core/control.py:38-70)."""

    u_min: Sequence[float] | Tensor
    u_max: Sequence[float] | Tensor
    active_tol: float = 1e-8

    def problem_bounds(self) -> Dict[str, object]:
        """Keyword arguments of :class:`DubinsDBaSProblem` for this box."""
        return {"u_min": _pair(self.u_min), "u_max": _pair(self.u_max), "active_tol": float(self.active_tol)}

    def _eval(self, u: Tensor, want_u: bool, want_mask: bool):
        from . import _points as P

        P.require_device(u)
        unbatched = u.ndim == 1
        us = u.unsqueeze(0) if unbatched else u
        ur, lead = P.rows(us, 2, us)
        n = ur.shape[0]
        uo = torch.empty_like(ur) if want_u else None
        m = torch.empty(n, 2, dtype=torch.bool, device=ur.device) if want_mask else None
        if n > 0:
            b = self.problem_bounds()
            sp = P.spec(u_min=b["u_min"], u_max=b["u_max"], active_tol=b["active_tol"])
            P.launch("dtmpc_box_clamp", P.dtype_code(ur), P.byref(sp), n, ur.data_ptr(), P.ptr(uo), P.ptr(m),
                     P.stream(ur))
        out = uo if want_u else m
        out = out.reshape(*lead, 2)
        return out.squeeze(0) if unbatched else out

    def clamp(self, u: Tensor) -> Tensor:
        """core/control.py:61-64: torch.clamp(u, u_min, u_max) (NaN propagates).  Differentiable like
        torch.clamp (_BoxClamp: the gradient passes where u_min <= u <= u_max)."""
        if torch.is_grad_enabled() and u.requires_grad:
            return _BoxClamp.apply(u, self)
        return self._eval(u, True, False)

    def active_mask(self, u: Tensor) -> Tensor:
        """core/control.py:66-70: bool [..., 2], u within active_tol of a bound."""
        return self._eval(u, False, True)


class _BoxClamp(torch.autograd.Function):
    """BoxClampControl.clamp as an autograd node: forward the dtmpc_box_clamp kernel, backward torch.clamp's
    rule (grad where u_min <= u <= u_max, 0 outside and for NaN), in torch ops on the saved input."""

    @staticmethod
    def forward(ctx, u: Tensor, box: "BoxClampControl"):
        ctx.save_for_backward(u)
        ctx.box = box
        return box._eval(u, True, False)

    @staticmethod
    def backward(ctx, g: Tensor):
        (u,) = ctx.saved_tensors
        lo, hi = _pair(ctx.box.u_min), _pair(ctx.box.u_max)
        lo_t = torch.tensor(lo, dtype=u.dtype, device=u.device)
        hi_t = torch.tensor(hi, dtype=u.dtype, device=u.device)
        return g * ((u >= lo_t) & (u <= hi_t)).to(g.dtype), None


@dataclass(frozen=True)
class BoxTanhControl:
    """Differentiable box via tanh (core/control.py:10-35)."""

    u_min: Sequence[float] | Tensor
    u_max: Sequence[float] | Tensor

    def __post_init__(self) -> None:
        _pair(self.u_min), _pair(self.u_max)  # two bounds per side (any values, as the reference)

    def problem(self, horizon: int = 1) -> DubinsDBaSProblem:
        return DubinsDBaSProblem(horizon=horizon, u_min=_pair(self.u_min), u_max=_pair(self.u_max))

    def u(self, v: Tensor) -> Tensor:
        """u_min + (u_max - u_min) (tanh(v) + 1) / 2 (core/control.py:22-27), v [..., 2]."""
        return tanh_box_eval(self, v)["u"]

    def du_dv_diag(self, v: Tensor) -> Tensor:
        """Elementwise du/dv (core/control.py:29-35), v [..., 2]."""
        return tanh_box_eval(self, v)["dudv"]


def tanh_box_eval(ctrl: BoxTanhControl, v: Tensor, *, cost: Optional[QuadraticCost] = None,
                  x_hat: Optional[Tensor] = None, x_ref: Optional[Tensor] = None,
                  u_ref: Optional[Tensor] = None) -> Dict[str, Tensor]:
    """One launch of ``dtmpc_tanh_cost_derivs`` over the points of v [..., 2] (a horizon-1 tape per
    point).  With ``cost`` it also returns the v-space stage-cost derivatives l_x [..., 4], l_v, and
    diag(l_vv) [..., 2] (x_hat [..., 4] required; x_ref [..., 3] / u_ref [..., 2] for a tracking cost)."""
    from .ddp import _dtype_code, _ptr, _require_device

    _require_device(v, x_hat, x_ref, u_ref)
    if v.shape[-1] != 2:
        raise ValueError("v must have a trailing dimension of 2")
    lead = v.shape[:-1]
    n = math.prod(lead)
    kw = dict(dtype=v.dtype, device=v.device)
    out = {k: torch.empty(*lead, 2, **kw) for k in ("u", "dudv")}
    if n == 0:
        if cost is not None:
            out.update(lx=torch.empty(*lead, 4, **kw), lv=torch.empty(*lead, 2, **kw), lvv=torch.empty(*lead, 2, **kw))
        return out
    cc = (cost if cost is not None else QuadraticCost()).to_c()
    Vd = v.reshape(n, 2).t().contiguous()  # [1][2][n] SoA
    Xs = Xr = Ur = lx = lv = lvv = None
    if cost is not None:
        if x_hat is None:
            raise ValueError("x_hat is required for the cost derivatives")
        # every per-point operand pairs with v's points: same leading shape (an unbatched one is
        # broadcast), never a reshape of a different layout with the same element count
        def per_point(t: Tensor, F: int, name: str) -> Tensor:
            if t.shape[-1] < F:
                raise ValueError(f"{name} must have a trailing dimension of at least {F}")
            if t.shape[:-1] != lead:
                if t.dim() != 1:
                    raise ValueError(f"{name} leading shape {tuple(t.shape[:-1])} does not match v's {tuple(lead)}")
                t = t.expand(*lead, t.shape[-1])
            return t[..., :F].to(v.dtype).reshape(n, F).t().contiguous()

        Xs = per_point(x_hat, 4, "x_hat")
        if cost.kind == "track":
            if x_ref is None or u_ref is None:
                raise ValueError("a tracking cost needs x_ref and u_ref")
            Xr = per_point(x_ref, 3, "x_ref")
            Ur = per_point(u_ref, 2, "u_ref")
        lx = torch.empty(4, n, **kw)
        lv = torch.empty(2, n, **kw)
        lvv = torch.empty(2, n, **kw)
    U = torch.empty(2, n, **kw)
    dU = torch.empty(2, n, **kw)
    lib = _lib.load()
    spec = ctrl.problem(1).to_c()
    _lib.check(lib.dtmpc_tanh_cost_derivs(_dtype_code(v), C.byref(spec), C.byref(cc), n, _ptr(Xs), Vd.data_ptr(),
                                          _ptr(Xr), _ptr(Ur), U.data_ptr(), dU.data_ptr(), _ptr(lx), _ptr(lv),
                                          _ptr(lvv), _lib.stream_of(v)), "dtmpc_tanh_cost_derivs")
    out["u"] = U.t().reshape(*lead, 2)
    out["dudv"] = dU.t().reshape(*lead, 2)
    if cost is not None:
        out["lx"] = lx.t().reshape(*lead, 4)
        out["lv"] = lv.t().reshape(*lead, 2)
        out["lvv"] = lvv.t().reshape(*lead, 2)
    return out
