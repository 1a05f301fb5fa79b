"""Cost derivatives (counterpart of the reference's core/cost_derivs.py, same names and keywords).

* u-form (the box-constrained solver's): ``nominal_cost_derivs_u`` / ``auxiliary_cost_derivs_u``
  (core/cost_derivs.py:58-76, 110-130) -> ``(l_x, l_u, l_xx, l_uu, l_ux)`` and
  ``nominal_terminal_derivs`` / ``auxiliary_terminal_derivs`` (:133-146) -> ``(phi_x, phi_xx)``: the
  gradients from the HIP kernel ``dtmpc_cost_derivs`` (include/dtmpc_systems.h), the constant Hessians
  diag(2Q, 2qb), diag(2R), 0 (terminal diag(2Qf, 0)) built in the working precision.
* v-form (tanh-box decision variable): ``nominal_cost_derivs`` / ``auxiliary_cost_derivs``
  (:27-107) with the reference's return tuple ``(l_x, l_v, l_xx, l_vv, l_vx)``.

Every argument may carry leading batch dimensions (x_hat [..., 4], u / v [..., 2], x_ref [..., 3],
u_ref [..., 2]); unbatched inputs give the reference's shapes ([4], [2], [4, 4], [2, 2], [2, 4]).
Q, R, Qf, qb and target are shared by the batch (tensors or floats).  The v-form derivatives come from
the HIP kernel of ``dtmpc_tanh_cost_derivs``; l_xx = diag(2Q, 2qb) and l_vx = 0 are constants.  The
solver kernels evaluate the u-form in place along their tapes (``core.ddp.linearize`` exposes that).
"""
from __future__ import annotations

from typing import Tuple

import torch
from torch import Tensor

from .control import BoxTanhControl, tanh_box_eval
from .problem import QuadraticCost

__all__ = ["nominal_cost_derivs", "auxiliary_cost_derivs", "nominal_cost_derivs_u", "auxiliary_cost_derivs_u",
           "nominal_terminal_derivs", "auxiliary_terminal_derivs"]


def _vals(t, n: int):
    vals = [float(x) for x in (t.reshape(-1).tolist() if isinstance(t, Tensor) else ([t] if n == 1 else t))]
    if len(vals) != n:
        raise ValueError(f"expected {n} weight values, got {len(vals)}")
    return vals


def _consts(v: Tensor, Q, qb) -> Tuple[Tensor, Tensor]:
    lead = v.shape[:-1]
    # 2 * [Q, qb] in the working precision, as the reference's tensors round it
    lxx_d = 2.0 * torch.tensor(_vals(Q, 3) + _vals(qb, 1), dtype=v.dtype, device=v.device)
    l_xx = torch.diag(lxx_d).expand(*lead, 4, 4).clone()
    l_vx = torch.zeros(*lead, 2, 4, dtype=v.dtype, device=v.device)
    return l_xx, l_vx


def nominal_cost_derivs(*, x_hat: Tensor, v: Tensor, target, Q, R, qb, ctrl: BoxTanhControl):
    """core/cost_derivs.py:27-55: target cost sum Q (x - target)^2 + R u(v)^2 + qb b^2 in v."""
    t = _vals(target, 3) if not (isinstance(target, Tensor) and target.dim() > 1) else None
    if t is None:
        raise ValueError("nominal_cost_derivs takes one target shared by the batch")
    cost = QuadraticCost(kind="target", Q=tuple(_vals(Q, 3)), R=tuple(_vals(R, 2)), qb=_vals(qb, 1)[0], target=tuple(t))
    o = tanh_box_eval(ctrl, v, cost=cost, x_hat=x_hat)
    l_xx, l_vx = _consts(v, Q, qb)
    return o["lx"], o["lv"], l_xx, torch.diag_embed(o["lvv"]), l_vx


def auxiliary_cost_derivs(*, x_hat: Tensor, v: Tensor, x_ref: Tensor, u_ref: Tensor, Q, R, qb, ctrl: BoxTanhControl):
    """core/cost_derivs.py:79-107: tracking cost sum Q (x - x_ref)^2 + R (u(v) - u_ref)^2 + qb b^2 in v."""
    cost = QuadraticCost(kind="track", Q=tuple(_vals(Q, 3)), R=tuple(_vals(R, 2)), qb=_vals(qb, 1)[0])
    lead = v.shape[:-1]
    o = tanh_box_eval(ctrl, v, cost=cost, x_hat=x_hat, x_ref=x_ref.expand(*lead, x_ref.shape[-1]),
                      u_ref=u_ref.expand(*lead, 2))
    l_xx, l_vx = _consts(v, Q, qb)
    return o["lx"], o["lv"], l_xx, torch.diag_embed(o["lvv"]), l_vx


# ------------------------------------------------------------------------------------------ u-form
def _u_form(x_hat: Tensor, u, x_ref, u_ref, *, kind: str, Q, R, qb, Qf, target, terminal: bool):
    from . import _points as P

    P.require_device(x_hat, u if isinstance(u, Tensor) else None, x_ref, u_ref)
    unbatched = x_hat.ndim == 1
    xs = x_hat.unsqueeze(0) if unbatched else x_hat
    xr, lead = P.rows(xs, 4, xs)
    n = xr.shape[0]
    ur = P.rows((u.unsqueeze(0) if u.ndim == 1 else u).expand(*lead, 2), 2, xs)[0] if not terminal else None
    rx = P.rows(x_ref[..., :3].expand(*lead, 3), 3, xs)[0] if kind == "track" else None
    ru = (P.rows(u_ref.expand(*lead, 2), 2, xs)[0] if (kind == "track" and not terminal) else None)
    cost = QuadraticCost(kind=kind, Q=tuple(_vals(Q, 3)) if Q is not None else (0.0, 0.0, 0.0),
                         R=tuple(_vals(R, 2)) if R is not None else (0.0, 0.0),
                         Qf=tuple(_vals(Qf, 3)) if Qf is not None else (0.0, 0.0, 0.0),
                         qb=_vals(qb, 1)[0] if qb is not None else 0.0,
                         target=tuple(_vals(target, 3)) if target is not None else (0.0, 0.0, 0.0))
    cc = cost.to_c()
    lx = torch.empty(n, 4, dtype=xr.dtype, device=xr.device)
    lu = torch.empty(n, 2, dtype=xr.dtype, device=xr.device) if not terminal else None
    if n > 0:
        P.launch("dtmpc_cost_derivs", P.dtype_code(xr), P.byref(cc), 1 if terminal else 0, n, xr.data_ptr(),
                 P.ptr(ur), P.ptr(rx), P.ptr(ru), lx.data_ptr(), P.ptr(lu), P.stream(xr))
    shape = lambda t, F: (t.reshape(*lead, F).squeeze(0) if unbatched else t.reshape(*lead, F))  # noqa: E731
    kw = dict(dtype=xr.dtype, device=xr.device)
    if terminal:
        d = 2.0 * torch.tensor(list(cost.Qf) + [0.0], **kw)
        return shape(lx, 4), torch.diag(d).expand(*(() if unbatched else lead), 4, 4).clone()
    dxx = 2.0 * torch.tensor(list(cost.Q) + [cost.qb], **kw)
    duu = 2.0 * torch.tensor(list(cost.R), **kw)
    L = () if unbatched else lead
    return (shape(lx, 4), shape(lu, 2), torch.diag(dxx).expand(*L, 4, 4).clone(),
            torch.diag(duu).expand(*L, 2, 2).clone(), torch.zeros(*L, 2, 4, **kw))


def nominal_cost_derivs_u(*, x_hat: Tensor, u: Tensor, target, Q, R, qb):
    """core/cost_derivs.py:58-76: l_x = [2Q (x - target), 2 qb b], l_u = 2R u, l_xx = diag(2Q, 2qb),
    l_uu = diag(2R), l_ux = 0.  x_hat [..., 4], u [..., 2] on a HIP device."""
    return _u_form(x_hat, u, None, None, kind="target", Q=Q, R=R, qb=qb, Qf=None, target=target, terminal=False)


def auxiliary_cost_derivs_u(*, x_hat: Tensor, u: Tensor, x_ref: Tensor, u_ref: Tensor, Q, R, qb):
    """core/cost_derivs.py:110-130: l_x = [2Q (x - x_ref), 2 qb b], l_u = 2R (u - u_ref), constant
    Hessians as the nominal form."""
    return _u_form(x_hat, u, x_ref, u_ref, kind="track", Q=Q, R=R, qb=qb, Qf=None, target=None, terminal=False)


def nominal_terminal_derivs(*, x_hat_N: Tensor, target, Qf):
    """core/cost_derivs.py:133-138: phi_x = [2Qf (x_N - target), 0], phi_xx = diag(2Qf, 0)."""
    return _u_form(x_hat_N, None, None, None, kind="target", Q=None, R=None, qb=None, Qf=Qf, target=target,
                   terminal=True)


def auxiliary_terminal_derivs(*, x_hat_N: Tensor, x_ref_N: Tensor, Qf):
    """core/cost_derivs.py:141-146: phi_x = [2Qf (x_N - x_ref_N), 0], phi_xx = diag(2Qf, 0)."""
    return _u_form(x_hat_N, None, x_ref_N, None, kind="track", Q=None, R=None, qb=None, Qf=Qf, target=None,
                   terminal=True)
