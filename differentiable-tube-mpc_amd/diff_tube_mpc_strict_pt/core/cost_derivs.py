"""Stage-cost derivatives in the tanh-box decision variable v (counterpart of the reference's
core/cost_derivs.py:27-107), with the reference's keyword signatures and return tuple
``(l_x, l_v, l_xx, l_vv, l_vx)``.

Every argument may carry leading batch dimensions (x_hat [..., 4], v [..., 2], target / x_ref [..., 3],
u_ref [..., 2]); unbatched inputs give the reference's shapes ([4], [2], [4, 4], [2, 2], [2, 4]).
Q, R, qb are the cost weights (tensors or floats, shared over the batch).  The derivatives are computed
by the HIP kernel of ``dtmpc_tanh_cost_derivs``; l_xx = diag(2Q, 2qb) and l_vx = 0 are constants.
The box-constrained ``*_cost_derivs_u`` forms (core/cost_derivs.py:58-76, 110-130) are fused into
the solver kernels (``core.ddp.linearize`` exposes them along a tape).
"""
from __future__ import annotations

from typing import Tuple

import torch
from torch import Tensor

from .control import BoxTanhControl, tanh_box_eval
from .problem import QuadraticCost

__all__ = ["nominal_cost_derivs", "auxiliary_cost_derivs"]


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
