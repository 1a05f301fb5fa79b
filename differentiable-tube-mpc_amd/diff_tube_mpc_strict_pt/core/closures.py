"""The reference's closure form of the solver API, as an adapter beside the typed one.

The reference's solvers take Python closures (``ilqr_solve(*, x0, V_init, cfg, f, f_jac, ctrl, stage_cost,
terminal_cost, stage_derivs, terminal_derivs, feasible_fn, ...)``, core/ddp.py:102-117;
``ddp_sensitivity(*, X, V, f, f_jac, ctrl, stage_hess, terminal_hess, upper_grad_x, upper_grad_u,
upper_grad_xN)``, :317-329; ``rollout(x0, V, *, f)``, :89) and call them point by point.  A HIP kernel
cannot call a Python closure, so the closures a caller hands over must SAY what they compute: this module
builds them as objects that are both

* callables with the reference's signatures, evaluated on the device through the per-function API
  (``f_hat(x_hat, u)`` -> x_hat', ``stage_cost(x_hat, u, k)``, ``stage_derivs(x_hat, u, k)``, ...), and
* carriers of the typed description the kernels consume (:class:`DubinsDBaSProblem`, :class:`QuadraticCost`).

``core.ddp.ilqr_solve`` / ``ddp_sensitivity`` / ``rollout`` accept the keyword form and resolve it here
(:func:`resolve_ilqr` / :func:`resolve_sensitivity`); closures that are not these objects are refused with
a TypeError (there is no Python-level solver to run them on).  :func:`nominal_closures` builds the set that
``run_nominal.py:284-324`` defines, so that file's solver call (:353-364) runs unchanged against this
package: ``ilqr_solve(x0=x_hat0, V_init=U_ws, cfg=ilqr_cfg, f=f_hat, ctrl=ctrl, f_jac=..., stage_cost=...,
terminal_cost=..., stage_derivs=..., terminal_derivs=...)``.

Mapping of the optional arguments:
* ``f_jac``: the reference's analytic Jacobian of ``f`` (``dubins_augmented_jacobian``); the device always
  linearises the resolved ``f`` with that same analytic Jacobian, so any callable is accepted in its place
  (the reference's call site passes a lambda around ``dubins_augmented_jacobian``);
* ``ctrl``: a :class:`BoxClampControl` gives the box and the active-set tolerance; ``None`` means no clamp
  (the reference skips ``ctrl.clamp`` then): unbounded box;
* ``feasible_fn``: no device counterpart (the reference's callers never pass it): NotImplementedError.
"""
from __future__ import annotations

import dataclasses
import math
from typing import Any, Callable, Dict, Optional, Tuple

import torch
from torch import Tensor

from .control import BoxClampControl
from .problem import DubinsDBaSProblem, ILQRConfig, QuadraticCost

__all__ = ["DBaSDynamics", "QuadraticClosures", "ParamClosures", "nominal_closures", "resolve_ilqr",
           "resolve_sensitivity", "resolve_ift", "ResolvedCall"]


def _wrap(e: Tensor) -> Tensor:
    """run_nominal.py:32-34: (e + pi) mod 2 pi - pi as atan2(sin e, cos e)."""
    return torch.atan2(torch.sin(e), torch.cos(e))


class DBaSDynamics:
    """f_hat(x_hat_k, u_k) -> x_hat_{k+1} = [f(x, u), B(h(f(x, u))) - gamma (B(h(x)) - b)] (core/barrier.py:75-108
    as wrapped by run_nominal.py:284-288 / core/tube_mpc.py:816-821) for the problem's dynamics, obstacles and
    DBaS; ``jacobian`` is its augmented Jacobian (core/systems/dubins_aug_jac.py:61-139).  x_hat [4] or
    [B, 4], u [2] or [B, 2] on a HIP device."""

    def __init__(self, problem: DubinsDBaSProblem):
        self.problem = problem
        self._one = dataclasses.replace(problem, horizon=1)

    def __call__(self, x_hat: Tensor, u: Tensor) -> Tensor:
        from .ddp import rollout

        single = x_hat.ndim == 1
        xs = x_hat.reshape(-1, 4)
        us = u.reshape(-1, 1, 2).expand(xs.shape[0], 1, 2).contiguous()
        out = rollout(self._one, xs, us)[:, 1]
        return out[0] if single else out

    def jacobian(self, x_hat: Tensor, u: Tensor) -> Tuple[Tensor, Tensor]:
        from .systems.dubins_aug_jac import _jac

        return _jac(x_hat, u, self._one.to_c())


class QuadraticClosures:
    """The cost closures of one QuadraticCost with the reference's signatures: stage_cost(x_hat, u, k),
    terminal_cost(x_hat_N), stage_derivs(x_hat, u, k) -> (l_x, l_u, l_xx, l_uu, l_ux), terminal_derivs(x_hat_N)
    -> (phi_x, phi_xx), stage_hess(x_hat, u, k) -> (l_xx, l_uu, l_ux), terminal_hess(x_hat_N) -> phi_xx.
    kind 'target' with wrap_angle is run_nominal.py:297-324 (the heading error wrapped, the derivatives taken
    at target_k = x_theta - wrap(x_theta - target_theta)); 'track' is core/tube_mpc.py:863-894 with X_ref
    [N+1, >=3] / U_ref [N, 2] (or [B, N+1, >=3] / [B, N, 2]) indexed by k.  The terminal derivatives include the barrier term 2 qb b
    (run_nominal.py:321-323)."""

    def __init__(self, cost: QuadraticCost, X_ref: Optional[Tensor] = None, U_ref: Optional[Tensor] = None):
        if cost.kind == "track" and (X_ref is None or U_ref is None):
            raise ValueError("a tracking cost needs X_ref and U_ref")
        self.cost, self.X_ref, self.U_ref = cost, X_ref, U_ref

    def _ref(self, x_hat: Tensor, k: Optional[int]) -> Tensor:
        c = self.cost
        if c.kind == "track":
            kk = k if k is not None else -1
            r = (self.X_ref[:, kk] if self.X_ref.ndim == 3 else self.X_ref[kk])[..., :3].to(x_hat)
            return r.expand(*x_hat.shape[:-1], 3)
        t = torch.tensor(c.target, dtype=x_hat.dtype, device=x_hat.device).expand(*x_hat.shape[:-1], 3)
        if not c.wrap_angle:
            return t
        th = x_hat[..., 2]
        return torch.stack([t[..., 0], t[..., 1], th - _wrap(th - t[..., 2])], -1)

    def _uref(self, u: Tensor, k: int) -> Tensor:
        if self.cost.kind == "track":
            r = self.U_ref[:, k] if self.U_ref.ndim == 3 else self.U_ref[k]
            return r.to(u).expand(*u.shape[:-1], 2)
        return torch.zeros_like(u)

    def _err(self, x_hat: Tensor, k: Optional[int]) -> Tensor:
        c = self.cost
        if c.kind == "track":
            return x_hat[..., :3] - self._ref(x_hat, k)
        dx = x_hat[..., :3] - torch.tensor(c.target, dtype=x_hat.dtype, device=x_hat.device)
        return torch.cat([dx[..., :2], _wrap(dx[..., 2:3])], -1) if c.wrap_angle else dx

    def _w(self, v, like: Tensor) -> Tensor:
        return torch.tensor(v, dtype=like.dtype, device=like.device)

    def stage_cost(self, x_hat: Tensor, u: Tensor, k: int) -> Tensor:
        from . import _points as P

        P.require_device(x_hat, u)
        c, dx, b = self.cost, self._err(x_hat, k), x_hat[..., 3]
        du = u - self._uref(u, k)
        return ((self._w(c.Q, x_hat) * dx * dx).sum(-1) + (self._w(c.R, x_hat) * du * du).sum(-1)
                + c.qb * (b * b))

    def terminal_cost(self, x_hat_N: Tensor) -> Tensor:
        from . import _points as P

        P.require_device(x_hat_N)
        c, dx, b = self.cost, self._err(x_hat_N, None), x_hat_N[..., 3]
        return (self._w(c.Qf, x_hat_N) * dx * dx).sum(-1) + c.qb * (b * b)

    def stage_derivs(self, x_hat: Tensor, u: Tensor, k: int):
        from .cost_derivs import auxiliary_cost_derivs_u

        c = self.cost
        return auxiliary_cost_derivs_u(x_hat=x_hat, u=u, x_ref=self._ref(x_hat, k), u_ref=self._uref(u, k),
                                       Q=c.Q, R=c.R, qb=c.qb)

    def terminal_derivs(self, x_hat_N: Tensor):
        from .cost_derivs import auxiliary_terminal_derivs

        c = self.cost
        phi_x, phi_xx = auxiliary_terminal_derivs(x_hat_N=x_hat_N, x_ref_N=self._ref(x_hat_N, None), Qf=c.Qf)
        phi_x = phi_x.clone()
        phi_x[..., 3] = phi_x[..., 3] + 2.0 * c.qb * x_hat_N[..., 3]
        phi_xx = phi_xx.clone()
        phi_xx[..., 3, 3] = phi_xx[..., 3, 3] + 2.0 * c.qb
        return phi_x, phi_xx

    def stage_hess(self, x_hat: Tensor, u: Tensor, k: int):
        c = self.cost
        kw = dict(dtype=x_hat.dtype, device=x_hat.device)
        lead = x_hat.shape[:-1]
        l_xx = torch.diag(2.0 * torch.tensor(list(c.Q) + [c.qb], **kw)).expand(*lead, 4, 4).clone()
        l_uu = torch.diag(2.0 * torch.tensor(list(c.R), **kw)).expand(*lead, 2, 2).clone()
        return l_xx, l_uu, torch.zeros(*lead, 2, 4, **kw)

    def terminal_hess(self, x_hat_N: Tensor) -> Tensor:
        return self.terminal_derivs(x_hat_N)[1]


def nominal_closures(cfg: Dict[str, Any]) -> Dict[str, Any]:
    """The closures run_nominal.py:231-324 builds from its config, as device objects: f_hat, f_jac (its
    Jacobian), ctrl, stage_cost, terminal_cost, stage_derivs, term_derivs, plus the ILQRConfig of :356-366
    (ilqr_cfg) -- keyed by the reference's local names."""
    from .receding import receding_setup_from_config

    problem, cost, icfg = receding_setup_from_config(cfg)
    f_hat = DBaSDynamics(problem)
    qc = QuadraticClosures(cost)
    return {"f_hat": f_hat, "f_jac": f_hat.jacobian,
            "ctrl": BoxClampControl(u_min=problem.u_min, u_max=problem.u_max, active_tol=problem.active_tol),
            "stage_cost": qc.stage_cost, "terminal_cost": qc.terminal_cost, "stage_derivs": qc.stage_derivs,
            "term_derivs": qc.terminal_derivs, "ilqr_cfg": icfg}


class ParamClosures:
    """The general path's gradient closures over raw parameters, for ift_gradient's keyword form
    (core/ift.py:35-43): the ancillary set of core/tube_mpc.py:469-489 (f_hat_aux_grad, stage_cost_aux_grad,
    terminal_cost_aux_grad over theta = AuxiliaryTheta and the reference tensors X_ref [N+1, 3] / U_ref
    [N, 2]) or, with ``target``, the nominal set of :556-585 over theta-bar = NominalTheta (with the
    tightening s).  ``f`` / ``stage_cost`` / ``terminal_cost`` have the reference's signatures and evaluate
    on the device with the parameters' current values (weights softplus(raw), alpha = softplus + 1e-6,
    gamma = tanh, core/params.py); the nominal ``f`` with a tightening s != 0 is not evaluated point-wise
    (its h - s lives in the fused kernels only)."""

    def __init__(self, problem: DubinsDBaSProblem, theta, *, X_ref: Optional[Tensor] = None,
                 U_ref: Optional[Tensor] = None, target: Optional[Tuple[float, float, float]] = None):
        if (X_ref is None) == (target is None):
            raise ValueError("pass X_ref / U_ref (the ancillary set) or target (the nominal set)")
        if X_ref is not None and U_ref is None:
            raise ValueError("the ancillary set needs X_ref and U_ref")
        self.problem, self.theta, self.X_ref, self.U_ref, self.target = problem, theta, X_ref, U_ref, target

    @property
    def nominal(self) -> bool:
        return self.target is not None

    def cost(self) -> QuadraticCost:
        return (QuadraticCost(kind="target", target=tuple(float(v) for v in self.target)) if self.nominal
                else QuadraticCost(kind="track"))

    def f(self, x_hat: Tensor, u: Tensor) -> Tensor:
        th = self.theta
        if self.nominal and float(th.tight()) != 0.0:
            raise NotImplementedError("point-wise f with the tightening h - s: use the typed general step")
        p = dataclasses.replace(self.problem, dbas_alpha=float(th.alpha()), dbas_gamma=float(th.gamma()))
        return DBaSDynamics(p)(x_hat, u)

    def _w(self, t: Tensor, like: Tensor) -> Tensor:
        return t.detach().to(dtype=like.dtype, device=like.device)

    def stage_cost(self, x_hat: Tensor, u: Tensor, k: int) -> Tensor:
        from . import _points as P

        P.require_device(x_hat, u)
        th = self.theta
        ref = (torch.tensor(self.target, dtype=x_hat.dtype, device=x_hat.device) if self.nominal
               else self.X_ref[k][..., :3].to(x_hat))
        dx = x_hat[..., :3] - ref
        du = u if self.nominal else u - self.U_ref[k].to(u)
        b = x_hat[..., 3]
        return ((self._w(th.Q(), x_hat) * dx * dx).sum(-1) + (self._w(th.R(), x_hat) * du * du).sum(-1)
                + self._w(th.qb(), x_hat) * (b * b))

    def terminal_cost(self, x_hat_N: Tensor) -> Tensor:
        from . import _points as P

        P.require_device(x_hat_N)
        th = self.theta
        ref = (torch.tensor(self.target, dtype=x_hat_N.dtype, device=x_hat_N.device) if self.nominal
               else self.X_ref[-1][..., :3].to(x_hat_N))
        dx = x_hat_N[..., :3] - ref
        b = x_hat_N[..., 3]
        return (self._w(th.Qf(), x_hat_N) * dx * dx).sum(-1) + self._w(th.qb(), x_hat_N) * (b * b)


def resolve_ift(*, theta_tensors, xi_fn, f_fn, stage_cost_fn, terminal_cost_fn) -> Tuple[ParamClosures, list]:
    """The keyword form of ift_gradient (core/ift.py:35-43) -> its closures' carrier and, per requested tensor,
    where its gradient sits: ("theta", index into IFTGradient.split()) or ("X_ref" | "U_ref", None)."""
    owners = {n: _owner(fn, ParamClosures, n) for n, fn in
              (("f_fn", f_fn), ("stage_cost_fn", stage_cost_fn), ("terminal_cost_fn", terminal_cost_fn))}
    pc = owners["f_fn"]
    if any(o is not pc for o in owners.values()):
        raise ValueError("f_fn, stage_cost_fn and terminal_cost_fn come from different ParamClosures")
    xi = xi_fn() if xi_fn is not None else None
    if xi is not None and isinstance(xi, Tensor) and xi.requires_grad:
        raise NotImplementedError("xi_fn must return a detached x_hat0 (the reference's callers pass "
                                  "x_hat0.detach(): xi contributes nothing)")
    params = pc.theta.tensors()
    where = []
    for t in theta_tensors:
        hit = [i for i, q in enumerate(params) if q is t]
        if hit:
            where.append(("theta", hit[0]))
        elif pc.X_ref is not None and t is pc.X_ref:
            where.append(("X_ref", None))
        elif pc.U_ref is not None and t is pc.U_ref:
            where.append(("U_ref", None))
        else:
            raise ValueError("theta_tensors holds a tensor the closures do not depend on")
    return pc, where


@dataclasses.dataclass(frozen=True)
class ResolvedCall:
    problem: DubinsDBaSProblem
    cost: QuadraticCost
    X_ref: Optional[Tensor]
    U_ref: Optional[Tensor]


def _owner(fn: Callable, cls, what: str):
    obj = fn if isinstance(fn, cls) else getattr(fn, "__self__", None)
    if not isinstance(obj, cls):
        raise TypeError(f"{what}: the device solver cannot call an arbitrary Python closure; build it with "
                        f"diff_tube_mpc_strict_pt.core.closures ({cls.__name__}, nominal_closures) so that it "
                        f"carries the typed problem it computes")
    return obj


def _cost_of(what: Dict[str, Callable]) -> QuadraticClosures:
    owners = {name: _owner(fn, QuadraticClosures, name) for name, fn in what.items() if fn is not None}
    if not owners:
        raise TypeError("the cost closures are required")
    first = next(iter(owners.values()))
    for name, o in owners.items():
        if o.cost != first.cost or o.X_ref is not first.X_ref or o.U_ref is not first.U_ref:
            raise ValueError(f"{name} describes a different cost than the other cost closures")
    return first


def _problem_of(f, ctrl: Optional[BoxClampControl], horizon: int) -> DubinsDBaSProblem:
    dyn = _owner(f, DBaSDynamics, "f")
    if ctrl is None:
        box = {"u_min": (-math.inf, -math.inf), "u_max": (math.inf, math.inf)}  # no clamp (core/ddp.py:128)
    elif isinstance(ctrl, BoxClampControl):
        box = ctrl.problem_bounds()
    else:
        raise TypeError("ctrl must be a BoxClampControl (or None)")
    return dataclasses.replace(dyn.problem, horizon=int(horizon), **box)


def resolve_ilqr(*, cfg: ILQRConfig, f, f_jac=None, ctrl=None, stage_cost=None, terminal_cost=None,
                 stage_derivs=None, terminal_derivs=None, feasible_fn=None) -> ResolvedCall:
    """The keyword form of ilqr_solve (core/ddp.py:102-117) -> the typed call's problem and cost."""
    if feasible_fn is not None:
        raise NotImplementedError("feasible_fn has no device counterpart (the reference's callers never pass it)")
    if f_jac is not None and not callable(f_jac):
        raise TypeError("f_jac must be callable")
    qc = _cost_of({"stage_cost": stage_cost, "terminal_cost": terminal_cost, "stage_derivs": stage_derivs,
                   "terminal_derivs": terminal_derivs})
    if stage_cost is None or terminal_cost is None or stage_derivs is None or terminal_derivs is None:
        raise TypeError("ilqr_solve needs stage_cost, terminal_cost, stage_derivs and terminal_derivs")
    return ResolvedCall(_problem_of(f, ctrl, cfg.horizon), qc.cost, qc.X_ref, qc.U_ref)


def resolve_sensitivity(*, f, f_jac=None, ctrl=None, stage_hess=None, terminal_hess=None,
                        horizon: int) -> ResolvedCall:
    """The keyword form of ddp_sensitivity (core/ddp.py:317-329) -> problem and cost (the cost's Hessians are
    what the sensitivity uses; its gradients enter only through the upper-level closures)."""
    if f_jac is not None and not callable(f_jac):
        raise TypeError("f_jac must be callable")
    if stage_hess is None or terminal_hess is None:
        raise TypeError("ddp_sensitivity needs stage_hess and terminal_hess")
    qc = _cost_of({"stage_hess": stage_hess, "terminal_hess": terminal_hess})
    return ResolvedCall(_problem_of(f, ctrl, horizon), qc.cost, qc.X_ref, qc.U_ref)
