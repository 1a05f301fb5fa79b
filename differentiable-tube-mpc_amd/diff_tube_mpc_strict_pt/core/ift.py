"""IFT gradient of the upper loss w.r.t. the raw parameters -- core/ift.py:35-92 for the typed problem.

The reference accumulates

    grad_theta L = xi_theta^T dlam_0 + sum_k ( L_theta_x dx_k + L_theta_u du_k + f_theta_k^T dlam_{k+1} )
                   + phi_theta_x dx_N

by autograd through its closures.  Here the closures are the typed Dubins + DBaS problem with
softplus / tanh parameterised weights (core/params.py, core/tube_mpc.py:461-500 and :556-585), and
every term has a closed form evaluated by the HIP kernel ``dtmpc_ift_gradient`` (derivation in
oracle/oracle_general.h); xi = x_hat0.detach() contributes nothing, as in the reference.
"""
from __future__ import annotations

import ctypes as C
import dataclasses
from dataclasses import dataclass
from typing import Optional, Sequence

import torch
from torch import Tensor

from .. import _abi, _lib
from .ddp import _dtype_code, _ptr, _require_device, from_soa, to_soa
from .problem import DubinsDBaSProblem, QuadraticCost

__all__ = ["IFTInputs", "IFTGradient", "ift_gradient", "P_NAMES"]

# raw parameter names in DTMPC_P_* order (core/params.py field order)
P_NAMES = ("Q_raw", "R_raw", "Qf_raw", "qb_raw", "alpha_raw", "gamma_raw", "tight_raw")


@dataclass(frozen=True)
class IFTInputs:
    """core/ift.py:10-20 with a leading batch dimension."""

    X: Tensor              # [B, N+1, 4]
    V: Tensor              # [B, N, 2]
    delta_X: Tensor        # [B, N+1, 4]
    delta_V: Tensor        # [B, N, 2]
    delta_lambda: Tensor   # [B, N+1, 4]


@dataclass(frozen=True)
class IFTGradient:
    theta: Tensor                 # [B, 12] d L / d raw (DTMPC_P_* layout)
    X_ref: Optional[Tensor]       # [B, N+1, 3] (tracking cost only)
    U_ref: Optional[Tensor]       # [B, N, 2]

    def split(self) -> list:
        """Per-tensor gradients in the reference's theta.tensors() order (Q, R, Qf, qb, alpha, gamma,
        tight), each [B, ...]."""
        t = self.theta
        return [t[:, 0:3], t[:, 3:5], t[:, 5:8], t[:, 8], t[:, 9], t[:, 10], t[:, 11]]


def ift_gradient(*, inputs: IFTInputs, problem: Optional[DubinsDBaSProblem] = None,
                 cost: Optional[QuadraticCost] = None, theta_raw: Sequence[float] | Tensor | None = None,
                 X_ref: Optional[Tensor] = None, U_ref: Optional[Tensor] = None, theta_tensors=None, xi_fn=None,
                 f_fn=None, stage_cost_fn=None, terminal_cost_fn=None):
    """ift_gradient (core/ift.py:35-92).

    The reference's keyword form -- ift_gradient(inputs=, theta_tensors=, xi_fn=, f_fn=, stage_cost_fn=,
    terminal_cost_fn=) with the closures of one core.closures.ParamClosures and unbatched inputs -- is resolved
    to this typed call and returns the reference's list: one gradient per tensor of theta_tensors, shaped like
    it (the raw parameters of the closures' theta, and the ancillary set's X_ref / U_ref).

    cost.kind 'track' = the ancillary closures (core/tube_mpc.py:461-500; also returns dL/dX_ref,
    dL/dU_ref), 'target' = the nominal ones (:556-585, with the tightening).  Weights and the DBaS
    alpha / gamma / tightening come from ``theta_raw`` [12] through core/params.py; ``cost`` supplies
    the kind and target, ``problem`` the system, obstacles, barrier type and eps."""
    if f_fn is not None:
        if problem is not None or cost is not None or theta_raw is not None:
            raise TypeError("pass either problem / cost / theta_raw (typed form) or the closures, not both")
        from .closures import resolve_ift

        pc, where = resolve_ift(theta_tensors=theta_tensors, xi_fn=xi_fn, f_fn=f_fn, stage_cost_fn=stage_cost_fn,
                                terminal_cost_fn=terminal_cost_fn)
        single = inputs.X.ndim == 2
        up = (lambda t: t[None]) if single else (lambda t: t)  # noqa: E731
        inb = IFTInputs(X=up(inputs.X), V=up(inputs.V), delta_X=up(inputs.delta_X), delta_V=up(inputs.delta_V),
                        delta_lambda=up(inputs.delta_lambda))
        Bn = inb.X.shape[0]
        Xr = Ur = None
        if not pc.nominal:
            Xr = pc.X_ref.detach()
            Ur = pc.U_ref.detach()
            Xr = (Xr[None].expand(Bn, *Xr.shape) if Xr.ndim == 2 else Xr).to(inb.X)
            Ur = (Ur[None].expand(Bn, *Ur.shape) if Ur.ndim == 2 else Ur).to(inb.X)
        g = ift_gradient(inputs=inb, problem=dataclasses.replace(pc.problem, horizon=inb.V.shape[1]),
                         cost=pc.cost(), theta_raw=pc.theta.raw(), X_ref=Xr, U_ref=Ur)
        parts = g.split()
        out = []
        for t, (kind, i) in zip(theta_tensors, where):
            v = parts[i] if kind == "theta" else (g.X_ref if kind == "X_ref" else g.U_ref)
            v = v[0] if single else v
            out.append(v.reshape(t.shape).to(dtype=t.dtype))
        return out
    if problem is None or cost is None or theta_raw is None:
        raise TypeError("ift_gradient needs problem, cost and theta_raw (typed form) or the closures (keyword form)")
    X, V = inputs.X, inputs.V
    _require_device(X, V, inputs.delta_X, inputs.delta_V, inputs.delta_lambda, X_ref, U_ref)
    B, N = X.shape[0], problem.horizon
    track = cost.kind == "track"
    if track and (X_ref is None or U_ref is None):
        raise ValueError("the ancillary (track) IFT needs X_ref and U_ref")
    lib = _lib.load()
    raw = torch.as_tensor(theta_raw, dtype=torch.float64).reshape(_abi.P_COUNT).tolist()
    th = (C.c_double * _abi.P_COUNT)(*raw)
    spec, cc = problem.to_c(), cost.to_c()
    dt = X.dtype
    args = [to_soa(t.to(dt)) for t in (X, V, inputs.delta_X, inputs.delta_V, inputs.delta_lambda)]
    Xr = to_soa(X_ref[..., :3].to(dt)) if track else None
    Ur = to_soa(U_ref.to(dt)) if track else None
    kw = dict(dtype=dt, device=X.device)
    g = torch.empty(_abi.P_COUNT, B, **kw)
    gxr = torch.empty(N + 1, 3, B, **kw) if track else None
    gur = torch.empty(N, 2, B, **kw) if track else None
    _lib.check(lib.dtmpc_ift_gradient(_dtype_code(X), C.byref(spec), C.byref(cc), th, B, *[a.data_ptr() for a in args],
                                      _ptr(Xr), _ptr(Ur), g.data_ptr(), _ptr(gxr), _ptr(gur), _lib.stream_of(X)),
               "dtmpc_ift_gradient")
    return IFTGradient(theta=g.t().contiguous(), X_ref=from_soa(gxr) if track else None,
                       U_ref=from_soa(gur) if track else None)
