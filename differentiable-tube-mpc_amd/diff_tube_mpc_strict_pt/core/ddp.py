"""Batched, typed DDP/iLQR entry points (HIP path).

Counterparts of the reference's core/ddp.py with the Python-closure arguments replaced by the typed
problem of :mod:`.problem`; every array carries a leading batch dimension B of independent
trajectories.  User-facing layout is trajectory-major ([B, N+1, 4] states, [B, N, 2] controls);
the C ABI (include/dtmpc.h) is SoA [step][field][B], converted here once per call.

Reference mapping:
  rollout           core/ddp.py:89-99        -> dtmpc_dbas_rollout
  linearize         core/systems/dubins_aug_jac.py:61-139 + core/cost_derivs.py -> dtmpc_linearize
  ilqr_solve        core/ddp.py:102-307      -> dtmpc_ilqr_solve
  ddp_sensitivity   core/ddp.py:317-427      -> dtmpc_ddp_sensitivity (paper upper loss) or
                                                dtmpc_ddp_sensitivity_upper (upper gradients as arrays)
  doc_gradient      core/tube_mpc.py:915-976 -> dtmpc_doc_grad

Errors follow the reference: FloatingPointError for non-finite values (core/ddp.py:138-159),
RuntimeError when the line search yields no candidate (core/ddp.py:298-299), ValueError for bad
arguments.  There is no CPU fallback: tensors must live on a HIP device.
"""
from __future__ import annotations

import ctypes as C
import dataclasses
from dataclasses import dataclass
from typing import Optional

import torch
from torch import Tensor

from .. import _abi, _lib
from .problem import DubinsDBaSProblem, ILQRConfig, QuadraticCost

__all__ = [
    "ILQRConfig",
    "ILQRResult",
    "SensitivityResult",
    "rollout",
    "dbas_init",
    "linearize",
    "ilqr_solve",
    "ddp_sensitivity",
    "doc_gradient",
    "raise_for_status",
]


def _dtype_code(t: Tensor) -> int:
    if t.dtype == torch.float32:
        return _abi.F32
    if t.dtype == torch.float64:
        return _abi.F64
    raise ValueError(f"unsupported dtype {t.dtype}; use float32 or float64")


def _require_device(*ts: Tensor) -> None:
    for t in ts:
        if t is not None and t.device.type != "cuda":
            raise ValueError(
                "the dtmpc HIP path needs device tensors (got %s); there is no CPU fallback" % t.device
            )


def to_soa(t: Tensor) -> Tensor:
    """[B, rows, F] -> contiguous [rows, F, B], always a fresh buffer: at B = 1 the permuted view is
    already "contiguous" and .contiguous() would hand the caller's own storage to kernels that write
    their in/out arrays (V_init must never be mutated, core/ddp.py:127)."""
    return t.permute(1, 2, 0).clone(memory_format=torch.contiguous_format)


def from_soa(t: Tensor) -> Tensor:
    """[rows, F, B] -> [B, rows, F] (contiguous copy)."""
    return t.permute(2, 0, 1).clone(memory_format=torch.contiguous_format)


def _ptr(t: Optional[Tensor]) -> Optional[int]:
    return None if t is None else t.data_ptr()


def raise_for_status(status: Tensor, what: str) -> None:
    """Map per-trajectory status words to the reference's exceptions (syncs the device)."""
    st = status.to("cpu")
    bad = torch.nonzero(st != 0).flatten().tolist()
    if not bad:
        return
    bits = 0
    for i in bad:
        bits |= int(st[i])
    idx = bad[:8]
    more = "" if len(bad) <= 8 else f" (+{len(bad) - 8} more)"
    if bits & _abi.ST_NONFINITE:
        raise FloatingPointError(f"{what}: non-finite detected in trajectories {idx}{more}")
    raise RuntimeError(f"{what}: line search failed to produce a candidate in trajectories {idx}{more}")


@dataclass(frozen=True)
class ILQRResult:
    X: Tensor  # [B, N+1, 4]
    V: Tensor  # [B, N, 2]
    K: Tensor  # [B, N, 2, 4] gains of the last backward pass
    k: Tensor  # [B, N, 2]
    iters: Tensor  # [B] int32
    status: Tensor  # [B] int32
    choices: Optional[Tensor] = None  # [B, max_iter] int8: winning alpha position per iteration, -1 not run
    costs: Optional[Tensor] = None  # [B, max_iter, 8]: every line-search candidate's cost by alpha position


@dataclass(frozen=True)
class SensitivityResult:
    """core/ddp.py:310-314 with a leading batch dimension."""

    delta_X: Tensor  # [B, N+1, 4]
    delta_V: Tensor  # [B, N, 2]
    delta_lambda: Optional[Tensor]  # [B, N+1, 4]


def _prep_x0(x0: Tensor) -> Tensor:
    if x0.dim() != 2 or x0.shape[1] != 4:
        raise ValueError("x0 must be [B, 4] (x, y, theta, b)")
    return x0.t().contiguous()


def rollout(problem, x0: Tensor, V: Optional[Tensor] = None, *, f=None) -> Tensor:
    """X[k+1] = f_hat(X[k], V[k]) for every trajectory (core/ddp.py:89-99, f = DBaS step).

    Typed form rollout(problem, x0 [B, 4], V [B, N, 2]); the reference's form rollout(x0, V, *, f) with f a
    core.closures.DBaSDynamics (x0 [4] / V [N, 2], or batched)."""
    if f is not None:
        from .closures import DBaSDynamics, _owner

        dyn = _owner(f, DBaSDynamics, "f")
        x0_, V_ = problem, x0
        single = x0_.ndim == 1
        xb, Vb = (x0_[None], V_[None]) if single else (x0_, V_)
        out = rollout(dataclasses.replace(dyn.problem, horizon=Vb.shape[1]), xb, Vb)
        return out[0] if single else out
    _require_device(x0, V)
    B, N = x0.shape[0], problem.horizon
    if V.shape != (B, N, 2):
        raise ValueError(f"V must be [{B}, {N}, 2]")
    lib = _lib.load()
    spec = problem.to_c()
    x0s = _prep_x0(x0)
    Us = to_soa(V.to(x0.dtype))
    Xs = torch.empty(N + 1, 4, B, dtype=x0.dtype, device=x0.device)
    _lib.check(lib.dtmpc_dbas_rollout(_dtype_code(x0), C.byref(spec), B, x0s.data_ptr(), Us.data_ptr(),
                                      Xs.data_ptr(), _lib.stream_of(x0)), "dtmpc_dbas_rollout")
    return from_soa(Xs)


def dbas_init(problem: DubinsDBaSProblem, x: Tensor) -> Tensor:
    """b0 = B(h(x0)) per trajectory (core/barrier.py:111-120).  x: [B, 3] -> [B]."""
    _require_device(x)
    B = x.shape[0]
    lib = _lib.load()
    spec = problem.to_c()
    xs = x[:, :3].t().contiguous()
    b = torch.empty(B, dtype=x.dtype, device=x.device)
    _lib.check(lib.dtmpc_dbas_init(_dtype_code(x), C.byref(spec), B, xs.data_ptr(), b.data_ptr(),
                                   _lib.stream_of(x)), "dtmpc_dbas_init")
    return b


def linearize(problem: DubinsDBaSProblem, cost: QuadraticCost, X: Tensor, V: Tensor,
              X_ref: Optional[Tensor] = None, U_ref: Optional[Tensor] = None):
    """Per-step A [B,N,4,4], B [B,N,4,2], l_x [B,N+1,4] (k = N is phi_x), l_u [B,N,2]."""
    _require_device(X, V, X_ref, U_ref)
    Bsz, N = X.shape[0], problem.horizon
    lib = _lib.load()
    spec, cc = problem.to_c(), cost.to_c()
    Xs, Us = to_soa(X), to_soa(V.to(X.dtype))
    Xr = to_soa(X_ref[..., :3].to(X.dtype)) if X_ref is not None else None
    Ur = to_soa(U_ref.to(X.dtype)) if U_ref is not None else None
    kw = dict(dtype=X.dtype, device=X.device)
    A = torch.empty(N, 16, Bsz, **kw)
    Bm = torch.empty(N, 8, Bsz, **kw)
    lx = torch.empty(N + 1, 4, Bsz, **kw)
    lu = torch.empty(N, 2, Bsz, **kw)
    _lib.check(lib.dtmpc_linearize(_dtype_code(X), C.byref(spec), C.byref(cc), Bsz, Xs.data_ptr(), Us.data_ptr(),
                                   _ptr(Xr), _ptr(Ur), A.data_ptr(), Bm.data_ptr(), lx.data_ptr(), lu.data_ptr(),
                                   _lib.stream_of(X)), "dtmpc_linearize")
    return (from_soa(A).view(Bsz, N, 4, 4), from_soa(Bm).view(Bsz, N, 4, 2), from_soa(lx), from_soa(lu))


def ilqr_solve(*, problem: Optional[DubinsDBaSProblem] = None, cost: Optional[QuadraticCost] = None,
               cfg: ILQRConfig, x0: Tensor, V_init: Tensor, X_ref: Optional[Tensor] = None,
               U_ref: Optional[Tensor] = None, check: bool = True, debug_name: str = "ilqr",
               record_choices: bool = False, lanes: int = 0, record_costs: bool = False,
               f=None, f_jac=None, ctrl=None, stage_cost=None, terminal_cost=None, stage_derivs=None,
               terminal_derivs=None, feasible_fn=None, debug: bool = False):
    """Batched box-clamped iLQR (core/ddp.py:102-307).

    The reference's keyword form -- ilqr_solve(x0=, V_init=, cfg=, f=, f_jac=, ctrl=, stage_cost=,
    terminal_cost=, stage_derivs=, terminal_derivs=) with closures from core.closures -- is resolved to this
    typed call and returns the reference's (X*, V*) pair (unbatched for x0 [4], V_init [N, 2]).

    x0 [B, 4], V_init [B, N, 2] (not mutated), X_ref [B, N+1, >=3] / U_ref [B, N, 2] for the tracking
    cost.  Returns X* [B, N+1, 4], V* [B, N, 2] and diagnostics; record_choices adds the decision
    record (the winning line-search alpha position of every iteration, core/ddp.py:293); record_costs
    the costs behind it (every candidate's J by alpha position [B, max_iter, 8], NaN not run; fused
    solver only -- None when the generic kernel runs).
    Runs dtmpc_ilqr_solve_ws: the tube step's fused solver on the paper configuration (f32 and f64:
    csrc/dtmpc_fast_ilqr.hip / dtmpc_fast64_ilqr.hip; DTMPC_FAST=0 / DTMPC_FAST64=0 switch it off) with
    ``lanes`` lanes per trajectory (0: dtmpc_tube_lanes(B); 1, 2 or 4), else the generic kernel
    (dtmpc_ilqr_fused_eligible says which)."""
    if f is not None:
        if problem is not None or cost is not None:
            raise TypeError("pass either problem / cost (typed form) or the closures (keyword form), not both")
        from .closures import resolve_ilqr

        r = resolve_ilqr(cfg=cfg, f=f, f_jac=f_jac, ctrl=ctrl, stage_cost=stage_cost, terminal_cost=terminal_cost,
                         stage_derivs=stage_derivs, terminal_derivs=terminal_derivs, feasible_fn=feasible_fn)
        single = x0.ndim == 1
        xb, Vb = (x0[None], V_init[None]) if single else (x0, V_init)
        Xr, Ur = r.X_ref, r.U_ref
        if Xr is not None and Xr.ndim == 2:
            Xr, Ur = Xr[None].expand(xb.shape[0], *Xr.shape), Ur[None].expand(xb.shape[0], *Ur.shape)
        res = ilqr_solve(problem=r.problem, cost=r.cost, cfg=cfg, x0=xb, V_init=Vb, X_ref=Xr, U_ref=Ur,
                         check=True, debug_name=debug_name, lanes=lanes)
        return (res.X[0], res.V[0]) if single else (res.X, res.V)
    if problem is None or cost is None:
        raise TypeError("ilqr_solve needs problem and cost (typed form) or f and the cost closures (keyword form)")
    _require_device(x0, V_init, X_ref, U_ref)
    B, N = x0.shape[0], problem.horizon
    if cfg.horizon != N:
        raise ValueError("cfg.horizon != problem.horizon")
    if V_init.shape != (B, N, 2):
        raise ValueError(f"V_init must be [{B}, {N}, 2]")
    lib = _lib.load()
    spec, cc, ic = problem.to_c(), cost.to_c(), cfg.to_c()
    dt = x0.dtype
    x0s = _prep_x0(x0)
    Us = to_soa(V_init.to(dt))
    Xr = to_soa(X_ref[..., :3].to(dt)) if X_ref is not None else None
    Ur = to_soa(U_ref.to(dt)) if U_ref is not None else None
    kw = dict(dtype=dt, device=x0.device)
    Xs = torch.empty(N + 1, 4, B, **kw)
    Ks = torch.zeros(N, 8, B, **kw)
    ks = torch.zeros(N, 2, B, **kw)
    iters = torch.zeros(B, dtype=torch.int32, device=x0.device)
    status = torch.zeros(B, dtype=torch.int32, device=x0.device)
    ch = torch.empty(max(cfg.max_iter, 1), B, dtype=torch.int8, device=x0.device) if record_choices else None
    fused = bool(lib.dtmpc_ilqr_fused_eligible(_dtype_code(x0), C.byref(spec), C.byref(cc), C.byref(ic)))
    cr = (torch.full((max(cfg.max_iter, 1), 8, B), float("nan"), **kw) if record_costs and fused else None)
    if lanes not in (0, 1, 2, 4):
        raise ValueError("lanes must be 0 (default), 1, 2 or 4")
    wb = int(lib.dtmpc_ilqr_workspace_bytes(_dtype_code(x0), N, B, lanes))
    work = torch.empty(max(wb, 1), dtype=torch.uint8, device=x0.device)
    _lib.check(lib.dtmpc_ilqr_solve_ws(_dtype_code(x0), C.byref(spec), C.byref(cc), C.byref(ic), B, x0s.data_ptr(),
                                       _ptr(Xr), _ptr(Ur), Xs.data_ptr(), Us.data_ptr(), Ks.data_ptr(), ks.data_ptr(),
                                       iters.data_ptr(), status.data_ptr(), _ptr(ch), _ptr(cr), lanes,
                                       work.data_ptr(), wb,
                                       _lib.stream_of(x0)),
               "dtmpc_ilqr_solve_ws")
    if check:
        raise_for_status(status, debug_name)
    return ILQRResult(X=from_soa(Xs), V=from_soa(Us), K=from_soa(Ks).view(B, N, 2, 4), k=from_soa(ks),
                      iters=iters, status=status,
                      choices=ch[:cfg.max_iter].t().contiguous() if ch is not None else None,
                      costs=cr[:cfg.max_iter].permute(2, 0, 1).contiguous() if cr is not None else None)


def ddp_sensitivity(*, problem: Optional[DubinsDBaSProblem] = None, cost: Optional[QuadraticCost] = None,
                    X: Tensor, V: Tensor, X_ref: Optional[Tensor] = None, U_ref: Optional[Tensor] = None,
                    X_bar: Optional[Tensor] = None, upper_grad_x=None, upper_grad_u=None,
                    want_lambda: bool = True, check: bool = True, f=None, f_jac=None, ctrl=None,
                    stage_hess=None, terminal_hess=None, upper_grad_xN=None) -> SensitivityResult:
    """DDP-structured KKT sensitivity with active set (core/ddp.py:317-427).

    The reference's keyword form -- ddp_sensitivity(X=, V=, f=, f_jac=, ctrl=, stage_hess=, terminal_hess=,
    upper_grad_x=, upper_grad_u=, upper_grad_xN=) with f / the Hessians from core.closures and the upper-level
    gradients as callables (x, k) / (u, k) / (x_N), evaluated along the tape -- is resolved to the array
    form below (unbatched result for X [N+1, 4]).

    Upper-level gradients either as arrays -- upper_grad_x [B, N+1, 4] (row N = upper_grad_xN) and
    upper_grad_u [B, N, 2], the reference's closures evaluated along the tape -- or, with X_bar, the
    paper upper loss L = sum ||x_k - xbar_k||^2 + b_k^2 (core/tube_mpc.py:915-957):
    g_x = [2(x - xbar), 2 b], g_u = 0."""
    if f is not None:
        if problem is not None or cost is not None:
            raise TypeError("pass either problem / cost (typed form) or the closures (keyword form), not both")
        from .closures import resolve_sensitivity

        if not (callable(upper_grad_x) and callable(upper_grad_u) and callable(upper_grad_xN)):
            raise TypeError("the keyword form takes upper_grad_x(x, k), upper_grad_u(u, k), upper_grad_xN(x_N)")
        single = X.ndim == 2
        Xb, Vb = (X[None], V[None]) if single else (X, V)
        N = Vb.shape[1]
        r = resolve_sensitivity(f=f, f_jac=f_jac, ctrl=ctrl, stage_hess=stage_hess, terminal_hess=terminal_hess,
                                horizon=N)
        # the closures see what the reference hands them: one trajectory's row (x [4], u [2]) for an
        # unbatched call, the batch's rows [B, 4] / [B, 2] otherwise
        if single:
            gX = torch.stack([upper_grad_x(X[k], k) for k in range(N)] + [upper_grad_xN(X[N])], 0)[None]
            gU = torch.stack([upper_grad_u(V[k], k) for k in range(N)], 0)[None]
        else:
            gX = torch.stack([upper_grad_x(Xb[:, k], k) for k in range(N)] + [upper_grad_xN(Xb[:, N])], 1)
            gU = torch.stack([upper_grad_u(Vb[:, k], k) for k in range(N)], 1)
        res = _ddp_sensitivity_upper(r.problem, r.cost, Xb, Vb, gX.to(Xb).expand(Xb.shape[0], N + 1, 4),
                                     gU.to(Xb).expand(Xb.shape[0], N, 2), want_lambda, check)
        if not single:
            return res
        return SensitivityResult(delta_X=res.delta_X[0], delta_V=res.delta_V[0],
                                 delta_lambda=res.delta_lambda[0] if res.delta_lambda is not None else None)
    if problem is None or cost is None:
        raise TypeError("ddp_sensitivity needs problem and cost (typed form) or f and the Hessian closures")
    if upper_grad_x is not None or upper_grad_u is not None:
        return _ddp_sensitivity_upper(problem, cost, X, V, upper_grad_x, upper_grad_u, want_lambda, check)
    if X_bar is None:
        raise ValueError("pass X_bar (paper upper loss) or upper_grad_x / upper_grad_u")
    _require_device(X, V, X_ref, U_ref, X_bar)
    B, N = X.shape[0], problem.horizon
    lib = _lib.load()
    spec, cc = problem.to_c(), cost.to_c()
    dt = X.dtype
    Xs, Us = to_soa(X), to_soa(V.to(dt))
    Xr = to_soa(X_ref[..., :3].to(dt)) if X_ref is not None else None
    Ur = to_soa(U_ref.to(dt)) if U_ref is not None else None
    Xb = to_soa(X_bar[..., :3].to(dt))
    kw = dict(dtype=dt, device=X.device)
    dX = torch.empty(N + 1, 4, B, **kw)
    dU = torch.empty(N, 2, B, **kw)
    dL = torch.empty(N + 1, 4, B, **kw) if want_lambda else None
    nbytes = lib.dtmpc_sensitivity_workspace_bytes(_dtype_code(X), N, B, 1 if want_lambda else 0)
    work = torch.empty(nbytes, dtype=torch.uint8, device=X.device)
    status = torch.zeros(B, dtype=torch.int32, device=X.device)
    _lib.check(lib.dtmpc_ddp_sensitivity(_dtype_code(X), C.byref(spec), C.byref(cc), B, Xs.data_ptr(), Us.data_ptr(),
                                         _ptr(Xr), _ptr(Ur), Xb.data_ptr(), dX.data_ptr(), dU.data_ptr(), _ptr(dL),
                                         work.data_ptr(), status.data_ptr(), _lib.stream_of(X)),
               "dtmpc_ddp_sensitivity")
    if check:
        raise_for_status(status, "ddp_sensitivity")
    return SensitivityResult(delta_X=from_soa(dX), delta_V=from_soa(dU),
                             delta_lambda=from_soa(dL) if dL is not None else None)


def _ddp_sensitivity_upper(problem, cost, X, V, gX, gU, want_lambda, check) -> SensitivityResult:
    if gX is None or gU is None:
        raise ValueError("upper_grad_x and upper_grad_u go together")
    _require_device(X, V, gX, gU)
    B, N = X.shape[0], problem.horizon
    if gX.shape != (B, N + 1, 4) or gU.shape != (B, N, 2):
        raise ValueError(f"upper_grad_x must be [{B}, {N + 1}, 4] and upper_grad_u [{B}, {N}, 2]")
    lib = _lib.load()
    spec, cc = problem.to_c(), cost.to_c()
    dt = X.dtype
    Xs, Us, gx, gu = to_soa(X), to_soa(V.to(dt)), to_soa(gX.to(dt)), to_soa(gU.to(dt))
    kw = dict(dtype=dt, device=X.device)
    dX = torch.empty(N + 1, 4, B, **kw)
    dU = torch.empty(N, 2, B, **kw)
    dL = torch.empty(N + 1, 4, B, **kw) if want_lambda else None
    work = torch.empty(lib.dtmpc_sensitivity_upper_workspace_bytes(_dtype_code(X), N, B), dtype=torch.uint8,
                       device=X.device)
    status = torch.zeros(B, dtype=torch.int32, device=X.device)
    _lib.check(lib.dtmpc_ddp_sensitivity_upper(_dtype_code(X), C.byref(spec), C.byref(cc), B, Xs.data_ptr(),
                                               Us.data_ptr(), gx.data_ptr(), gu.data_ptr(), dX.data_ptr(),
                                               dU.data_ptr(), _ptr(dL), work.data_ptr(), status.data_ptr(),
                                               _lib.stream_of(X)), "dtmpc_ddp_sensitivity_upper")
    if check:
        raise_for_status(status, "ddp_sensitivity")
    return SensitivityResult(delta_X=from_soa(dX), delta_V=from_soa(dU),
                             delta_lambda=from_soa(dL) if dL is not None else None)


def doc_gradient(X_aux: Tensor, U_aux: Tensor, X_nom: Tensor, U_nom: Tensor, dX: Tensor, dU: Tensor) -> Tensor:
    """Per-trajectory [L, gQ(3), gR(2), g_qb] (core/tube_mpc.py:915-919, 963-976).  -> [B, 7]"""
    _require_device(X_aux, U_aux, X_nom, U_nom, dX, dU)
    B, N = X_aux.shape[0], X_aux.shape[1] - 1
    lib = _lib.load()
    dt = X_aux.dtype
    args = [to_soa(t.to(dt)) for t in (X_aux, U_aux, X_nom, U_nom, dX, dU)]
    out = torch.empty(7, B, dtype=dt, device=X_aux.device)
    _lib.check(lib.dtmpc_doc_grad(_dtype_code(X_aux), N, B, *[a.data_ptr() for a in args], out.data_ptr(),
                                  _lib.stream_of(X_aux)), "dtmpc_doc_grad")
    return out.t().contiguous()
