"""Shared plumbing of the per-point entry points (include/dtmpc_systems.h): batch flattening, dtype /
device checks and the launch.  Every array is point-major [n, F] (the reference's [B, F] layout), so a
caller's tensor goes to the kernel as is when it is already contiguous.  There is no CPU fallback:
host tensors raise ValueError, a missing library NativeLibraryError.

Autograd: the reference's per-function API is plain torch, so autograd differentiates through it (its
``core/ddp.py`` ``_linearize_autograd`` and ``core/autodiff.py`` rely on that).  The functions whose
reference bodies are differentiable maps -- ``dubins_step``, the h aggregations, the barriers and the box
clamp -- are ``torch.autograd.Function``s here whose backward uses the analytic derivative the library
already computes (the kernels' grad h / dB outputs, the Dubins Jacobian).  Every other entry point
(Jacobians, cost derivatives, the tanh map) refuses an input that requires grad while grad mode is on
(``require_device``), so a caller never gets an output silently cut from the graph."""
from __future__ import annotations

import ctypes as C
import math
from typing import Optional, Sequence, Tuple

import torch
from torch import Tensor

from .. import _abi, _lib
from .problem import CircleObstacle, DubinsDBaSProblem


def dtype_code(t: Tensor) -> int:
    if t.dtype == torch.float32:
        return _abi.F32
    if t.dtype == torch.float64:
        return _abi.F64
    raise ValueError(f"unsupported dtype {t.dtype}; use float32 or float64")


def require_device(*ts: Optional[Tensor]) -> None:
    """Device tensors only; and no input that autograd would have to differentiate (see the module
    docstring: the differentiable entry points call this inside their autograd.Function's forward,
    where grad mode is off)."""
    for t in ts:
        if t is not None and t.device.type != "cuda":
            raise ValueError("the dtmpc HIP path needs device tensors (got %s); there is no CPU fallback" % t.device)
    forbid_grad(*ts)


def forbid_grad(*ts) -> None:
    if torch.is_grad_enabled() and any(isinstance(t, Tensor) and t.requires_grad for t in ts):
        raise RuntimeError("this dtmpc entry point is a HIP kernel without an autograd formula and an input "
                           "requires grad: its output would be cut from the graph.  Differentiate through "
                           "dubins_step / h_* / the barriers / BoxClampControl.clamp (autograd Functions), or "
                           "call under torch.no_grad() / with detached inputs")


def rows(t: Tensor, F: int, like: Tensor) -> Tuple[Tensor, Tuple[int, ...]]:
    """[..., F] -> contiguous [n, F] in like's dtype / device, and the leading shape."""
    if t.shape[-1] != F:
        raise ValueError(f"expected a trailing dimension of {F}, got shape {tuple(t.shape)}")
    lead = tuple(t.shape[:-1])
    n = math.prod(lead)
    return t.to(device=like.device, dtype=like.dtype).reshape(n, F).contiguous(), lead


def scalar(v) -> float:
    """A float or a one-element tensor (the reference's ScalarLike)."""
    if isinstance(v, Tensor):
        forbid_grad(v)
        if v.numel() != 1:
            raise NotImplementedError("per-point (batched) DBaS parameters are not supported; pass a scalar")
        return float(v.reshape(()).item())
    return float(v)


def spec(*, dt: float = 0.01, obstacles: Sequence[CircleObstacle] = (), aggregation: str = "none", beta: float = 20.0,
         barrier_type: str = "inverse", alpha=0.0, gamma=0.0, eps: float = 1e-4,
         u_min=(-10.0, -math.pi), u_max=(10.0, math.pi), active_tol: float = 1e-8) -> _abi.DtmpcSpec:
    if len(obstacles) > _abi.MAX_OBS:
        raise NotImplementedError(f"at most {_abi.MAX_OBS} obstacles per call")
    obs = tuple(CircleObstacle(center=(float(o.center[0]), float(o.center[1])), radius=float(o.radius))
                for o in obstacles)
    p = DubinsDBaSProblem(horizon=1, dt=float(dt), obstacles=obs, obs_beta=float(beta), obs_aggregation=aggregation,
                          barrier_type=barrier_type, dbas_alpha=scalar(alpha), dbas_gamma=scalar(gamma),
                          dbas_eps=float(eps), u_min=tuple(float(v) for v in u_min),
                          u_max=tuple(float(v) for v in u_max), active_tol=float(active_tol))
    return p.to_c()


def launch(name: str, *args) -> None:
    lib = _lib.load()
    _lib.check(getattr(lib, name)(*args), name)


def ptr(t: Optional[Tensor]):
    return None if t is None else t.data_ptr()


def stream(t: Tensor) -> int:
    return _lib.stream_of(t)


def byref(s):
    return C.byref(s)
