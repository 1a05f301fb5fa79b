"""Batched receding-horizon nominal MPC -- run_nominal.py:204-415 for B independent starts.

The reference runs one trajectory: per closed-loop step an iLQR solve with the angle-wrapped nominal
cost (run_nominal.py:297-324), the first control applied through the DBaS-augmented plant, a
collision check (true min over the circles <= 0) and a success check (||x[:2] - target[:2]|| <= 0.25),
then the warm-start shift.  Here the whole task horizon of all B runs is ONE kernel launch
(``dtmpc_nominal_receding``): each lane runs its own loop and stops at its own exit.
"""
from __future__ import annotations

import ctypes as C
import math
from dataclasses import dataclass
from typing import Any, Dict, Optional, Tuple

import torch
from torch import Tensor

from .. import _lib
from .ddp import _dtype_code, _require_device, from_soa, raise_for_status, to_soa
from .problem import DubinsDBaSProblem, ILQRConfig, QuadraticCost, problem_from_config

__all__ = ["RecedingResult", "nominal_receding", "receding_setup_from_config", "SUCCESS_RADIUS"]

SUCCESS_RADIUS = 0.25  # run_nominal.py:382


@dataclass(frozen=True)
class RecedingResult:
    x: Tensor          # [B, H, 3] recorded states (rows >= h_ran are NaN)
    u: Tensor          # [B, H, 2] applied controls u0
    b: Tensor          # [B, H] barrier states
    h_ran: Tensor      # [B] recorded steps
    success_t: Tensor  # [B] step of the success exit, -1 if none
    collided: Tensor   # [B] bool
    status: Tensor     # [B] DTMPC_ST_* bits
    U_last: Tensor     # [B, N, 2] last (shifted) plan
    iters: Optional[Tensor] = None  # [B] total iLQR iterations of each run (dtmpc_nominal_receding_it)


def receding_setup_from_config(cfg: Dict[str, Any]) -> Tuple[DubinsDBaSProblem, QuadraticCost, ILQRConfig]:
    """run_nominal.py:231-366: obstacles / DBaS from the config (alpha, gamma, barrier type as given),
    nominal weights, angle-wrapped target cost, ILQRConfig(tol = 1e-3, reg = ilqr_reg, the config's
    line-search alphas)."""
    sc = cfg["system"]
    env = cfg.get("environment", {})
    if "obstacles" not in env and "obstacle" not in env:
        import dataclasses

        base = problem_from_config(cfg)
        problem = dataclasses.replace(base, obstacles=(), obs_aggregation="none")  # h = 1 (run_nominal.py:256)
    else:
        problem = problem_from_config(cfg)
    cn = cfg["cost_nominal"]
    cost = QuadraticCost(kind="target", Q=tuple(float(v) for v in cn["Q"]), R=tuple(float(v) for v in cn["R"]),
                         Qf=tuple(float(v) for v in cn["Qf"]), qb=float(cn["q_b"]),
                         target=tuple(float(v) for v in sc["target"]), wrap_angle=True)
    icfg = ILQRConfig(horizon=int(sc["horizon_N"]), max_iter=int(sc.get("nominal_max_iter", 10)), tol=1e-3,
                      reg=float(sc.get("ilqr_reg", 1e-6)),
                      line_search_alphas=tuple(float(a) for a in sc.get("line_search_alphas", [1.0, 0.5, 0.25, 0.1])))
    return problem, cost, icfg


def nominal_receding(*, problem: DubinsDBaSProblem, cost: QuadraticCost, cfg: ILQRConfig, x0: Tensor, H: int,
                     success_radius: float = SUCCESS_RADIUS, U_init: Optional[Tensor] = None,
                     check: bool = True) -> RecedingResult:
    """B receding-horizon runs from x0 [B, 3] (b0 = B(h(x0)) derived).  U_init [B, N, 2] defaults to the
    reference's warm start v = v_max, omega = 0 (run_nominal.py:368-369)."""
    _require_device(x0, U_init)
    if cost.kind != "target":
        raise ValueError("the receding nominal MPC uses a target cost")
    B, N = x0.shape[0], problem.horizon
    if x0.shape != (B, 3):
        raise ValueError("x0 must be [B, 3]")
    dt = x0.dtype
    kw = dict(dtype=dt, device=x0.device)
    if U_init is None:
        U_init = torch.zeros(B, N, 2, **kw)
        U_init[:, :, 0] = float(problem.u_max[0])
    lib = _lib.load()
    spec, cc, ic = problem.to_c(), cost.to_c(), cfg.to_c()
    xs = x0.t().contiguous()
    Us = to_soa(U_init.to(dt))
    log = torch.full((H, 6, B), math.nan, **kw)
    ints = [torch.zeros(B, dtype=torch.int32, device=x0.device) for _ in range(5)]
    work = torch.empty(lib.dtmpc_receding_workspace_bytes(_dtype_code(x0), N, B), dtype=torch.uint8, device=x0.device)
    _lib.check(lib.dtmpc_nominal_receding_it(_dtype_code(x0), C.byref(spec), C.byref(cc), C.byref(ic), B, int(H),
                                             float(success_radius), xs.data_ptr(), Us.data_ptr(), log.data_ptr(),
                                             *[t.data_ptr() for t in ints], work.data_ptr(), _lib.stream_of(x0)),
               "dtmpc_nominal_receding")
    h_ran, success_t, collided, status, iters = ints
    if check:
        raise_for_status(status, "nominal_receding")
    lg = from_soa(log)
    return RecedingResult(x=lg[:, :, 0:3], u=lg[:, :, 3:5], b=lg[:, :, 5], h_ran=h_ran, success_t=success_t,
                          collided=collided.bool(), status=status, U_last=from_soa(Us), iters=iters)
