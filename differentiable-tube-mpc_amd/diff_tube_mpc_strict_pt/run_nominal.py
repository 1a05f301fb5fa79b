"""Drop-ins for the reference's run_nominal.py entry points on the HIP path.

* :func:`run_nominal_receding` (run_nominal.py:204-415): receding-horizon nominal MPC from the paper
  start (0, 0, pi/4), f64, writing x_bar / u_bar / x_real / u_real / b_real / loss .npy files and the
  same summary.  The batched form is :func:`diff_tube_mpc_strict_pt.core.receding.nominal_receding`.
* :func:`run_nominal_once` (run_nominal.py:37-201): one nominal solve (f32, as the reference), writing
  x_bar_single.npy / u_bar_single.npy.
"""
from __future__ import annotations

import os
from typing import Any, Dict

import numpy as np
import torch

from .core.ddp import ilqr_solve
from .core.receding import SUCCESS_RADIUS, nominal_receding, receding_setup_from_config

__all__ = ["run_nominal_receding", "run_nominal_once"]

_X0 = (0.0, 0.0, float(np.pi / 4))  # run_nominal.py:91, 276


def run_nominal_receding(cfg: Dict[str, Any], *, device: torch.device, run_dir: str) -> Dict[str, Any]:
    system_cfg = cfg["system"]
    assert system_cfg["name"] == "dubins"
    problem, cost, icfg = receding_setup_from_config(cfg)
    H = int(system_cfg["task_horizon_H"])
    dtype = torch.float64  # run_nominal.py:220
    x0 = torch.tensor([_X0], dtype=dtype, device=device)
    r = nominal_receding(problem=problem, cost=cost, cfg=icfg, x0=x0, H=H, success_radius=SUCCESS_RADIUS)
    n = int(r.h_ran[0])
    xs_np = r.x[0, :n].cpu().numpy().astype(np.float64)
    us_np = r.u[0, :n].cpu().numpy().astype(np.float64)
    bs_np = r.b[0, :n].cpu().numpy().astype(np.float64)
    os.makedirs(run_dir, exist_ok=True)
    np.save(os.path.join(run_dir, "x_bar.npy"), xs_np)
    np.save(os.path.join(run_dir, "u_bar.npy"), us_np)
    np.save(os.path.join(run_dir, "x_real.npy"), xs_np)
    np.save(os.path.join(run_dir, "u_real.npy"), us_np)
    np.save(os.path.join(run_dir, "b_real.npy"), bs_np)
    np.save(os.path.join(run_dir, "loss.npy"), np.zeros((xs_np.shape[0],), dtype=np.float64))
    st = int(r.success_t[0])
    return {
        "summary": {
            "system": "dubins",
            "mode": "nominal_receding",
            "H_ran": int(xs_np.shape[0]),
            "success": st >= 0,
            "success_t": None if st < 0 else st,
            "collided": bool(r.collided[0]),
            "final_state": xs_np[-1].tolist() if xs_np.size else list(_X0),
        }
    }


def run_nominal_once(cfg: Dict[str, Any], *, device: torch.device, run_dir: str) -> Dict[str, Any]:
    from .core.ddp import dbas_init

    problem, cost, icfg = receding_setup_from_config(cfg)
    N = problem.horizon
    dtype = torch.float32  # run_nominal.py:87-124
    x0 = torch.tensor([_X0], dtype=dtype, device=device)
    b0 = dbas_init(problem, x0)
    x_hat0 = torch.cat([x0, b0[:, None]], 1)
    U_ws = torch.zeros(1, N, 2, dtype=dtype, device=device)
    U_ws[:, :, 0] = float(problem.u_max[0])
    res = ilqr_solve(problem=problem, cost=cost, cfg=icfg, x0=x_hat0, V_init=U_ws, debug_name="iLQR-nominal")
    x_bar = res.X[0, :, :-1].cpu().numpy()
    u_bar = res.V[0].cpu().numpy()
    os.makedirs(run_dir, exist_ok=True)
    np.save(os.path.join(run_dir, "x_bar_single.npy"), x_bar)
    np.save(os.path.join(run_dir, "u_bar_single.npy"), u_bar)
    return {"summary": {"system": "dubins", "mode": "nominal_only", "N": N, "x0": x_bar[0].tolist(),
                        "xN": x_bar[-1].tolist()}}
