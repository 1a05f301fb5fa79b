"""Pin the oracle's receding-horizon nominal MPC (oracle_nominal_receding) to run_nominal.py:204-415
run by the reference (tests/golden/make_golden_receding.py): the paper field, the success exit, the
collision exit, and exact-min / log-barrier / gamma / alpha variants.  CPU only, f64 (the reference's
precision for this driver); states at 1e-9 relative."""
from __future__ import annotations

import json

import numpy as np
import pytest

from _common import golden, rel


def receding_inputs(g):
    from diff_tube_mpc_strict_pt.core.receding import receding_setup_from_config

    cfg = json.loads(str(g["config"]))
    problem, cost, icfg = receding_setup_from_config(cfg)
    H = int(cfg["system"]["task_horizon_H"])
    N = problem.horizon
    U = np.zeros((1, N, 2))
    U[0, :, 0] = problem.u_max[0]
    return problem, cost, icfg, H, U


@pytest.mark.parametrize("name", ["R1", "R2", "R3", "R4"])
def test_receding_vs_run_nominal(oracle_lib, name):
    g = golden(f"receding_{name}")
    problem, cost, icfg, H, U = receding_inputs(g)
    o = oracle_lib.Oracle(np.float64)
    log, h_ran, st_t, coll, status, _ = o.nominal_receding(problem.to_c(), cost.to_c(), icfg.to_c(),
                                                           np.array([[0.0, 0.0, np.pi / 4]]), H, 0.25, U)
    assert status[0] == 0
    n = int(g["H_ran"])
    assert h_ran[0] == n
    assert bool(coll[0]) == bool(g["collided"])
    assert (st_t[0] >= 0) == bool(g["success"])
    if bool(g["success"]):
        assert st_t[0] == int(g["success_t"])
    assert rel(log[0, :n, 0:3], g["x_bar"]) < 1e-9
    assert rel(log[0, :n, 3:5], g["u_bar"]) < 1e-9
    assert rel(log[0, :n, 5], g["b_real"]) < 1e-9
    assert rel(log[0, n - 1, 0:3], g["final_state"]) < 1e-9


def test_receding_exits_are_covered():
    assert bool(golden("receding_R2")["success"]) and bool(golden("receding_R3")["collided"])
