"""The lane forms of the fused solver compute the same numbers (GPU).  One, two and four lanes per trajectory split the
line search's candidates and the backward pass's linearisation differently, but every value is produced by the same
operations in the same order; since round 6 the backward step (the Jacobian and the Riccati step) compiles without
implicit FMA contraction, every multiply-add an explicit fma at a fixed place (DTMPC_FAST_RIC_FMA), so the compiler
cannot round it differently per form (reference core/ddp.py:213-254).
Two closed-loop steps of the paper setup (fixed iterations, B = 700, theta held) at 1, 2 and 4 lanes: every state,
tape, log row (the per-trajectory DOC gradient rows included) and status bitwise equal; the standalone batched iLQR (core.ddp.ilqr_solve, BASELINE config 2's solve) the
same over its lane forms."""
import dataclasses

import numpy as np
import pytest
import torch

from _common import ilqr_cfg, paper_setup

pytestmark = pytest.mark.gpu
NAMES = ("x", "b", "xbar", "bbar", "Xnom", "Unom", "Xaux", "Uaux", "status", "log")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


def _x0(B, tdt, dev, seed=5):
    rng = np.random.default_rng(seed)
    return torch.as_tensor(np.stack([rng.uniform(0, 1, B), rng.uniform(0, 1, B), rng.uniform(0, np.pi / 2, B)], 1),
                           dtype=tdt, device=dev)


def _same(a, b):
    return torch.equal(a, b) or (a.is_floating_point() and torch.equal(torch.isnan(a), torch.isnan(b)) and
                                 torch.equal(torch.nan_to_num(a), torch.nan_to_num(b)))


@pytest.mark.parametrize("tag", ["f32", "f64"])
def test_tube_step_lane_forms_bitwise(dev, tag, monkeypatch):
    from diff_tube_mpc_strict_pt.core import TubeMPC

    st = paper_setup()
    st = dataclasses.replace(st, ilqr_nom=dataclasses.replace(st.ilqr_nom, tol=-1.0),
                             ilqr_aux=dataclasses.replace(st.ilqr_aux, tol=-1.0))
    tdt = torch.float64 if tag == "f64" else torch.float32
    B = 700
    x = _x0(B, tdt, dev)
    runs = {}
    for lanes in ("1", "2", "4"):
        monkeypatch.setenv("DTMPC_TUBE_LANES", lanes)
        m = TubeMPC(st, batch=B, device=dev, dtype=tdt, disturbance="philox", seed=4, write_log=True)
        assert m.lanes == int(lanes)
        m.reset(x)
        # theta held (adapt=False): the batch-mean gradient's sum runs over workgroups whose size in trajectories
        # depends on the lane form, so its rounding -- and with it every later step -- legitimately differs
        m.step(adapt=False)
        m.step(adapt=False)
        torch.cuda.synchronize()
        runs[lanes] = {k: getattr(m, k).clone() for k in NAMES if getattr(m, k, None) is not None}
    assert (runs["1"]["status"] == 0).all()
    for lanes in ("2", "4"):
        bad = [k for k in runs["1"] if not _same(runs["1"][k], runs[lanes][k])]
        assert not bad, (lanes, bad)


@pytest.mark.parametrize("tag", ["f32", "f64"])
def test_ilqr_lane_forms_bitwise(dev, tag):
    from diff_tube_mpc_strict_pt.core import ilqr_solve
    from diff_tube_mpc_strict_pt.core.ddp import dbas_init

    st = paper_setup()
    tdt = torch.float64 if tag == "f64" else torch.float32
    B, N = 1000, st.problem.horizon
    x3 = _x0(B, tdt, dev, seed=9)
    x0 = torch.cat([x3, dbas_init(st.problem, x3)[:, None]], 1)
    V0 = torch.zeros(B, N, 2, dtype=tdt, device=dev)
    cfg = ilqr_cfg(10, -1.0)
    out = {}
    for lanes in (1, 2, 4):
        r = ilqr_solve(problem=st.problem, cost=st.nominal_cost, cfg=cfg, x0=x0, V_init=V0, lanes=lanes)
        torch.cuda.synchronize()
        out[lanes] = (r.X.clone(), r.V.clone(), r.K.clone(), r.k.clone(), r.iters.clone(), r.status.clone())
    for lanes in (2, 4):
        for i, (a, b) in enumerate(zip(out[1], out[lanes])):
            assert _same(a, b), (lanes, i)
