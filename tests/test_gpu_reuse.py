"""The fused tube step must not read device memory it has not written (GPU).  Two closed-loop steps of the paper
setup (fixed iterations, B = 700) run twice in one process, the second time with the step's workspace pre-filled
with 0xff bytes (NaN in either precision): every state, tape, log row, partial sum and theta must be bitwise
equal.  Round 5 found the two-lane f64 step with the one-block asm exp failing this on one trajectory
(csrc/dtmpc_fast.hip xasm_flag; scripts/diag_reuse.py is the diagnostic form)."""
import dataclasses

import numpy as np
import pytest
import torch

from _common import paper_setup

pytestmark = pytest.mark.gpu
NAMES = ("x", "b", "xbar", "bbar", "Xnom", "Unom", "Xaux", "Uaux", "theta", "status", "log", "partials")


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from diff_tube_mpc_strict_pt import _lib

    assert _lib.load().dtmpc_device_count() >= 1
    return torch.device("cuda:0")


@pytest.mark.parametrize("lanes", ["1", "2", "4"])
@pytest.mark.parametrize("tag", ["f32", "f64"])
def test_tube_step_reads_only_what_it_wrote(dev, tag, lanes, monkeypatch):
    from diff_tube_mpc_strict_pt.core import TubeMPC

    monkeypatch.setenv("DTMPC_TUBE_LANES", lanes)
    st = paper_setup()
    st = dataclasses.replace(st, ilqr_nom=dataclasses.replace(st.ilqr_nom, tol=-1.0),
                             ilqr_aux=dataclasses.replace(st.ilqr_aux, tol=-1.0))
    tdt = torch.float64 if tag == "f64" else torch.float32
    B = 700
    rng = np.random.default_rng(5)
    x = torch.as_tensor(np.stack([rng.uniform(0, 1, B), rng.uniform(0, 1, B), rng.uniform(0, np.pi / 2, B)], 1),
                        dtype=tdt, device=dev)
    runs = []
    for fill in (None, 0xFF):
        m = TubeMPC(st, batch=B, device=dev, dtype=tdt, disturbance="philox", seed=4, write_log=True)
        if fill is not None:
            m.work.fill_(fill)
        m.reset(x)
        m.step()
        m.step()
        torch.cuda.synchronize()
        runs.append({k: getattr(m, k).clone() for k in NAMES if getattr(m, k, None) is not None})
    assert (runs[0]["status"] == 0).all()
    for k in runs[0]:
        assert torch.equal(runs[0][k], runs[1][k]) or (
            runs[0][k].is_floating_point() and torch.equal(torch.isnan(runs[0][k]), torch.isnan(runs[1][k])) and
            torch.equal(torch.nan_to_num(runs[0][k]), torch.nan_to_num(runs[1][k]))), k
