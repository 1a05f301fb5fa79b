"""Receding-horizon nominal MPC on the HIP device (run_nominal.py:204-415): the single-run drop-in vs
the reference's own runs, and the batched driver vs the oracle.  Needs an MI355X: -m gpu.

Tolerances: f64 vs the reference at 1e-9 relative; batched f64 vs the oracle: exits identical, states
within the oracle-build agreement (base 1e-9); f32: agreement on >= 90 % of runs (the tol = 1e-3 exit
sits at fp32 resolution of the cost, see tests/test_gpu_parity.py)."""
from __future__ import annotations

import json
import os

import numpy as np
import pytest
import torch

from _common import agreement, golden, oracles, rel

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from diff_tube_mpc_strict_pt import _lib

    assert _lib.load().dtmpc_device_count() >= 1
    return torch.device("cuda:0")


@pytest.mark.parametrize("name", ["R1", "R2", "R3", "R4"])
def test_run_nominal_receding_vs_reference(dev, tmp_path, name):
    from diff_tube_mpc_strict_pt.run_nominal import run_nominal_receding

    g = golden(f"receding_{name}")
    cfg = json.loads(str(g["config"]))
    res = run_nominal_receding(cfg, device=dev, run_dir=str(tmp_path))
    s = res["summary"]
    assert s["H_ran"] == int(g["H_ran"])
    assert s["collided"] == bool(g["collided"]) and s["success"] == bool(g["success"])
    if s["success"]:
        assert s["success_t"] == int(g["success_t"])
    for f, key in (("x_bar", "x_bar"), ("u_bar", "u_bar"), ("b_real", "b_real"), ("x_real", "x_bar")):
        assert rel(np.load(os.path.join(tmp_path, f + ".npy")), g[key]) < 1e-9, f
    assert rel(np.array(s["final_state"]), g["final_state"]) < 1e-9


@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_nominal_receding_batched_vs_oracle(dev, oracle_lib, tag):
    """B = 257 starts over the obstacle field (some inside an obstacle -> collision at t = 0) with the
    target moved next to a cluster of starts (success exits), H = 15, against the oracle builds."""
    from diff_tube_mpc_strict_pt.core import nominal_receding
    from diff_tube_mpc_strict_pt.core.receding import receding_setup_from_config
    from _common import config

    npdt, tdt = (np.float64, torch.float64) if tag == "f64" else (np.float32, torch.float32)
    cfg = json.loads(json.dumps(config()))
    cfg["system"]["target"] = [1.0, 1.0, 0.7853981633974483]
    problem, cost, icfg = receding_setup_from_config(cfg)
    B, H, N = 257, 15, problem.horizon
    rng = np.random.default_rng(3)
    x0 = np.stack([rng.uniform(0, 5, B), rng.uniform(0, 5, B), rng.uniform(-np.pi, np.pi, B)], 1)
    x0[:40, :2] = 1.0 + rng.uniform(-0.5, 0.5, (40, 2))  # near the target
    x0[40:50, :2] = np.array([4.0, 2.0]) + rng.uniform(-0.3, 0.3, (10, 2))  # inside obstacle 0
    x0 = x0.astype(npdt)
    U = np.zeros((B, N, 2), npdt)
    U[:, :, 0] = problem.u_max[0]
    r = nominal_receding(problem=problem, cost=cost, cfg=icfg, x0=torch.as_tensor(x0, device=dev), H=H, check=False)
    torch.cuda.synchronize()
    outs = [o.nominal_receding(problem.to_c(), cost.to_c(), icfg.to_c(), x0, H, 0.25, U.copy()) for o in oracles(npdt)]
    h_dev = r.h_ran.cpu().numpy()
    # f32: a few runs driven into an obstacle overflow the relaxed barrier (b ~ 1e38) in the device and
    # the oracle alike (the reference's f32 path raises FloatingPointError there); they are set aside
    ok = (r.status.cpu().numpy() == 0) & np.all([o[4] == 0 for o in outs], axis=0)
    assert ok.mean() >= (1.0 if tag == "f64" else 0.9), ok.mean()
    assert r.collided[40:50].all() and (h_dev[40:50] == 1).all()
    assert (r.success_t.cpu().numpy() >= 0).sum() >= 20
    # The exits are knife-edge events (a plan grazing an obstacle, b ~ 1e8): the three oracle builds
    # themselves disagree on ~5 % of these runs at f64.  Exits are judged where the builds agree (the
    # well-conditioned runs, >= 85 % of the batch), and the device must match one build elsewhere.
    ex_dev = np.stack([h_dev, r.success_t.cpu().numpy(), r.collided.cpu().numpy().astype(np.int32)], 1)
    ex_or = [np.stack([o[1], o[2], o[3]], 1) for o in outs]
    cons = np.all([(e == ex_or[0]).all(1) for e in ex_or[1:]], axis=0) & ok
    assert cons.mean() >= (0.85 if tag == "f64" else 0.75), cons.mean()
    # the device's libm (sincos/exp/log) is a fourth valid rounding: plain-vs-fma builds already agree
    # on only ~95 % of all runs, so >= 97 % on the consensus set is the f64 bar (measured 97.9 %)
    need = 0.97 if tag == "f64" else 0.9
    assert (ex_dev[cons] == ex_or[0][cons]).all(1).mean() >= need
    any_build = np.any([(ex_dev == e).all(1) for e in ex_or], axis=0)[ok]
    assert any_build.mean() >= (0.95 if tag == "f64" else 0.85), any_build.mean()
    # recorded trajectories (common prefix with the plain build) within the oracle-build agreement
    same = (ex_dev == ex_or[0]).all(1) & ok
    h_or = outs[0][1]
    n = np.minimum(h_dev, h_or)
    mask = np.arange(H)[None, :] < n[:, None]
    dev_log = torch.cat([r.x, r.u, r.b[..., None]], -1).cpu().numpy()
    dev_log = np.where(mask[..., None], dev_log, 0)
    # a build whose own exit came earlier has NaN rows inside this mask: it cannot be the matching
    # build there (np.min over builds must not propagate its NaN)
    refs = [np.nan_to_num(np.where(mask[..., None], o[0], 0), nan=1e30) for o in outs]
    frac, e, _ = agreement(dev_log[same], [x[same] for x in refs], 1e-9 if tag == "f64" else 1e-4)
    assert frac >= need, (frac, np.sort(e)[-5:])


def test_run_nominal_once(dev, tmp_path):
    """run_nominal.py:37-201: one f32 nominal solve from the paper start, saved as *_single.npy."""
    from diff_tube_mpc_strict_pt.run_nominal import run_nominal_once
    from _common import config

    res = run_nominal_once(config(), device=dev, run_dir=str(tmp_path))
    xb = np.load(os.path.join(tmp_path, "x_bar_single.npy"))
    ub = np.load(os.path.join(tmp_path, "u_bar_single.npy"))
    assert xb.shape == (51, 3) and ub.shape == (50, 2) and np.isfinite(xb).all()
    g = golden("receding_R1")
    assert rel(ub[0], g["u_bar"][0]) < 1e-3  # the f64 reference's first applied control
    assert res["summary"]["mode"] == "nominal_only"


def test_receding_f32_failure_set_vs_oracle(dev, oracle_lib):
    """The f32 receding driver's failure SET at scale: B = 4,096 runs of the benchmark's
    start distribution (x0 ~ U[0,1]^2 x U[0, pi/2], paper configuration, H = 20), where about 10 % of the
    runs end non-finite in f32 (a line-search candidate pushed deep into an obstacle overflows the relaxed
    barrier's b^2, where the reference's f32 path raises FloatingPointError).

    Whether a run fails is a threshold event (a candidate's cost crossing 3.4e38), so the three oracle
    builds -- the same algorithm in three valid roundings -- agree with EACH OTHER on only ~85 % of the runs
    (measured: 0.851-0.856), and a 99 % device-vs-oracle agreement is not a property of the algorithm.  The
    test pins what is: the device agrees with every build at least as well as the builds agree with each
    other (minus 2 points), its failure count is within 15 % of theirs, and in f64 (no overflow) the failure
    sets are identical (empty).  Round 3 (generic kernel): device-vs-build 0.832-0.843; failures 463 vs 416-425,
    of them late in the horizon (h > 10) 100 vs ~51; the h > 10 split is asserted too since round 4 (the
    driver on the fused solver)."""
    import math

    from diff_tube_mpc_strict_pt.core import nominal_receding
    from diff_tube_mpc_strict_pt.core.receding import receding_setup_from_config
    from _common import config

    problem, cost, icfg = receding_setup_from_config(json.loads(json.dumps(config())))
    B, H, N = 4096, 20, problem.horizon
    g = torch.Generator().manual_seed(0)
    u = torch.rand(B, 3, generator=g, dtype=torch.float64)
    x0 = torch.stack([u[:, 0], u[:, 1], u[:, 2] * (math.pi / 2)], 1)
    fails = {}
    for tag, tdt, npdt in (("f32", torch.float32, np.float32), ("f64", torch.float64, np.float64)):
        r = nominal_receding(problem=problem, cost=cost, cfg=icfg, x0=x0.to(tdt).to(dev), H=H, check=False)
        torch.cuda.synchronize()
        U = np.zeros((B, N, 2), npdt)
        U[:, :, 0] = problem.u_max[0]
        outs = [o.nominal_receding(problem.to_c(), cost.to_c(), icfg.to_c(), x0.numpy().astype(npdt), H, 0.25, U.copy())
                for o in oracles(npdt)]
        fails[tag] = [r.status.cpu().numpy() != 0] + [o[4] != 0 for o in outs]
        if tag == "f32":
            hs = [r.h_ran.cpu().numpy()] + [o[1] for o in outs]
    f = fails["f32"]
    inter = min(float((f[i] == f[j]).mean()) for i in range(1, 4) for j in range(i + 1, 4))
    dev_vs = [float((f[0] == f[k]).mean()) for k in range(1, 4)]
    counts = [int(x.sum()) for x in f]
    # where in the horizon the runs fail (the h > 10 split): h_ran is the step of the failure
    late = [int((fk & (hk > 10)).sum()) for fk, hk in zip(f, hs)]
    print(f"[receding f32 B={B} H={H}] failures device / oracle builds {counts}, of them at h > 10 {late}; builds "
          f"agree with each other >= {inter:.4f}; device agrees with each build {[round(v, 4) for v in dev_vs]}")
    assert 0.02 <= f[0].mean() <= 0.3, f[0].mean()  # the regime the benchmark reports (~11 %)
    assert min(dev_vs) >= inter - 0.02, (dev_vs, inter)
    mean_or = np.mean(counts[1:])
    assert abs(counts[0] - mean_or) <= 0.15 * mean_or, counts
    mean_late = np.mean(late[1:])
    assert abs(late[0] - mean_late) <= max(0.15 * mean_late, 8), late  # the late-horizon split too
    assert all((x == fails["f64"][0]).all() for x in fails["f64"][1:])  # f64: the same (empty) set


@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_receding_fused_vs_generic(dev, tag, monkeypatch):
    """The receding driver on the tube step's fused solver (csrc/dtmpc_fast.hip receding_fast_kernel, the
    wrapped target cost compiled in) against the generic receding_kernel (DTMPC_FAST=0) from the same starts:
    the same algorithm in two roundings (the fused solver's FMA-contracted forward passes and its own sin /
    cos), so exits are identical and the recorded runs agree to 1e-8 (f64) / 1e-4 (f32) relative on the
    runs where no knife-edge exit intervenes (>= 97 % f64, >= 90 % f32)."""
    import math

    from diff_tube_mpc_strict_pt.core import nominal_receding
    from diff_tube_mpc_strict_pt.core.receding import receding_setup_from_config
    from _common import config

    tdt = torch.float64 if tag == "f64" else torch.float32
    problem, cost, icfg = receding_setup_from_config(json.loads(json.dumps(config())))
    B, H = 1024, 20
    g = torch.Generator().manual_seed(5)
    u = torch.rand(B, 3, generator=g, dtype=torch.float64)
    x0 = torch.stack([u[:, 0] * 3, u[:, 1] * 3, u[:, 2] * (math.pi / 2)], 1).to(tdt).to(dev)
    runs = []
    for fast in ("1", "0"):
        monkeypatch.setenv("DTMPC_FAST", fast)
        r = nominal_receding(problem=problem, cost=cost, cfg=icfg, x0=x0, H=H, check=False)
        torch.cuda.synchronize()
        runs.append(r)
    a, b = runs
    ex = [np.stack([r.h_ran.cpu().numpy(), r.success_t.cpu().numpy(), r.collided.cpu().numpy()], 1) for r in runs]
    same = (ex[0] == ex[1]).all(1) & (a.status.cpu().numpy() == 0) & (b.status.cpu().numpy() == 0)
    la = torch.cat([a.x, a.u, a.b[..., None]], -1).cpu().numpy()
    lb = torch.cat([b.x, b.u, b.b[..., None]], -1).cpu().numpy()
    mask = np.arange(H)[None, :] < a.h_ran.cpu().numpy()[:, None]
    d = np.where(mask[..., None], np.abs(la - lb), 0).reshape(B, -1).max(1)
    sc = np.where(mask[..., None], np.abs(lb), 0).reshape(B, -1).max(1) + 1.0
    tol = 1e-8 if tag == "f64" else 1e-4
    frac_ex = float((ex[0] == ex[1]).all(1).mean())
    frac = float((d[same] / sc[same] <= tol).mean())
    print(f"[receding fused vs generic {tag}] exits equal {frac_ex:.4f}; runs within {tol:g} {frac:.4f} "
          f"(of {int(same.sum())})")
    need = 0.97 if tag == "f64" else 0.90
    assert frac_ex >= need and frac >= need, (frac_ex, frac)
