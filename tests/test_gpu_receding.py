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


def test_receding_f32_failure_set_vs_oracle(dev, oracle_lib, monkeypatch):
    """The f32 receding driver's failure SET at scale: B = 4,096 runs of the
    benchmark's start distribution (x0 ~ U[0,1]^2 x U[0, pi/2], paper configuration, H = 20).

    Root cause of the reference's f32 failures: the warm start (v = 10, w = 0) drives most
    of these runs straight into an obstacle, deep in the relaxed barrier's quadratic branch, where B's barrier
    row is ~1e10.  Q_uu = l_uu + B^T V_xx B is then numerically rank one in f32 (its small eigenvalue, 2 + reg,
    lies below the resolution of the large one, ~1e20), so the gains are rounding noise, and the antisymmetric
    part of V_xx that the reference's order leaves (core/ddp.py:252, never symmetrised) grows through the
    closed loop until it overflows: one step before the first non-finite gain Q_uu = [[2, 1.9e34],
    [-1.9e34, 3e25]] in one of them (oracle, second backward pass of the first solve); all 422 of the plain
    build's failures are a non-finite Riccati step.  Whether a run fails is therefore a property of
    the evaluation order, not of the algorithm: liboracle_sym.so -- the plain build with V_xx mirrored from its
    upper triangle after every step, equal in exact arithmetic -- fails on ~0.5 % of the runs against ~10 % for
    the plain / fma / ulp builds, and the fused solver's order (csrc/dtmpc_fast.hip riccati_pk: fma chains,
    the gamma = 0 structure) on none.  The reference configuration is f64 (configs/dubins.yaml:8), where no
    run fails anywhere.

    Asserted: the reference-form builds' failure rate (the regime) and the symmetric build's; the fused
    driver fails on no more runs than the symmetric build, in total and at h > 10 (+8 runs); the generic
    kernel (DTMPC_FAST=0, the reference's order of the recursion) against the reference-form builds (total
    within 15 %); f64: every failure set identical (empty)."""
    import math

    from diff_tube_mpc_strict_pt.core import nominal_receding
    from diff_tube_mpc_strict_pt.core.receding import receding_setup_from_config
    from _common import config
    from oracle.oracle import Oracle

    problem, cost, icfg = receding_setup_from_config(json.loads(json.dumps(config())))
    B, H, N = 4096, 20, problem.horizon
    g = torch.Generator().manual_seed(0)
    u = torch.rand(B, 3, generator=g, dtype=torch.float64)
    x0 = torch.stack([u[:, 0], u[:, 1], u[:, 2] * (math.pi / 2)], 1)
    fails, hs = {}, {}
    for tag, tdt, npdt in (("f32", torch.float32, np.float32), ("f64", torch.float64, np.float64)):
        devs = []
        for fast in ("1", "0"):
            monkeypatch.setenv("DTMPC_FAST", fast)
            r = nominal_receding(problem=problem, cost=cost, cfg=icfg, x0=x0.to(tdt).to(dev), H=H, check=False)
            torch.cuda.synchronize()
            devs.append((r.status.cpu().numpy() != 0, r.h_ran.cpu().numpy()))
        monkeypatch.delenv("DTMPC_FAST")
        U = np.zeros((B, N, 2), npdt)
        U[:, :, 0] = problem.u_max[0]
        builds = oracles(npdt) + [Oracle(npdt, nthreads=8, variant="sym")]
        outs = [o.nominal_receding(problem.to_c(), cost.to_c(), icfg.to_c(), x0.numpy().astype(npdt), H, 0.25, U.copy())
                for o in builds]
        # [fused, generic, plain, fma, ulp, sym]
        fails[tag] = [d[0] for d in devs] + [o[4] != 0 for o in outs]
        hs[tag] = [d[1] for d in devs] + [o[1] for o in outs]
    f, h = fails["f32"], hs["f32"]
    counts = [int(x.sum()) for x in f]
    late = [int((fk & (hk > 10)).sum()) for fk, hk in zip(f, h)]  # h_ran is the step of the failure
    inter = min(float((f[i] == f[j]).mean()) for i in range(2, 5) for j in range(i + 1, 5))
    print(f"[receding f32 B={B} H={H}] failures fused / generic / plain, fma, ulp builds / symmetric-V_xx build "
          f"{counts}, of them at h > 10 {late}; reference-form builds agree with each other >= {inter:.4f}; "
          f"fused vs symmetric build {float((f[0] == f[5]).mean()):.4f}")
    assert all(0.02 <= x.mean() <= 0.3 for x in f[2:5]), counts  # the regime (the reference form, ~10 %)
    assert f[5].mean() <= 0.015, counts  # ... of which the unsymmetrised V_xx accounts for ~95 %
    assert counts[0] <= counts[5] + 8, counts
    assert late[0] <= late[5] + 8, late
    assert float((f[0] == f[5]).mean()) >= inter - 0.02
    mean_ref = np.mean(counts[2:5])
    assert abs(counts[1] - mean_ref) <= 0.15 * mean_ref, counts  # the generic kernel keeps the reference form
    assert all(not x.any() for x in fails["f64"]), [int(x.sum()) for x in fails["f64"]]  # f64: empty sets


@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_receding_fused_vs_generic(dev, oracle_lib, tag, monkeypatch):
    """The receding driver on the tube step's fused solver (csrc/dtmpc_fast.hip receding_fast_kernel, the
    wrapped target cost compiled in) against the generic receding_kernel (DTMPC_FAST=0) from the same starts
    (x0 ~ U[0,3]^2 x U[0, pi/2], paper configuration, H = 20).

    This workload is chaotic: many starts see an obstacle within the horizon and the closed loop passes close
    to others, so the oracle's own builds (plain / fma / ulp: the same algorithm in three valid roundings)
    agree on the exits of only ~80 % of the runs (f64) and on the whole recorded run at 1e-8 on only ~16 %
    (measured 0.798-0.811 / 0.162-0.164).  The two device kernels are two more roundings: their agreement is
    held to the builds' own (runs where nothing fails; minus 3 points for exits, 5 for the row fraction).
    Row-level parity is pinned on the well-conditioned workloads above (the reference runs at 1e-9,
    test_nominal_receding_batched_vs_oracle)."""
    import math

    from diff_tube_mpc_strict_pt.core import nominal_receding
    from diff_tube_mpc_strict_pt.core.receding import receding_setup_from_config
    from _common import config

    tdt, npdt = (torch.float64, np.float64) if tag == "f64" else (torch.float32, np.float32)
    problem, cost, icfg = receding_setup_from_config(json.loads(json.dumps(config())))
    B, H, N = 1024, 20, problem.horizon
    g = torch.Generator().manual_seed(5)
    u = torch.rand(B, 3, generator=g, dtype=torch.float64)
    x0 = torch.stack([u[:, 0] * 3, u[:, 1] * 3, u[:, 2] * (math.pi / 2)], 1)
    runs = []
    for fast in ("1", "0"):
        monkeypatch.setenv("DTMPC_FAST", fast)
        r = nominal_receding(problem=problem, cost=cost, cfg=icfg, x0=x0.to(tdt).to(dev), H=H, check=False)
        torch.cuda.synchronize()
        runs.append((torch.cat([r.x, r.u, r.b[..., None]], -1).cpu().numpy(), r.h_ran.cpu().numpy(),
                     r.success_t.cpu().numpy(), r.collided.cpu().numpy().astype(np.int32), r.status.cpu().numpy()))
    monkeypatch.delenv("DTMPC_FAST")
    U = np.zeros((B, N, 2), npdt)
    U[:, :, 0] = problem.u_max[0]
    for o in oracles(npdt):
        runs.append(o.nominal_receding(problem.to_c(), cost.to_c(), icfg.to_c(), x0.numpy().astype(npdt), H, 0.25,
                                       U.copy())[:5])
    ok = np.all([r[4] == 0 for r in runs], axis=0)  # runs where nothing fails (f32: see the test above)
    tol = 1e-8 if tag == "f64" else 1e-4

    def pair(a, b):
        ex = (a[1] == b[1]) & (a[2] == b[2]) & (a[3] == b[3])
        same = ex & ok
        mask = np.arange(H)[None, :] < a[1][:, None]
        d = np.where(mask[..., None], np.abs(np.nan_to_num(a[0]) - np.nan_to_num(b[0])), 0).reshape(B, -1).max(1)
        sc = np.where(mask[..., None], np.abs(np.nan_to_num(b[0])), 0).reshape(B, -1).max(1) + 1.0
        return float(ex[ok].mean()), float((d[same] / sc[same] <= tol).mean())

    dv = pair(runs[0], runs[1])
    bl = [pair(runs[i], runs[j]) for i in range(2, 5) for j in range(i + 1, 5)]
    print(f"[receding fused vs generic {tag}] on {int(ok.sum())} runs: exits equal {dv[0]:.4f}, runs within {tol:g} "
          f"{dv[1]:.4f}; oracle builds pairwise {[(round(a, 4), round(b, 4)) for a, b in bl]}")
    assert ok.mean() >= (1.0 if tag == "f64" else 0.7), ok.mean()  # f32: the builds fail on ~8 % each (union ~25 %)
    assert dv[0] >= min(b[0] for b in bl) - 0.03, (dv, bl)
    assert dv[1] >= min(b[1] for b in bl) - 0.05, (dv, bl)


def test_reference_call_pattern(dev):
    """run_nominal.py:344-410 with its solver call (:353-364) in the reference's keyword form -- closures
    from core.closures.nominal_closures, the f_jac lambda, single-trajectory tensors -- on the device in f64,
    against the reference's own run (tests/golden/nominal_receding.npz, H = 2) at 1e-9."""
    import math

    from diff_tube_mpc_strict_pt.core import ilqr_solve
    from diff_tube_mpc_strict_pt.core.closures import nominal_closures
    from diff_tube_mpc_strict_pt.core.ddp import dbas_init
    from _common import config

    cfg = json.loads(json.dumps(config()))
    cfg["system"]["task_horizon_H"] = 2
    cl = nominal_closures(cfg)
    f_hat, ctrl, ilqr_cfg, jac = cl["f_hat"], cl["ctrl"], cl["ilqr_cfg"], cl["f_jac"]
    stage_cost, terminal_cost, stage_derivs, term_derivs = (cl["stage_cost"], cl["terminal_cost"],
                                                            cl["stage_derivs"], cl["term_derivs"])
    kw = dict(dtype=torch.float64, device=dev)
    N, H = ilqr_cfg.horizon, 2
    x = torch.tensor([0.0, 0.0, math.pi / 4], **kw)
    b = dbas_init(f_hat.problem, x[None])[0]
    U_ws = torch.zeros(N, 2, **kw)
    U_ws[:, 0] = float(ctrl.u_max[0])
    xs, us, bs = [], [], []
    for t in range(H):
        x_hat0 = torch.cat([x, b.view(1)], dim=0)
        X_hat, U = ilqr_solve(
            x0=x_hat0,
            V_init=U_ws,
            cfg=ilqr_cfg,
            f=f_hat,
            ctrl=ctrl,
            f_jac=lambda xh, uk: jac(xh, uk),
            stage_cost=stage_cost,
            terminal_cost=terminal_cost,
            stage_derivs=stage_derivs,
            terminal_derivs=term_derivs,
        )
        assert X_hat.shape == (N + 1, 4) and U.shape == (N, 2)
        u0 = U[0]
        xs.append(x.cpu().numpy())
        us.append(u0.cpu().numpy())
        bs.append(float(b))
        xn = f_hat(x_hat0, u0)
        x, b = xn[:3], xn[3]
        U_ws = torch.cat([U[1:], U[-1:]], dim=0)
    g = golden("nominal_receding")
    assert rel(np.array(xs), g["x_bar"]) < 1e-9
    assert rel(np.array(us), g["u_bar"]) < 1e-9
    assert rel(np.array(bs), g["b_real"]) < 1e-9
    # the closures themselves evaluate on the device: cost and derivatives at the last plan's first point
    J0 = stage_cost(X_hat[0], U[0], 0)
    lx, lu, lxx, luu, lux = stage_derivs(X_hat[0], U[0], 0)
    phi_x, phi_xx = term_derivs(X_hat[N])
    assert torch.isfinite(J0) and lx.shape == (4,) and lu.shape == (2,) and phi_xx.shape == (4, 4)
    assert float(phi_xx[3, 3]) == 2.0 * stage_cost.__self__.cost.qb


@pytest.mark.parametrize("m,gamma,alpha", [(m, 0.0, 0.0) for m in range(1, 9)] + [(3, 0.3, 0.05), (4, 0.3, 0.05),
                                                                                (5, 0.3, 0.05), (8, 0.3, 0.05)])
def test_receding_fused_instantiations_vs_generic(dev, oracle_lib, m, gamma, alpha):
    """The fused receding driver's other instantiations -- every obstacle count 1-8 (compile-time M) and the
    general gain records (gamma != 0, alpha > 0: receding_fast_kernel<M, 0>) -- against the generic kernel and
    the oracle (plain build), f64, B = 256, H = 10, x0 ~ U[0,1]^2 x U[0, pi/2]; and the fused driver run
    twice on the same inputs, bitwise equal.  This test found the M = 8 f64 defect of round 4 (run-to-run
    different results with the obstacle table pinned in VGPRs).

    The obstacles sit off the diagonal the runs move along (barrier active, no decision close to a tie): there
    the three oracle builds agree on every run to 1e-14 (measured on the CPU; with obstacles on the paths, as
    in the paper field's (4, 2) / (6, 6), the builds themselves agree on only 56-79 % of the runs at 1e-9 --
    the chaotic regime of test_receding_fused_vs_generic).  Asserted: exits identical and every recorded run
    within 1e-9 on >= 99 % of the runs, fused vs generic and both vs the oracle."""
    from diff_tube_mpc_strict_pt.core import nominal_receding
    from diff_tube_mpc_strict_pt.core.receding import receding_setup_from_config
    from _common import config
    from oracle.oracle import Oracle

    cfg = json.loads(json.dumps(config()))
    ring = [(8.0, 2.5), (2.5, 8.0), (9.5, 4.5), (4.5, 9.5), (6.5, 1.5), (1.5, 6.5), (9.0, 7.5), (7.5, 9.0)]
    cfg["environment"]["obstacles"] = [{"center": list(c), "radius": 0.8} for c in ring[:m]]
    cfg["dbas"]["gamma"], cfg["dbas"]["alpha"] = gamma, alpha
    problem, cost, icfg = receding_setup_from_config(cfg)
    assert len(problem.obstacles) == m
    B, H, N = 256, 10, problem.horizon
    rng = np.random.default_rng(11)
    x0 = np.stack([rng.uniform(0, 1, B), rng.uniform(0, 1, B), rng.uniform(0, np.pi / 2, B)], 1)
    runs = []
    for fast in ("1", "1", "0"):
        monkey = pytest.MonkeyPatch()
        monkey.setenv("DTMPC_FAST", fast)
        r = nominal_receding(problem=problem, cost=cost, cfg=icfg, x0=torch.as_tensor(x0, device=dev), H=H, check=False)
        torch.cuda.synchronize()
        monkey.undo()
        runs.append((torch.cat([r.x, r.u, r.b[..., None]], -1).cpu().numpy(), r.h_ran.cpu().numpy(),
                     r.success_t.cpu().numpy(), r.collided.cpu().numpy().astype(np.int32), r.status.cpu().numpy()))
    for k in range(5):  # the fused driver twice: bitwise
        assert np.array_equal(runs[0][k], runs[1][k], equal_nan=True), k
    del runs[1]
    U = np.zeros((B, N, 2))
    U[:, :, 0] = problem.u_max[0]
    runs.append(Oracle(np.float64, nthreads=8).nominal_receding(problem.to_c(), cost.to_c(), icfg.to_c(), x0.copy(),
                                                                H, 0.25, U)[:5])

    def pair(a, b):
        ex = (a[1] == b[1]) & (a[2] == b[2]) & (a[3] == b[3]) & (a[4] == b[4])
        mask = np.arange(H)[None, :] < a[1][:, None]
        d = np.where(mask[..., None], np.abs(a[0] - b[0]), 0).reshape(B, -1).max(1)
        sc = np.where(mask[..., None], np.abs(b[0]), 0).reshape(B, -1).max(1) + 1.0
        return float(ex.mean()), float((d[ex] / sc[ex] <= 1e-9).mean())

    res = {"fused-generic": pair(runs[0], runs[1]), "fused-oracle": pair(runs[0], runs[2]),
           "generic-oracle": pair(runs[1], runs[2])}
    print(f"[receding instantiation M={m} gamma={gamma} alpha={alpha}] (exits equal, runs within 1e-9): {res}")
    for k, (e, f) in res.items():
        assert e == 1.0 and f >= 0.99, (k, res)
