"""HIP (gfx950) path vs the C oracle and the reference's golden vectors.  Needs an MI355X: -m gpu.

Tolerances: f64 kernels vs reference/oracle at 1e-9 relative (x 100 the reference's own
few-ulp conditioning on a case, tests/_common.tol_for); f32 kernels at 1e-3 relative on solves
(the reference's own f32-vs-f64 spread) and 1e-5 on single-step kernels.
Chaotic cases (the reference moves by > 1e-2 under a few-ulp input nudge) are checked for
status / finiteness only."""
from __future__ import annotations

import dataclasses

import numpy as np
import pytest
import torch

from _common import (CHAOTIC, agreement, decision_agreement, f64_truth, f64_truth_line, golden, ilqr_cfg, oracles,
                     paper_setup, rel, tie_aware_decisions, tol_for)

pytestmark = pytest.mark.gpu

DT = {"f64": (np.float64, torch.float64), "f32": (np.float32, torch.float32)}


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from diff_tube_mpc_strict_pt import _lib

    lib = _lib.load()
    assert lib.dtmpc_device_count() >= 1
    return torch.device("cuda:0")


def _t(a, dt, dev):
    return torch.as_tensor(np.asarray(a), dtype=dt, device=dev)


def random_batch(B, seed, dtype=np.float64, spread=1.0):
    """Starts in the safe region around the origin + random warm starts; ragged B on purpose."""
    from oracle.oracle import Oracle

    st = paper_setup()
    rng = np.random.default_rng(seed)
    x = np.stack([rng.uniform(0, 1.5 * spread, B), rng.uniform(0, 1.5 * spread, B), rng.uniform(0, np.pi / 2, B)], 1)
    o = Oracle(np.float64)
    sp = st.problem.to_c()
    b = o.barrier(sp, o.h_eval(sp, x[:, 0], x[:, 1])[0])[0]
    x0 = np.concatenate([x, b[:, None]], 1).astype(dtype)
    V0 = np.stack([rng.uniform(-1, 3, (B, st.problem.horizon)), rng.uniform(-1, 1, (B, st.problem.horizon))], 2)
    return x0, V0.astype(dtype)


# ------------------------------------------------------------------------------------ KAT level
@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_rollout_linearize_init_vs_oracle(dev, oracle_lib, tag):
    from diff_tube_mpc_strict_pt.core import dbas_init, linearize, rollout, tracking_cost

    npdt, tdt = DT[tag]
    o = oracle_lib.Oracle(npdt)
    st = paper_setup()
    x0, V = random_batch(333, 1, npdt, spread=6.0)
    Xg = rollout(st.problem, _t(x0, tdt, dev), _t(V, tdt, dev)).cpu().numpy()
    Xo = o.dbas_rollout(st.problem.to_c(), x0, V)
    tol = 1e-12 if tag == "f64" else 2e-5
    assert rel(Xg, Xo) < tol
    bg = dbas_init(st.problem, _t(x0[:, :3], tdt, dev)).cpu().numpy()
    assert rel(bg, x0[:, 3]) < tol
    for cost, ref in ((st.nominal_cost, None), (tracking_cost((0.7, 1.3, 0.2, 0.5, 2.0, 0.8)), Xo)):
        Xr = None if ref is None else ref[:, :, :3] + 0.01
        Ur = None if ref is None else V[:, ::-1, :].copy()
        outs_g = linearize(st.problem, cost, _t(Xo, tdt, dev), _t(V, tdt, dev),
                           None if Xr is None else _t(Xr, tdt, dev), None if Ur is None else _t(Ur, tdt, dev))
        outs_o = o.linearize(st.problem.to_c(), cost.to_c(), Xo, V, Xr, Ur)
        for a, b in zip(outs_g, outs_o):
            assert rel(a.cpu().numpy(), b) < (1e-12 if tag == "f64" else 1e-5)


# ------------------------------------------------------------------------------------ solvers vs golden
def _golden_tol(npdt, cond, spread):
    return max(tol_for(npdt, cond), 10.0 * spread)


@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_ilqr_nominal_vs_reference_golden(dev, oracle_lib, tag):
    from diff_tube_mpc_strict_pt.core import ilqr_solve

    npdt, tdt = DT[tag]
    g = golden(f"ilqr_{tag}")
    st = paper_setup()
    ok = [i for i in range(g["x0"].shape[0]) if np.isfinite(g["X_nom"][i]).all()]
    ors = oracles(npdt)
    for mi, tl, xk, vk, ck in ((3, -1.0, "X_nom_fixed", "V_nom_fixed", "cond_nom_fixed"),
                               (10, 1e-3, "X_nom", "V_nom", "cond_nom")):
        r = ilqr_solve(problem=st.problem, cost=st.nominal_cost, cfg=ilqr_cfg(mi, tl), x0=_t(g["x0"][ok], tdt, dev),
                       V_init=_t(g["Vinit_nom"][ok], tdt, dev))
        Xs = [o.ilqr_solve(st.problem.to_c(), st.nominal_cost.to_c(), ilqr_cfg(mi, tl).to_c(), g["x0"][ok],
                           g["Vinit_nom"][ok])[0] for o in ors]
        X, V = r.X.cpu().numpy(), r.V.cpu().numpy()
        n = 0
        for j, i in enumerate(ok):
            if g[ck][i] > CHAOTIC:
                continue
            t = _golden_tol(npdt, g[ck][i], max(rel(x[j], Xs[0][j]) for x in Xs[1:]))
            assert rel(X[j], g[xk][i]) < t, (i, xk)
            assert rel(V[j], g[vk][i]) < t, (i, vk)
            n += 1
        assert n >= 5


@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_ilqr_ancillary_sensitivity_grad_vs_reference_golden(dev, oracle_lib, tag):
    from diff_tube_mpc_strict_pt.core import ddp_sensitivity, doc_gradient, ilqr_solve, tracking_cost

    npdt, tdt = DT[tag]
    g = golden(f"ilqr_{tag}")
    st = paper_setup()
    ors = oracles(npdt)
    sp = st.problem.to_c()
    n = 0
    for i in range(g["x0"].shape[0]):
        if not np.isfinite(g["X_aux"][i]).all():
            continue
        cost = tracking_cost(g["theta"][i])
        sl = slice(i, i + 1)
        Xr, Ur = _t(g["X_nom"][sl], tdt, dev), _t(g["V_nom"][sl], tdt, dev)
        for mi, tl, xk, vk, ck in ((4, -1.0, "X_aux_fixed", "V_aux_fixed", "cond_aux_fixed"),
                                   (20, 1e-3, "X_aux", "V_aux", "cond_aux")):
            r = ilqr_solve(problem=st.problem, cost=cost, cfg=ilqr_cfg(mi, tl), x0=_t(g["x0_aux"][sl], tdt, dev),
                           V_init=_t(g["Vinit_aux"][sl], tdt, dev), X_ref=Xr, U_ref=Ur)
            if g[ck][i] > CHAOTIC:
                continue
            args = (sp, cost.to_c(), ilqr_cfg(mi, tl).to_c(), g["x0_aux"][sl], g["Vinit_aux"][sl], g["X_nom"][sl], g["V_nom"][sl])
            Xs = [o.ilqr_solve(*args)[0] for o in ors]
            t = _golden_tol(npdt, g[ck][i], max(rel(x, Xs[0]) for x in Xs[1:]))
            assert rel(r.X[0].cpu().numpy(), g[xk][i]) < t, (i, xk)
            assert rel(r.V[0].cpu().numpy(), g[vk][i]) < t, (i, vk)
        Xa, Va = _t(g["X_aux"][sl], tdt, dev), _t(g["V_aux"][sl], tdt, dev)
        s = ddp_sensitivity(problem=st.problem, cost=cost, X=Xa, V=Va, X_ref=Xr, U_ref=Ur, X_bar=Xr)
        gr = doc_gradient(Xa, Va, Xr, Ur, s.delta_X, s.delta_V)
        if g["cond_sens"][i] > CHAOTIC:
            continue
        ds = [o.ddp_sensitivity(sp, cost.to_c(), g["X_aux"][sl], g["V_aux"][sl], g["X_nom"][sl]) for o in ors]
        t = _golden_tol(npdt, g["cond_sens"][i], max(rel(d[j], ds[0][j]) for d in ds[1:] for j in range(3)))
        assert rel(s.delta_X[0].cpu().numpy(), g["dX"][i]) < t, i
        assert rel(s.delta_V[0].cpu().numpy(), g["dV"][i]) < t, i
        assert rel(s.delta_lambda[0].cpu().numpy(), g["dlam"][i]) < t, i
        assert rel(gr[0].cpu().numpy(), g["grad"][i]) < t, i
        n += 1
    assert n >= 5


# ------------------------------------------------------------------------------------ solvers vs oracle, batched
# decision-record gate (the chosen alpha of every iteration + the final active set) on the
# determinate trajectories, those on which the three oracle builds agree (tests/_common.py
# decision_agreement; near-ties of line-search costs at the working precision make the rest
# rounding-dependent in the oracle itself)
# Measured (round 3, profiles/r03/decisions.txt): f64 >= 0.99 everywhere.  In f32 the device's own rounding
# (hardware exp / log / rcp, fused multiply-adds) is none of the three builds', and the f32 line-search
# costs tie at fp32 resolution near convergence, so even where the builds agree the device's decision
# differs on a few percent of iLQR solves and on ~10 % of the 30-iteration tube steps (late iterations,
# alpha = 0.01 vs keep); the f32 gates are set below those measurements, the rates are printed.
# Round 4 added the stronger f32 gates (_f32_vs_truth: f64 truth + tie-aware decisions, >= 0.99 of trajectories);
# these raw-rate gates stay as a second, weaker check of the same decision records (a regression floor on the
# exact-match rate, whose f32 shortfall the tie-aware gate attributes to near-ties).
DECISION_GATE = {"f64": 0.99, "f32": 0.95}
DECISION_GATE_TUBE = {"f64": 0.99, "f32": 0.84}
# the 20-iteration tracking solve with the tol exit compares tiny cost decreases (warm start next to the
# reference): in f32 many iterations are near-ties that the device's summation order decides differently
# from all three oracle builds (measured 0.945 on determinate trajectories, 0.79 overall; f64 >= 0.99)
DECISION_GATE_TRACK = {"f64": 0.99, "f32": 0.92}
# the raw per-trajectory X band of that 20-iteration tracking solve, calibrated on the oracle builds themselves
# (scripts/calib_f32_truth.py ilqr, profiles/r06/calib_f32_ilqr.txt): valid f32 roundings of the same algorithm reach
# 0.954 / 0.968 / 0.973 against the other two builds and 0.991 (the symmetric-V_xx build) against all three, so f32
# is held to the lowest of them; the principled f32 gates (f64 truth, tie-aware decisions) run beside it.  Rounds 2-5
# held 0.98 there, which the round-6 deterministic Riccati rounding (0.978) and two of the three builds miss.
TRACK_X_GATE = {"f64": 0.98, "f32": 0.95}

@pytest.mark.parametrize("tag,variant", [("f64", "generic"), ("f64", "l4"), ("f64", "l2"), ("f64", "l1"),
                                         ("f32", "l4"), ("f32", "l2"), ("f32", "l1"), ("f32", "generic")])
def test_ilqr_batched_vs_oracle(dev, oracle_lib, tag, variant, monkeypatch):
    """Ragged batch (B = 1000) of random starts / warm starts; nominal cost with fixed iterations and
    with the tol exit, then a tracking solve of the oracle's nominal plans.  Each trajectory must agree
    with the oracle within max(base, 10 x the spread of the three oracle builds on that trajectory).
    Both precisions run the fused solver (dtmpc_ilqr_solve_ws; f64: csrc/dtmpc_fast64_ilqr.hip) at 4 / 2 / 1
    lanes per trajectory and the generic kernel (DTMPC_FAST=0).  The last backward pass's gains K, k are
    checked too (the same per-trajectory band)."""
    from diff_tube_mpc_strict_pt.core import ilqr_solve, tracking_cost

    lanes = {"l4": 4, "l2": 2, "l1": 1}.get(variant, 0)
    if variant == "generic":
        monkeypatch.setenv("DTMPC_FAST", "0")
    npdt, tdt = DT[tag]
    ors = oracles(npdt)
    st = paper_setup()
    sp = st.problem.to_c()
    B = 1000
    base = 1e-9 if tag == "f64" else 1e-3
    x0, V0 = random_batch(B, 5, npdt)
    fused = variant != "generic"
    truth_o = oracles(np.float64)[0] if tag == "f32" else None
    for cost, mi, tl in ((st.nominal_cost, 5, -1.0), (st.nominal_cost, 10, 1e-3)):
        r = ilqr_solve(problem=st.problem, cost=cost, cfg=ilqr_cfg(mi, tl), x0=_t(x0, tdt, dev), V_init=_t(V0, tdt, dev),
                       check=False, record_choices=True, lanes=lanes, record_costs=True)
        outs = [o.ilqr_solve(sp, cost.to_c(), ilqr_cfg(mi, tl).to_c(), x0, V0, choices=True, costs=True) for o in ors]
        if tag == "f32":
            _f32_vs_truth(r, outs, truth_o.ilqr_solve(sp, cost.to_c(), ilqr_cfg(mi, tl).to_c(), x0.astype(np.float64),
                                                      V0.astype(np.float64)), tl, fused, f"ilqr {variant} max_iter={mi} tol={tl}")
        Xp, Vp, so = outs[0][0], outs[0][1], outs[0][5]
        keep = (so == 0) & (r.status.cpu().numpy() == 0)
        assert keep.mean() > 0.995
        frac, e, s = agreement(r.X.cpu().numpy()[keep], [o[0][keep] for o in outs], base)
        # the tol exit (|J_prev - J_best| < tol) in f32: J ~ 1e3-1e4 carries ~1e-4 of rounding, so about
        # 1-4 % of the trajectories sit on the knife edge and stop one iteration earlier or later than the
        # oracle (iteration counts: measured 0.96-0.98 agreement, X 0.988 on the fused solver's summation
        # order); fixed iteration counts and f64 keep the 0.99 bar
        knife = tl > 0 and tag == "f32"
        assert frac >= (0.98 if knife else 0.99), (mi, tl, frac, np.sort(e)[-5:])
        n = int(keep.sum())
        gk = np.concatenate([r.K.cpu().numpy()[keep].reshape(n, -1), r.k.cpu().numpy()[keep].reshape(n, -1)], 1)
        gref = [np.concatenate([o[2][keep].reshape(n, -1), o[3][keep].reshape(n, -1)], 1) for o in outs]
        frac, e, s = agreement(gk, gref, base * 10)
        assert frac >= 0.97, ("gains", mi, tl, frac, np.sort(e)[-5:])
        assert (r.iters.cpu().numpy()[keep] == outs[0][4][keep]).mean() >= (0.95 if knife else 0.99)
        # decision record: winning alpha per iteration + final active set
        dec = decision_agreement(r.choices.cpu().numpy()[keep], [o[6][keep] for o in outs], r.V.cpu().numpy()[keep],
                                 [o[1][keep] for o in outs], label=f"ilqr {tag} max_iter={mi} tol={tl}")
        assert dec["on_determinate"] >= DECISION_GATE[tag], dec
    cost = tracking_cost((0.7, 1.3, 0.2, 0.5, 2.0, 0.8))
    xa = x0.copy()
    xa[:, :2] += 0.02
    Va0 = np.roll(Vp, -1, axis=1)
    r = ilqr_solve(problem=st.problem, cost=cost, cfg=ilqr_cfg(20, 1e-3), x0=_t(xa, tdt, dev), V_init=_t(Va0, tdt, dev),
                   X_ref=_t(Xp, tdt, dev), U_ref=_t(Vp, tdt, dev), check=False, record_choices=True, lanes=lanes,
                   record_costs=True)
    args = (sp, cost.to_c(), ilqr_cfg(20, 1e-3).to_c(), xa, Va0, Xp, Vp)
    outs = [o.ilqr_solve(*args, choices=True, costs=True) for o in ors]
    if tag == "f32":
        a64 = tuple(a.astype(np.float64) if isinstance(a, np.ndarray) else a for a in args)
        _f32_vs_truth(r, outs, truth_o.ilqr_solve(*a64), 1e-3, fused, f"ilqr {variant} tracking")
    keep = (outs[0][5] == 0) & (r.status.cpu().numpy() == 0)
    assert keep.mean() > 0.99
    frac, e, s = agreement(r.X.cpu().numpy()[keep], [o[0][keep] for o in outs], base)
    assert frac >= TRACK_X_GATE[tag], (frac, np.sort(e)[-5:])
    dec = decision_agreement(r.choices.cpu().numpy()[keep], [o[6][keep] for o in outs], r.V.cpu().numpy()[keep],
                             [o[1][keep] for o in outs], label=f"ilqr {tag} tracking")
    assert dec["on_determinate"] >= DECISION_GATE_TRACK[tag], dec


# f32 against f64 truth: the device's f32 solution must be as close to the f64 oracle (the
# reference's configured precision) as a valid f32 evaluation is -- no more often the worst than the builds are
# among themselves, quantiles within 2 x the builds', the §8c 1e-3 share within 3 points of the lowest build's
# (tests/_common.f64_truth; the per-trajectory "1.5 x the worst build on 99 %" fails for the builds themselves,
# scripts/calib_f32_truth.py) -- and its line-search decisions must equal a build's or split from it only at a
# near-tie (tests/_common.tie_aware_decisions), on >= 99 % (the builds among themselves: 0.996-0.999) -- or, where
# the builds themselves split from each other by more than ties (the 20-iteration tracking solve from perturbed
# starts: chaotic from the first iteration), on >= the builds' own pass rate under the same rule - 2 points.
F32_TRUTH_GATE = 1.0
TIE_GATE = 0.99


def _f32_vs_truth(r, outs, truth, tol, fused, label):
    keep = (outs[0][5] == 0) & (r.status.cpu().numpy() == 0) & (truth[5] == 0)
    for name, dv, k in (("X", r.X, 0), ("U", r.V, 1)):
        res = f64_truth(dv.cpu().numpy()[keep], [o[k][keep] for o in outs], truth[k][keep])
        print(f"[f32 vs f64 truth {label}] {name}: " + f64_truth_line(res))
        assert res["frac_ok"] >= F32_TRUTH_GATE, (label, name, f64_truth_line(res), res["bad"][:8])
    if fused:  # the candidate-cost record is written by the fused solver
        tie = tie_aware_decisions(r.choices.cpu().numpy()[keep], r.costs.cpu().numpy()[keep],
                                  [o[6][keep] for o in outs], [o[7][keep] for o in outs], tol=tol, label=label)
        assert tie["frac_ok"] >= min(TIE_GATE, min(tie["builds_rate"]) - 0.02), (label, tie["frac_ok"], tie["fail"][:8])


@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_sensitivity_batched_vs_oracle(dev, oracle_lib, tag):
    from diff_tube_mpc_strict_pt.core import ddp_sensitivity, doc_gradient, tracking_cost

    npdt, tdt = DT[tag]
    ors = oracles(npdt)
    st = paper_setup()
    sp = st.problem.to_c()
    B = 513
    x0, V0 = random_batch(B, 9, npdt)
    cost = tracking_cost((1.0, 0.8, 1.2, 0.6, 1.1, 0.9))
    op = ors[0]
    Xn, Vn, _, _, _, _ = op.ilqr_solve(sp, st.nominal_cost.to_c(), ilqr_cfg(4, -1.0).to_c(), x0, V0)
    xa = x0.copy()
    xa[:, 1] -= 0.03
    Xa, Va, _, _, _, _ = op.ilqr_solve(sp, cost.to_c(), ilqr_cfg(6, -1.0).to_c(), xa, np.roll(Vn, -1, 1), Xn, Vn)
    res = [o.ddp_sensitivity(sp, cost.to_c(), Xa, Va, Xn) for o in ors]
    grads = [o.doc_grad(Xa, Va, Xn, Vn, r_[0], r_[1]) for o, r_ in zip(ors, res)]
    keep = np.all(np.isfinite(res[0][0]), axis=(1, 2))
    s = ddp_sensitivity(problem=st.problem, cost=cost, X=_t(Xa, tdt, dev), V=_t(Va, tdt, dev), X_ref=_t(Xn, tdt, dev),
                        U_ref=_t(Vn, tdt, dev), X_bar=_t(Xn, tdt, dev), check=False)
    gg = doc_gradient(_t(Xa, tdt, dev), _t(Va, tdt, dev), _t(Xn, tdt, dev), _t(Vn, tdt, dev), s.delta_X, s.delta_V)
    base = 1e-9 if tag == "f64" else 1e-4
    for a, outs in ((s.delta_X, [r_[0] for r_ in res]), (s.delta_V, [r_[1] for r_ in res]),
                    (s.delta_lambda, [r_[2] for r_ in res]), (gg, grads)):
        frac, e, sp_ = agreement(a.cpu().numpy()[keep], [o[keep] for o in outs], base)
        assert frac >= (0.99 if tag == "f64" else 0.98), (frac, np.sort(e)[-5:])


# ------------------------------------------------------------------------------------ problem variants
def _variant(name):
    """SURVEY §8f-4 problem variants (core/systems/dubins_obstacles.py:16-117, core/barrier.py:36-108,
    run_nominal.py:297-324) plus an obstacle field larger than the kernels' compile-time fast path."""
    from diff_tube_mpc_strict_pt.core.problem import CircleObstacle, QuadraticCost

    st = paper_setup()
    p, c = st.problem, st.nominal_cost
    if name == "min_alpha_gamma":
        p = dataclasses.replace(p, obs_aggregation="min", dbas_alpha=0.05, dbas_gamma=0.3)
    elif name == "log_barrier":
        p = dataclasses.replace(p, barrier_type="log", dbas_gamma=-0.5)
    elif name == "smoothmin_11_obstacles":
        extra = tuple(CircleObstacle((o.center[0] + 1.7, o.center[1] - 1.1), 0.6) for o in p.obstacles)
        p = dataclasses.replace(p, obstacles=p.obstacles + extra + (CircleObstacle((-2.0, 3.0), 0.8),))
    elif name == "single":
        p = dataclasses.replace(p, obs_aggregation="single")
    elif name == "no_obstacles":
        p = dataclasses.replace(p, obs_aggregation="none", obstacles=())
    elif name == "wrap_angle_cost":
        c = QuadraticCost(kind="target", Q=(1.0, 1.0, 0.5), R=(0.1, 0.1), Qf=(50.0, 50.0, 5.0), qb=1.0,
                          target=(4.0, 4.0, 3.0), wrap_angle=True)
    return p, c



@pytest.mark.parametrize("name", ["min_alpha_gamma", "log_barrier", "smoothmin_11_obstacles", "single",
                                  "no_obstacles", "wrap_angle_cost"])
def test_problem_variants_vs_oracle(dev, oracle_lib, name):
    """f64 device path on each variant: rollout + linearisation (1e-12), a 4-iteration iLQR and its DDP
    sensitivity (per trajectory within 10x the spread of the three oracle builds plus oracle reruns on
    inputs nudged by 1e-13, base 1e-9, on >= 99 %).  Starts are in free space (h > 0.5): starts inside
    an obstacle put b ~ 1e12 and costs ~ 1e24 into the line search, where candidates tie at rounding
    level.  The nudged reruns measure each trajectory's own chaos (log barrier + random warm starts:
    ~40 % of trajectories move by > 1e-6 under a 1e-13 nudge)."""
    from diff_tube_mpc_strict_pt.core import ddp_sensitivity, ilqr_solve, linearize, rollout

    p, c = _variant(name)
    sp = p.to_c()
    ors = oracles(np.float64)
    o = ors[0]
    B = 384
    rng = np.random.default_rng(17)
    x = np.stack([rng.uniform(-1, 5, B), rng.uniform(-1, 5, B), rng.uniform(-np.pi, np.pi, B)], 1)
    b = o.barrier(sp, o.h_eval(sp, x[:, 0], x[:, 1])[0])[0]
    x0 = np.concatenate([x, b[:, None]], 1)
    V0 = np.stack([rng.uniform(-1, 3, (B, p.horizon)), rng.uniform(-1, 1, (B, p.horizon))], 2)
    fin = np.isfinite(x0).all(1) & (o.h_eval(sp, x[:, 0], x[:, 1])[0] > 0.5)
    x0, V0 = x0[fin], V0[fin]
    assert len(x0) >= 150
    Xo = o.dbas_rollout(sp, x0, V0)
    assert rel(rollout(p, _t(x0, torch.float64, dev), _t(V0, torch.float64, dev)).cpu().numpy(), Xo) < 1e-12
    for a_, b_ in zip(linearize(p, c, _t(Xo, torch.float64, dev), _t(V0, torch.float64, dev)),
                      o.linearize(sp, c.to_c(), Xo, V0)):
        assert rel(a_.cpu().numpy(), b_) < 1e-12
    cfg = ilqr_cfg(4, -1.0)
    r = ilqr_solve(problem=p, cost=c, cfg=cfg, x0=_t(x0, torch.float64, dev), V_init=_t(V0, torch.float64, dev),
                   check=False)
    outs = [o_.ilqr_solve(sp, c.to_c(), cfg.to_c(), x0, V0) for o_ in ors]
    for xs, vs in ((x0 * (1 + 1e-13), V0), (x0 * (1 - 1e-13), V0), (x0, V0 * (1 + 1e-13))):
        outs.append(o.ilqr_solve(sp, c.to_c(), cfg.to_c(), xs, vs))
    keep = (outs[0][5] == 0) & (r.status.cpu().numpy() == 0)
    assert keep.mean() > 0.98
    # log barrier: B = -log(max(h, eps)) is flat inside an obstacle while the reference's augmented
    # Jacobian keeps the relaxed-inverse slope there (core/systems/dubins_aug_jac.py:31-40); with random
    # warm starts ~45 % of these trajectories move under a 1e-13 nudge and a few % sit beyond every
    # nudged rerun.  Its dynamics / Jacobians are held to 1e-12 above.
    need = 0.95 if name == "log_barrier" else 0.99
    frac, e, _ = agreement(r.X.cpu().numpy()[keep], [o_[0][keep] for o_ in outs], 1e-9)
    assert frac >= need, (name, frac, np.sort(e)[-5:])
    Xa, Va = outs[0][0][keep], outs[0][1][keep]
    Xbar = Xa[:, :, :3] + 0.05
    s = ddp_sensitivity(problem=p, cost=c, X=_t(Xa, torch.float64, dev), V=_t(Va, torch.float64, dev), X_ref=None,
                        U_ref=None, X_bar=_t(Xbar, torch.float64, dev), check=False)
    res = [o_.ddp_sensitivity(sp, c.to_c(), Xa, Va, Xbar) for o_ in ors]
    for xs, vs in ((Xa * (1 + 1e-13), Va), (Xa * (1 - 1e-13), Va), (Xa, Va * (1 + 1e-13))):
        res.append(o.ddp_sensitivity(sp, c.to_c(), xs, vs, Xbar))
    ok = np.all(np.isfinite(res[0][0]), axis=(1, 2))
    for got, k in ((s.delta_X, 0), (s.delta_V, 1), (s.delta_lambda, 2)):
        frac, e, _ = agreement(got.cpu().numpy()[ok], [r_[k][ok] for r_ in res], 1e-9)
        assert frac >= need, (name, k, frac, np.sort(e)[-5:])


# ------------------------------------------------------------------------------------ fused closed loop
def _oracle_state(x0, N, dt):
    B = x0.shape[0]
    xs = x0[:, :3].T.astype(dt).copy()
    return {"x": xs, "b": x0[:, 3].astype(dt).copy(), "xbar": xs.copy(), "bbar": x0[:, 3].astype(dt).copy(),
            "Xnom": np.zeros((N + 1, 4, B), dt), "Unom": np.zeros((N, 2, B), dt),
            "Xaux": np.zeros((N + 1, 4, B), dt), "Uaux": np.zeros((N, 2, B), dt)}


def _oracle_tube(o, st, x0b, steps, B, seed):
    from diff_tube_mpc_strict_pt import _abi

    tcfg = _abi.DtmpcTubeCfg()
    tcfg.nominal, tcfg.nom_ilqr, tcfg.aux_ilqr = st.nominal_cost.to_c(), st.ilqr_nom.to_c(), st.ilqr_aux.to_c()
    tcfg.disturbance, tcfg.seed = 1, seed
    for f in range(3):
        tcfg.w_low[f], tcfg.w_high[f] = st.w_low[f], st.w_high[f]
    state = _oracle_state(x0b, st.problem.horizon, o.dt)
    theta = np.array(st.theta0, o.dt)
    vel = np.zeros(6, o.dt)
    xs, ths, sts = [], [], []
    status = np.zeros(B, np.int32)
    for t in range(steps):
        gout, _, so, _ = o.tube_step(st.problem.to_c(), tcfg, state, theta, step=t)
        status |= so
        sums = np.zeros(8, o.dt)
        sums[:7] = gout.sum(1)
        theta, vel = o.theta_update(st.adapt.to_c(), 1.0 / B, sums, theta, vel)
        xs.append(state["x"].T.copy())
        ths.append(theta.copy())
        sts.append(status.copy())
    return xs, ths, sts


@pytest.mark.parametrize("lanes", ["4", "2", "1"])
@pytest.mark.parametrize("mode", ["paper", "bench"])
@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_tube_step_vs_oracle(dev, oracle_lib, tag, mode, lanes, monkeypatch):
    """Fused Algorithm-2 step (device Philox disturbances) on the bench workload's start distribution
    (x0 ~ U[0,1]^2 x U[0, pi/2], zero warm starts), ragged batch, 3 closed-loop steps: per-trajectory
    plant / nominal states, warm starts and the shared theta, against the three oracle builds.
    lanes (DTMPC_TUBE_LANES): "4" (this batch size's own form: one line-search pair per lane, candidate
    tapes kept instead of a commit, the backward's per-point linearisation split over the lanes), "2"
    (paired line search) and "1" (the one-lane kernel of the large batches).  The three forms run the same
    operations; they differ only in where the compiler fuses the backward pass's multiply-adds (a build
    without implicit contraction gives bitwise-identical results at 1, 2 and 4 lanes), so each is held to
    the oracle band on its own.
    mode paper: tol = 1e-3 early exit (core/tube_mpc.py:757-768); bench: fixed iterations (tol = -1).
    In f32 the paper's absolute tol test sits at fp32 resolution of the cost, so
    iteration counts flip on a few % of trajectories there; the bench mode has no such decision."""
    monkeypatch.setenv("DTMPC_TUBE_LANES", lanes)
    import dataclasses

    from diff_tube_mpc_strict_pt.core import TubeMPC

    npdt, tdt = DT[tag]
    st = paper_setup()
    if mode == "bench":
        st = dataclasses.replace(st, ilqr_nom=dataclasses.replace(st.ilqr_nom, tol=-1.0),
                                 ilqr_aux=dataclasses.replace(st.ilqr_aux, tol=-1.0))
    # f32: line-search candidates' costs tie at fp32 resolution near convergence (alpha = 0.01 vs 0), so
    # which one wins is rounding-dependent.  Measured on this batch: the three CPU oracle builds already
    # differ by > 1e-4 (up to 0.34) in U on 16-23 % of trajectories after ONE step; the device must agree
    # within 10x that spread on 95 % (f64: 99 %, base 1e-9).
    need = 0.99 if tag == "f64" else 0.95
    B = 700
    rng = np.random.default_rng(11)
    x = np.stack([rng.uniform(0, 1, B), rng.uniform(0, 1, B), rng.uniform(0, np.pi / 2, B)], 1).astype(npdt)
    mpc = TubeMPC(st, batch=B, device=dev, dtype=tdt, disturbance="philox", seed=3, write_log=True,
                  record_choices=True, record_costs=True)
    mpc.reset(_t(x, tdt, dev))
    ors = oracles(npdt)
    truth_o = oracles(np.float64)[0] if tag == "f32" else None
    base = 1e-9 if tag == "f64" else 1e-4
    names = ("x", "b", "xbar", "bbar", "Xnom", "Unom", "Xaux", "Uaux")
    for t in range(3):
        # the oracle's one-step map from the device's exact pre-step state (theta is a batch mean, so
        # comparing free-running loops would compound differences from the first step on)
        pre = {k: getattr(mpc, k).cpu().numpy().copy() for k in names}
        th0, vel0 = mpc.theta.cpu().numpy(), mpc.vel.cpu().numpy()
        mpc.step()
        torch.cuda.synchronize()
        outs = []
        for o in ors:
            state = {k: v.copy() for k, v in pre.items()}
            gout, _, so, _, ch, cc = o.tube_step(st.problem.to_c(), _tube_cfg(st, 3), state, th0, step=t,
                                                 choices=True, costs=True)
            sums = np.zeros(8, npdt)
            sums[:7] = gout.sum(1)
            theta, _ = o.theta_update(st.adapt.to_c(), 1.0 / B, sums, th0, vel0)
            outs.append((state, theta, so, gout, ch, cc))
        keep = (mpc.status.cpu().numpy() == 0) & (outs[0][2] == 0)
        assert keep.mean() > 0.99
        if tag == "f32":  # against f64 truth from the same pre-step state
            tstate = {k: v.astype(np.float64) for k, v in pre.items()}
            tg, _, tso, _ = truth_o.tube_step(st.problem.to_c(), _tube_cfg(st, 3), tstate, th0.astype(np.float64), step=t)
            kt = keep & (tso == 0)
            lab = f"tube {mode} lanes={lanes} step {t}"
            for k in ("x", "Unom", "Uaux", "grad"):
                if k == "grad":
                    dv, bo, tr = mpc.log.cpu().numpy()[11:18].T, [o_[3].T for o_ in outs], tg.T
                elif k == "x":
                    dv, bo, tr = mpc.x.cpu().numpy().T, [o_[0]["x"].T for o_ in outs], tstate["x"].T
                else:
                    f = lambda a: np.transpose(a, (2, 0, 1))  # noqa: E731
                    dv, bo, tr = f(getattr(mpc, k).cpu().numpy()), [f(o_[0][k]) for o_ in outs], f(tstate[k])
                res = f64_truth(dv[kt], [b_[kt] for b_ in bo], tr[kt])
                print(f"[f32 vs f64 truth {lab}] {k}: " + f64_truth_line(res))
                assert res["frac_ok"] >= F32_TRUTH_GATE, (lab, k, f64_truth_line(res), res["bad"][:8])
            tie = tie_aware_decisions(mpc.choices.cpu().numpy().T[keep],
                                      np.transpose(mpc.costs.cpu().numpy(), (2, 0, 1))[keep],
                                      [o_[4].T[keep] for o_ in outs], [o_[5][keep] for o_ in outs],
                                      tol=st.ilqr_nom.tol, label=lab, starts=(0, st.ilqr_nom.max_iter))
            assert tie["frac_ok"] >= min(TIE_GATE, min(tie["builds_rate"]) - 0.02), (lab, tie["frac_ok"], tie["fail"][:8])
        # decision record: the nominal then ancillary winning alphas of every iteration and
        # the final ancillary active set, against the oracle builds from the same pre-step state
        # (active sets of the ancillary plans as the step leaves them: shifted warm starts on both sides)
        dch = mpc.choices.cpu().numpy().T[keep]
        dU = np.transpose(mpc.Uaux.cpu().numpy(), (2, 0, 1))[keep]
        dec = decision_agreement(dch, [o_[4].T[keep] for o_ in outs], dU,
                                 [np.transpose(o_[0]["Uaux"], (2, 0, 1))[keep] for o_ in outs],
                                 label=f"tube {tag} {mode} lanes={lanes} step {t}")
        assert dec["on_determinate"] >= DECISION_GATE_TUBE[tag], dec
        for k in ("x", "xbar", "b"):
            dev_k = getattr(mpc, k).cpu().numpy()
            dev_k = dev_k.T if dev_k.ndim == 2 else dev_k[:, None]
            ref = [(o_[0][k].T if o_[0][k].ndim == 2 else o_[0][k][:, None])[keep] for o_ in outs]
            frac, e, s = agreement(dev_k[keep], ref, base)
            assert frac >= need, (t, k, frac, np.sort(e)[-5:])
        for k in ("Uaux", "Unom"):
            dev_k = np.transpose(getattr(mpc, k).cpu().numpy(), (2, 0, 1))[keep]
            frac, e, s = agreement(dev_k, [np.transpose(o_[0][k], (2, 0, 1))[keep] for o_ in outs], base)
            assert frac >= need, (t, k, frac, np.sort(e)[-5:])
        # per-trajectory DOC loss + gradient rows [L, gQ(3), gR(2), gqb] (log rows 11..17)
        log = mpc.log.cpu().numpy()
        frac, e, s = agreement(log[11:18].T[keep], [o_[3].T[keep] for o_ in outs], base)
        assert frac >= need, (t, "grad", frac, np.sort(e)[-5:])
        # shared theta: momentum + projection applied to the device's own batch sums.  (Comparing it
        # with the oracle's theta instead would be a lottery: the batch mean is dominated by the few
        # obstacle-grazing trajectories whose gradients are chaotic -- the three CPU builds' thetas
        # already differ by up to 3e4 relative on this batch.)
        healthy = mpc.status.cpu().numpy() == 0
        gb = mpc.cfg.grad_bound  # the health policy's bound on the gradient components (f32 default)
        if gb > 0:
            healthy &= (np.abs(log[12:18]) <= gb).all(0)
        g = np.where(healthy, log[11:18], 0).astype(np.float64)
        sums = np.zeros(8)
        sums[:7] = g.sum(1)
        sums[7] = healthy.sum()
        assert int(round(float(mpc.sums[7]))) == int(healthy.sum())  # the device's healthy count
        # inv_batch 0: the mean over the healthy trajectories, as TubeMPC.step asks the device for
        th_ref, _ = ors[0].theta_update(st.adapt.to_c(), 0.0, sums.astype(npdt), th0, vel0)
        th = mpc.theta.cpu().numpy()
        eta = st.adapt.lr_eta
        scale = np.abs(th0) + eta * (np.abs(vel0) + np.abs(g).sum(1)[1:] / B) + 1e-30
        tol_th = 1e-12 if tag == "f64" else 1e-5
        assert (np.abs(th - th_ref) <= tol_th * scale).all(), (t, th, th_ref)


def _tube_cfg(st, seed):
    from diff_tube_mpc_strict_pt import _abi

    tcfg = _abi.DtmpcTubeCfg()
    tcfg.nominal, tcfg.nom_ilqr, tcfg.aux_ilqr = st.nominal_cost.to_c(), st.ilqr_nom.to_c(), st.ilqr_aux.to_c()
    tcfg.disturbance, tcfg.seed = 1, seed
    for f in range(3):
        tcfg.w_low[f], tcfg.w_high[f] = st.w_low[f], st.w_high[f]
    return tcfg


def test_philox_disturbance_matches_oracle(dev, oracle_lib):
    """Device Philox stream == oracle stream, keyed by global index (sharding invariance)."""
    from diff_tube_mpc_strict_pt.core import TubeMPC

    st = paper_setup()
    B = 300
    x0, _ = random_batch(B, 2)
    full = TubeMPC(st, batch=B, device=dev, dtype=torch.float64, disturbance="philox", seed=11)
    full.reset(_t(x0[:, :3], torch.float64, dev))
    full.step()
    halves = []
    for lo, hi in ((0, 137), (137, B)):
        m = TubeMPC(st, batch=hi - lo, device=dev, dtype=torch.float64, disturbance="philox", seed=11,
                    global_offset=lo, global_batch=B)
        m.reset(_t(x0[lo:hi, :3], torch.float64, dev))
        m.step()
        halves.append(m.x.cpu().numpy())
    torch.cuda.synchronize()
    assert np.array_equal(np.concatenate(halves, 1), full.x.cpu().numpy())
    # the stream itself (bit-exact with the oracle) is exercised by test_tube_step_vs_oracle
    bits = oracle_lib.philox_bits(11, 5, 0)
    w = -0.05 + 0.1 * ((bits[:3] >> 8) * (1.0 / 16777216.0))
    assert np.all(np.abs(w) <= 0.05)


def test_closed_loop_vs_reference_loop_f64(dev):
    """TubeMPC(B=1) driven with the golden disturbances reproduces the reference's own paper-mode loop."""
    from diff_tube_mpc_strict_pt.core import TubeMPC

    g = golden("closed_loop_f64")
    st = paper_setup()
    mpc = TubeMPC(st, batch=1, device=dev, dtype=torch.float64, disturbance="injected", write_log=True)
    mpc.reset(torch.tensor([[0.0, 0.0, np.pi / 4]], dtype=torch.float64))
    logs, th = [], []
    for t in range(g["loss"].shape[0]):
        mpc.step(_t(g["w"][t:t + 1], torch.float64, dev))
        logs.append(mpc.log[:, 0].cpu().numpy())
        th.append(mpc.theta.cpu().numpy())
    mpc.check()
    logs, th = np.array(logs), np.array(th)
    t = 1e-8
    assert rel(logs[:, 0:3], g["x_real"]) < t
    assert rel(logs[:, 3:5], g["u_real"]) < t
    assert rel(logs[:, 5:8], g["x_bar"]) < t
    assert rel(logs[:, 8:10], g["u_bar"]) < t
    assert rel(logs[:, 10], g["b_real"]) < t
    assert rel(logs[:, 11], g["loss"]) < t
    assert rel(th[:, 0:3], g["Qa_history"]) < t
    assert rel(th[:, 3:5], g["Ra_history"]) < t
    assert rel(th[:, 5], g["qba_history"]) < t


def test_closed_loop_vs_reference_loop_f32_health_policy(dev):
    """TubeMPC(B=1) in f32 with the default health policy (grad_bound 1e6) reproduces the reference's own
    f32 paper-mode loop: the bound never triggers there, so every theta update is the reference's
    (core/tube_mpc.py:978-984) exactly as computed from the trajectory's gradient."""
    from diff_tube_mpc_strict_pt.core import TubeMPC

    g = golden("closed_loop_f32")
    st = paper_setup()
    mpc = TubeMPC(st, batch=1, device=dev, dtype=torch.float32, disturbance="injected", write_log=True)
    assert mpc.cfg.grad_bound == 1e6
    mpc.reset(torch.tensor([[0.0, 0.0, np.pi / 4]], dtype=torch.float32))
    logs, th = [], []
    for t in range(g["loss"].shape[0]):
        mpc.step(_t(g["w"][t:t + 1], torch.float32, dev))
        assert mpc.healthy_count == 1
        logs.append(mpc.log[:, 0].cpu().numpy())
        th.append(mpc.theta.cpu().numpy())
    logs, th = np.array(logs), np.array(th)
    t = 5e-4  # the oracle's f32 tolerance against the same fixture (tests/test_oracle_golden.py)
    assert rel(logs[:, 0:3], g["x_real"]) < t
    assert rel(logs[:, 11], g["loss"]) < t
    assert rel(th[:, 0:3], g["Qa_history"]) < t
    assert rel(th[:, 3:5], g["Ra_history"]) < t
    assert rel(th[:, 5], g["qba_history"]) < t


def test_free_running_loop_f32_theta_bounded(dev, monkeypatch):
    """The steady-state workload of bench.py: B = 65,536 f32, fixed iterations, 20 free-running closed-loop
    steps (warm-started, theta updated every step under the f32 health policy) keep theta finite and
    bounded and nearly every trajectory healthy (measured: 98.4-99.9 % per step; the rest are flagged or
    obstacle-grazing outliers the health policy drops), and the loop's theta stays as close to the f64 loop's as
    the other valid evaluations do (scripts/theta_loop.py)."""
    import dataclasses

    from diff_tube_mpc_strict_pt.core import TubeMPC

    st = paper_setup()
    st = dataclasses.replace(st, ilqr_nom=dataclasses.replace(st.ilqr_nom, tol=-1.0),
                             ilqr_aux=dataclasses.replace(st.ilqr_aux, tol=-1.0))
    B = 65536
    g = torch.Generator().manual_seed(0)
    u = torch.rand(B, 3, generator=g, dtype=torch.float64)
    x0 = torch.stack([u[:, 0], u[:, 1], u[:, 2] * (np.pi / 2)], 1).float()
    m = TubeMPC(st, batch=B, device=dev, dtype=torch.float32, disturbance="philox", seed=0)
    m.reset(x0)
    thetas, healthy = [], []
    for _ in range(20):
        m.step()
        thetas.append(m.theta.double().cpu().numpy())
        healthy.append(m.healthy_count / B)
    thetas = np.array(thetas)
    # the same loop in f64 (the reference's configured precision) under the same health policy, on the fused
    # f64 kernel and on the generic one (DTMPC_FAST64=0: a second f64 rounding of the same algorithm).  The
    # shared theta is a batch mean dominated by the few obstacle-grazing trajectories' large gradients, so
    # after a few steps it is as sensitive to rounding as they are: the f32 loop must track f64 as closely
    # as the two f64 evaluations track each other
    def loop64(fast):
        monkeypatch.setenv("DTMPC_FAST64", fast)
        m64 = TubeMPC(st, batch=B, device=dev, dtype=torch.float64, disturbance="philox", seed=0,
                      grad_bound=m.cfg.grad_bound)
        m64.reset(x0.double())
        out = []
        for _ in range(20):
            m64.step()
            out.append(m64.theta.cpu().numpy())
        return np.array(out)

    th64, th64g = loop64("1"), loop64("0")
    monkeypatch.delenv("DTMPC_FAST64")
    # and a second f32 rounding of the same loop: the generic f32 kernel (DTMPC_FAST=0)
    monkeypatch.setenv("DTMPC_FAST", "0")
    mg = TubeMPC(st, batch=B, device=dev, dtype=torch.float32, disturbance="philox", seed=0)
    mg.reset(x0)
    th32g = []
    for _ in range(20):
        mg.step()
        th32g.append(mg.theta.double().cpu().numpy())
    monkeypatch.delenv("DTMPC_FAST")
    th32g = np.array(th32g)
    rel_d = lambda a, b: (np.abs(a - b) / np.maximum(np.abs(b), 1e-3)).max(1)  # noqa: E731
    d32, d64, d32g = rel_d(thetas, th64), rel_d(th64g, th64), rel_d(th32g, th64)
    print(f"[free-running f32 B={B}] theta after 20 steps {thetas[-1].round(4).tolist()} (f64 loop "
          f"{th64[-1].round(4).tolist()}, generic f64 {th64g[-1].round(4).tolist()}, generic f32 "
          f"{th32g[-1].round(4).tolist()}), max |theta| {np.abs(thetas).max():.4g}, healthy fraction min "
          f"{min(healthy):.5f}; relative theta distance from the f64 loop per step: f32 {[float(f'{v:.2g}') for v in d32]}, "
          f"generic f32 {[float(f'{v:.2g}') for v in d32g]}, generic f64 {[float(f'{v:.2g}') for v in d64]}")
    assert np.isfinite(thetas).all() and np.abs(thetas).max() < 1e2, thetas.max(0)
    assert min(healthy) > 0.97, healthy
    assert d32[0] <= 1e-3, d32  # one step: the batch-mean update of the same theta0
    # later steps: the loop is chaotic (a theta component meets its projection bound in one evaluation and not in
    # another, and the relative distance spikes by 1e2-1e3 for a step or two -- in the generic f32 loop as well,
    # profiles/r06/theta_loop.txt), so the step at which a spike comes is not a property of the arithmetic.  The f32
    # loop is held to the other valid evaluations' envelope instead: at its worst and at its end no further from the
    # f64 loop than 10 x the farther of the generic f64 and the generic f32 loops (or 1e-2)
    other = np.maximum(d64, d32g)
    assert d32.max() <= max(10.0 * other.max(), 1e-2), (d32, d64, d32g)
    assert d32[-1] <= max(10.0 * other[-1], 1e-2), (d32, d64, d32g)


def test_run_closed_loop_experiment_outputs(dev, tmp_path):
    import os

    from diff_tube_mpc_strict_pt.core import run_closed_loop_experiment
    from diff_tube_mpc_strict_pt.core.problem import paper_config

    cfg = paper_config()
    cfg["system"]["task_horizon_H"] = 4
    torch.manual_seed(0)
    res = run_closed_loop_experiment(cfg, device=dev, run_dir=str(tmp_path))
    for name in ("x_real", "u_real", "x_bar", "u_bar", "b_real", "loss", "Qa_history", "Ra_history", "qba_history"):
        a = np.load(os.path.join(tmp_path, name + ".npy"))
        assert a.shape[0] == 4 and np.isfinite(a).all()
    assert set(res["summary"]) == {"system", "H", "N", "final_state", "final_barrier_state", "final_loss", "note"}
    assert abs(np.load(os.path.join(tmp_path, "loss.npy"))[0] - 14.4392417) < 1e-6  # loss(t=0), SURVEY.md §6


# ------------------------------------------------------------------------------------ full-size properties
@pytest.mark.parametrize("B", [65536, 8192])
def test_full_batch_properties(dev, B):
    """B = 65,536 (the bench size, one lane per trajectory) and 8,192 (one GPU's shard of it at 8-way,
    four lanes), f32, fixed iterations: all trajectories finite and OK; the fused step is deterministic
    (bitwise); each iLQR never ends above its warm-start cost (the alpha = 0 candidate, core/ddp.py:293)."""
    import dataclasses

    from diff_tube_mpc_strict_pt.core import TubeMPC, ilqr_solve

    st = paper_setup()
    st = dataclasses.replace(st, ilqr_nom=dataclasses.replace(st.ilqr_nom, tol=-1.0),
                             ilqr_aux=dataclasses.replace(st.ilqr_aux, tol=-1.0))
    g = torch.Generator().manual_seed(0)
    u = torch.rand(B, 3, generator=g, dtype=torch.float64)
    x0 = torch.stack([u[:, 0], u[:, 1], u[:, 2] * (np.pi / 2)], 1).float()
    runs = []
    for _ in range(2):
        m = TubeMPC(st, batch=B, device=dev, dtype=torch.float32, disturbance="philox", seed=0)
        m.reset(x0)
        m.step()
        m.step()
        torch.cuda.synchronize()
        runs.append((m.x.clone(), m.Xaux.clone(), m.theta.clone(), m.status.clone()))
    # f32 overflows on trajectories driven deep into an obstacle's relaxed barrier (the reference's own
    # f32 path raises FloatingPointError there): they must be rare, flagged, and everything else finite
    ok = runs[0][3] == 0
    assert int((~ok).sum()) <= B // 1000
    assert torch.isfinite(runs[0][1][:, :, ok]).all() and torch.isfinite(runs[0][2]).all()
    for a, b in zip(runs[0], runs[1]):
        assert torch.equal(a, b)
    # cost never increases: J(X*, V*) <= J(rollout(V_init)) for every trajectory
    x0h = torch.cat([x0, torch.zeros(B, 1)], 1).to(dev)
    from diff_tube_mpc_strict_pt.core import dbas_init, rollout

    x0h[:, 3] = dbas_init(st.problem, x0h[:, :3])
    V0 = torch.zeros(B, st.problem.horizon, 2, device=dev)
    V0[:, :, 0] = 2.0
    r = ilqr_solve(problem=st.problem, cost=st.nominal_cost, cfg=ilqr_cfg(10, -1.0), x0=x0h, V_init=V0)

    def J(X, V):
        c = st.nominal_cost
        X, V = X.double(), V.double()
        tq = torch.tensor(c.target, dtype=torch.float64, device=dev)
        d = X[:, :-1, :3] - tq
        Q = torch.tensor(c.Q, dtype=torch.float64, device=dev)
        R = torch.tensor(c.R, dtype=torch.float64, device=dev)
        Qf = torch.tensor(c.Qf, dtype=torch.float64, device=dev)
        dN = X[:, -1, :3] - tq
        return ((Q * d * d).sum((1, 2)) + (R * V * V).sum((1, 2)) + c.qb * (X[:, :-1, 3] ** 2).sum(1)
                + (Qf * dN * dN).sum(1) + c.qb * X[:, -1, 3] ** 2)

    J0 = J(rollout(st.problem, x0h, V0), V0)
    J1 = J(r.X, r.V)
    assert bool((J1 <= J0 * (1 + 1e-5) + 1e-3).all())


@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_tube_reset_fused_matches_stepwise(dev, tag):
    """dtmpc_tube_reset (the episode start in one launch) writes exactly what the step-by-step reset
    does (copies, dtmpc_dbas_init, zero warm starts, theta0, zero momentum and status), from a dirty
    state."""
    from diff_tube_mpc_strict_pt.core import TubeMPC

    npdt, tdt = DT[tag]
    st = paper_setup()
    B = 333
    rng = np.random.default_rng(2)
    x = np.stack([rng.uniform(0, 1, B), rng.uniform(0, 1, B), rng.uniform(0, np.pi / 2, B)], 1).astype(npdt)
    N = st.problem.horizon
    names = ("x", "b", "xbar", "bbar", "Unom", "Uaux", "theta", "vel", "status")
    outs = []
    for fused in (True, False):
        m = TubeMPC(st, batch=B, device=dev, dtype=tdt, disturbance="philox", seed=1)
        m.reset(_t(x, tdt, dev))
        m.step()
        m.status.fill_(3)
        m.vel.fill_(1.0)
        if fused:
            m.reset(_t(x, tdt, dev))
        else:
            z = torch.zeros(B, N, 2, dtype=tdt, device=dev)
            m.reset(_t(x, tdt, dev), U_nom0=z, U_aux0=z)
        torch.cuda.synchronize()
        outs.append({k: getattr(m, k).clone() for k in names})
    for k in names:
        assert torch.equal(outs[0][k], outs[1][k]), k


@pytest.mark.parametrize("tag", ["f32", "f64"])
@pytest.mark.parametrize("lanes", ["1", "2", "4"])
def test_tube_step_fast_chunked_bitwise(dev, lanes, tag, monkeypatch):
    """The f32 fast kernel keeps its per-lane records in one buffer resource (< 2^31 bytes), so a batch
    whose records exceed that runs in chunks of trajectories (dtmpc_fast.hip tube_fast_chunk).  Forcing
    chunks of 256 (DTMPC_FAST_CHUNK) on a ragged batch of 700 = 256 + 256 + 188 must give bitwise the
    single-launch results: states, tapes, log rows, partial sums and the shared theta."""
    import dataclasses

    from diff_tube_mpc_strict_pt.core import TubeMPC

    monkeypatch.setenv("DTMPC_TUBE_LANES", lanes)
    st = paper_setup()
    st = dataclasses.replace(st, ilqr_nom=dataclasses.replace(st.ilqr_nom, tol=-1.0),
                             ilqr_aux=dataclasses.replace(st.ilqr_aux, tol=-1.0))
    B = 700
    npdt, tdt = DT[tag]  # f64: the same kernel source instantiated in f64 (csrc/dtmpc_fast64.hip)
    rng = np.random.default_rng(5)
    x = np.stack([rng.uniform(0, 1, B), rng.uniform(0, 1, B), rng.uniform(0, np.pi / 2, B)], 1).astype(npdt)
    names = ("x", "b", "xbar", "bbar", "Xnom", "Unom", "Xaux", "Uaux", "theta", "status", "log", "partials")
    runs = []
    for chunk in (None, "256"):
        if chunk:
            monkeypatch.setenv("DTMPC_FAST_CHUNK", chunk)
        m = TubeMPC(st, batch=B, device=dev, dtype=tdt, disturbance="philox", seed=4, write_log=True)
        m.reset(_t(x, tdt, dev))
        m.step()
        m.step()
        torch.cuda.synchronize()
        runs.append({k: getattr(m, k).clone() for k in names if getattr(m, k, None) is not None})
    assert (runs[0]["status"] == 0).all()
    for k in runs[0]:
        assert torch.equal(runs[0][k], runs[1][k]), k


@pytest.mark.parametrize("tag", ["f32", "f64"])
@pytest.mark.parametrize("lanes", ["1", "2", "4"])
def test_tube_step_fast_gamma0_records(dev, lanes, tag, monkeypatch):
    """gamma = 0 (the paper's DBaS) makes the column of K for the barrier state exactly zero, and the
    fast kernel then keeps K and k in one 32-byte record per step (dtmpc_fast.hip fk::Gains).  The
    general 40-byte records (DTMPC_FAST_G0=0) must give the same values -- an exact zero term dropped
    from the feedback sum changes nothing but, at most, the sign of a zero -- over two closed-loop
    steps: states, tapes, log rows, partial sums and the shared theta.  DTMPC_FAST_G0=1 is the compact
    records with the general Riccati step; the default at gamma = 0 also drops the barrier state's zero
    column from the recursion (riccati_pk<true>, an FMA rounding of it), which test_tube_step_vs_oracle
    checks against the oracle builds.  (Round 5 v2 ran the f64 general records at four lanes on the generic
    kernel and skipped that case; the store-data hazard fix put them back on the fused kernel)"""
    import dataclasses

    from diff_tube_mpc_strict_pt.core import TubeMPC

    monkeypatch.setenv("DTMPC_TUBE_LANES", lanes)
    st = paper_setup()
    assert st.problem.dbas_gamma == 0.0
    st = dataclasses.replace(st, ilqr_nom=dataclasses.replace(st.ilqr_nom, tol=-1.0),
                             ilqr_aux=dataclasses.replace(st.ilqr_aux, tol=-1.0))
    B = 700
    npdt, tdt = DT[tag]
    rng = np.random.default_rng(6)
    x = np.stack([rng.uniform(0, 1, B), rng.uniform(0, 1, B), rng.uniform(0, np.pi / 2, B)], 1).astype(npdt)
    names = ("x", "b", "xbar", "bbar", "Xnom", "Unom", "Xaux", "Uaux", "theta", "status", "log", "partials")
    runs = []
    for g0 in ("1", "0"):
        monkeypatch.setenv("DTMPC_FAST_G0", g0)
        m = TubeMPC(st, batch=B, device=dev, dtype=tdt, disturbance="philox", seed=4, write_log=True)
        m.reset(_t(x, tdt, dev))
        m.step()
        m.step()
        torch.cuda.synchronize()
        runs.append({k: getattr(m, k).clone() for k in names if getattr(m, k, None) is not None})
    assert (runs[0]["status"] == 0).all()
    for k in runs[0]:
        assert torch.equal(runs[0][k], runs[1][k]), k


@pytest.mark.parametrize("lanes", ["1", "2", "4"])
def test_tube_step_fast64_vs_generic(dev, lanes, monkeypatch):
    """The f64 instantiation of the fused kernel (csrc/dtmpc_fast64.hip) against the generic f64 kernel
    (DTMPC_FAST64=0, tube_step_kernel<double>) from the same start, one closed-loop step at the paper
    settings: the same algorithm in two roundings (FMA contraction in the backward pass, the fdlibm sin/cos
    kernels against OCML's), so states, plans and log rows agree to 1e-8 relative to each trajectory's
    largest entry on >= 99 % of trajectories (the chaotic obstacle-grazing ones aside, test_tube_step_vs_oracle's band).  One step:
    the next one runs on the batch-mean theta, which the few chaotic trajectories' gradients dominate."""
    from diff_tube_mpc_strict_pt.core import TubeMPC

    monkeypatch.setenv("DTMPC_TUBE_LANES", lanes)
    st = paper_setup()
    B = 700
    rng = np.random.default_rng(21)
    x = np.stack([rng.uniform(0, 1, B), rng.uniform(0, 1, B), rng.uniform(0, np.pi / 2, B)], 1)
    names = ("x", "b", "xbar", "bbar", "Xnom", "Unom", "Xaux", "Uaux", "log")
    runs = []
    for fast in ("1", "0"):
        monkeypatch.setenv("DTMPC_FAST64", fast)
        m = TubeMPC(st, batch=B, device=dev, dtype=torch.float64, disturbance="philox", seed=5, write_log=True)
        m.reset(_t(x, torch.float64, dev))
        m.step()
        torch.cuda.synchronize()
        assert (m.status == 0).all()
        runs.append({k: getattr(m, k).cpu().numpy() for k in names})
    for k in names:
        a, b = runs[0][k], runs[1][k]
        a = a.reshape(-1, B) if a.ndim > 1 else a[None]
        b = b.reshape(-1, B) if b.ndim > 1 else b[None]
        e = np.abs(a - b).max(0) / (np.abs(b).max(0) + 1e-30)
        frac = float((e <= 1e-8).mean())
        print(f"[fast64 vs generic lanes={lanes}] {k}: {frac:.4f} within 1e-8, max {e.max():.3g}")
        assert frac >= 0.99, (k, frac, np.sort(e)[-5:])


@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_status_and_errors(dev, tag):
    """Non-finite inputs raise FloatingPointError (core/ddp.py:138-159); bad arguments ValueError."""
    import dataclasses

    from diff_tube_mpc_strict_pt.core import ilqr_solve

    npdt, tdt = DT[tag]
    st = paper_setup()
    x0, V0 = random_batch(5, 3, npdt)
    x0[2, 0] = np.nan
    with pytest.raises(FloatingPointError):
        ilqr_solve(problem=st.problem, cost=st.nominal_cost, cfg=ilqr_cfg(2, -1.0), x0=_t(x0, tdt, dev),
                   V_init=_t(V0, tdt, dev))
    r = ilqr_solve(problem=st.problem, cost=st.nominal_cost, cfg=ilqr_cfg(2, -1.0), x0=_t(x0, tdt, dev),
                   V_init=_t(V0, tdt, dev), check=False)
    s = r.status.cpu().numpy()
    assert s[2] & 1 and (np.delete(s, 2) == 0).all()
    with pytest.raises(ValueError):
        ilqr_solve(problem=st.problem, cost=st.nominal_cost,
                   cfg=dataclasses.replace(ilqr_cfg(2, -1.0), line_search_alphas=tuple([1.0] * 9)),
                   x0=_t(x0, tdt, dev), V_init=_t(V0, tdt, dev))
