"""The fused solver's general gain records in f64 and its reference handling (round 5).

* f64, smooth-min, gamma = 0.3 (core/barrier.py:75-108: b' = B(h') - gamma (B(h) - b)), M in {4, 8}: the
  instantiations that ended trajectories non-finite in round 4 (tube_fast_kernel<M, P, 0>).
  TubeMPC, ilqr_solve and nominal_receding each against the three oracle builds at 1e-9 (f64: every trajectory
  within max(1e-9, 10 x the builds' own spread) on >= 99 %), on the ring field of tests/test_gpu_instantiations.py
  (obstacles of radius 0.8 off the diagonal the starts move along, where the builds agree to ~1e-14), at each lane
  form of the tube step and the iLQR.  With gamma != 0 TubeMPC's fused kernel runs the general records -- the
  product configuration the round-4 xfail said was unreachable.
* Tracking iLQR with caller references that are NOT a rollout of each other: the f32 line
  search re-rolls its reference states from U_ref only when they are the device's own rollout (Solve::rroll);
  ilqr_solve must price the candidates against the X_ref it was given, as the oracle does.
* The receding driver with an unwrapped target cost: the fused receding kernel compiles
  the wrapped heading error in, so wrap_angle = 0 runs the generic kernel -- the plans must match the oracle's
  unwrapped run, and differ from the wrapped one where the heading error passes pi.
Needs an MI355X: -m gpu."""
from __future__ import annotations

import json

import numpy as np
import pytest
import torch

from _common import agreement, config, decision_agreement, oracles

pytestmark = pytest.mark.gpu

RING = [(8.0, 2.5), (2.5, 8.0), (9.5, 4.5), (4.5, 9.5), (6.5, 1.5), (1.5, 6.5), (9.0, 7.5), (7.5, 9.0)]


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


def _cfg(m, gamma=0.3, alpha=0.05):
    cfg = json.loads(json.dumps(config()))
    cfg["environment"]["obstacles"] = [{"center": list(c), "radius": 0.8} for c in RING[:m]]
    cfg["dbas"]["gamma"], cfg["dbas"]["alpha"] = gamma, alpha
    return cfg


def _gamma_setup(m, gamma=0.3, alpha=0.05):
    """The paper setup on the ring field with a DBaS of gamma != 0 (paper_setup_from_config fixes alpha = gamma =
    0, core/tube_mpc.py:666-768; a TubeMPC built on this setup runs the fused kernel's general records)."""
    import dataclasses

    from diff_tube_mpc_strict_pt.core.problem import paper_setup_from_config

    st = paper_setup_from_config(_cfg(m))
    return dataclasses.replace(st, problem=dataclasses.replace(st.problem, dbas_gamma=gamma, dbas_alpha=alpha))


def _starts(B, seed=21):
    rng = np.random.default_rng(seed)
    return np.stack([rng.uniform(0, 1, B), rng.uniform(0, 1, B), rng.uniform(0, np.pi / 2, B)], 1)


def _tube_cfg(st, seed):
    from diff_tube_mpc_strict_pt import _abi

    tcfg = _abi.DtmpcTubeCfg()
    tcfg.nominal, tcfg.nom_ilqr, tcfg.aux_ilqr = st.nominal_cost.to_c(), st.ilqr_nom.to_c(), st.ilqr_aux.to_c()
    tcfg.disturbance, tcfg.seed = 1, seed
    for f in range(3):
        tcfg.w_low[f], tcfg.w_high[f] = st.w_low[f], st.w_high[f]
    return tcfg


@pytest.mark.parametrize("lanes", ["4", "2", "1"])
@pytest.mark.parametrize("m", [4, 8])
def test_tube_step_f64_gamma_vs_oracle(dev, oracle_lib, m, lanes, monkeypatch):
    """Two closed-loop steps of TubeMPC (f64, gamma = 0.3, alpha = 0.05: the fused kernel's general records at
    one, two and four lanes -- four lanes ran the generic f64 kernel in round 5 v2 until the store-data hazard was
    found)
    from the device's own pre-step state, against the oracle's one-step map; status all 0, x / xbar / b, both plans
    and the per-trajectory DOC gradient rows within the f64 band."""
    monkeypatch.setenv("DTMPC_TUBE_LANES", lanes)
    monkeypatch.setenv("DTMPC_FAST", "1")
    from diff_tube_mpc_strict_pt.core import TubeMPC

    st = _gamma_setup(m)
    assert st.problem.dbas_gamma == 0.3 and len(st.problem.obstacles) == m
    B = 384
    mpc = TubeMPC(st, batch=B, device=dev, dtype=torch.float64, disturbance="philox", seed=4, write_log=True)
    mpc.reset(torch.as_tensor(_starts(B), device=dev))
    ors = oracles(np.float64)
    names = ("x", "b", "xbar", "bbar", "Xnom", "Unom", "Xaux", "Uaux")
    for t in range(2):
        pre = {k: getattr(mpc, k).cpu().numpy().copy() for k in names}
        th0 = mpc.theta.cpu().numpy()
        mpc.step()
        torch.cuda.synchronize()
        assert (mpc.status.cpu().numpy() == 0).all(), (t, np.flatnonzero(mpc.status.cpu().numpy())[:10])
        outs = []
        for o in ors:
            state = {k: v.copy() for k, v in pre.items()}
            gout, _, so, _ = o.tube_step(st.problem.to_c(), _tube_cfg(st, 4), state, th0, step=t)
            assert (so == 0).all()
            outs.append((state, gout))
        for k in ("x", "xbar", "b"):
            d = getattr(mpc, k).cpu().numpy()
            d = d.T if d.ndim == 2 else d[:, None]
            ref = [o_[0][k].T if o_[0][k].ndim == 2 else o_[0][k][:, None] for o_ in outs]
            frac, e, _ = agreement(d, ref, 1e-9)
            assert frac >= 0.99, (t, k, frac, np.sort(e)[-5:])
        for k in ("Unom", "Uaux", "Xaux"):
            d = np.transpose(getattr(mpc, k).cpu().numpy(), (2, 0, 1))
            frac, e, _ = agreement(d, [np.transpose(o_[0][k], (2, 0, 1)) for o_ in outs], 1e-9)
            assert frac >= 0.99, (t, k, frac, np.sort(e)[-5:])
        frac, e, _ = agreement(mpc.log.cpu().numpy()[11:18].T, [o_[1].T for o_ in outs], 1e-9)
        print(f"[tube f64 gamma=0.3 M={m} lanes={lanes} step {t}] gradient rows within band: {frac:.4f}")
        assert frac >= 0.99, (t, "grad", frac, np.sort(e)[-5:])


@pytest.mark.parametrize("lanes", [4, 2, 1])
@pytest.mark.parametrize("m", [4, 8])
def test_ilqr_f64_gamma_vs_oracle(dev, oracle_lib, m, lanes):
    """ilqr_solve (f64, gamma = 0.3: ilqr_fast_kernel<M, P, TRACK, 0>), nominal from a constant warm start and a
    tracking solve of the oracle's nominal plans, against the three oracle builds (X, V, gains; decisions)."""
    from diff_tube_mpc_strict_pt.core import ilqr_solve, tracking_cost
    from diff_tube_mpc_strict_pt.core.ddp import dbas_init
    from diff_tube_mpc_strict_pt.core.problem import ILQRConfig

    st = _gamma_setup(m)
    B, N = 400, st.problem.horizon
    x3 = _starts(B, 5)
    b0 = dbas_init(st.problem, torch.as_tensor(x3, device=dev)).cpu().numpy()
    x0 = np.concatenate([x3, b0[:, None]], 1)
    V0 = np.zeros((B, N, 2))
    V0[:, :, 0] = 2.0
    ic = ILQRConfig(horizon=N, max_iter=10, tol=-1.0, line_search_alphas=st.ilqr_nom.line_search_alphas)
    ors = oracles(np.float64)
    sp = st.problem.to_c()
    r = ilqr_solve(problem=st.problem, cost=st.nominal_cost, cfg=ic, x0=torch.as_tensor(x0, device=dev),
                   V_init=torch.as_tensor(V0, device=dev), check=False, record_choices=True, lanes=lanes)
    outs = [o.ilqr_solve(sp, st.nominal_cost.to_c(), ic.to_c(), x0, V0, choices=True) for o in ors]
    assert (r.status.cpu().numpy() == 0).all() and all((o[5] == 0).all() for o in outs)
    for name, dv, k in (("X", r.X, 0), ("V", r.V, 1), ("K", r.K, 2)):
        frac, e, _ = agreement(dv.cpu().numpy().reshape(B, -1), [o[k].reshape(B, -1) for o in outs], 1e-9)
        assert frac >= 0.99, (name, frac, np.sort(e)[-5:])
    dec = decision_agreement(r.choices.cpu().numpy(), [o[6] for o in outs], label=f"ilqr f64 gamma M={m} l{lanes}")
    assert dec["on_determinate"] >= 0.99, dec
    Xp, Vp = outs[0][0], outs[0][1]
    cost = tracking_cost((0.7, 1.3, 0.2, 0.5, 2.0, 0.8))
    xa = x0.copy()
    xa[:, :2] += 0.02
    Va0 = np.roll(Vp, -1, axis=1)
    ic2 = ILQRConfig(horizon=N, max_iter=20, tol=-1.0, line_search_alphas=st.ilqr_aux.line_search_alphas)
    r = ilqr_solve(problem=st.problem, cost=cost, cfg=ic2, x0=torch.as_tensor(xa, device=dev),
                   V_init=torch.as_tensor(Va0, device=dev), X_ref=torch.as_tensor(Xp[:, :, :3].copy(), device=dev),
                   U_ref=torch.as_tensor(Vp, device=dev), check=False, lanes=lanes)
    outs = [o.ilqr_solve(sp, cost.to_c(), ic2.to_c(), xa, Va0, Xp[:, :, :3].copy(), Vp) for o in ors]
    assert (r.status.cpu().numpy() == 0).all()
    frac, e, _ = agreement(r.X.cpu().numpy().reshape(B, -1), [o[0].reshape(B, -1) for o in outs], 1e-9)
    print(f"[ilqr f64 gamma=0.3 M={m} lanes={lanes}] tracking X within band: {frac:.4f}")
    assert frac >= 0.99, ("tracking", frac, np.sort(e)[-5:])


@pytest.mark.parametrize("m", [4, 8])
def test_receding_f64_gamma_vs_oracle(dev, oracle_lib, m):
    """nominal_receding (f64, gamma = 0.3, alpha = 0.05: receding_fast_kernel<M, 0>) against the oracle: exits
    identical and every recorded run within 1e-9; the fused driver twice bitwise equal (the round-4 M = 8 defect
    was run-to-run)."""
    from diff_tube_mpc_strict_pt.core import nominal_receding
    from diff_tube_mpc_strict_pt.core.receding import receding_setup_from_config
    from oracle.oracle import Oracle

    problem, cost, icfg = receding_setup_from_config(_cfg(m))
    B, H, N = 256, 10, problem.horizon
    x0 = _starts(B, 11)
    runs = []
    for _ in range(2):
        r = nominal_receding(problem=problem, cost=cost, cfg=icfg, x0=torch.as_tensor(x0, device=dev), H=H, check=False)
        torch.cuda.synchronize()
        runs.append((torch.cat([r.x, r.u, r.b[..., None]], -1).cpu().numpy(), r.h_ran.cpu().numpy(),
                     r.success_t.cpu().numpy(), r.collided.cpu().numpy().astype(np.int32), r.status.cpu().numpy()))
    for k in range(5):
        assert np.array_equal(runs[0][k], runs[1][k], equal_nan=True), k
    U = np.zeros((B, N, 2))
    U[:, :, 0] = problem.u_max[0]
    ref = Oracle(np.float64, nthreads=8).nominal_receding(problem.to_c(), cost.to_c(), icfg.to_c(), x0.copy(), H, 0.25, U)
    a = runs[0]
    ex = (a[1] == ref[1]) & (a[2] == ref[2]) & (a[3] == ref[3]) & (a[4] == ref[4])
    mask = np.arange(H)[None, :] < a[1][:, None]
    d = np.where(mask[..., None], np.abs(a[0] - ref[0]), 0).reshape(B, -1).max(1)
    sc = np.where(mask[..., None], np.abs(ref[0]), 0).reshape(B, -1).max(1) + 1.0
    print(f"[receding f64 gamma=0.3 M={m}] exits equal {ex.mean():.4f}, runs within 1e-9 {(d[ex] / sc[ex] <= 1e-9).mean():.4f}")
    assert ex.mean() == 1.0 and (d[ex] / sc[ex] <= 1e-9).mean() >= 0.99


@pytest.mark.parametrize("tag", ["f32", "f64"])
@pytest.mark.parametrize("lanes", [1, 2, 4])
def test_ilqr_tracking_inconsistent_refs_vs_oracle(dev, oracle_lib, tag, lanes):
    """Tracking iLQR whose X_ref is NOT a rollout of U_ref (random perturbations of both, independently): the
    fused solver must price its candidates against the X_ref it was given (the f32 line search used to
    re-roll X_ref from U_ref).  Against the three oracle builds: f64 at 1e-9 on >= 99 %, f32 at 1e-3 on >= 97 %
    (the f32 band of the existing tracking test, tests/test_gpu_parity.py); a re-rolled reference would be off by
    the perturbation (1e-1) on every trajectory."""
    from diff_tube_mpc_strict_pt.core import ilqr_solve, tracking_cost
    from diff_tube_mpc_strict_pt.core.problem import ILQRConfig

    from _common import paper_setup

    npdt = np.float64 if tag == "f64" else np.float32
    tdt = torch.float64 if tag == "f64" else torch.float32
    st = paper_setup()
    B, N = 500, st.problem.horizon
    rng = np.random.default_rng(31)
    o64 = oracles(np.float64)[0]
    sp = st.problem.to_c()
    x3 = np.stack([rng.uniform(0, 1, B), rng.uniform(0, 1, B), rng.uniform(0, np.pi / 2, B)], 1)
    b0 = o64.barrier(sp, o64.h_eval(sp, x3[:, 0], x3[:, 1])[0])[0]
    x0 = np.concatenate([x3, b0[:, None]], 1)
    V0 = np.zeros((B, N, 2))
    V0[:, :, 0] = 2.0
    ic = ILQRConfig(horizon=N, max_iter=10, tol=-1.0, line_search_alphas=st.ilqr_nom.line_search_alphas)
    Xp, Vp = o64.ilqr_solve(sp, st.nominal_cost.to_c(), ic.to_c(), x0, V0)[:2]
    Xr = Xp[:, :, :3] + rng.normal(0, 0.1, Xp[:, :, :3].shape)  # no longer the rollout of Ur
    Ur = Vp + rng.normal(0, 0.1, Vp.shape)
    cost = tracking_cost((0.7, 1.3, 0.2, 0.5, 2.0, 0.8))
    ic2 = ILQRConfig(horizon=N, max_iter=20, tol=-1.0, line_search_alphas=st.ilqr_aux.line_search_alphas)
    xa, Va0 = x0.astype(npdt), np.roll(Vp, -1, axis=1).astype(npdt)
    Xr, Ur = Xr.astype(npdt), Ur.astype(npdt)
    r = ilqr_solve(problem=st.problem, cost=cost, cfg=ic2, x0=torch.as_tensor(xa, device=dev),
                   V_init=torch.as_tensor(Va0, device=dev), X_ref=torch.as_tensor(Xr, device=dev),
                   U_ref=torch.as_tensor(Ur, device=dev), check=False, lanes=lanes)
    outs = [o.ilqr_solve(sp, cost.to_c(), ic2.to_c(), xa, Va0, Xr, Ur) for o in oracles(npdt)]
    keep = (r.status.cpu().numpy() == 0) & (outs[0][5] == 0)
    assert keep.mean() > 0.99
    base, need = (1e-9, 0.99) if tag == "f64" else (1e-3, 0.97)
    frac, e, _ = agreement(r.X.cpu().numpy()[keep].reshape(int(keep.sum()), -1),
                           [o[0][keep].reshape(int(keep.sum()), -1) for o in outs], base)
    print(f"[ilqr {tag} lanes={lanes} inconsistent refs] X within band: {frac:.4f}")
    assert frac >= need, (frac, np.sort(e)[-5:])


@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_receding_unwrapped_cost(dev, oracle_lib, tag):
    """nominal_receding with wrap_angle = False: the generic receding kernel runs (the fused
    one compiles the wrapped cost in), its runs match the oracle's unwrapped run, and from a heading beyond pi of the
    target the two costs plan differently."""
    import dataclasses

    from diff_tube_mpc_strict_pt.core import nominal_receding
    from diff_tube_mpc_strict_pt.core.receding import receding_setup_from_config
    from oracle.oracle import Oracle

    npdt = np.float64 if tag == "f64" else np.float32
    problem, cost, icfg = receding_setup_from_config(_cfg(5, gamma=0.0, alpha=0.0))
    ucost = dataclasses.replace(cost, wrap_angle=False)
    B, H, N = 128, 6, problem.horizon
    rng = np.random.default_rng(3)
    x0 = np.stack([rng.uniform(0, 1, B), rng.uniform(0, 1, B), rng.uniform(3.5, 6.0, B)], 1).astype(npdt)
    xs = torch.as_tensor(x0, device=dev)
    ru = nominal_receding(problem=problem, cost=ucost, cfg=icfg, x0=xs, H=H, check=False)
    rw = nominal_receding(problem=problem, cost=cost, cfg=icfg, x0=xs, H=H, check=False)
    torch.cuda.synchronize()
    U = np.zeros((B, N, 2), npdt)
    U[:, :, 0] = problem.u_max[0]
    ref = Oracle(npdt, nthreads=8).nominal_receding(problem.to_c(), ucost.to_c(), icfg.to_c(), x0.copy(), H, 0.25, U)
    du = torch.cat([ru.x, ru.u, ru.b[..., None]], -1).cpu().numpy()
    ok = ru.h_ran.cpu().numpy() == ref[1]
    mask = np.arange(H)[None, :] < ref[1][:, None]
    d = np.where(mask[..., None], np.abs(du - ref[0]), 0).reshape(B, -1).max(1)
    sc = np.where(mask[..., None], np.abs(ref[0]), 0).reshape(B, -1).max(1) + 1.0
    tol = 1e-9 if tag == "f64" else 1e-3
    within = float((d[ok] / sc[ok] <= tol).mean())
    print(f"[receding {tag} unwrapped] exits equal {ok.mean():.4f}, runs within {tol:g}: {within:.4f}")
    assert ok.mean() >= 0.98 and within >= 0.95
    # the wrapped and unwrapped costs plan differently from these headings (error beyond pi)
    dw = torch.cat([rw.x, rw.u, rw.b[..., None]], -1).cpu().numpy()
    assert np.nanmax(np.abs(dw[:, 0, 3:5] - du[:, 0, 3:5])) > 1e-2
