"""GENERAL IFT path on the HIP device (core/tube_mpc.py:40-663) vs the reference's golden vectors
and the C oracle.  Needs an MI355X: -m gpu.

Tolerances (stated per test): f64 against the reference at 1e-8 relative on states / plans and
1e-7 relative + 1e-9 absolute on gradients (closed forms vs autograd differ only by rounding;
entries that are analytically 0 come out as +-1e-30 noise in the reference); f32 through the
oracle-build agreement of tests/_common.agreement."""
from __future__ import annotations

import dataclasses
import json

import numpy as np
import pytest
import torch

from _common import agreement, config, golden, oracles, rel

pytestmark = pytest.mark.gpu

DT = {"f64": (np.float64, torch.float64), "f32": (np.float32, torch.float32)}
SL = {"Q": slice(0, 3), "R": slice(3, 5), "Qf": slice(5, 8), "qb": slice(8, 9), "alpha": slice(9, 10),
      "gamma": slice(10, 11), "tight": slice(11, 12)}
AUX = ("Q", "R", "Qf", "qb", "alpha", "gamma")
NOM = AUX + ("tight",)


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from diff_tube_mpc_strict_pt import _lib

    assert _lib.load().dtmpc_device_count() >= 1
    return torch.device("cuda:0")


def _t(a, dt, dev):
    return torch.as_tensor(np.asarray(a), dtype=dt, device=dev)


def close(a, b, rtol, atol):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return bool(np.all(np.abs(a - b) <= atol + rtol * np.abs(b)))


def general_cfg(**over):
    cfg = json.loads(json.dumps(config()))
    cfg["paper_dubins_mode"] = False
    cfg["adaptation"]["adapt_nominal"] = True
    for k, v in over.items():
        sec, key = k.split("__")
        cfg[sec][key] = v
    return cfg


@pytest.mark.parametrize("tag", ["A_f64", "B_f64", "C_f64"])
def test_general_closed_loop_vs_reference(dev, tag):
    """GeneralTubeMPC(B = 1) driven by the golden disturbances reproduces the reference's general loop:
    plant / nominal states, plans, loss, and the raw theta / theta-bar after every update."""
    from diff_tube_mpc_strict_pt.core import GeneralTubeMPC
    from diff_tube_mpc_strict_pt.core.problem import general_setup_from_config

    g = golden(f"general_{tag}")
    cfg = json.loads(str(g["config"]))
    st = general_setup_from_config(cfg)
    mpc = GeneralTubeMPC(st, batch=1, device=dev, dtype=torch.float64, disturbance="injected", write_log=True)
    mpc.reset(torch.tensor([list(st.x0)], dtype=torch.float64))
    H = g["loss"].shape[0]
    an = bool(cfg["adaptation"]["adapt_nominal"])
    for t in range(H):
        th_before = mpc.theta.cpu().numpy()
        for nm in AUX:
            assert close(th_before[0][SL[nm]], g[f"theta_aux_{nm}"][t], 1e-10, 1e-13), (t, nm)
        if an:
            for nm in NOM:
                assert close(th_before[1][SL[nm]], g[f"theta_nom_{nm}"][t], 1e-10, 1e-13), (t, nm)
        mpc.step(_t(g["w"][t:t + 1], torch.float64, dev))
        torch.cuda.synchronize()
        assert rel(mpc.Xnom[:, :, 0].cpu().numpy(), g["nom_X"][t]) < 1e-8, t
        assert rel(mpc.Xaux[:, :, 0].cpu().numpy(), g["aux_X"][t]) < 1e-8, t
        gout = mpc.gout[:, 0].cpu().numpy()
        for nm in AUX:
            ref = np.ravel(g[f"gaux_{nm}"][t])
            got = gout[1:12][SL[nm]]
            if np.isnan(ref).all():  # None in the reference (alpha unused under the log barrier)
                assert np.all(got == 0)
                continue
            assert close(got, ref, 1e-7, 1e-9), (t, nm, got, ref)
        if an:
            for nm in NOM:
                assert close(gout[12:24][SL[nm]], np.ravel(g[f"gnom_{nm}"][t]), 1e-7, 1e-9), (t, nm)
        lg = mpc.log[:, 0].cpu().numpy()
        assert rel(lg[0:3], g["x_real"][t]) < 1e-12
        assert rel(lg[3:5], g["u_real"][t]) < 1e-8
        assert rel(lg[5:8], g["x_bar"][t]) < 1e-12
        assert rel(lg[8:10], g["u_bar"][t]) < 1e-8
        assert close(lg[10], g["b_real"][t], 1e-10, 0)
        assert close(lg[11], g["loss"][t], 1e-10, 0)
        Qa = torch.nn.functional.softplus(mpc.theta[0, 0:3]).cpu().numpy()
        assert close(Qa, g["Qa_history"][t], 1e-10, 1e-13)
    mpc.check()
    th = mpc.theta.cpu().numpy()
    for nm in AUX:
        assert close(th[0][SL[nm]], g[f"theta_aux_final_{nm}"], 1e-9, 1e-12), nm
    if an:
        for nm in NOM:
            assert close(th[1][SL[nm]], g[f"theta_nom_final_{nm}"], 1e-9, 1e-12), nm


@pytest.mark.parametrize("tag,solver,gamma", [("f64", "generic", 0.3), ("f64", "fast", 0.3), ("f64", "fast", 0.0),
                                               ("f32", "fast", 0.3), ("f32", "generic", 0.3), ("f32", "fast", 0.0)])
def test_general_step_batched_vs_oracle(dev, oracle_lib, tag, solver, gamma, monkeypatch):
    """Batched general step (B = 300, ragged) from starts spread over the obstacle field (relaxed
    barrier, alpha / gamma / tightening gradients exercised), non-trivial raw parameters, 2 steps:
    per-trajectory plans, the 24 gradient rows, the shared theta update (applied to the device's own
    batch sums) and the plant step, against the three oracle builds from the device's pre-step state.
    Both precisions run both solvers: the fused one (general_solve_fast_kernel: gamma != 0 gain records, the
    tightened nominal barrier; f64: csrc/dtmpc_fast64_general.hip) and the generic kernel (DTMPC_FAST=0); raw
    gamma 0 (tanh 0 = 0 exactly) runs the fused solver's gamma = 0 records in both solves."""
    from diff_tube_mpc_strict_pt.core import GeneralTubeMPC
    from diff_tube_mpc_strict_pt.core.problem import general_setup_from_config

    if solver == "generic":
        monkeypatch.setenv("DTMPC_FAST", "0")
    npdt, tdt = DT[tag]
    cfg = general_cfg(dbas__gamma=gamma, dbas__alpha=-1.0, dbas__nominal_tightening=-0.5,
                      adaptation__grad_clip_norm=2.0)
    st = general_setup_from_config(cfg)
    B = 300
    rng = np.random.default_rng(5)
    x = np.stack([rng.uniform(0, 9, B), rng.uniform(0, 9, B), rng.uniform(-np.pi, np.pi, B)], 1).astype(npdt)
    mpc = GeneralTubeMPC(st, batch=B, device=dev, dtype=tdt, disturbance="philox", seed=9, write_log=True)
    mpc.reset(_t(x, tdt, dev))
    ors = oracles(npdt)
    need = 0.99 if tag == "f64" else 0.93
    base = 1e-9 if tag == "f64" else 1e-4
    names = ("x", "b", "xbar", "bbar", "Xnom", "Unom", "Xaux", "Uaux")
    sp, gc = st.problem.to_c(), st.to_c(disturbance=1, seed=9)
    for t in range(2):
        pre = {k: getattr(mpc, k).cpu().numpy().copy() for k in names}
        th0, vel0 = mpc.theta.cpu().numpy(), mpc.vel.cpu().numpy()
        mpc.step()
        torch.cuda.synchronize()
        outs = []
        for o in ors:
            state = {k: v.copy() for k, v in pre.items()}
            gout, so, _ = o.general_step(sp, gc, state, th0)
            outs.append((state, gout, so))
        keep = (mpc.status.cpu().numpy() == 0) & (outs[0][2] == 0)
        assert keep.mean() > 0.9, keep.mean()
        for k in ("Xnom", "Xaux"):
            dk = np.transpose(getattr(mpc, k).cpu().numpy(), (2, 0, 1))[keep]
            frac, e, _ = agreement(dk, [np.transpose(o_[0][k], (2, 0, 1))[keep] for o_ in outs], base)
            assert frac >= need, (t, k, frac, np.sort(e)[-5:])
        gdev = mpc.gout.cpu().numpy()
        frac, e, _ = agreement(gdev.T[keep], [o_[1].T[keep] for o_ in outs], base)
        assert frac >= need, (t, "gout", frac, np.sort(e)[-5:])
        # theta update on the device's own (masked) batch sums
        sums = gdev.astype(np.float64).sum(1).astype(npdt)
        assert sums[-1] == (mpc.status.cpu().numpy() == 0).sum()  # healthy count (last gout row)
        # inv_batch 0: the mean over the healthy trajectories, as GeneralTubeMPC.step asks for
        th_ref, vel_ref = ors[0].general_update(sp, gc, 0.0, sums, th0, vel0)
        th = mpc.theta.cpu().numpy()
        tol = 1e-10 if tag == "f64" else 2e-5
        assert np.allclose(th, th_ref, rtol=tol, atol=tol * 0.05 * (np.abs(vel_ref) + 1)), (t, th - th_ref)
        # plant step with the updated theta from the device's pre-step plant state and plans
        # (the device plans are shifted by now: the step's first controls come from the log)
        lg = mpc.log.cpu().numpy()
        u_aux0 = lg[3:5]
        u_nom0 = lg[8:10]
        st2 = {k: pre[k].copy() for k in ("x", "b", "xbar", "bbar")}
        N = st.problem.horizon
        st2["Unom"] = np.zeros((N, 2, B), npdt)
        st2["Uaux"] = np.zeros((N, 2, B), npdt)
        st2["Unom"][0] = u_nom0
        st2["Uaux"][0] = u_aux0
        ors[0].general_plant(sp, gc, st2, th, gdev[0], step=t)
        for k in ("x", "xbar", "b", "bbar"):
            a = getattr(mpc, k).cpu().numpy()
            assert rel(a, st2[k]) < (1e-12 if tag == "f64" else 1e-5), (t, k)


def test_ift_gradient_device_vs_reference_kats(dev):
    """dtmpc_ift_gradient (f64) on the reference's ift_gradient KATs (tapes in / near the obstacles,
    relaxed branch, log barrier), both closure sets."""
    from diff_tube_mpc_strict_pt.core import IFTInputs, QuadraticCost, ift_gradient
    from diff_tube_mpc_strict_pt.core.problem import general_setup_from_config

    k = golden("ift_general_f64")
    base = general_setup_from_config(general_cfg())
    n, N = k["X"].shape[0], k["X"].shape[1] - 1
    T = torch.float64
    for c in range(n):
        prob = dataclasses.replace(base.problem, horizon=N, barrier_type="log" if int(k["btype"][c]) else "inverse")
        inp = IFTInputs(X=_t(k["X"][c:c + 1], T, dev), V=_t(k["V"][c:c + 1], T, dev),
                        delta_X=_t(k["dX"][c:c + 1], T, dev), delta_V=_t(k["dV"][c:c + 1], T, dev),
                        delta_lambda=_t(k["dlam"][c:c + 1], T, dev))
        ga = ift_gradient(inputs=inp, problem=prob, cost=QuadraticCost(kind="track"),
                          theta_raw=np.concatenate([k["raw_aux"][c], [0.0]]), X_ref=_t(k["Xref"][c:c + 1], T, dev),
                          U_ref=_t(k["Uref"][c:c + 1], T, dev))
        ref = k["g_aux"][c]
        assert close(ga.theta[0, :11].cpu().numpy(), ref[:11], 1e-9, 1e-10), c
        assert close(ga.X_ref[0].cpu().numpy().reshape(-1), ref[11:11 + 3 * (N + 1)], 1e-12, 1e-13), c
        assert close(ga.U_ref[0].cpu().numpy().reshape(-1), ref[11 + 3 * (N + 1):], 1e-12, 1e-13), c
        gn = ift_gradient(inputs=inp, problem=prob, cost=QuadraticCost(kind="target", target=base.target),
                          theta_raw=k["raw_nom"][c])
        assert close(gn.theta[0].cpu().numpy(), k["g_nom"][c], 1e-9, 1e-10), c


@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_sensitivity_upper_vs_oracle(dev, oracle_lib, tag):
    """ddp_sensitivity with array upper gradients (the nominal solve's form, g_u != 0) vs the oracle,
    on the reference's own ancillary optima, with random upper gradients."""
    from diff_tube_mpc_strict_pt.core import ddp_sensitivity, paper_setup_from_config, tracking_cost

    npdt, tdt = DT[tag]
    g = golden("ilqr_f64")
    st = paper_setup_from_config(config())
    rng = np.random.default_rng(2)
    X, V = g["X_aux"].astype(npdt), g["V_aux"].astype(npdt)
    B = X.shape[0]
    gX = rng.normal(size=X.shape).astype(npdt)
    gU = rng.normal(size=V.shape).astype(npdt)
    cost = tracking_cost(g["theta"][0])
    r = ddp_sensitivity(problem=st.problem, cost=cost, X=_t(X, tdt, dev), V=_t(V, tdt, dev),
                        upper_grad_x=_t(gX, tdt, dev), upper_grad_u=_t(gU, tdt, dev))
    outs = [o.ddp_sensitivity_upper(st.problem.to_c(), cost.to_c(), X, V, gX, gU) for o in oracles(npdt)]
    base = 1e-10 if tag == "f64" else 1e-4
    for j, got in enumerate((r.delta_X, r.delta_V, r.delta_lambda)):
        frac, e, _ = agreement(got.cpu().numpy(), [o[j] for o in outs], base)
        assert frac == 1.0, (j, np.sort(e)[-3:])
    assert B == 8


def test_run_closed_loop_experiment_general_outputs(dev, tmp_path):
    """The general branch of run_closed_loop_experiment (core/tube_mpc.py:40-663): output files and
    summary as the reference writes them."""
    import os

    from diff_tube_mpc_strict_pt.core import run_closed_loop_experiment

    cfg = general_cfg()
    cfg["system"]["task_horizon_H"] = 3
    torch.manual_seed(0)
    res = run_closed_loop_experiment(cfg, device=dev, run_dir=str(tmp_path))
    for name in ("x_real", "u_real", "x_bar", "u_bar", "b_real", "loss", "Qa_history", "Ra_history", "qba_history"):
        a = np.load(os.path.join(tmp_path, name + ".npy"))
        assert a.shape[0] == 3 and np.isfinite(a).all()
    assert set(res["summary"]) == {"system", "H", "N", "final_state", "final_barrier_state", "final_loss"}
    g = golden("general_A_f64")
    assert abs(np.load(os.path.join(tmp_path, "loss.npy"))[0] - g["loss"][0]) < 1e-9  # step 0 has no disturbance


def test_ift_gradient_keyword_form_vs_reference_kats(dev):
    """ift_gradient in the reference's keyword form (core/ift.py:35-43): closures from core.closures.ParamClosures
    over the raw parameter tensors (and the ancillary set's X_ref / U_ref tensors), unbatched IFTInputs, a
    detached xi -- on the reference's own ift_gradient KATs, the same figures as the typed call."""
    from diff_tube_mpc_strict_pt.core import IFTInputs, ift_gradient
    from diff_tube_mpc_strict_pt.core.closures import ParamClosures
    from diff_tube_mpc_strict_pt.core.params import theta_from_raw
    from diff_tube_mpc_strict_pt.core.problem import general_setup_from_config

    k = golden("ift_general_f64")
    base = general_setup_from_config(general_cfg())
    n, N = k["X"].shape[0], k["X"].shape[1] - 1
    T = torch.float64
    for c in range(n):
        prob = dataclasses.replace(base.problem, horizon=N, barrier_type="log" if int(k["btype"][c]) else "inverse")
        inp = IFTInputs(X=_t(k["X"][c], T, dev), V=_t(k["V"][c], T, dev), delta_X=_t(k["dX"][c], T, dev),
                        delta_V=_t(k["dV"][c], T, dev), delta_lambda=_t(k["dlam"][c], T, dev))
        x0 = inp.X[0].clone()
        th = theta_from_raw(np.concatenate([k["raw_aux"][c], [0.0]]), False, dtype=T, device=dev)
        Xr, Ur = _t(k["Xref"][c], T, dev), _t(k["Uref"][c], T, dev)
        pc = ParamClosures(prob, th, X_ref=Xr, U_ref=Ur)
        g = ift_gradient(inputs=inp, theta_tensors=th.tensors() + [Xr, Ur], xi_fn=lambda: x0.detach(), f_fn=pc.f,
                         stage_cost_fn=pc.stage_cost, terminal_cost_fn=pc.terminal_cost)
        assert [tuple(a.shape) for a in g] == [tuple(t.shape) for t in th.tensors() + [Xr, Ur]]
        flat = torch.cat([a.reshape(-1) for a in g[:6]]).cpu().numpy()
        ref = k["g_aux"][c]
        assert close(flat, ref[:11], 1e-9, 1e-10), c
        assert close(g[6].cpu().numpy().reshape(-1), ref[11:11 + 3 * (N + 1)], 1e-12, 1e-13), c
        assert close(g[7].cpu().numpy().reshape(-1), ref[11 + 3 * (N + 1):], 1e-12, 1e-13), c
        thn = theta_from_raw(k["raw_nom"][c], True, dtype=T, device=dev)
        pn = ParamClosures(prob, thn, target=base.target)
        gn = ift_gradient(inputs=inp, theta_tensors=thn.tensors(), xi_fn=lambda: x0.detach(), f_fn=pn.f,
                          stage_cost_fn=pn.stage_cost, terminal_cost_fn=pn.terminal_cost)
        assert close(torch.cat([a.reshape(-1) for a in gn]).cpu().numpy(), k["g_nom"][c], 1e-9, 1e-10), c
