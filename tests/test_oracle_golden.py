"""Pin the C oracle to the reference: every oracle function vs the golden vectors produced by running
the reference itself (tests/golden/make_golden.py).  CPU only."""
from __future__ import annotations

import dataclasses

import numpy as np
import pytest

from _common import CHAOTIC, config, golden, ilqr_cfg, paper_setup, rel, tol_for

DTYPES = [("f64", np.float64), ("f32", np.float32)]


def kat_spec(setting: str):
    from diff_tube_mpc_strict_pt.core.problem import problem_from_config

    base = problem_from_config(config(), barrier_type="inverse", alpha=0.0, gamma=0.0)
    return {
        "s0": base,
        "s1": dataclasses.replace(base, obs_aggregation="min", dbas_alpha=0.05, dbas_gamma=0.3),
        "s2": dataclasses.replace(base, barrier_type="log", dbas_gamma=-0.5),
    }[setting]


@pytest.mark.parametrize("tag,dt", DTYPES)
def test_kat_safety_function(oracle_lib, tag, dt):
    o = oracle_lib.Oracle(dt)
    k = golden(f"kat_{tag}")
    base = kat_spec("s0")
    tol = 1e-13 if dt == np.float64 else 2e-6
    for agg, key in (("smoothmin", "smoothmin"), ("min", "min"), ("single", "single")):
        sp = dataclasses.replace(base, obs_aggregation=agg).to_c()
        h, gx, gy = o.h_eval(sp, k["xh"][:, 0], k["xh"][:, 1])
        assert rel(h, k[f"h_{key}"]) < tol, agg
        assert rel(np.stack([gx, gy], 1), k[f"gh_{key}"][:, :2]) < tol, agg
        assert np.all(k[f"gh_{key}"][:, 2] == 0)


@pytest.mark.parametrize("tag,dt", DTYPES)
def test_kat_barriers(oracle_lib, tag, dt):
    o = oracle_lib.Oracle(dt)
    k = golden(f"kat_{tag}")
    tol = 1e-14 if dt == np.float64 else 1e-6
    for name, alpha in (("a0", 0.0), ("a05", 0.05)):
        sp = dataclasses.replace(kat_spec("s0"), dbas_alpha=alpha).to_c()
        _, Br, dB = o.barrier(sp, k["z"])
        assert np.allclose(Br, k[f"B_relaxed_{name}"], rtol=tol, atol=0), name
        assert np.allclose(dB, k[f"dB_relaxed_{name}"], rtol=tol, atol=0), name
    sp = dataclasses.replace(kat_spec("s0"), barrier_type="log").to_c()
    Bd, _, _ = o.barrier(sp, k["z"])
    assert np.allclose(Bd, k["B_log"], rtol=tol, atol=tol)


@pytest.mark.parametrize("tag,dt", DTYPES)
@pytest.mark.parametrize("setting", ["s0", "s1", "s2"])
def test_kat_dbas_step_and_jacobian(oracle_lib, tag, dt, setting):
    o = oracle_lib.Oracle(dt)
    k = golden(f"kat_{tag}")
    sp = kat_spec(setting).to_c()
    tol = 1e-13 if dt == np.float64 else 1e-5
    f = o.fhat(sp, k["xh"], k["u"])
    assert np.allclose(f, k[f"fhat_{setting}"], rtol=tol, atol=tol)
    A, Bm = o.aug_jac(sp, k["xh"], k["u"])
    assert rel(A, k[f"A_{setting}"]) < tol
    assert rel(Bm, k[f"B_{setting}"]) < tol
    Bd, _, _ = o.barrier(sp, o.h_eval(sp, k["xh"][:, 0], k["xh"][:, 1])[0])
    assert np.allclose(Bd, k[f"b0_{setting}"], rtol=tol, atol=0)
    # dubins_step is the first three components of f_hat
    assert np.allclose(f[:, :3], k["dubins_step"], rtol=tol, atol=tol)


def _cases(g, key):
    return [i for i in range(g["x0"].shape[0]) if np.isfinite(g[key][i]).all()]


@pytest.mark.parametrize("tag,dt", DTYPES)
def test_ilqr_nominal_vs_reference(oracle_lib, tag, dt):
    o = oracle_lib.Oracle(dt)
    g = golden(f"ilqr_{tag}")
    st = paper_setup()
    sp, cn = st.problem.to_c(), st.nominal_cost.to_c()
    for mi, tl, xk, vk, ck in ((3, -1.0, "X_nom_fixed", "V_nom_fixed", "cond_nom_fixed"),
                               (10, 1e-3, "X_nom", "V_nom", "cond_nom")):
        X, V, K, kk, it, status = o.ilqr_solve(sp, cn, ilqr_cfg(mi, tl).to_c(), g["x0"], g["Vinit_nom"])
        checked = 0
        for i in range(X.shape[0]):
            if not np.isfinite(g[xk][i]).all():  # the reference raised FloatingPointError here
                continue
            assert status[i] == 0
            if g[ck][i] > CHAOTIC:
                continue
            t = tol_for(dt, g[ck][i])
            assert rel(X[i], g[xk][i]) < t, (i, xk)
            assert rel(V[i], g[vk][i]) < t, (i, vk)
            if tl > 0:
                assert it[i] == g["it_nom"][i]
            checked += 1
        assert checked >= 5


@pytest.mark.parametrize("tag,dt", DTYPES)
def test_ilqr_ancillary_sensitivity_gradient_vs_reference(oracle_lib, tag, dt):
    from diff_tube_mpc_strict_pt.core.problem import tracking_cost

    o = oracle_lib.Oracle(dt)
    g = golden(f"ilqr_{tag}")
    sp = paper_setup().problem.to_c()
    checked = 0
    for i in _cases(g, "X_aux"):
        cost = tracking_cost(g["theta"][i]).to_c()
        sl = slice(i, i + 1)
        for mi, tl, xk, vk, ck in ((4, -1.0, "X_aux_fixed", "V_aux_fixed", "cond_aux_fixed"),
                                   (20, 1e-3, "X_aux", "V_aux", "cond_aux")):
            X, V, _, _, it, status = o.ilqr_solve(sp, cost, ilqr_cfg(mi, tl).to_c(), g["x0_aux"][sl], g["Vinit_aux"][sl],
                                                  g["X_nom"][sl], g["V_nom"][sl])
            assert status[0] == 0
            if g[ck][i] > CHAOTIC:
                continue
            t = tol_for(dt, g[ck][i])
            assert rel(X[0], g[xk][i]) < t, (i, xk)
            assert rel(V[0], g[vk][i]) < t, (i, vk)
            if tl > 0:
                assert it[0] == g["it_aux"][i]
        # sensitivity on the reference's own optimum
        dX, dU, dL, status = o.ddp_sensitivity(sp, cost, g["X_aux"][sl], g["V_aux"][sl], g["X_nom"][sl])
        assert status[0] == 0
        gr = o.doc_grad(g["X_aux"][sl], g["V_aux"][sl], g["X_nom"][sl], g["V_nom"][sl], dX, dU)
        if g["cond_sens"][i] > CHAOTIC:
            continue
        t = tol_for(dt, g["cond_sens"][i])
        assert rel(dX[0], g["dX"][i]) < t, i
        assert rel(dU[0], g["dV"][i]) < t, i
        assert rel(dL[0], g["dlam"][i]) < t, i
        assert rel(gr[0], g["grad"][i]) < t, i
        checked += 1
    assert checked >= 5


@pytest.mark.parametrize("tag,dt", DTYPES)
def test_nonfinite_inputs_are_flagged(oracle_lib, tag, dt):
    """NaN in x0 or V_init -> FloatingPointError in the reference (core/ddp.py:138-159) -> status bit.
    +inf in V_init is clamped to the box (core/ddp.py:128-129) and stays finite."""
    o = oracle_lib.Oracle(dt)
    g = golden(f"ilqr_{tag}")
    st = paper_setup()
    x0 = np.array(g["x0"][[0, 2, 3]])
    V = np.array(g["Vinit_nom"][[0, 2, 3]])
    x0[0, 1] = np.nan
    V[1, 7, 1] = np.nan
    V[2, 4, 0] = np.inf
    _, Vo, _, _, _, status = o.ilqr_solve(st.problem.to_c(), st.nominal_cost.to_c(), ilqr_cfg(3, -1.0).to_c(), x0, V)
    assert status[0] & 1 and status[1] & 1
    assert status[2] == 0 and np.isfinite(Vo[2]).all()


def _oracle_closed_loop(o, dt, g, H):
    """Drive the oracle tube step like core/tube_mpc.py:803-1023 (B = 1)."""
    from diff_tube_mpc_strict_pt import _abi

    st = paper_setup()
    N = st.problem.horizon
    sp = st.problem.to_c()
    tcfg = _abi.DtmpcTubeCfg()
    tcfg.nominal = st.nominal_cost.to_c()
    tcfg.nom_ilqr = st.ilqr_nom.to_c()
    tcfg.aux_ilqr = st.ilqr_aux.to_c()
    tcfg.disturbance = 0
    x0 = np.array([[0.0, 0.0, np.pi / 4]], dt)
    _, _, b0s = None, None, None
    h, _, _ = o.h_eval(sp, x0[:, 0], x0[:, 1])
    b0 = o.barrier(sp, h)[0]
    state = {
        "x": x0.T.copy(), "b": b0.astype(dt), "xbar": x0.T.copy(),
        "bbar": b0.astype(dt).copy(), "Xnom": np.zeros((N + 1, 4, 1), dt), "Unom": np.zeros((N, 2, 1), dt),
        "Xaux": np.zeros((N + 1, 4, 1), dt), "Uaux": np.zeros((N, 2, 1), dt),
    }
    theta = np.array(st.theta0, dt)
    vel = np.zeros(6, dt)
    logs, thetas = [], []
    for t in range(H):
        gout, log, status, iters = o.tube_step(sp, tcfg, state, theta, w=g["w"][t:t + 1], step=t)
        assert status[0] == 0
        sums = np.zeros(8, dt)
        sums[:7] = gout[:, 0]
        theta, vel = o.theta_update(st.adapt.to_c(), 1.0, sums, theta, vel)
        logs.append(log[:, 0].copy())
        thetas.append(theta.copy())
    return np.array(logs), np.array(thetas)


@pytest.mark.parametrize("tag,dt", DTYPES)
def test_closed_loop_vs_reference_loop(oracle_lib, tag, dt):
    o = oracle_lib.Oracle(dt)
    g = golden(f"closed_loop_{tag}")
    H = g["loss"].shape[0]
    logs, thetas = _oracle_closed_loop(o, dt, g, H)
    t = 1e-9 if dt == np.float64 else 5e-4
    assert rel(logs[:, 0:3], g["x_real"]) < t
    assert rel(logs[:, 3:5], g["u_real"]) < t
    assert rel(logs[:, 5:8], g["x_bar"]) < t
    assert rel(logs[:, 8:10], g["u_bar"]) < t
    assert rel(logs[:, 10], g["b_real"]) < t
    assert rel(logs[:, 11], g["loss"]) < t
    assert rel(thetas[:, 0:3], g["Qa_history"]) < t
    assert rel(thetas[:, 3:5], g["Ra_history"]) < t
    assert rel(thetas[:, 5], g["qba_history"]) < t


def test_nominal_receding_vs_run_nominal(oracle_lib):
    """run_nominal.py:204-415 (config #1): angle-wrapped nominal MPC, reg = ilqr_reg, v_max warm start."""
    from diff_tube_mpc_strict_pt.core.problem import ILQRConfig, QuadraticCost, problem_from_config

    cfg = config()
    g = golden("nominal_receding")
    o = oracle_lib.Oracle(np.float64)
    sc = cfg["system"]
    prob = problem_from_config(cfg)
    cn = cfg["cost_nominal"]
    cost = QuadraticCost(kind="target", Q=tuple(cn["Q"]), R=tuple(cn["R"]), Qf=tuple(cn["Qf"]), qb=float(cn["q_b"]),
                         target=tuple(sc["target"]), wrap_angle=True)
    N = prob.horizon
    icfg = ILQRConfig(horizon=N, max_iter=int(sc["nominal_max_iter"]), tol=1e-3, reg=float(sc["ilqr_reg"]),
                      line_search_alphas=tuple(sc["line_search_alphas"])).to_c()
    sp = prob.to_c()
    x = np.array([0.0, 0.0, np.pi / 4])
    b = o.barrier(sp, o.h_eval(sp, x[:1], x[1:2])[0])[0][0]
    U = np.zeros((1, N, 2))
    U[0, :, 0] = prob.u_max[0]
    xs, us = [], []
    for t in range(int(g["H_ran"])):
        X, V, _, _, _, status = o.ilqr_solve(sp, cost.to_c(), icfg, np.array([[*x, b]]), U)
        assert status[0] == 0
        xs.append(x.copy())
        us.append(V[0, 0].copy())
        nxt = o.fhat(sp, np.array([[*x, b]]), V[:, 0])[0]
        x, b = nxt[:3], nxt[3]
        U = np.concatenate([V[:, 1:], V[:, -1:]], axis=1)
    assert rel(np.array(xs), g["x_bar"]) < 1e-9
    assert rel(np.array(us), g["u_bar"]) < 1e-9


def test_symmetric_vxx_build_is_the_same_algorithm(oracle_lib):
    """liboracle_sym.so (V_xx mirrored from its upper triangle after every Riccati step; the receding f32
    failure-set test's fourth rounding) solves the reference's golden nominal iLQR cases like the plain build:
    f64, well-conditioned cases, within the golden tolerance -- it is a rounding of the same recursion."""
    g = golden("ilqr_f64")
    st = paper_setup()
    sp, cn = st.problem.to_c(), st.nominal_cost.to_c()
    outs = [oracle_lib.Oracle(np.float64, variant=v).ilqr_solve(sp, cn, ilqr_cfg(10, 1e-3).to_c(), g["x0"],
                                                                 g["Vinit_nom"]) for v in ("plain", "sym")]
    n = 0
    for i in range(g["x0"].shape[0]):
        if not np.isfinite(g["X_nom"][i]).all() or g["cond_nom"][i] > CHAOTIC:
            continue
        t = tol_for(np.float64, g["cond_nom"][i])
        assert rel(outs[1][0][i], outs[0][0][i]) < t and rel(outs[1][0][i], g["X_nom"][i]) < t, i
        n += 1
    assert n >= 5
