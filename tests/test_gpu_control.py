"""Tanh-box control map and v-space cost derivatives on the HIP device (dtmpc_tanh_cost_derivs,
include/dtmpc_control.h): vs the reference's golden vectors (core/control.py:10-35,
core/cost_derivs.py:16-107; tests/golden/make_golden_tanh.py), vs the oracle on a full tape batch, and
the Python mirror's reference signatures and shapes.  Needs an MI355X: -m gpu.

Tolerance: f64 1e-13 relative to max(1, |reference|); f32 2e-6 (device tanhf vs the reference's tanh:
one ulp, amplified at most by the 1 - tanh^2 cancellation)."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from _common import golden, rel

pytestmark = pytest.mark.gpu

DTYPES = [("f64", np.float64, torch.float64), ("f32", np.float32, torch.float32)]


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from diff_tube_mpc_strict_pt import _lib

    assert _lib.load().dtmpc_device_count() >= 1
    return torch.device("cuda:0")


def _ctrl(g):
    from diff_tube_mpc_strict_pt.core import BoxTanhControl

    return BoxTanhControl(u_min=tuple(g["umin"]), u_max=tuple(g["umax"]))


@pytest.mark.parametrize("tag,npdt,tdt", DTYPES)
def test_tanh_cost_derivs_vs_reference(dev, tag, npdt, tdt):
    from diff_tube_mpc_strict_pt.core import auxiliary_cost_derivs, nominal_cost_derivs

    g = golden(f"tanh_{tag}")
    tol = 1e-13 if tag == "f64" else 2e-6
    t = lambda a: torch.as_tensor(np.asarray(a), dtype=tdt, device=dev)  # noqa: E731
    ctrl = _ctrl(g)
    N = g["Vd"].shape[1]
    X, Vd = t(g["X"][:, :N]), t(g["Vd"])
    assert rel(ctrl.u(Vd).cpu().numpy(), g["u"]) < tol
    assert rel(ctrl.du_dv_diag(Vd).cpu().numpy(), g["dudv"]) < tol
    lx, lv, lxx, lvv, lvx = nominal_cost_derivs(x_hat=X, v=Vd, target=g["target"], Q=g["Q"], R=g["R"], qb=g["qb"],
                                                ctrl=ctrl)
    assert rel(lx.cpu().numpy(), g["lx_nom"]) < tol
    assert rel(lv.cpu().numpy(), g["lv_nom"]) < tol
    assert rel(torch.diagonal(lvv, dim1=-2, dim2=-1).cpu().numpy(), g["lvv_nom"]) < tol
    assert lxx.shape == (*Vd.shape[:-1], 4, 4) and lvx.shape == (*Vd.shape[:-1], 2, 4) and not lvx.any()
    q2 = 2 * torch.tensor(list(g["Q"]) + [float(g["qb"])], dtype=tdt)
    assert torch.equal(lxx[0, 0].cpu(), torch.diag(q2))
    lx, lv, lxx, lvv, lvx = auxiliary_cost_derivs(x_hat=X, v=Vd, x_ref=t(g["Xr"][:, :N]), u_ref=t(g["Ur"]), Q=g["Qa"],
                                                  R=g["Ra"], qb=g["qba"], ctrl=ctrl)
    assert rel(lx.cpu().numpy(), g["lx_aux"]) < tol
    assert rel(lv.cpu().numpy(), g["lv_aux"]) < tol
    assert rel(torch.diagonal(lvv, dim1=-2, dim2=-1).cpu().numpy(), g["lvv_aux"]) < tol
    # unbatched call: the reference's own shapes
    lx, lv, lxx, lvv, lvx = nominal_cost_derivs(x_hat=X[1, 2], v=Vd[1, 2], target=g["target"], Q=g["Q"], R=g["R"],
                                                qb=g["qb"], ctrl=ctrl)
    assert (lx.shape, lv.shape, lxx.shape, lvv.shape, lvx.shape) == ((4,), (2,), (4, 4), (2, 2), (2, 4))
    assert rel(lv.cpu().numpy(), g["lv_nom"][1, 2]) < tol


@pytest.mark.parametrize("tag,npdt,tdt", DTYPES)
@pytest.mark.parametrize("kind", ["target", "track"])
def test_tanh_cost_derivs_tape_vs_oracle(dev, oracle_lib, tag, npdt, tdt, kind):
    """Full tapes (B = 1,000 ragged against the 256-lane blocks, N = 50) through the C ABI vs the oracle."""
    import ctypes as C

    from diff_tube_mpc_strict_pt import _abi, _lib
    from diff_tube_mpc_strict_pt.core.problem import DubinsDBaSProblem, QuadraticCost

    rng = np.random.default_rng(3)
    B, N = 1000, 50
    X = rng.uniform(-5, 5, (B, N + 1, 4)).astype(npdt)
    Vd = rng.normal(0, 3, (B, N, 2)).astype(npdt)
    Xr = rng.uniform(-5, 5, (B, N + 1, 3)).astype(npdt)
    Ur = rng.uniform(-5, 5, (B, N, 2)).astype(npdt)
    prob = DubinsDBaSProblem(horizon=N)
    cost = QuadraticCost(kind=kind, Q=(1.0, 2.0, 0.1), R=(0.01, 0.3), qb=0.05, target=(4.0, 4.0, 0.5))
    refs = {"Xref": Xr, "Uref": Ur} if kind == "track" else {}
    want = oracle_lib.Oracle(npdt).tanh_cost_derivs(prob.to_c(), cost.to_c(), X, Vd, **refs)
    soa = lambda a: torch.as_tensor(np.ascontiguousarray(np.transpose(a, (1, 2, 0))), device=dev)  # noqa: E731
    Xs, Vs = soa(X), soa(Vd)
    Xrs, Urs = (soa(Xr), soa(Ur)) if kind == "track" else (None, None)
    outs = {k: torch.full((N, w, B), float("nan"), dtype=tdt, device=dev)
            for k, w in (("u", 2), ("dudv", 2), ("lx", 4), ("lv", 2), ("lvv", 2))}
    lib = _lib.load()
    p = lambda x: None if x is None else x.data_ptr()  # noqa: E731
    rc = lib.dtmpc_tanh_cost_derivs(_abi.F64 if tag == "f64" else _abi.F32, C.byref(prob.to_c()), C.byref(cost.to_c()),
                                    B, Xs.data_ptr(), Vs.data_ptr(), p(Xrs), p(Urs), *(outs[k].data_ptr() for k in
                                                                                        ("u", "dudv", "lx", "lv", "lvv")),
                                    None)
    assert rc == 0, lib.dtmpc_last_error()
    torch.cuda.synchronize()
    tol = 1e-13 if tag == "f64" else 2e-6
    for k, o in outs.items():
        got = np.transpose(o.cpu().numpy(), (2, 0, 1))
        assert np.isfinite(got).all(), k
        assert rel(got, want[k]) < tol, k


@pytest.mark.parametrize("tag,npdt,tdt", DTYPES)
def test_ocp_total_cost_and_rollout(dev, oracle_lib, tag, npdt, tdt):
    """core.ocp.total_cost (dtmpc_tape_cost) vs the reference's total_cost with the paper closures
    (golden ocp_*.npz) and vs the oracle; rollout_dynamics batched / unbatched vs core.ddp.rollout."""
    from diff_tube_mpc_strict_pt.core import DubinsDBaSProblem
    from diff_tube_mpc_strict_pt.core.ocp import rollout_dynamics, total_cost
    from test_oracle_ocp import ocp_case

    g, spec, nom, aux = ocp_case(tag)
    tol = 1e-13 if tag == "f64" else 1e-6
    t = lambda a: torch.as_tensor(np.asarray(a), dtype=tdt, device=dev)  # noqa: E731
    X, U = t(g["X"]), t(g["U"])
    J = total_cost(X=X, U=U, cost=nom).cpu().numpy()
    np.testing.assert_allclose(J, g["J_nom"], rtol=tol)
    o = oracle_lib.Oracle(npdt)
    np.testing.assert_allclose(J, o.tape_cost(spec, nom.to_c(), g["X"], g["U"]), rtol=tol)
    Ja = total_cost(X=X, U=U, cost=aux, X_ref=t(g["Xr"]), U_ref=t(g["Ur"])).cpu().numpy()
    np.testing.assert_allclose(Ja, g["J_aux"], rtol=tol)
    J1 = total_cost(X=X[2], U=U[2], cost=nom)
    assert J1.dim() == 0 and abs(float(J1) - float(g["J_one"])) <= tol * abs(float(g["J_one"]))
    prob = DubinsDBaSProblem(horizon=U.shape[1])
    from diff_tube_mpc_strict_pt.core import rollout

    Xr = rollout_dynamics(X[:, 0], U, f=prob)
    assert torch.equal(Xr, rollout(prob, X[:, 0], U))
    assert torch.equal(rollout_dynamics(X[3, 0], U[3], f=prob), Xr[3])
