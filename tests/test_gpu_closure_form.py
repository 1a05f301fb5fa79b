"""The reference's keyword (closure) form on the device (core/closures.py): ddp_sensitivity and rollout through
closures against the typed calls on the same tapes, and the closures' own point evaluations against the
typed kernels.  f64, single-trajectory inputs as the reference passes them.  Needs an MI355X: -m gpu."""
from __future__ import annotations

import json

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda:0")


def _setup(dev):
    from diff_tube_mpc_strict_pt.core import ilqr_solve
    from diff_tube_mpc_strict_pt.core.closures import nominal_closures
    from diff_tube_mpc_strict_pt.core.ddp import dbas_init
    from _common import config

    cl = nominal_closures(json.loads(json.dumps(config())))
    f_hat, ctrl, icfg = cl["f_hat"], cl["ctrl"], cl["ilqr_cfg"]
    kw = dict(dtype=torch.float64, device=dev)
    x = torch.tensor([0.3, 0.2, 0.6], **kw)
    b = dbas_init(f_hat.problem, x[None])[0]
    x0 = torch.cat([x, b.view(1)])
    U = torch.zeros(icfg.horizon, 2, **kw)
    U[:, 0] = 10.0
    X, V = ilqr_solve(x0=x0, V_init=U, cfg=icfg, f=f_hat, ctrl=ctrl, f_jac=cl["f_jac"],
                      stage_cost=cl["stage_cost"], terminal_cost=cl["terminal_cost"],
                      stage_derivs=cl["stage_derivs"], terminal_derivs=cl["term_derivs"])
    return cl, x0, X, V


def test_sensitivity_keyword_form_vs_typed(dev):
    """ddp_sensitivity(X=, V=, f=, f_jac=, ctrl=, stage_hess=, terminal_hess=, upper_grad_x=, upper_grad_u=,
    upper_grad_xN=) with the paper upper loss as closures (g_x = [2 (x - xbar_k), 2 b], g_u = 0) against the
    typed call with X_bar (core/tube_mpc.py:915-957): 1e-12 relative."""
    from diff_tube_mpc_strict_pt.core import ddp_sensitivity

    cl, _, X, V = _setup(dev)
    qc = cl["stage_cost"].__self__
    Xbar = X + 0.01 * torch.sin(torch.arange(X.numel(), dtype=X.dtype, device=X.device)).view_as(X)

    def gx(x, k):
        return torch.cat([2.0 * (x[:3] - Xbar[k, :3]), 2.0 * x[3:4]])

    res = ddp_sensitivity(X=X, V=V, f=cl["f_hat"], f_jac=cl["f_jac"], ctrl=cl["ctrl"], stage_hess=qc.stage_hess,
                          terminal_hess=qc.terminal_hess, upper_grad_x=gx, upper_grad_u=lambda u, k: torch.zeros_like(u),
                          upper_grad_xN=lambda x: gx(x, X.shape[0] - 1))
    ref = ddp_sensitivity(problem=dataclass_problem(cl), cost=qc.cost, X=X[None], V=V[None], X_bar=Xbar[None])
    assert res.delta_X.shape == X.shape and res.delta_V.shape == V.shape
    for a, b in ((res.delta_X, ref.delta_X[0]), (res.delta_V, ref.delta_V[0]), (res.delta_lambda, ref.delta_lambda[0])):
        a, b = a.cpu().numpy(), b.cpu().numpy()
        assert np.max(np.abs(a - b)) <= 1e-12 * max(1.0, np.max(np.abs(b))), np.max(np.abs(a - b))


def dataclass_problem(cl):
    import dataclasses

    p = cl["f_hat"].problem
    return dataclasses.replace(p, **cl["ctrl"].problem_bounds())


def test_rollout_and_point_closures(dev):
    """rollout(x0, V, *, f) vs the typed rollout (bitwise: the same kernel); f_hat(x, u) step by step vs the
    rolled-out tape (bitwise); stage / terminal cost closures summed along the tape vs core.ocp.total_cost
    (the tape-cost kernel) at 1e-12; the wrapped-heading derivative at target_k (run_nominal.py:311-315)."""
    from diff_tube_mpc_strict_pt.core import rollout
    from diff_tube_mpc_strict_pt.core.ocp import total_cost

    cl, x0, X, V = _setup(dev)
    f_hat = cl["f_hat"]
    Xr = rollout(x0, V, f=f_hat)
    Xt = rollout(dataclass_problem(cl), x0[None], V[None])[0]
    assert torch.equal(Xr, Xt)
    x = x0
    for k in range(V.shape[0]):
        x = f_hat(x, V[k])
        assert torch.equal(x, Xr[k + 1]), k
    qc = cl["stage_cost"].__self__
    J = sum(float(cl["stage_cost"](Xr[k], V[k], k)) for k in range(V.shape[0])) + float(cl["terminal_cost"](Xr[-1]))
    Jt = float(total_cost(X=Xr[None], U=V[None], cost=qc.cost)[0])
    assert abs(J - Jt) <= 1e-12 * max(1.0, abs(Jt)), (J, Jt)
    # a heading 2 pi + 0.1 from the target: the wrapped cost and derivative see an error of 0.1
    import dataclasses

    from diff_tube_mpc_strict_pt.core.closures import QuadraticClosures

    q1 = QuadraticClosures(dataclasses.replace(qc.cost, Q=(1.0, 1.0, 1.0)))
    t2 = qc.cost.target[2]
    xh = torch.tensor([qc.cost.target[0], qc.cost.target[1], t2 + 2 * np.pi + 0.1, 0.0], dtype=torch.float64,
                      device=dev)
    u0 = torch.zeros(2, dtype=torch.float64, device=dev)
    lx, lu, *_ = q1.stage_derivs(xh, u0, 0)
    assert abs(float(lx[2]) - 0.2) <= 1e-12 and abs(float(lx[0])) <= 1e-12
    assert abs(float(q1.stage_cost(xh, u0, 0)) - 0.01) <= 1e-12


def test_ilqr_keyword_form_batched_vs_typed(dev):
    """The keyword form with a batch (x0 [B, 4], V_init [B, N, 2]) returns the typed call's X*, V* bit for bit
    (the same kernel); ctrl=None is the unclamped box."""
    import dataclasses

    from diff_tube_mpc_strict_pt.core import ilqr_solve

    cl, x0, X, V = _setup(dev)
    icfg = cl["ilqr_cfg"]
    B = 5
    xb = x0[None].repeat(B, 1)
    xb[:, 0] += torch.linspace(0.0, 0.2, B, dtype=xb.dtype, device=dev)
    Ub = torch.zeros(B, icfg.horizon, 2, dtype=xb.dtype, device=dev)
    Ub[:, :, 0] = 10.0
    kw = dict(cfg=icfg, f=cl["f_hat"], f_jac=cl["f_jac"], stage_cost=cl["stage_cost"],
              terminal_cost=cl["terminal_cost"], stage_derivs=cl["stage_derivs"], terminal_derivs=cl["term_derivs"])
    Xk, Vk = ilqr_solve(x0=xb, V_init=Ub, ctrl=cl["ctrl"], **kw)
    qc = cl["stage_cost"].__self__
    r = ilqr_solve(problem=dataclass_problem(cl), cost=qc.cost, cfg=icfg, x0=xb, V_init=Ub)
    assert torch.equal(Xk, r.X) and torch.equal(Vk, r.V)
    Xn, Vn = ilqr_solve(x0=xb, V_init=Ub, ctrl=None, **kw)
    p_unb = dataclasses.replace(cl["f_hat"].problem, u_min=(-np.inf, -np.inf), u_max=(np.inf, np.inf))
    r2 = ilqr_solve(problem=p_unb, cost=qc.cost, cfg=icfg, x0=xb, V_init=Ub)
    assert torch.isfinite(Xn).all() and torch.equal(Xn, r2.X) and torch.equal(Vn, r2.V)
