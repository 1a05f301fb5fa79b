"""The reference's keyword (closure) form of ilqr_solve / ddp_sensitivity / rollout (core/ddp.py:89, 102-117,
317-329) resolving against the package, on CPU: no device call is made -- resolution happens
before dispatch, and the dispatch then refuses host tensors (there is no CPU fallback).  The device run of the
same call pattern against the reference's fixture is tests/test_gpu_receding.py::test_reference_call_pattern."""
from __future__ import annotations

import json
import math

import numpy as np
import pytest
import torch

from _common import config, golden


def _closures():
    from diff_tube_mpc_strict_pt.core.closures import nominal_closures

    cfg = json.loads(json.dumps(config()))
    cfg["system"]["task_horizon_H"] = 2  # the fixture nominal_receding.npz (tests/golden/make_golden.py)
    return cfg, nominal_closures(cfg)


def test_run_nominal_call_pattern_resolves():
    """run_nominal.py:353-364, argument for argument (the f_jac lambda included), resolves to the typed
    problem and cost that the package's own receding setup builds from the same config."""
    from diff_tube_mpc_strict_pt.core import ilqr_solve
    from diff_tube_mpc_strict_pt.core.closures import resolve_ilqr
    from diff_tube_mpc_strict_pt.core.receding import receding_setup_from_config

    cfg, cl = _closures()
    f_hat, ctrl, ilqr_cfg = cl["f_hat"], cl["ctrl"], cl["ilqr_cfg"]
    stage_cost, terminal_cost, stage_derivs, term_derivs = (cl["stage_cost"], cl["terminal_cost"],
                                                            cl["stage_derivs"], cl["term_derivs"])
    jac = cl["f_jac"]
    kwargs = dict(cfg=ilqr_cfg, f=f_hat, ctrl=ctrl, f_jac=lambda xh, uk: jac(xh, uk), stage_cost=stage_cost,
                  terminal_cost=terminal_cost, stage_derivs=stage_derivs, terminal_derivs=term_derivs)
    r = resolve_ilqr(**kwargs)
    problem, cost, icfg = receding_setup_from_config(cfg)
    assert r.problem == problem and r.cost == cost and icfg == ilqr_cfg
    assert cost.wrap_angle and cost.kind == "target"
    # the call itself: resolved, then refused at dispatch on host tensors (no CPU fallback)
    N = ilqr_cfg.horizon
    x_hat0 = torch.tensor([0.0, 0.0, math.pi / 4, 0.05], dtype=torch.float64)
    U_ws = torch.zeros(N, 2, dtype=torch.float64)
    U_ws[:, 0] = 10.0
    with pytest.raises(ValueError, match="device tensors"):
        ilqr_solve(x0=x_hat0, V_init=U_ws, **kwargs)
    # the fixture the device test compares against exists with the expected shapes
    g = golden("nominal_receding")
    assert g["x_bar"].shape == (2, 3) and g["u_bar"].shape == (2, 2) and int(g["H_ran"]) == 2


def test_keyword_form_refusals():
    from diff_tube_mpc_strict_pt.core import ddp_sensitivity, ilqr_solve, rollout
    from diff_tube_mpc_strict_pt.core.closures import QuadraticClosures, resolve_ilqr, resolve_sensitivity
    from diff_tube_mpc_strict_pt.core.problem import QuadraticCost

    _, cl = _closures()
    base = dict(cfg=cl["ilqr_cfg"], f=cl["f_hat"], ctrl=cl["ctrl"], stage_cost=cl["stage_cost"],
                terminal_cost=cl["terminal_cost"], stage_derivs=cl["stage_derivs"],
                terminal_derivs=cl["term_derivs"])
    # an arbitrary Python closure cannot run in the device solver
    with pytest.raises(TypeError, match="arbitrary Python closure"):
        resolve_ilqr(**{**base, "stage_cost": lambda x, u, k: (x * x).sum()})
    with pytest.raises(TypeError, match="arbitrary Python closure"):
        resolve_ilqr(**{**base, "f": lambda x, u: x})
    # cost closures of two different costs
    other = QuadraticClosures(QuadraticCost(kind="target", target=(1.0, 1.0, 0.0)))
    with pytest.raises(ValueError, match="different cost"):
        resolve_ilqr(**{**base, "terminal_cost": other.terminal_cost})
    with pytest.raises(NotImplementedError):
        resolve_ilqr(**base, feasible_fn=lambda x, k: True)
    with pytest.raises(TypeError, match="needs"):
        resolve_ilqr(**{**base, "terminal_derivs": None})
    # typed and keyword forms do not mix
    with pytest.raises(TypeError, match="not both"):
        ilqr_solve(problem=cl["f_hat"].problem, x0=torch.zeros(4), V_init=torch.zeros(50, 2), **base)
    # ctrl = None: no clamp (core/ddp.py:128), an unbounded box
    r = resolve_ilqr(**{**base, "ctrl": None})
    assert r.problem.u_min == (-math.inf, -math.inf) and r.problem.u_max == (math.inf, math.inf)
    # sensitivity: Hessian closures resolve, the upper-level gradients must be callables
    qc = cl["stage_cost"].__self__
    rs = resolve_sensitivity(f=cl["f_hat"], ctrl=cl["ctrl"], stage_hess=qc.stage_hess,
                             terminal_hess=qc.terminal_hess, horizon=50)
    assert rs.cost == qc.cost
    X, V = torch.zeros(51, 4, dtype=torch.float64), torch.zeros(50, 2, dtype=torch.float64)
    with pytest.raises(TypeError, match="upper_grad"):
        ddp_sensitivity(X=X, V=V, f=cl["f_hat"], ctrl=cl["ctrl"], stage_hess=qc.stage_hess,
                        terminal_hess=qc.terminal_hess, upper_grad_x=None, upper_grad_u=None, upper_grad_xN=None)
    with pytest.raises(ValueError, match="device tensors"):
        ddp_sensitivity(X=X, V=V, f=cl["f_hat"], ctrl=cl["ctrl"], stage_hess=qc.stage_hess,
                        terminal_hess=qc.terminal_hess, upper_grad_x=lambda x, k: torch.zeros_like(x),
                        upper_grad_u=lambda u, k: torch.zeros_like(u), upper_grad_xN=lambda x: torch.zeros_like(x))
    # rollout(x0, V, *, f): the reference's form, refused on host tensors after resolution
    with pytest.raises(ValueError, match="device tensors"):
        rollout(torch.zeros(4, dtype=torch.float64), V, f=cl["f_hat"])
    with pytest.raises(TypeError, match="arbitrary Python closure"):
        rollout(torch.zeros(4), V, f=lambda x, u: x)
    # the closures' own evaluation is device-only too
    with pytest.raises(ValueError, match="device tensors"):
        cl["stage_cost"](torch.zeros(4, dtype=torch.float64), torch.zeros(2, dtype=torch.float64), 0)


def test_ift_keyword_form_resolution():
    """ift_gradient(inputs=, theta_tensors=, xi_fn=, f_fn=, stage_cost_fn=, terminal_cost_fn=) (core/ift.py:35-43):
    the closures of one ParamClosures resolve, theta_tensors map by identity onto the raw parameters and the
    reference tensors; a foreign tensor, mixed closure sets, a xi that needs gradients, or a mix with the typed
    arguments are refused; the call reaches dispatch and refuses host tensors."""
    from diff_tube_mpc_strict_pt.core import IFTInputs, ift_gradient
    from diff_tube_mpc_strict_pt.core.closures import ParamClosures, resolve_ift
    from diff_tube_mpc_strict_pt.core.params import theta_from_raw
    from diff_tube_mpc_strict_pt.core.problem import DubinsDBaSProblem

    N = 6
    prob = DubinsDBaSProblem(horizon=N)
    th = theta_from_raw(np.linspace(-0.5, 0.5, 12), False)
    Xr, Ur = torch.zeros(N + 1, 3, dtype=torch.float64), torch.zeros(N, 2, dtype=torch.float64)
    pc = ParamClosures(prob, th, X_ref=Xr, U_ref=Ur)
    x0 = torch.zeros(4, dtype=torch.float64)
    kw = dict(xi_fn=lambda: x0, f_fn=pc.f, stage_cost_fn=pc.stage_cost, terminal_cost_fn=pc.terminal_cost)
    got, where = resolve_ift(theta_tensors=th.tensors() + [Xr, Ur], **kw)
    assert got is pc and where == [("theta", i) for i in range(6)] + [("X_ref", None), ("U_ref", None)]
    with pytest.raises(ValueError, match="do not depend"):
        resolve_ift(theta_tensors=[torch.zeros(3)], **kw)
    other = ParamClosures(prob, th, target=(1.0, 1.0, 0.0))
    with pytest.raises(ValueError, match="different"):
        resolve_ift(theta_tensors=th.tensors(), **{**kw, "terminal_cost_fn": other.terminal_cost})
    with pytest.raises(NotImplementedError, match="detached"):
        resolve_ift(theta_tensors=th.tensors(), **{**kw, "xi_fn": lambda: x0.clone().requires_grad_(True)})
    with pytest.raises(TypeError, match="arbitrary Python closure"):
        resolve_ift(theta_tensors=th.tensors(), **{**kw, "f_fn": lambda x, u: x})
    with pytest.raises(ValueError, match="X_ref / U_ref"):
        ParamClosures(prob, th)
    inp = IFTInputs(X=torch.zeros(N + 1, 4, dtype=torch.float64), V=torch.zeros(N, 2, dtype=torch.float64),
                    delta_X=torch.zeros(N + 1, 4, dtype=torch.float64), delta_V=torch.zeros(N, 2, dtype=torch.float64),
                    delta_lambda=torch.zeros(N + 1, 4, dtype=torch.float64))
    with pytest.raises(TypeError, match="not both"):
        ift_gradient(inputs=inp, problem=prob, theta_tensors=th.tensors(), **kw)
    with pytest.raises(ValueError, match="device tensors"):
        ift_gradient(inputs=inp, theta_tensors=th.tensors(), **kw)
