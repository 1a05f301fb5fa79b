"""The reference's public names resolve under its own module paths in this package (CPU, import only).

The lists are the reference's own imports and exports:
  run_nominal.py:38-49 and :209-221 (run_nominal_once / run_nominal_receding),
  run_experiment.py:52, core/__init__.py:9-52 (the ddp / ift exports on the hot path), and the
  per-function modules core/barrier.py, core/systems/*.py, core/control.py, core/cost_derivs.py.
Their numerics are checked on the device in tests/test_gpu_systems.py (reference KAT vectors)."""
from __future__ import annotations

import importlib

import pytest

NAMES = {
    # run_nominal.py:38-49, 209-221
    "core.barrier": ["DBaSConfig", "dbas_init_b0", "dbas_step", "relaxed_inverse_barrier_B_alpha", "barrier_B"],
    "core.control": ["BoxClampControl", "BoxTanhControl"],
    "core.cost_derivs": ["nominal_cost_derivs_u", "nominal_terminal_derivs", "auxiliary_cost_derivs_u",
                         "auxiliary_terminal_derivs", "nominal_cost_derivs", "auxiliary_cost_derivs"],
    "core.ddp": ["ILQRConfig", "ilqr_solve", "ddp_sensitivity", "rollout", "SensitivityResult"],
    "core.systems.dubins": ["DubinsConfig", "dubins_step", "clamp_control", "sample_disturbance",
                            "default_safe_h_no_obstacles"],
    "core.systems.dubins_aug_jac": ["dubins_augmented_jacobian", "dubins_f_jac", "_B_inv", "_dB_inv_dz",
                                    "_dB_relaxed_inv_dz"],
    "core.systems.dubins_obstacles": ["CircleObstacle", "h_circle_obstacle", "grad_h_circle_obstacle",
                                      "h_multi_circle_obstacles", "grad_h_multi_circle_obstacles",
                                      "h_min_circle_obstacles", "grad_h_min_circle_obstacles"],
    # run_experiment.py:52
    "core.tube_mpc": ["run_closed_loop_experiment", "ExperimentTrajectories"],
    # core/__init__.py:9-20 (hot-path exports)
    "core": ["ILQRConfig", "SensitivityResult", "ilqr_solve", "ddp_sensitivity", "rollout", "IFTInputs",
             "ift_gradient",
             # core/__init__.py:22-31: the autograd fallbacks and the utils (round 5)
             "grad_hess_xu", "grad_hess_x", "compute_jacobian", "solve_psd", "regularize_matrix",
             "quadratic_cost_derivs_diagonal"],
    "core.autodiff": ["grad_hess_xu", "grad_hess_x", "compute_jacobian"],
    "core.utils": ["solve_psd", "regularize_matrix", "quadratic_cost_derivs_diagonal"],
    "core.ift": ["IFTInputs", "ift_gradient"],
    "core.ocp": ["rollout_dynamics", "total_cost"],
    "core.params": ["NominalTheta", "AuxiliaryTheta"],
}


@pytest.mark.parametrize("module", sorted(NAMES))
def test_reference_names_resolve(module):
    m = importlib.import_module(f"diff_tube_mpc_strict_pt.{module}")
    missing = [n for n in NAMES[module] if not hasattr(m, n)]
    assert not missing, (module, missing)


def test_reference_dataclass_defaults():
    """DBaSConfig (core/barrier.py:16-33) and DubinsConfig (core/systems/dubins.py:10-21) keep the
    reference's fields and defaults; the per-point functions refuse host tensors (no CPU fallback)."""
    import math

    import torch

    from diff_tube_mpc_strict_pt.core.barrier import DBaSConfig, relaxed_inverse_barrier_B_alpha
    from diff_tube_mpc_strict_pt.core.control import BoxClampControl
    from diff_tube_mpc_strict_pt.core.systems.dubins import DubinsConfig, dubins_step

    d = DBaSConfig()
    assert (d.barrier_type, d.alpha, d.gamma, d.eps) == ("inverse", 0.1, 0.0, 1e-6)
    c = DubinsConfig()
    assert c.dt == 0.01 and c.v_max == 10.0 and abs(c.omega_max - math.pi) < 1e-12
    assert c.w_low == (-0.05, -0.05, -0.05) and c.x_target[:2] == (10.0, 10.0)
    with pytest.raises(ValueError, match="no CPU fallback"):
        dubins_step(torch.zeros(3), torch.zeros(2), cfg=c)
    with pytest.raises(ValueError, match="no CPU fallback"):
        relaxed_inverse_barrier_B_alpha(torch.zeros(4), alpha=0.0)
    with pytest.raises(ValueError, match="no CPU fallback"):
        BoxClampControl(u_min=(-1.0, -1.0), u_max=(1.0, 1.0)).clamp(torch.zeros(2))


def test_reference_utils_semantics():
    """core.utils (core/utils.py:15-91) and core.autodiff (core/autodiff.py:9-82): plain torch helpers, checked
    here on small CPU tensors against their closed forms (the device checks: tests/test_gpu_systems.py)."""
    import torch

    from diff_tube_mpc_strict_pt.core import (compute_jacobian, grad_hess_x, grad_hess_xu,
                                              quadratic_cost_derivs_diagonal, regularize_matrix, solve_psd)

    g = torch.Generator().manual_seed(0)
    M = torch.randn(4, 4, generator=g, dtype=torch.float64)
    A = M @ M.T + 0.1 * torch.eye(4, dtype=torch.float64)
    b = torch.randn(4, 2, generator=g, dtype=torch.float64)
    assert torch.allclose(A @ solve_psd(A, b), b, atol=1e-10)
    assert torch.allclose(A @ solve_psd(A, b[:, 0]), b[:, 0], atol=1e-10)
    S = torch.zeros(3, 3, dtype=torch.float64)  # singular: the regularised LU branch
    assert torch.allclose(solve_psd(S, torch.ones(3, dtype=torch.float64), reg=0.5), torch.full((3,), 2.0, dtype=torch.float64))
    assert torch.equal(regularize_matrix(S, 0.25), 0.25 * torch.eye(3, dtype=torch.float64))
    x, u = torch.randn(4, generator=g, dtype=torch.float64), torch.randn(2, generator=g, dtype=torch.float64)
    Q, R = torch.tensor([1.0, 2.0, 3.0, 0.5], dtype=torch.float64), torch.tensor([0.1, 0.2], dtype=torch.float64)
    xr, ur = torch.randn(4, generator=g, dtype=torch.float64), torch.randn(2, generator=g, dtype=torch.float64)
    ref = quadratic_cost_derivs_diagonal(x, u, Q, R, xr, ur)
    auto = grad_hess_xu(lambda xx, uu, k: (Q * (xx - xr) ** 2).sum() + (R * (uu - ur) ** 2).sum(), x, u, 0)
    for a, r in zip(auto, ref):
        assert torch.allclose(a, r, atol=1e-12)
    gx, Hx = grad_hess_x(lambda xx: (Q * xx ** 2).sum(), x)
    assert torch.allclose(gx, 2 * Q * x) and torch.allclose(Hx, torch.diag(2 * Q))
    Ja, Jb = compute_jacobian(lambda xx, uu: torch.stack([xx[0] + uu[0] * torch.cos(xx[2]), xx[1] * uu[1]]),
                              x[:3], u)
    assert torch.allclose(Ja, torch.tensor([[1.0, 0.0, -u[0] * torch.sin(x[2])], [0.0, u[1], 0.0]], dtype=torch.float64))
    assert torch.allclose(Jb, torch.tensor([[torch.cos(x[2]), 0.0], [0.0, x[1]]], dtype=torch.float64))
