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
             "ift_gradient"],
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
