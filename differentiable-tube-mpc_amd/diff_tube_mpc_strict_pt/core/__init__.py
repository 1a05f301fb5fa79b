"""Core API: typed problem (problem), batched DDP/IFT entry points (ddp), closed loop (tube_mpc),
control parameterisations (control) and tanh-box cost derivatives (cost_derivs); the reference's autograd
fallbacks (autodiff) and helpers (utils) under its own names (/root/reference core/__init__.py:22-31)."""
from .autodiff import compute_jacobian, grad_hess_x, grad_hess_xu
from .control import BoxClampControl, BoxTanhControl, tanh_box_eval
from .cost_derivs import auxiliary_cost_derivs, nominal_cost_derivs
from .ddp import (
    ILQRResult,
    SensitivityResult,
    dbas_init,
    ddp_sensitivity,
    doc_gradient,
    ilqr_solve,
    linearize,
    raise_for_status,
    rollout,
)
from .ift import IFTGradient, IFTInputs, ift_gradient
from .params import AuxiliaryTheta, NominalTheta, theta_from_raw
from .problem import (
    AdaptConfig,
    CircleObstacle,
    DubinsDBaSProblem,
    GeneralSetup,
    ILQRConfig,
    PaperSetup,
    QuadraticCost,
    general_setup_from_config,
    paper_setup_from_config,
    problem_from_config,
    tracking_cost,
)
from .receding import RecedingResult, nominal_receding, receding_setup_from_config
from .utils import quadratic_cost_derivs_diagonal, regularize_matrix, solve_psd
from .tube_mpc import ExperimentTrajectories, GeneralTubeMPC, TubeMPC, allreduce_sums, run_closed_loop_experiment, shard_range

__all__ = [
    "compute_jacobian",
    "grad_hess_x",
    "grad_hess_xu",
    "quadratic_cost_derivs_diagonal",
    "regularize_matrix",
    "solve_psd",
    "BoxClampControl",
    "BoxTanhControl",
    "auxiliary_cost_derivs",
    "nominal_cost_derivs",
    "tanh_box_eval",
    "AdaptConfig",
    "AuxiliaryTheta",
    "GeneralSetup",
    "GeneralTubeMPC",
    "IFTGradient",
    "IFTInputs",
    "NominalTheta",
    "general_setup_from_config",
    "RecedingResult",
    "nominal_receding",
    "receding_setup_from_config",
    "ift_gradient",
    "theta_from_raw",
    "CircleObstacle",
    "DubinsDBaSProblem",
    "ExperimentTrajectories",
    "ILQRConfig",
    "ILQRResult",
    "PaperSetup",
    "QuadraticCost",
    "SensitivityResult",
    "TubeMPC",
    "allreduce_sums",
    "dbas_init",
    "ddp_sensitivity",
    "doc_gradient",
    "ilqr_solve",
    "linearize",
    "paper_setup_from_config",
    "problem_from_config",
    "raise_for_status",
    "rollout",
    "run_closed_loop_experiment",
    "shard_range",
    "tracking_cost",
]
