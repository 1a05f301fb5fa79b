"""Typed problem description consumed by the HIP kernels.

The reference hands its solver Python closures (core/tube_mpc.py:814-957).  A GPU kernel cannot call
a closure, so this module captures exactly what those closures compute as plain data:

* Dubins dynamics + DBaS barrier state + circle obstacles  -> :class:`DubinsDBaSProblem`
  (core/systems/dubins.py, core/barrier.py, core/systems/dubins_obstacles.py,
  core/systems/dubins_aug_jac.py)
* diagonal quadratic nominal / tracking costs              -> :class:`QuadraticCost`
  (core/cost_derivs.py, core/tube_mpc.py:823-894, run_nominal.py:297-324)
* iLQR settings                                            -> :class:`ILQRConfig` (core/ddp.py:12-20)
* Algorithm-2 adaptation                                    -> :class:`AdaptConfig` (core/tube_mpc.py:746-752, 978-984)

:func:`paper_setup_from_config` reproduces the paper-mode wiring of core/tube_mpc.py:674-768.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Any, Dict, Optional, Sequence, Tuple

from .. import _abi


@dataclass(frozen=True)
class CircleObstacle:
    """core/systems/dubins_obstacles.py:10-13"""

    center: Tuple[float, float]
    radius: float


@dataclass(frozen=True)
class DubinsDBaSProblem:
    horizon: int = 50
    dt: float = 0.01
    u_min: Tuple[float, float] = (-10.0, -math.pi)
    u_max: Tuple[float, float] = (10.0, math.pi)
    obstacles: Tuple[CircleObstacle, ...] = ()
    obs_beta: float = 20.0
    obs_aggregation: str = "smoothmin"  # smoothmin | min | single | none
    barrier_type: str = "inverse"  # inverse (relaxed B_alpha) | log
    dbas_alpha: float = 0.0
    dbas_gamma: float = 0.0
    dbas_eps: float = 1e-4
    active_tol: float = 1e-8

    def __post_init__(self) -> None:
        if not (1 <= self.horizon <= _abi.MAX_HORIZON):
            raise ValueError(f"horizon must be in [1, {_abi.MAX_HORIZON}]")
        if len(self.obstacles) > _abi.MAX_OBS:
            raise ValueError(f"at most {_abi.MAX_OBS} obstacles")
        if self.obs_aggregation not in _abi.OBS_AGGREGATIONS:
            raise ValueError(f"unknown obstacle aggregation {self.obs_aggregation!r}")
        if self.barrier_type not in _abi.BARRIERS:
            raise ValueError(f"Unknown barrier_type: {self.barrier_type}")  # core/barrier.py:72
        if self.dbas_alpha < 0:
            raise ValueError("alpha must be >= 0")  # core/barrier.py:43-44
        if not (-1.0 <= self.dbas_gamma <= 1.0):
            raise ValueError("gamma must be in [-1, 1]")  # core/barrier.py:90-91

    def to_c(self) -> _abi.DtmpcSpec:
        s = _abi.DtmpcSpec()
        s.horizon = int(self.horizon)
        s.n_obstacles = len(self.obstacles)
        s.obs_aggregation = _abi.OBS_AGGREGATIONS[self.obs_aggregation]
        s.barrier_type = _abi.BARRIERS[self.barrier_type]
        s.dt = float(self.dt)
        s.u_min[0], s.u_min[1] = (float(v) for v in self.u_min)
        s.u_max[0], s.u_max[1] = (float(v) for v in self.u_max)
        s.active_tol = float(self.active_tol)
        s.obs_beta = float(self.obs_beta)
        for i, o in enumerate(self.obstacles):
            s.obs_cx[i] = float(o.center[0])
            s.obs_cy[i] = float(o.center[1])
            s.obs_r[i] = float(o.radius)
        s.dbas_alpha = float(self.dbas_alpha)
        s.dbas_gamma = float(self.dbas_gamma)
        s.dbas_eps = float(self.dbas_eps)
        return s


@dataclass(frozen=True)
class QuadraticCost:
    """kind='target': sum Q (x - target)^2 + R u^2 + qb b^2, terminal Qf.
    kind='track': sum Q (x - x_ref_k)^2 + R (u - u_ref_k)^2 + qb b^2, terminal Qf."""

    kind: str = "target"
    Q: Tuple[float, float, float] = (1.0, 1.0, 0.0)
    R: Tuple[float, float] = (1.0, 1.0)
    Qf: Tuple[float, float, float] = (1000.0, 1000.0, 1000.0)
    qb: float = 1.0
    target: Tuple[float, float, float] = (0.0, 0.0, 0.0)
    wrap_angle: bool = False

    def to_c(self) -> _abi.DtmpcCost:
        c = _abi.DtmpcCost()
        if self.kind not in ("target", "track"):
            raise ValueError(f"unknown cost kind {self.kind!r}")
        c.kind = _abi.COST_TARGET if self.kind == "target" else _abi.COST_TRACK
        c.wrap_angle = 1 if self.wrap_angle else 0
        for i in range(3):
            c.Q[i] = float(self.Q[i])
            c.Qf[i] = float(self.Qf[i])
            c.target[i] = float(self.target[i])
        c.R[0], c.R[1] = float(self.R[0]), float(self.R[1])
        c.qb = float(self.qb)
        return c


@dataclass(frozen=True)
class ILQRConfig:
    """core/ddp.py:12-20 (same fields and defaults)."""

    horizon: int
    nx: int = 4
    nu: int = 2
    max_iter: int = 30
    tol: float = 1e-6
    reg: float = 1e-6
    line_search_alphas: Tuple[float, ...] = (1.0, 0.5, 0.25, 0.1)

    def to_c(self) -> _abi.DtmpcIlqrCfg:
        if not (1 <= len(self.line_search_alphas) <= _abi.MAX_ALPHAS):
            raise ValueError(f"1..{_abi.MAX_ALPHAS} line-search alphas supported")
        c = _abi.DtmpcIlqrCfg()
        c.max_iter = int(self.max_iter)
        c.n_alphas = len(self.line_search_alphas)
        c.tol = float(self.tol)
        c.reg = float(self.reg)
        for i, a in enumerate(self.line_search_alphas):
            c.alphas[i] = float(a)
        return c


@dataclass(frozen=True)
class AdaptConfig:
    lr_eta: float = 1e-2
    momentum: float = 0.9
    q_min: float = 0.0
    r_min: float = 1e-4
    qb_min: float = 0.0
    qb_max: float = 1.0

    def to_c(self) -> _abi.DtmpcAdaptCfg:
        c = _abi.DtmpcAdaptCfg()
        c.lr_eta, c.momentum = float(self.lr_eta), float(self.momentum)
        c.q_min, c.r_min, c.qb_min, c.qb_max = float(self.q_min), float(self.r_min), float(self.qb_min), float(self.qb_max)
        return c


@dataclass(frozen=True)
class PaperSetup:
    """Everything core/tube_mpc.py:674-768 derives from the config in paper mode."""

    problem: DubinsDBaSProblem
    nominal_cost: QuadraticCost
    theta0: Tuple[float, ...]  # Qa(3), Ra(2), qba
    ilqr_nom: ILQRConfig
    ilqr_aux: ILQRConfig
    adapt: AdaptConfig
    w_low: Tuple[float, float, float]
    w_high: Tuple[float, float, float]
    x0: Tuple[float, float, float] = (0.0, 0.0, math.pi / 4)
    use_float64: bool = False
    task_horizon: int = 300


def problem_from_config(cfg: Dict[str, Any], *, barrier_type: Optional[str] = None,
                        alpha: Optional[float] = None, gamma: Optional[float] = None) -> DubinsDBaSProblem:
    """System + environment + DBaS part of the config (core/tube_mpc.py:680-712, run_nominal.py:231-273)."""
    sc = cfg["system"]
    env = cfg.get("environment", {})
    beta = float(env.get("obstacle_smoothmin_beta", 20.0))
    agg = str(env.get("obstacle_aggregation", "min"))
    if "obstacles" in env:
        obs = tuple(CircleObstacle(center=tuple(o["center"]), radius=float(o["radius"])) for o in env["obstacles"])
        agg = "smoothmin" if agg == "smoothmin" else "min"
    else:
        o = env.get("obstacle", {"center": [5.0, 5.0], "radius": 1.5})
        obs = (CircleObstacle(center=tuple(o["center"]), radius=float(o["radius"])),)
        agg = "single"
    cb = sc["control_bounds"]
    v_max = float(cb["v_max"])
    om = float(cb.get("omega_max", math.pi))
    v_min = float(cb.get("v_min", -v_max))
    db = cfg.get("dbas", {})
    return DubinsDBaSProblem(
        horizon=int(sc["horizon_N"]),
        dt=float(sc["dt"]),
        u_min=(v_min, -om),
        u_max=(v_max, om),
        obstacles=obs,
        obs_beta=beta,
        obs_aggregation=agg,
        barrier_type=barrier_type if barrier_type is not None else str(db.get("barrier_type", "inverse")),
        dbas_alpha=float(db.get("alpha", 0.0)) if alpha is None else float(alpha),
        dbas_gamma=float(db.get("gamma", 0.0)) if gamma is None else float(gamma),
        dbas_eps=float(db.get("eps", 1e-6)),
    )


def paper_setup_from_config(cfg: Dict[str, Any]) -> PaperSetup:
    """Paper-aligned Dubins setting (core/tube_mpc.py:666-768): inverse barrier with alpha = gamma = 0,
    fixed nominal weights, ancillary weights initialised from ``cost_auxiliary``, reg = 1e-6
    (ILQRConfig default; the config's ilqr_reg is not used in this mode), tol = 1e-3."""
    sc = cfg["system"]
    problem = problem_from_config(cfg, barrier_type="inverse", alpha=0.0, gamma=0.0)
    cn = cfg["cost_nominal"]
    nominal = QuadraticCost(
        kind="target",
        Q=tuple(float(v) for v in cn["Q"]),
        R=tuple(float(v) for v in cn["R"]),
        Qf=tuple(float(v) for v in cn["Qf"]),
        qb=float(cn["q_b"]),
        target=tuple(float(v) for v in sc["target"]),
    )
    ac = cfg.get("cost_auxiliary", {})
    Qa = tuple(float(v) for v in ac["Q"]) if "Q" in ac else (1.0, 1.0, 1.0)
    Ra = tuple(float(v) for v in ac["R"]) if "R" in ac else (1.0, 1.0)
    qba = float(ac["q_b"]) if "q_b" in ac else 1.0
    ad = cfg.get("adaptation", {})
    alphas = tuple(float(a) for a in sc.get("line_search_alphas", [1.0]))
    N = int(sc["horizon_N"])
    dist = sc.get("disturbance", {})
    return PaperSetup(
        problem=problem,
        nominal_cost=nominal,
        theta0=Qa + Ra + (qba,),
        ilqr_nom=ILQRConfig(horizon=N, max_iter=int(sc.get("nominal_max_iter", 10)), tol=1e-3, line_search_alphas=alphas),
        ilqr_aux=ILQRConfig(horizon=N, max_iter=int(sc.get("aux_max_iter", 10)), tol=1e-3, line_search_alphas=alphas),
        adapt=AdaptConfig(lr_eta=float(ad.get("lr_eta", 1e-2)), momentum=float(ad.get("momentum", 0.9))),
        w_low=tuple(float(v) for v in dist.get("w_low", (-0.05, -0.05, -0.05))),
        w_high=tuple(float(v) for v in dist.get("w_high", (0.05, 0.05, 0.05))),
        use_float64=bool(cfg.get("use_float64", False)),
        task_horizon=int(sc.get("task_horizon_H", 300)),
    )


def paper_config() -> Dict[str, Any]:
    """The experiment configuration of the reference (values of configs/dubins.yaml:1-85), as a dict
    in the same schema run_closed_loop_experiment reads (core/tube_mpc.py:48-181, 674-768)."""
    return {
        "seed": 0,
        "device": "cuda",
        "use_float64": True,
        "paper_dubins_mode": True,
        "system": {
            "name": "dubins", "dt": 0.01, "horizon_N": 50, "task_horizon_H": 300,
            "nominal_max_iter": 10, "aux_max_iter": 20, "ilqr_reg": 1.0e-3,
            "line_search_alphas": [1.0, 0.5, 0.25, 0.1, 0.05, 0.01, 0.0],
            "control_bounds": {"v_min": -10.0, "v_max": 10.0, "omega_max": math.pi},
            "disturbance": {"w_low": [-0.05, -0.05, -0.05], "w_high": [0.05, 0.05, 0.05]},
            "target": [10.0, 10.0, math.pi / 4],
        },
        "dbas": {"barrier_type": "inverse", "alpha": 0.0, "gamma": 0.0, "nominal_tightening": 0.0, "eps": 1.0e-4},
        "environment": {
            "obstacles": [{"center": c, "radius": 1.0} for c in ([4.0, 2.0], [2.0, 4.0], [4.0, 8.0], [8.0, 4.0], [6.0, 6.0])],
            "obstacle_smoothmin_beta": 20.0,
            "obstacle_aggregation": "smoothmin",
        },
        "cost_nominal": {"Q": [1.0, 1.0, 0.0], "R": [1.0, 1.0], "q_b": 1.0, "Qf": [1000.0, 1000.0, 1000.0]},
        "cost_auxiliary": {"Q": [1.0, 1.0, 1.0], "R": [1.0, 1.0], "q_b": 1.0},
        "adaptation": {"lr_eta": 5.0e-2, "steps": 1, "momentum": 0.9, "adapt_nominal": False,
                       "adapt_ancillary": True, "project_params": True},
    }


def tracking_cost(theta: Sequence[float]) -> QuadraticCost:
    """Ancillary tracking cost with weights theta = (Qa, Ra, qba); terminal weight Qa
    (core/tube_mpc.py:875-894)."""
    Q = tuple(float(v) for v in theta[:3])
    return QuadraticCost(kind="track", Q=Q, R=(float(theta[3]), float(theta[4])), Qf=Q, qb=float(theta[5]))


# ---------------------------------------------------------------------------------------------
# general (softplus / tanh parameterised) path, core/tube_mpc.py:40-663

@dataclass(frozen=True)
class GeneralSetup:
    """Everything core/tube_mpc.py:48-188 derives from the config on the general path.

    theta0 is the [2][12] raw parameter block of include/dtmpc.h (DTMPC_P_* layout): row 0 the
    ancillary AuxiliaryTheta (Q, R, Qf, q_b, alpha, gamma; tight slot unused), row 1 the nominal
    NominalTheta (+ tight).  Both start from cost_nominal's raw weights (:111-131; the ancillary
    q_b from cost_auxiliary.q_b when given) and the DBaS alpha / gamma / nominal_tightening."""

    problem: DubinsDBaSProblem        # system + obstacles + barrier type + eps (alpha/gamma from theta)
    target: Tuple[float, float, float]
    theta0: Tuple[Tuple[float, ...], Tuple[float, ...]]
    ilqr_nom: ILQRConfig
    ilqr_aux: ILQRConfig
    adapt_nominal: bool
    adapt_ancillary: bool
    lr_eta: float
    momentum: float
    clip_norm: float
    project_params: bool
    w_low: Tuple[float, float, float]
    w_high: Tuple[float, float, float]
    x0: Tuple[float, float, float] = (0.0, 0.0, math.pi / 4)
    use_float64: bool = False
    task_horizon: int = 300
    adapt_steps: int = 1

    def to_c(self, *, disturbance: int = 0, seed: int = 0, write_log: bool = False) -> _abi.DtmpcGeneralCfg:
        c = _abi.DtmpcGeneralCfg()
        for i in range(3):
            c.target[i] = float(self.target[i])
            c.w_low[i] = float(self.w_low[i])
            c.w_high[i] = float(self.w_high[i])
        c.nom_ilqr = self.ilqr_nom.to_c()
        c.aux_ilqr = self.ilqr_aux.to_c()
        c.adapt_nominal = 1 if self.adapt_nominal else 0
        c.adapt_ancillary = 1 if self.adapt_ancillary else 0
        c.project_params = 1 if self.project_params else 0
        c.disturbance = int(disturbance)
        c.write_log = 1 if write_log else 0
        c.seed = int(seed) & ((1 << 64) - 1)
        c.lr_eta = float(self.lr_eta)
        c.momentum = float(self.momentum)
        c.clip_norm = float(self.clip_norm)
        return c


def general_setup_from_config(cfg: Dict[str, Any]) -> GeneralSetup:
    """General-path wiring of core/tube_mpc.py:48-188."""
    sc = cfg["system"]
    env = cfg.get("environment", {})
    if "obstacles" not in env and "obstacle" not in env:
        # the reference mixes h = 1 in the dynamics with a (5, 5, 1.5) circle in the Jacobian here
        # (core/tube_mpc.py:82-84); that combination has no typed equivalent
        raise NotImplementedError("the general path needs an obstacle set ('obstacles' or 'obstacle')")
    problem = problem_from_config(cfg, alpha=0.0, gamma=0.0)
    db = cfg["dbas"]
    cn = cfg["cost_nominal"]
    Q0 = tuple(float(v) for v in cn["Q"])
    R0 = tuple(float(v) for v in cn["R"])
    Qf0 = tuple(float(v) for v in cn["Qf"])
    qb0 = float(cn["q_b"])
    qb_aux0 = float(cfg.get("cost_auxiliary", {}).get("q_b", qb0))
    a0, g0, s0 = float(db["alpha"]), float(db["gamma"]), float(db.get("nominal_tightening", 0.0))
    aux = Q0 + R0 + Qf0 + (qb_aux0, a0, g0, 0.0)
    nom = Q0 + R0 + Qf0 + (qb0, a0, g0, s0)
    ad = cfg.get("adaptation", {})
    N = int(sc["horizon_N"])
    reg = float(sc.get("ilqr_reg", 1e-6))
    dist = sc.get("disturbance", {})
    return GeneralSetup(
        problem=problem,
        target=tuple(float(v) for v in sc["target"]),
        theta0=(aux, nom),
        # ILQRConfig(horizon, nx, nu, max_iter, reg): tol and line-search alphas keep the dataclass
        # defaults (core/tube_mpc.py:161-162, core/ddp.py:12-20)
        ilqr_nom=ILQRConfig(horizon=N, max_iter=int(sc.get("nominal_max_iter", 10)), reg=reg),
        ilqr_aux=ILQRConfig(horizon=N, max_iter=int(sc.get("aux_max_iter", 10)), reg=reg),
        adapt_nominal=bool(ad.get("adapt_nominal", True)),
        adapt_ancillary=bool(ad.get("adapt_ancillary", True)),
        lr_eta=float(ad.get("lr_eta", 1e-3)),
        momentum=float(ad.get("momentum", 0.0)),
        clip_norm=float(ad.get("grad_clip_norm", 0.0)),
        project_params=bool(ad.get("project_params", False)),
        w_low=tuple(float(v) for v in dist.get("w_low", (-0.05, -0.05, -0.05))),
        w_high=tuple(float(v) for v in dist.get("w_high", (0.05, 0.05, 0.05))),
        use_float64=bool(cfg.get("use_float64", False)),
        task_horizon=int(sc.get("task_horizon_H", 300)),
        adapt_steps=int(ad.get("steps", 1)),
    )


def softplus(x: float) -> float:
    """torch.nn.functional.softplus (beta 1, threshold 20), core/params.py:9-11"""
    return x if x > 20.0 else math.log1p(math.exp(x))
