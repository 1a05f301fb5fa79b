"""ctypes mirror of include/dtmpc.h (the C ABI of libdtmpc.so).

Only plain data lives here: struct layouts, enum values and status-word decoding.  The library
loader is :mod:`diff_tube_mpc_strict_pt._lib`.
"""
from __future__ import annotations

import ctypes as C

ABI_VERSION = 7
MAX_OBS = 16
MAX_ALPHAS = 8
MAX_HORIZON = 512
LOG_FIELDS = 18
GEN_LOG_FIELDS = 12
GEN_SUMS = 25  # L, ancillary grads (11), nominal grads (12), healthy count
TUBE_SUMS = 8  # L, gQ(3), gR(2), gqb, healthy count
# raw parameter layout of the general path (include/dtmpc.h DTMPC_P_*)
P_Q, P_R, P_QF, P_QB, P_ALPHA, P_GAMMA, P_TIGHT, P_COUNT = 0, 3, 5, 8, 9, 10, 11, 12

F32, F64 = 0, 1
OBS_SMOOTHMIN, OBS_MIN, OBS_SINGLE, OBS_NONE = 0, 1, 2, 3
BARRIER_INVERSE, BARRIER_LOG = 0, 1
COST_TARGET, COST_TRACK = 0, 1
OK, ERR_BAD_ARG, ERR_HIP = 0, 3, 4
ST_NONFINITE, ST_NO_CANDIDATE = 1, 2
BARRIER_INVERSE_PLAIN = 2  # include/dtmpc_systems.h: dtmpc_barrier_eval's plain 1 / max(z, eps)

OBS_AGGREGATIONS = {"smoothmin": OBS_SMOOTHMIN, "min": OBS_MIN, "single": OBS_SINGLE, "none": OBS_NONE}
BARRIERS = {"inverse": BARRIER_INVERSE, "log": BARRIER_LOG}


class DtmpcSpec(C.Structure):
    _fields_ = [
        ("horizon", C.c_int32),
        ("n_obstacles", C.c_int32),
        ("obs_aggregation", C.c_int32),
        ("barrier_type", C.c_int32),
        ("dt", C.c_double),
        ("u_min", C.c_double * 2),
        ("u_max", C.c_double * 2),
        ("active_tol", C.c_double),
        ("obs_beta", C.c_double),
        ("obs_cx", C.c_double * MAX_OBS),
        ("obs_cy", C.c_double * MAX_OBS),
        ("obs_r", C.c_double * MAX_OBS),
        ("dbas_alpha", C.c_double),
        ("dbas_gamma", C.c_double),
        ("dbas_eps", C.c_double),
        ("h_offset", C.c_double),
    ]


class DtmpcCost(C.Structure):
    _fields_ = [
        ("kind", C.c_int32),
        ("wrap_angle", C.c_int32),
        ("Q", C.c_double * 3),
        ("R", C.c_double * 2),
        ("Qf", C.c_double * 3),
        ("qb", C.c_double),
        ("target", C.c_double * 3),
    ]


class DtmpcIlqrCfg(C.Structure):
    _fields_ = [
        ("max_iter", C.c_int32),
        ("n_alphas", C.c_int32),
        ("tol", C.c_double),
        ("reg", C.c_double),
        ("alphas", C.c_double * MAX_ALPHAS),
    ]


class DtmpcAdaptCfg(C.Structure):
    _fields_ = [
        ("lr_eta", C.c_double),
        ("momentum", C.c_double),
        ("q_min", C.c_double),
        ("r_min", C.c_double),
        ("qb_min", C.c_double),
        ("qb_max", C.c_double),
    ]


class DtmpcTubeCfg(C.Structure):
    _fields_ = [
        ("nominal", DtmpcCost),
        ("nom_ilqr", DtmpcIlqrCfg),
        ("aux_ilqr", DtmpcIlqrCfg),
        ("disturbance", C.c_int32),
        ("write_log", C.c_int32),
        ("seed", C.c_uint64),
        ("w_low", C.c_double * 3),
        ("w_high", C.c_double * 3),
        ("grad_bound", C.c_double),
    ]


class DtmpcTubeState(C.Structure):
    _fields_ = [
        ("x", C.c_void_p),
        ("b", C.c_void_p),
        ("xbar", C.c_void_p),
        ("bbar", C.c_void_p),
        ("Xnom", C.c_void_p),
        ("Unom", C.c_void_p),
        ("Xaux", C.c_void_p),
        ("Uaux", C.c_void_p),
        ("work", C.c_void_p),
        ("theta", C.c_void_p),
        ("partials", C.c_void_p),
        ("log", C.c_void_p),
        ("status", C.c_void_p),
        ("iters", C.c_void_p),
        ("lanes", C.c_int32),
        ("phase", C.c_int32),
        ("n_partials", C.c_int64),
        ("chunk", C.c_int64),
        ("work_bytes", C.c_int64),
        ("choices", C.c_void_p),
        ("costs", C.c_void_p),
    ]


class DtmpcGeneralCfg(C.Structure):
    _fields_ = [
        ("target", C.c_double * 3),
        ("nom_ilqr", DtmpcIlqrCfg),
        ("aux_ilqr", DtmpcIlqrCfg),
        ("adapt_nominal", C.c_int32),
        ("adapt_ancillary", C.c_int32),
        ("project_params", C.c_int32),
        ("disturbance", C.c_int32),
        ("write_log", C.c_int32),
        ("pad_", C.c_int32),
        ("seed", C.c_uint64),
        ("w_low", C.c_double * 3),
        ("w_high", C.c_double * 3),
        ("lr_eta", C.c_double),
        ("momentum", C.c_double),
        ("clip_norm", C.c_double),
    ]


class DtmpcGeneralState(C.Structure):
    _fields_ = [
        ("x", C.c_void_p),
        ("b", C.c_void_p),
        ("xbar", C.c_void_p),
        ("bbar", C.c_void_p),
        ("Xnom", C.c_void_p),
        ("Unom", C.c_void_p),
        ("Xaux", C.c_void_p),
        ("Uaux", C.c_void_p),
        ("work", C.c_void_p),
        ("theta", C.c_void_p),
        ("velocity", C.c_void_p),
        ("partials", C.c_void_p),
        ("sums", C.c_void_p),
        ("gout", C.c_void_p),
        ("log", C.c_void_p),
        ("status", C.c_void_p),
        ("iters", C.c_void_p),
        ("n_partials", C.c_int64),
    ]


# Exported symbols and their ctypes prototypes: (restype, argtypes).  Both the loader and the
# "library exports every declared symbol" test read this table.
P = C.c_void_p
I64 = C.c_int64
I32 = C.c_int32
PROTOTYPES = {
    "dtmpc_abi_version": (C.c_int, []),
    "dtmpc_last_error": (C.c_char_p, []),
    "dtmpc_device_count": (C.c_int, []),
    "dtmpc_dbas_rollout": (C.c_int, [C.c_int, C.POINTER(DtmpcSpec), I64, P, P, P, P]),
    "dtmpc_dbas_init": (C.c_int, [C.c_int, C.POINTER(DtmpcSpec), I64, P, P, P]),
    "dtmpc_linearize": (C.c_int, [C.c_int, C.POINTER(DtmpcSpec), C.POINTER(DtmpcCost), I64, P, P, P, P, P, P, P, P, P]),
    # include/dtmpc_control.h
    "dtmpc_tape_cost": (C.c_int, [C.c_int, C.POINTER(DtmpcSpec), C.POINTER(DtmpcCost), I64, P, P, P, P, P, P]),
    "dtmpc_tanh_cost_derivs": (
        C.c_int,
        [C.c_int, C.POINTER(DtmpcSpec), C.POINTER(DtmpcCost), I64, P, P, P, P, P, P, P, P, P, P],
    ),
    "dtmpc_ilqr_solve": (
        C.c_int,
        [C.c_int, C.POINTER(DtmpcSpec), C.POINTER(DtmpcCost), C.POINTER(DtmpcIlqrCfg), I64, P, P, P, P, P, P, P, P, P, P,
         P],
    ),
    "dtmpc_ilqr_workspace_bytes": (C.c_size_t, [C.c_int, I32, I64, I32]),
    "dtmpc_ilqr_fused_eligible": (I32, [C.c_int, C.POINTER(DtmpcSpec), C.POINTER(DtmpcCost), C.POINTER(DtmpcIlqrCfg)]),
    "dtmpc_ilqr_solve_ws": (
        C.c_int,
        [C.c_int, C.POINTER(DtmpcSpec), C.POINTER(DtmpcCost), C.POINTER(DtmpcIlqrCfg), I64, P, P, P, P, P, P, P, P, P, P,
         P, I32, P, C.c_size_t, P],
    ),
    "dtmpc_sensitivity_workspace_bytes": (C.c_size_t, [C.c_int, I32, I64, I32]),
    "dtmpc_ddp_sensitivity": (
        C.c_int,
        [C.c_int, C.POINTER(DtmpcSpec), C.POINTER(DtmpcCost), I64, P, P, P, P, P, P, P, P, P, P, P],
    ),
    "dtmpc_doc_grad": (C.c_int, [C.c_int, I32, I64, P, P, P, P, P, P, P, P]),
    "dtmpc_tube_chunk": (I64, [I32, I32]),
    "dtmpc_tube_workspace_bytes": (C.c_size_t, [C.c_int, I32, I64, I32, I64]),
    "dtmpc_tube_lanes": (I32, [I64]),
    "dtmpc_tube_lanes_dtype": (I32, [I64, C.c_int]),
    "dtmpc_tube_split_supported": (I32, [C.c_int, C.POINTER(DtmpcSpec), C.POINTER(DtmpcTubeCfg), I32]),
    "dtmpc_tube_split_ok": (I32, [C.c_int, C.POINTER(DtmpcSpec), C.POINTER(DtmpcTubeCfg), C.c_int64, I32, C.c_int64]),
    "dtmpc_tube_partials_count": (I64, [I64, I32]),
    "dtmpc_tube_step": (
        C.c_int,
        [C.c_int, C.POINTER(DtmpcSpec), C.POINTER(DtmpcTubeCfg), I64, I64, I64, C.POINTER(DtmpcTubeState), P, P],
    ),
    "dtmpc_tube_reset": (C.c_int, [C.c_int, C.POINTER(DtmpcSpec), I64, P, C.POINTER(DtmpcTubeState), P, P, P, P]),
    "dtmpc_partials_reduce": (C.c_int, [C.c_int, I64, P, P, P]),
    "dtmpc_theta_update": (C.c_int, [C.c_int, C.POINTER(DtmpcAdaptCfg), C.c_double, P, P, P, P]),
    "dtmpc_sensitivity_upper_workspace_bytes": (C.c_size_t, [C.c_int, I32, I64]),
    "dtmpc_ddp_sensitivity_upper": (
        C.c_int,
        [C.c_int, C.POINTER(DtmpcSpec), C.POINTER(DtmpcCost), I64, P, P, P, P, P, P, P, P, P, P],
    ),
    "dtmpc_ift_gradient": (
        C.c_int,
        [C.c_int, C.POINTER(DtmpcSpec), C.POINTER(DtmpcCost), C.POINTER(C.c_double), I64, P, P, P, P, P, P, P, P, P,
         P, P],
    ),
    "dtmpc_general_workspace_bytes": (C.c_size_t, [C.c_int, I32, I64]),
    "dtmpc_general_partials_count": (I64, [I64]),
    "dtmpc_general_step": (
        C.c_int, [C.c_int, C.POINTER(DtmpcSpec), C.POINTER(DtmpcGeneralCfg), I64, C.POINTER(DtmpcGeneralState), P]),
    "dtmpc_partials_reduce_n": (C.c_int, [C.c_int, I64, I32, P, P, P]),
    "dtmpc_general_update": (
        C.c_int, [C.c_int, C.POINTER(DtmpcSpec), C.POINTER(DtmpcGeneralCfg), C.c_double,
                  C.POINTER(DtmpcGeneralState), P]),
    "dtmpc_general_plant": (
        C.c_int, [C.c_int, C.POINTER(DtmpcSpec), C.POINTER(DtmpcGeneralCfg), I64, I64, I64,
                  C.POINTER(DtmpcGeneralState), P, P]),
    # include/dtmpc_systems.h
    "dtmpc_dubins_step": (C.c_int, [C.c_int, C.POINTER(DtmpcSpec), I64, I32, P, P, P, P]),
    "dtmpc_h_eval": (C.c_int, [C.c_int, C.POINTER(DtmpcSpec), I64, I32, P, P, P, P]),
    "dtmpc_barrier_eval": (C.c_int, [C.c_int, I32, C.c_double, C.c_double, I64, P, P, P, P]),
    "dtmpc_fhat": (C.c_int, [C.c_int, C.POINTER(DtmpcSpec), I64, P, P, P, P]),
    "dtmpc_aug_jac": (C.c_int, [C.c_int, C.POINTER(DtmpcSpec), I64, P, P, P, P, P]),
    "dtmpc_box_clamp": (C.c_int, [C.c_int, C.POINTER(DtmpcSpec), I64, P, P, P, P]),
    "dtmpc_cost_derivs": (C.c_int, [C.c_int, C.POINTER(DtmpcCost), I32, I64, P, P, P, P, P, P, P]),
    "dtmpc_receding_workspace_bytes": (C.c_size_t, [C.c_int, I32, I64]),
    "dtmpc_nominal_receding": (
        C.c_int, [C.c_int, C.POINTER(DtmpcSpec), C.POINTER(DtmpcCost), C.POINTER(DtmpcIlqrCfg), I64, I32, C.c_double,
                  P, P, P, P, P, P, P, P, P]),
    "dtmpc_nominal_receding_it": (
        C.c_int, [C.c_int, C.POINTER(DtmpcSpec), C.POINTER(DtmpcCost), C.POINTER(DtmpcIlqrCfg), I64, I32, C.c_double,
                  P, P, P, P, P, P, P, P, P, P]),
}


def status_messages(bits: int) -> list[str]:
    out = []
    if bits & ST_NONFINITE:
        out.append("non-finite value")
    if bits & ST_NO_CANDIDATE:
        out.append("line search failed to produce a candidate")
    return out
