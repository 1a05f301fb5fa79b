"""Pin the oracle's tape cost (oracle_tape_cost, the typed stage / terminal costs the solvers price
candidates with) to the reference's core/ocp.py:63-85 `total_cost` driven by the paper's cost closures
(core/tube_mpc.py:823-832, 875-885) -- golden vectors of tests/golden/make_golden_ocp.py.  CPU only.

Tolerance: f64 1e-13, f32 1e-6 relative (a 50-term f32 sum of costs of order 1e5)."""
from __future__ import annotations

import numpy as np
import pytest

from _common import golden

DTYPES = [("f64", np.float64), ("f32", np.float32)]


def ocp_case(tag):
    from diff_tube_mpc_strict_pt.core.problem import DubinsDBaSProblem, QuadraticCost

    g = golden(f"ocp_{tag}")
    N = g["U"].shape[1]
    spec = DubinsDBaSProblem(horizon=N).to_c()
    nom = QuadraticCost(kind="target", Q=tuple(g["Qn"]), R=tuple(g["Rn"]), Qf=tuple(g["Qfn"]), qb=float(g["qbn"]),
                        target=tuple(g["target"]))
    aux = QuadraticCost(kind="track", Q=tuple(g["Qa"]), R=tuple(g["Ra"]), Qf=tuple(g["Qa"]), qb=float(g["qba"]))
    return g, spec, nom, aux


@pytest.mark.parametrize("tag,dt", DTYPES)
def test_oracle_tape_cost_vs_reference(oracle_lib, tag, dt):
    g, spec, nom, aux = ocp_case(tag)
    tol = 1e-13 if dt == np.float64 else 1e-6
    o = oracle_lib.Oracle(dt)
    J = o.tape_cost(spec, nom.to_c(), g["X"], g["U"])
    np.testing.assert_allclose(J, g["J_nom"], rtol=tol)
    J = o.tape_cost(spec, aux.to_c(), g["X"], g["U"], Xref=g["Xr"], Uref=g["Ur"])
    np.testing.assert_allclose(J, g["J_aux"], rtol=tol)
    assert abs(float(g["J_one"]) - float(g["J_nom"][2])) <= tol * abs(float(g["J_one"]))


def test_tape_cost_abi_arguments_validated():
    """dtmpc_tape_cost rejects bad arguments with DTMPC_ERR_BAD_ARG before any HIP call."""
    import ctypes as C

    from diff_tube_mpc_strict_pt import _abi, _lib

    lib = _lib.load()
    g, spec, nom, aux = ocp_case("f64")
    sp, cn, ca = spec, nom.to_c(), aux.to_c()
    rc = lib.dtmpc_tape_cost(_abi.F64, C.byref(sp), C.byref(ca), 4, 1, 1, None, None, 1, None)
    assert rc == _abi.ERR_BAD_ARG and b"Xref" in lib.dtmpc_last_error()
    rc = lib.dtmpc_tape_cost(_abi.F64, C.byref(sp), C.byref(cn), 4, 1, 1, None, None, None, None)
    assert rc == _abi.ERR_BAD_ARG and b"NULL" in lib.dtmpc_last_error()
    rc = lib.dtmpc_tape_cost(_abi.F64, C.byref(sp), C.byref(cn), 0, 1, 1, None, None, 1, None)
    assert rc == _abi.ERR_BAD_ARG and b"batch" in lib.dtmpc_last_error()
    rc = lib.dtmpc_tape_cost(9, C.byref(sp), C.byref(cn), 4, 1, 1, None, None, 1, None)
    assert rc == _abi.ERR_BAD_ARG and b"dtype" in lib.dtmpc_last_error()


def test_ocp_host_side_checks():
    """core.ocp refuses host tensors (no CPU fallback) and mismatched horizons before any launch."""
    import torch

    from diff_tube_mpc_strict_pt.core import DubinsDBaSProblem, QuadraticCost
    from diff_tube_mpc_strict_pt.core.ocp import rollout_dynamics, total_cost

    X = torch.zeros(2, 6, 4)
    U = torch.zeros(2, 5, 2)
    with pytest.raises(ValueError, match="no CPU fallback"):
        total_cost(X=X, U=U, cost=QuadraticCost())
    with pytest.raises(ValueError, match="horizon"):
        rollout_dynamics(X[:, 0], U, f=DubinsDBaSProblem(horizon=7))
