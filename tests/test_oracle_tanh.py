"""Pin the oracle's tanh-box restatement (oracle_tanh_cost_derivs) to the reference: BoxTanhControl.u /
du_dv_diag (core/control.py:10-35), _d2u_dv2_diag and the v-space cost derivatives
nominal_cost_derivs / auxiliary_cost_derivs (core/cost_derivs.py:16-107), on the golden vectors of
tests/golden/make_golden_tanh.py.  Also the argument checks of the C ABI entry (no device call).  CPU only.

Tolerance: f64 1e-13, f32 2e-6 relative to max(1, |reference|) (one tanhf ulp, amplified at most by the
1 - tanh^2 cancellation near saturation)."""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

from _common import golden, rel

DTYPES = [("f64", np.float64), ("f32", np.float32)]


def tanh_case(tag):
    from diff_tube_mpc_strict_pt.core.problem import DubinsDBaSProblem, QuadraticCost

    g = golden(f"tanh_{tag}")
    N = g["Vd"].shape[1]
    spec = DubinsDBaSProblem(horizon=N, u_min=tuple(g["umin"]), u_max=tuple(g["umax"])).to_c()
    nom = QuadraticCost(kind="target", Q=tuple(g["Q"]), R=tuple(g["R"]), qb=float(g["qb"]), target=tuple(g["target"]))
    aux = QuadraticCost(kind="track", Q=tuple(g["Qa"]), R=tuple(g["Ra"]), qb=float(g["qba"]))
    return g, spec, nom, aux


@pytest.mark.parametrize("tag,dt", DTYPES)
def test_oracle_tanh_cost_derivs_vs_reference(oracle_lib, tag, dt):
    g, spec, nom, aux = tanh_case(tag)
    tol = 1e-13 if dt == np.float64 else 2e-6
    o = oracle_lib.Oracle(dt)
    for cost, sfx, refs in ((nom, "nom", {}), (aux, "aux", {"Xref": g["Xr"], "Uref": g["Ur"]})):
        r = o.tanh_cost_derivs(spec, cost.to_c(), g["X"], g["Vd"], **refs)
        assert rel(r["u"], g["u"]) < tol
        assert rel(r["dudv"], g["dudv"]) < tol
        assert rel(r["lx"], g[f"lx_{sfx}"]) < tol, sfx
        assert rel(r["lv"], g[f"lv_{sfx}"]) < tol, sfx
        assert rel(r["lvv"], g[f"lvv_{sfx}"]) < tol, sfx
    # saturated point: u hits the box, du/dv = 0 (f32) or tiny (f64)
    assert abs(r["u"][0, 0, 0] - g["umax"][0]) < 1e-5 and abs(r["u"][0, 0, 1] - g["umin"][1]) < 1e-5


def test_tanh_abi_arguments_validated(oracle_lib):
    """dtmpc_tanh_cost_derivs rejects bad arguments with DTMPC_ERR_BAD_ARG before any HIP call."""
    from diff_tube_mpc_strict_pt import _abi, _lib

    lib = _lib.load()
    g, spec, nom, aux = tanh_case("f64")
    sp, cn, ca = spec, nom.to_c(), aux.to_c()
    rc = lib.dtmpc_tanh_cost_derivs(_abi.F64, C.byref(sp), C.byref(ca), 4, 1, 1, None, None, 1, 1, 1, 1, 1, None)
    assert rc == _abi.ERR_BAD_ARG and b"Xref" in lib.dtmpc_last_error()
    cw = nom.to_c()
    cw.wrap_angle = 1
    rc = lib.dtmpc_tanh_cost_derivs(_abi.F64, C.byref(sp), C.byref(cw), 4, 1, 1, None, None, 1, 1, 1, 1, 1, None)
    assert rc == _abi.ERR_BAD_ARG and b"unwrapped" in lib.dtmpc_last_error()
    rc = lib.dtmpc_tanh_cost_derivs(_abi.F64, C.byref(sp), C.byref(cn), 4, None, 1, None, None, 1, 1, 1, 1, 1, None)
    assert rc == _abi.ERR_BAD_ARG and b"NULL" in lib.dtmpc_last_error()
    rc = lib.dtmpc_tanh_cost_derivs(_abi.F64, C.byref(sp), C.byref(cn), 0, 1, 1, None, None, 1, 1, 1, 1, 1, None)
    assert rc == _abi.ERR_BAD_ARG and b"batch" in lib.dtmpc_last_error()
    rc = lib.dtmpc_tanh_cost_derivs(7, C.byref(sp), C.byref(cn), 4, 1, 1, None, None, 1, 1, 1, 1, 1, None)
    assert rc == _abi.ERR_BAD_ARG and b"dtype" in lib.dtmpc_last_error()


def test_box_controls_host_side():
    from diff_tube_mpc_strict_pt.core import BoxClampControl, BoxTanhControl, DubinsDBaSProblem

    b = BoxClampControl(u_min=(-10.0, -np.pi), u_max=(10.0, np.pi))
    p = DubinsDBaSProblem(**b.problem_bounds())
    assert p.u_max == (10.0, np.pi) and p.active_tol == 1e-8
    # any bounds, as the reference's map takes them (core/control.py:10-35 has no ordering check)
    BoxTanhControl(u_min=(1.0, 0.0), u_max=(1.0, 1.0))
    with pytest.raises(ValueError):
        BoxTanhControl(u_min=(1.0, 0.0, 2.0), u_max=(1.0, 1.0))


def test_tanh_mirror_refuses_host_tensors():
    """core.control / core.cost_derivs have no CPU fallback: host tensors raise before any launch."""
    import torch

    from diff_tube_mpc_strict_pt.core import BoxTanhControl, nominal_cost_derivs

    ctrl = BoxTanhControl(u_min=(-10.0, -np.pi), u_max=(10.0, np.pi))
    v = torch.zeros(3, 2, dtype=torch.float64)
    with pytest.raises(ValueError, match="no CPU fallback"):
        ctrl.u(v)
    with pytest.raises(ValueError, match="no CPU fallback"):
        nominal_cost_derivs(x_hat=torch.zeros(3, 4, dtype=torch.float64), v=v, target=(1.0, 1.0, 0.0),
                            Q=(1.0, 1.0, 0.0), R=(1.0, 1.0), qb=1.0, ctrl=ctrl)
