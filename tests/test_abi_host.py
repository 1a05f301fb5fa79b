"""CPU tests of the drop-in boundary and the host logic: libdtmpc.so loads and exports exactly the
symbols include/dtmpc.h declares, the ctypes structs match the C layout, argument validation happens
before any device call, and the config -> typed-problem mapping follows the reference."""
from __future__ import annotations

import ctypes as C
import glob
import math
import os
import re
import subprocess

import numpy as np
import pytest

from _common import config

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "dtmpc.h")
HEADERS = sorted(glob.glob(os.path.join(REPO, "include", "*.h")))


def header_functions() -> set:
    """Every dtmpc_* function declared in include/*.h."""
    src = "\n".join(open(h).read() for h in HEADERS)
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return set(re.findall(r"^\s*(?:const\s+)?[\w]+[\s\*]+(dtmpc_\w+)\s*\(", src, flags=re.M))


@pytest.fixture(scope="module")
def lib():
    from diff_tube_mpc_strict_pt import _lib

    return _lib.load()


def test_library_exports_every_declared_symbol(lib):
    from diff_tube_mpc_strict_pt import _abi

    declared = header_functions()
    assert len(declared) >= 15
    missing = [n for n in declared if not hasattr(lib, n)]
    assert not missing, missing
    assert declared == set(_abi.PROTOTYPES), declared ^ set(_abi.PROTOTYPES)
    out = subprocess.run(["nm", "-D", "--defined-only", os.path.join(REPO, "differentiable-tube-mpc_amd",
                                                                        "diff_tube_mpc_strict_pt", "libdtmpc.so")],
                         capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (dtmpc_\w+)", out))
    assert declared <= exported
    assert lib.dtmpc_abi_version() == _abi.ABI_VERSION


def test_struct_layouts_match_header(tmp_path):
    """sizeof / offsetof of every ABI struct, compiled from include/dtmpc.h by gcc, vs the ctypes mirror."""
    from diff_tube_mpc_strict_pt import _abi

    structs = {"dtmpc_spec": _abi.DtmpcSpec, "dtmpc_cost": _abi.DtmpcCost, "dtmpc_ilqr_cfg": _abi.DtmpcIlqrCfg,
               "dtmpc_adapt_cfg": _abi.DtmpcAdaptCfg, "dtmpc_tube_cfg": _abi.DtmpcTubeCfg,
               "dtmpc_tube_state": _abi.DtmpcTubeState}
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HEADER}"', "int main(void){"]
    for cname, py in structs.items():
        lines.append(f'printf("{cname} sizeof %zu\\n", sizeof({cname}));')
        for fname, _ in py._fields_:
            lines.append(f'printf("{cname} {fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append("return 0;}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-o", str(exe), str(src)], check=True)
    got = {}
    for line in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.splitlines():
        s, f, v = line.split()
        got[(s, f)] = int(v)
    for cname, py in structs.items():
        assert got[(cname, "sizeof")] == C.sizeof(py), cname
        for fname, _ in py._fields_:
            assert got[(cname, fname)] == getattr(py, fname).offset, (cname, fname)


def test_header_constants_match_ctypes_mirror():
    from diff_tube_mpc_strict_pt import _abi

    defines = dict(re.findall(r"^#define DTMPC_(\w+) (-?\d+)", open(HEADER).read(), flags=re.M))
    checked = 0
    for name, val in defines.items():
        if hasattr(_abi, name):
            assert getattr(_abi, name) == int(val), name
            checked += 1
    assert checked >= 5 and _abi.LOG_FIELDS == 18


def test_arguments_validated_before_any_device_call(lib):
    """Bad arguments return DTMPC_ERR_BAD_ARG with a message; no HIP call is made (safe without GPU)."""
    from diff_tube_mpc_strict_pt import _abi
    from diff_tube_mpc_strict_pt.core.problem import ILQRConfig, paper_config, paper_setup_from_config

    st = paper_setup_from_config(paper_config())
    spec, cost = st.problem.to_c(), st.nominal_cost.to_c()
    cfg = st.ilqr_nom.to_c()
    cfg.n_alphas = 0
    rc = lib.dtmpc_ilqr_solve(_abi.F32, C.byref(spec), C.byref(cost), C.byref(cfg), 4, 1, None, None, 1, 1, 1, 1, None,
                              1, None, None)
    assert rc == _abi.ERR_BAD_ARG and b"n_alphas" in lib.dtmpc_last_error()
    bad = st.problem.to_c()
    bad.dbas_gamma = 1.5
    rc = lib.dtmpc_dbas_rollout(_abi.F64, C.byref(bad), 4, 1, 1, 1, None)
    assert rc == _abi.ERR_BAD_ARG and b"gamma" in lib.dtmpc_last_error()
    track = st.nominal_cost.to_c()
    track.kind = _abi.COST_TRACK
    rc = lib.dtmpc_linearize(_abi.F32, C.byref(spec), C.byref(track), 4, 1, 1, None, None, 1, 1, 1, 1, None)
    assert rc == _abi.ERR_BAD_ARG and b"Xref" in lib.dtmpc_last_error()
    tc = _abi.DtmpcTubeCfg()
    tc.nominal = cost
    tc.nom_ilqr = st.ilqr_nom.to_c()
    tc.aux_ilqr = ILQRConfig(horizon=50, line_search_alphas=(1.0, 0.5)).to_c()
    state = _abi.DtmpcTubeState()
    rc = lib.dtmpc_tube_step(_abi.F32, C.byref(spec), C.byref(tc), 8, 0, 0, C.byref(state), None, None)
    assert rc == _abi.ERR_BAD_ARG and b"same width" in lib.dtmpc_last_error()
    # f32: the larger of the generic kernel's scratch (30 values per step) and the fast kernel's per-lane
    # records (two tapes of (N+1) x 16 B + N x 8 B, gains and sensitivity scratch of N x 40 B per
    # trajectory; four lanes: twelve tape slots per solve), for one launch chunk
    # (+ 12 B: the split step's hand-over of the nominal solve to its phase-2 launch, dtmpc_tube_state.phase, ABI 6)
    per1, per4 = 51 * 32 + 50 * 96 + 12, 12 * (51 * 32 + 50 * 16) + 50 * 80 + 12
    c1, c4 = lib.dtmpc_tube_chunk(50, 1), lib.dtmpc_tube_chunk(50, 4)
    assert c1 == (0x7FFFFFFF // per1) // 256 * 256 and c4 == (0x7FFFFFFF // per4) // 256 * 256
    assert lib.dtmpc_tube_chunk(50, 3) == 0
    assert lib.dtmpc_tube_workspace_bytes(_abi.F32, 50, 65536, 1, c1) == max(4 * 50 * 30, per1) * 65536
    assert lib.dtmpc_tube_workspace_bytes(_abi.F32, 50, 4096, 4, c4) == per4 * 4096
    # f64 (csrc/dtmpc_fast64.hip): the same records in doubles, so twice the bytes and at most half the chunk
    per1d, per4d = 2 * (per1 - 12) + 12, 2 * (per4 - 12) + 12
    c1d, c4d = (0x7FFFFFFF // per1d) // 256 * 256, (0x7FFFFFFF // per4d) // 256 * 256
    assert lib.dtmpc_tube_workspace_bytes(_abi.F64, 50, 65536, 1, c1) == max(8 * 50 * 30, per1d) * 65536
    assert lib.dtmpc_tube_workspace_bytes(_abi.F64, 50, 4096, 4, c4) == per4d * 4096
    assert lib.dtmpc_tube_workspace_bytes(_abi.F64, 50, 1 << 20, 1, c1) == max(8 * 50 * 30 * (1 << 20), per1d * c1d)
    assert lib.dtmpc_tube_workspace_bytes(_abi.F64, 50, 100000, 4, c4) == per4d * min(c4, c4d)
    # above 2^31 bytes of records the fast kernel runs in chunks: the workspace holds one chunk
    assert lib.dtmpc_tube_workspace_bytes(_abi.F32, 50, 1 << 22, 1, c1) == 4 * 50 * 30 * (1 << 22)
    assert lib.dtmpc_tube_workspace_bytes(_abi.F32, 50, 100000, 4, c4) == per4 * c4
    # a chunk no dtmpc_tube_chunk returns (too large, not a workgroup multiple) or a bad lane count: 0
    assert lib.dtmpc_tube_workspace_bytes(_abi.F32, 50, 65536, 4, c1) == 0
    assert lib.dtmpc_tube_workspace_bytes(_abi.F32, 50, 65536, 1, 1000) == 0
    assert lib.dtmpc_tube_workspace_bytes(_abi.F32, 50, 65536, 3, c1) == 0
    assert lib.dtmpc_tube_partials_count(65536, 1) == 256
    # 64-thread workgroups below the device's wave slots (65,536 on MI355X; the same without a device)
    assert lib.dtmpc_tube_partials_count(1000, 2) == 32
    assert lib.dtmpc_tube_partials_count(1000, 3) == 0
    assert lib.dtmpc_general_partials_count(1000) == 4
    assert lib.dtmpc_tube_partials_count(1000, 4) == 63
    assert lib.dtmpc_tube_lanes(65536) in (1, 2, 4) and lib.dtmpc_tube_lanes(4096) in (1, 2, 4)
    # ABI 6: the precision's rule (no device: the MI355X lane slots, 65,536) -- f32 as dtmpc_tube_lanes, f64 four
    # lanes up to a quarter of the slots, two up to half (round 6), then one
    if not os.environ.get("DTMPC_TUBE_LANES"):
        assert [lib.dtmpc_tube_lanes_dtype(b, 0) for b in (4096, 16384, 65536)] == [4, 2, 1]
        assert [lib.dtmpc_tube_lanes_dtype(b, 1) for b in (4096, 16384, 32768, 65536)] == [4, 4, 2, 1]
        assert lib.dtmpc_tube_lanes_dtype(4096, 7) == 0
    # the lane count and the partials size come from the state (resolved once by the caller)
    tc.aux_ilqr = st.ilqr_aux.to_c()
    for f in ("x", "b", "xbar", "bbar", "Xnom", "Unom", "Xaux", "Uaux", "work", "theta", "partials", "status"):
        setattr(state, f, 1)
    state.lanes, state.n_partials = 3, 1
    rc = lib.dtmpc_tube_step(_abi.F32, C.byref(spec), C.byref(tc), 8, 0, 0, C.byref(state), None, None)
    assert rc == _abi.ERR_BAD_ARG and b"lanes" in lib.dtmpc_last_error()
    state.lanes, state.n_partials = 2, 0
    rc = lib.dtmpc_tube_step(_abi.F32, C.byref(spec), C.byref(tc), 8, 0, 0, C.byref(state), None, None)
    assert rc == _abi.ERR_BAD_ARG and b"n_partials" in lib.dtmpc_last_error()
    # the chunk and the workspace size come from the state and are checked against each other (a chunk
    # changed after the workspace was sized cannot make the kernel address past it)
    state.n_partials = lib.dtmpc_tube_partials_count(8, 2)
    state.chunk, state.work_bytes = 300, 1 << 30
    rc = lib.dtmpc_tube_step(_abi.F32, C.byref(spec), C.byref(tc), 8, 0, 0, C.byref(state), None, None)
    assert rc == _abi.ERR_BAD_ARG and b"chunk" in lib.dtmpc_last_error()
    state.chunk = lib.dtmpc_tube_chunk(50, 2)
    state.work_bytes = lib.dtmpc_tube_workspace_bytes(_abi.F32, 50, 8, 2, state.chunk) - 1
    rc = lib.dtmpc_tube_step(_abi.F32, C.byref(spec), C.byref(tc), 8, 0, 0, C.byref(state), None, None)
    assert rc == _abi.ERR_BAD_ARG and b"work_bytes" in lib.dtmpc_last_error()
    assert lib.dtmpc_sensitivity_workspace_bytes(_abi.F64, 50, 10, 1) == 8 * 10 * (50 * 20 + 51 * 20)
    # the standalone fused iLQR: X / U tape slots (12 at four lanes), gains 40 B per step, references
    ip1, ip4 = (51 * 16 + 50 * 8) + 50 * 40 + 51 * 16 + 50 * 8, 12 * (51 * 16 + 50 * 8) + 50 * 40 + 51 * 16 + 50 * 8
    assert lib.dtmpc_ilqr_workspace_bytes(_abi.F32, 50, 4096, 4) == ip4 * 4096
    assert lib.dtmpc_ilqr_workspace_bytes(_abi.F32, 50, 65536, 1) == ip1 * 65536
    assert lib.dtmpc_ilqr_workspace_bytes(_abi.F32, 50, 1 << 20, 4) == ((0x7FFFFFFF // ip4) // 256 * 256) * ip4
    assert lib.dtmpc_ilqr_workspace_bytes(_abi.F32, 50, 4096, 3) == 0
    # f64 (csrc/dtmpc_fast64_ilqr.hip): the same records in doubles
    assert lib.dtmpc_ilqr_workspace_bytes(_abi.F64, 50, 4096, 4) == 2 * ip4 * 4096
    assert lib.dtmpc_ilqr_workspace_bytes(_abi.F64, 50, 65536, 0) == 2 * ip1 * 65536
    rc = lib.dtmpc_ilqr_solve_ws(_abi.F32, C.byref(spec), C.byref(cost), C.byref(st.ilqr_nom.to_c()), 4, 1, None, None,
                                 1, 1, 1, 1, None, 1, None, None, 3, None, 0, None)
    assert rc == _abi.ERR_BAD_ARG and b"lanes" in lib.dtmpc_last_error()
    rc = lib.dtmpc_ilqr_solve_ws(_abi.F32, C.byref(spec), C.byref(cost), C.byref(st.ilqr_nom.to_c()), 4, 1, None, None,
                                 1, 1, 1, 1, None, 1, None, None, 4, None, 100, None)
    assert rc == _abi.ERR_BAD_ARG and b"work_bytes" in lib.dtmpc_last_error()
    # the fused episode reset validates before launching
    rc = lib.dtmpc_tube_reset(_abi.F32, C.byref(spec), 8, None, C.byref(state), 1, 1, 1, None)
    assert rc == _abi.ERR_BAD_ARG and b"NULL" in lib.dtmpc_last_error()
    empty = _abi.DtmpcTubeState()
    rc = lib.dtmpc_tube_reset(_abi.F32, C.byref(spec), 8, 1, C.byref(empty), 1, 1, 1, None)
    assert rc == _abi.ERR_BAD_ARG and b"state" in lib.dtmpc_last_error()
    rc = lib.dtmpc_tube_reset(_abi.F32, C.byref(spec), 0, 1, C.byref(state), 1, 1, 1, None)
    assert rc == _abi.ERR_BAD_ARG


def test_split_step_gate_uses_the_precisions_chunk(lib):
    """a split step (dtmpc_tube_state.phase 1 / 2, TubeMPC overlap) keeps the nominal records of the whole
    batch in the workspace between its two launches, so B must fit ONE launch chunk of the precision -- and the f64
    records are twice as large, so its chunk is about half the f32 one.  dtmpc_tube_split_ok (ABI 7) decides it with
    the clamped chunk; dtmpc_tube_step refuses a phase != 0 launch it rejects, before any device call."""
    from diff_tube_mpc_strict_pt import _abi
    from diff_tube_mpc_strict_pt.core.problem import paper_config, paper_setup_from_config

    st = paper_setup_from_config(paper_config())
    spec = st.problem.to_c()
    tc = _abi.DtmpcTubeCfg()
    tc.nominal, tc.nom_ilqr, tc.aux_ilqr = st.nominal_cost.to_c(), st.ilqr_nom.to_c(), st.ilqr_aux.to_c()
    tc.disturbance = 1  # Philox: no injected w needed
    c1 = lib.dtmpc_tube_chunk(50, 1)  # the f32 chunk, the one TubeMPC keeps in its state in both precisions
    per1d = 2 * (51 * 32 + 50 * 96) + 12  # f64 records per trajectory at one lane (see the test above)
    c1d = (0x7FFFFFFF // per1d) // 256 * 256
    assert c1d < c1
    ok = lambda dt, B: lib.dtmpc_tube_split_ok(dt, C.byref(spec), C.byref(tc), B, 1, c1)  # noqa: E731
    for dt in (_abi.F32, _abi.F64):
        assert ok(dt, 1000) == 1 and ok(dt, 65536) == 1
    assert ok(_abi.F32, c1) == 1 and ok(_abi.F32, c1 + 1) == 0
    assert ok(_abi.F64, c1d) == 1 and ok(_abi.F64, c1d + 1) == 0 and ok(_abi.F64, c1) == 0
    # the launch refuses it (validation order: state arrays, lanes, partials, workspace, disturbance, then the phase)
    B = c1d + 256
    state = _abi.DtmpcTubeState()
    for f in ("x", "b", "xbar", "bbar", "Xnom", "Unom", "Xaux", "Uaux", "work", "theta", "partials", "status"):
        setattr(state, f, 1)
    state.lanes, state.chunk, state.phase = 1, c1, 1
    state.n_partials = lib.dtmpc_tube_partials_count(B, 1)
    state.work_bytes = lib.dtmpc_tube_workspace_bytes(_abi.F64, 50, B, 1, c1)
    rc = lib.dtmpc_tube_step(_abi.F64, C.byref(spec), C.byref(tc), B, 0, 0, C.byref(state), None, None)
    assert rc == _abi.ERR_BAD_ARG and b"split_ok" in lib.dtmpc_last_error()
    # a non-fused configuration never splits
    other = st.problem.to_c()
    other.n_obstacles = 9
    assert lib.dtmpc_tube_split_ok(_abi.F32, C.byref(other), C.byref(tc), 1000, 1, c1) == 0


def test_no_cpu_fallback():
    """The product path refuses host tensors and a missing native library, loudly."""
    import torch

    from diff_tube_mpc_strict_pt import _lib
    from diff_tube_mpc_strict_pt.core import TubeMPC, ilqr_solve
    from diff_tube_mpc_strict_pt.core.problem import paper_config, paper_setup_from_config

    st = paper_setup_from_config(paper_config())
    with pytest.raises(ValueError, match="no CPU fallback"):
        ilqr_solve(problem=st.problem, cost=st.nominal_cost, cfg=st.ilqr_nom, x0=torch.zeros(2, 4),
                   V_init=torch.zeros(2, 50, 2))
    with pytest.raises(ValueError, match="no CPU fallback"):
        TubeMPC(st, batch=4, device="cpu")
    saved_lib, saved_path = _lib._lib, _lib.LIB_PATH
    try:
        _lib._lib, _lib.LIB_PATH = None, "/nonexistent/libdtmpc.so"
        with pytest.raises(_lib.NativeLibraryError):
            _lib.load()
    finally:
        _lib._lib, _lib.LIB_PATH = saved_lib, saved_path


def test_paper_setup_follows_reference_wiring():
    """core/tube_mpc.py:674-768: inverse barrier alpha = gamma = 0, 5 smooth-min circles, reg = 1e-6 (the
    config's ilqr_reg is not used in paper mode), tol = 1e-3, theta0 = cost_auxiliary, Qf_aux = Qa."""
    from diff_tube_mpc_strict_pt.core.problem import paper_config, paper_setup_from_config, tracking_cost

    st = paper_setup_from_config(config())
    assert st == paper_setup_from_config(paper_config())
    p = st.problem
    assert (p.barrier_type, p.dbas_alpha, p.dbas_gamma, p.dbas_eps) == ("inverse", 0.0, 0.0, 1e-4)
    assert p.obs_aggregation == "smoothmin" and len(p.obstacles) == 5 and p.obs_beta == 20.0
    assert p.u_min == (-10.0, -math.pi) and p.u_max == (10.0, math.pi)
    assert st.ilqr_nom.reg == 1e-6 and st.ilqr_nom.tol == 1e-3 and st.ilqr_nom.max_iter == 10
    assert st.ilqr_aux.max_iter == 20 and len(st.ilqr_aux.line_search_alphas) == 7
    assert st.theta0 == (1.0, 1.0, 1.0, 1.0, 1.0, 1.0)
    assert st.adapt.lr_eta == 0.05 and st.adapt.momentum == 0.9
    tc = tracking_cost((1, 2, 3, 4, 5, 6))
    assert tc.Qf == tc.Q == (1.0, 2.0, 3.0) and tc.kind == "track"
    c = tc.to_c()
    assert list(c.Qf) == [1.0, 2.0, 3.0] and c.qb == 6.0


def test_problem_validation_mirrors_reference_errors():
    import dataclasses

    from diff_tube_mpc_strict_pt.core.problem import ILQRConfig, problem_from_config

    base = problem_from_config(config())
    with pytest.raises(ValueError, match="gamma"):
        dataclasses.replace(base, dbas_gamma=1.2)  # core/barrier.py:90-91
    with pytest.raises(ValueError, match="alpha"):
        dataclasses.replace(base, dbas_alpha=-0.1)  # core/barrier.py:43-44
    with pytest.raises(ValueError, match="barrier_type"):
        dataclasses.replace(base, barrier_type="quadratic")  # core/barrier.py:72
    with pytest.raises(ValueError):
        ILQRConfig(horizon=50, line_search_alphas=tuple([1.0] * 9)).to_c()
    single = problem_from_config({**config(), "environment": {"obstacle": {"center": [5, 5], "radius": 1.5}}})
    assert single.obs_aggregation == "single" and single.obstacles[0].radius == 1.5


def test_shard_range_partitions_global_batch():
    from diff_tube_mpc_strict_pt.core import shard_range

    for Bg in (1, 7, 4096, 65536, 65537):
        for W in (1, 2, 3, 8):
            if Bg < W:
                continue
            parts = [shard_range(Bg, r, W) for r in range(W)]
            assert parts[0][0] == 0 and parts[-1][1] == Bg
            assert all(parts[r][1] == parts[r + 1][0] for r in range(W - 1))
            sizes = [hi - lo for lo, hi in parts]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(10, 2, 2)


def test_philox_stream_is_keyed_by_global_index(oracle_lib):
    a = oracle_lib.philox_bits(0, 5, 3)
    assert not np.array_equal(a, oracle_lib.philox_bits(0, 6, 3))
    assert not np.array_equal(a, oracle_lib.philox_bits(0, 5, 4))
    assert not np.array_equal(a, oracle_lib.philox_bits(1, 5, 3))
    assert np.array_equal(a, oracle_lib.philox_bits(0, 5, 3))
