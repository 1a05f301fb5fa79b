"""Shared helpers for the parity tests (golden fixtures, tolerances, problem builders)."""
from __future__ import annotations

import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")

# A golden case whose reference output moves by more than this under a few-ulp input perturbation
# (cond_* fields written by tests/golden/make_golden.py) is chaotic in the reference itself: only
# finiteness / status / cost-decrease properties are compared there.
CHAOTIC = 1e-2


def config() -> dict:
    with open(os.path.join(GOLDEN, "config.json")) as f:
        return json.load(f)


def golden(name: str):
    return np.load(os.path.join(GOLDEN, name + ".npz"))


def paper_setup():
    from diff_tube_mpc_strict_pt.core.problem import paper_setup_from_config

    return paper_setup_from_config(config())


def ilqr_cfg(max_iter: int, tol: float):
    from diff_tube_mpc_strict_pt.core.problem import ILQRConfig

    st = paper_setup()
    return ILQRConfig(horizon=st.problem.horizon, max_iter=max_iter, tol=tol,
                      line_search_alphas=st.ilqr_nom.line_search_alphas)


def rel(a, b) -> float:
    """max |a - b| / max(1, max |b|)"""
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b)) / max(1.0, float(np.max(np.abs(b)))))


def rel_rows(a, b) -> np.ndarray:
    """rel() per trajectory (leading axis)."""
    return np.array([rel(a[i], b[i]) for i in range(len(a))])


VARIANTS = ("plain", "fma", "ulp")


def oracles(npdt, nthreads: int = 8):
    """The oracle in its three builds (oracle/Makefile): plain IEEE order, FMA-contracted, and +-1 ulp on
    every transcendental result."""
    from oracle.oracle import Oracle

    return [Oracle(npdt, nthreads=nthreads, variant=v) for v in VARIANTS]


def agreement(dev_out, outs, base: float, k: float = 10.0):
    """Per-trajectory agreement of a device result with the oracle.

    outs = results of the three oracle builds (plain, fma, ulp).  Valid evaluations of the same algorithm
    already differ by s_i = max(|fma - plain|, |ulp - plain|) on trajectory i (line-search near-ties,
    tol-exit knife edges, trajectories grazing an obstacle where B' = -1/h^2 reaches 1e8).  The device
    result is accepted when it is within max(base, k * s_i) of one of the builds.
    Returns (fraction ok, per-trajectory errors, spreads)."""
    e = np.min(np.stack([rel_rows(dev_out, o) for o in outs]), axis=0)
    s = np.max(np.stack([rel_rows(o, outs[0]) for o in outs[1:]]), axis=0)
    return float(np.mean(e <= np.maximum(base, k * s))), e, s


def tol_for(dtype, cond: float) -> float:
    """Comparison tolerance from the reference's own conditioning on that case."""
    base = 1e-9 if np.dtype(dtype) == np.float64 else 2e-3
    return max(base, 100.0 * float(cond))


def active_set(U, u_min=(-10.0, -np.pi), u_max=(10.0, np.pi), tol: float = 1e-8):
    """BoxClampControl.active_mask (core/control.py:66-70) of plans U [..., 2]."""
    U = np.asarray(U, np.float64)
    lo, hi = np.asarray(u_min, np.float64), np.asarray(u_max, np.float64)
    return (U <= lo + tol) | (U >= hi - tol)


def decision_agreement(dev_ch, oracle_chs, dev_U=None, oracle_Us=None, label: str = "", show: int = 6):
    """Decision record agreement.  dev_ch / oracle_chs: per trajectory the sequence of
    winning line-search alpha positions ([B, I] int, -1 = iteration not run) of the device and of each
    oracle build; dev_U / oracle_Us: final plans [B, N, 2] whose active sets (core/control.py:66-70) are
    compared too.  Near-ties of the line-search costs make the decision rounding-dependent, so the
    oracle builds (same algorithm, three roundings) disagree among themselves on part of the batch; the
    gate is therefore taken on the DETERMINATE trajectories -- those on which all builds agree -- where
    the device must make the same decisions, and the overall rate (device = at least one build) is
    reported beside the builds' own mutual agreement.  Prints a summary and the first disagreements."""
    dev_ch = np.asarray(dev_ch)
    chs = [np.asarray(c) for c in oracle_chs]
    B = dev_ch.shape[0]
    eq = np.stack([(dev_ch == c).all(1) for c in chs])  # [builds, B]
    det = np.stack([(c == chs[0]).all(1) for c in chs[1:]]).all(0)
    ok_any = eq.any(0)
    if dev_U is not None:
        da = active_set(dev_U).reshape(B, -1)
        acts = [active_set(u).reshape(B, -1) for u in oracle_Us]
        aeq = np.stack([(da == a).all(1) for a in acts])
        det = det & np.stack([(a == acts[0]).all(1) for a in acts[1:]]).all(0)
        ok_any = ok_any & (eq & aeq).any(0)
        eq0 = eq[0] & aeq[0]
    else:
        eq0 = eq[0]
    n_det = int(det.sum())
    res = {"n": int(B), "determinate": n_det / B, "on_determinate": float(eq0[det].mean()) if n_det else 1.0,
           "overall": float(ok_any.mean()), "oracle_builds_agree": n_det / B}
    bad = np.nonzero(det & ~eq0)[0]
    res["disagree_determinate"] = bad.tolist()
    print(f"[decisions{(' ' + label) if label else ''}] B={B}: alpha sequence"
          + (" + active set" if dev_U is not None else "")
          + f" -- on the {n_det} determinate trajectories (all oracle builds agree) {res['on_determinate']:.4f}; "
          f"overall (device = one of the builds) {res['overall']:.4f}; {len(bad)} determinate disagreements")
    for i in bad[:show]:
        print(f"    traj {i}: device {dev_ch[i].tolist()} oracle {chs[0][i].tolist()}")
    return res
