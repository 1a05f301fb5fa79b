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
