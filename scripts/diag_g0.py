"""Diagnostic (GPU): where do configurations of the fast tube step differ?  usage:
  python scripts/diag_g0.py run OUT.npz "G0=1,L=1"     one and two closed-loop steps of a B = 700 batch (f32;
                                                      "DT=f64" for f64; "SEED=5" the start states' seed) under DTMPC_FAST_G0 / DTMPC_TUBE_LANES /
                                                      DTMPC_FAST64 ("F64=0": the generic f64 kernel) and the
                                                      library named by DTMPC_LIBRARY, saved
  python scripts/diag_g0.py cmp BASE.npz A.npz ...    per state array: bitwise equal or the max difference"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "differentiable-tube-mpc_amd"), os.path.join(REPO, "tests")]
NAMES = ("x", "b", "xbar", "bbar", "Xnom", "Unom", "Xaux", "Uaux", "log", "theta", "status", "iters")


def run(out, cfg):
    import dataclasses

    import torch

    dt_name = "f32"
    seed = 6
    for kv in cfg.split(","):
        k, v = kv.split("=")
        if k == "DT":
            dt_name = v
            continue
        if k == "SEED":
            seed = int(v)
            continue
        os.environ[{"G0": "DTMPC_FAST_G0", "L": "DTMPC_TUBE_LANES", "F64": "DTMPC_FAST64"}[k]] = v
    from _common import paper_setup
    from diff_tube_mpc_strict_pt.core import TubeMPC

    st = paper_setup()
    st = dataclasses.replace(st, ilqr_nom=dataclasses.replace(st.ilqr_nom, tol=-1.0),
                             ilqr_aux=dataclasses.replace(st.ilqr_aux, tol=-1.0))
    B = 700
    rng = np.random.default_rng(seed)
    tdt = torch.float32 if dt_name == "f32" else torch.float64
    x = torch.tensor(np.stack([rng.uniform(0, 1, B), rng.uniform(0, 1, B), rng.uniform(0, np.pi / 2, B)], 1),
                     dtype=tdt)
    m = TubeMPC(st, batch=B, device="cuda", dtype=tdt, disturbance="philox", seed=4, write_log=True)
    m.reset(x.cuda())
    res = {}
    for s in range(2):
        m.step()
        torch.cuda.synchronize()
        for k in NAMES:
            res[f"{k}_{s}"] = getattr(m, k).cpu().numpy()
    np.savez(out, **res)


def cmp(base, others):
    b = np.load(base)
    for o in others:
        d = np.load(o)
        for s in range(2):
            diffs = []
            for k in NAMES:
                A, Bv = b[f"{k}_{s}"], d[f"{k}_{s}"]
                if not np.array_equal(A, Bv, equal_nan=True):
                    e = np.abs(A.astype(np.float64) - Bv.astype(np.float64))
                    if e.ndim > 1:  # trajectories off by more than 1e-8 of their own scale
                        r = (e.reshape(-1, e.shape[-1]).max(0) /
                             (np.abs(A.astype(np.float64)).reshape(-1, e.shape[-1]).max(0) + 1e-30))
                        far = f" traj>1e-8: {int((r > 1e-8).sum())}/{r.size}"
                    else:
                        far = ""
                    diffs.append(f"{k}: max {np.nanmax(e):.2e} n={int((e > 0).sum())}{far}")
            print(f"{os.path.basename(base)} vs {os.path.basename(o)} step {s + 1}: "
                  + ("bitwise equal" if not diffs else "; ".join(diffs)))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], sys.argv[3])
    else:
        cmp(sys.argv[2], sys.argv[3:])
