"""Diagnostic (GPU): the tube step's results must not depend on what earlier runs left in reused device memory.
One process runs the same two closed-loop steps (paper setup, fixed iterations, B = 700, DT / L / SEED as in
scripts/diag_g0.py) several times -- fresh TubeMPC each time, the caching allocator handing back the previous runs'
blocks -- optionally with DTMPC_FAST_CHUNK set for some runs, and compares every array with the first run.
usage: python scripts/diag_reuse.py DT=f64,L=2,SEED=5 [chunk ...]   (chunk 0 = one launch; env FILL=0xff pre-fills
the workspace of every run after the first)"""
import dataclasses
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "differentiable-tube-mpc_amd"), os.path.join(REPO, "tests")]
NAMES = ("x", "b", "xbar", "bbar", "Xnom", "Unom", "Xaux", "Uaux", "theta", "status", "log", "partials")


def main():
    cfg = dict(kv.split("=") for kv in sys.argv[1].split(","))
    chunks = [int(c) for c in sys.argv[2:]] or [0, 0, 256, 0]
    os.environ["DTMPC_TUBE_LANES"] = cfg.get("L", "1")
    from _common import paper_setup
    from diff_tube_mpc_strict_pt.core import TubeMPC

    st = paper_setup()
    st = dataclasses.replace(st, ilqr_nom=dataclasses.replace(st.ilqr_nom, tol=-1.0),
                             ilqr_aux=dataclasses.replace(st.ilqr_aux, tol=-1.0))
    tdt = torch.float64 if cfg.get("DT", "f32") == "f64" else torch.float32
    B = 700
    rng = np.random.default_rng(int(cfg.get("SEED", "5")))
    x = torch.tensor(np.stack([rng.uniform(0, 1, B), rng.uniform(0, 1, B), rng.uniform(0, np.pi / 2, B)], 1),
                     dtype=tdt, device="cuda")
    first = None
    for r, ch in enumerate(chunks):
        if ch:
            os.environ["DTMPC_FAST_CHUNK"] = str(ch)
        else:
            os.environ.pop("DTMPC_FAST_CHUNK", None)
        m = TubeMPC(st, batch=B, device="cuda", dtype=tdt, disturbance="philox", seed=4, write_log=True)
        if os.environ.get("FILL") and r > 0:  # the workspace pre-filled with a byte pattern (0xff: NaN in either precision)
            m.work.fill_(int(os.environ["FILL"], 0))
        m.reset(x)
        for _ in range(int(os.environ.get("STEPS", "2"))):
            m.step()
        torch.cuda.synchronize()
        out = {k: getattr(m, k).cpu().numpy().copy() for k in NAMES if getattr(m, k, None) is not None}
        if first is None:
            first = out
            print(f"run {r} (chunk {ch}): reference")
            continue
        diff = {}
        for k, v in out.items():
            a = first[k]
            if not np.array_equal(a, v, equal_nan=True):
                bad = ~((a == v) | (np.isnan(a) & np.isnan(v)))
                tr = np.unique(np.argwhere(bad)[:, -1])
                diff[k] = (int(bad.sum()), tr[:8].tolist())
        print(f"run {r} (chunk {ch}):", "bitwise equal" if not diff else diff)
        if "log" in diff:
            t = diff["log"][1][0]
            print(f"  log rows of trajectory {t}: first run {first['log'][:, t].tolist()}\n  this run {out['log'][:, t].tolist()}")
            print(f"  status {first['status'][t]} {out['status'][t]}")
        del m


if __name__ == "__main__":
    main()
