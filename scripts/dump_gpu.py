"""Debug helper (GPU box): dump HIP solver outputs for offline comparison with the oracle.

python scripts/dump_gpu.py  -> gpurun_out/dump_ilqr.npz
"""
from __future__ import annotations

import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "differentiable-tube-mpc_amd"), os.path.join(REPO, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from _common import ilqr_cfg, paper_setup  # noqa: E402
from diff_tube_mpc_strict_pt.core import ilqr_solve  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    st = paper_setup()
    rng = np.random.default_rng(5)
    B, N = 1000, st.problem.horizon
    from oracle.oracle import Oracle

    o = Oracle(np.float64)
    sp = st.problem.to_c()
    x = np.stack([rng.uniform(0, 1.5, B), rng.uniform(0, 1.5, B), rng.uniform(0, np.pi / 2, B)], 1)
    b = o.barrier(sp, o.h_eval(sp, x[:, 0], x[:, 1])[0])[0]
    x0 = np.concatenate([x, b[:, None]], 1)
    V0 = np.stack([rng.uniform(-1, 3, (B, N)), rng.uniform(-1, 1, (B, N))], 2)
    out = {"x0": x0, "V0": V0}
    for tag, dt in (("f64", torch.float64), ("f32", torch.float32)):
        for mi in range(1, 6):
            r = ilqr_solve(problem=st.problem, cost=st.nominal_cost, cfg=ilqr_cfg(mi, -1.0),
                           x0=torch.as_tensor(x0, dtype=dt, device=dev), V_init=torch.as_tensor(V0, dtype=dt, device=dev),
                           check=False)
            out[f"X_{tag}_{mi}"] = r.X.cpu().numpy()
            out[f"V_{tag}_{mi}"] = r.V.cpu().numpy()
            out[f"K_{tag}_{mi}"] = r.K.cpu().numpy()
            out[f"k_{tag}_{mi}"] = r.k.cpu().numpy()
            out[f"st_{tag}_{mi}"] = r.status.cpu().numpy()
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    np.savez_compressed(os.path.join(REPO, "gpurun_out", "dump_ilqr.npz"), **out)
    print("dumped")


if __name__ == "__main__":
    main()
