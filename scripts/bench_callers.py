"""Throughput of the callers either side of the hot path, f32 on one GPU.

* General IFT path (adapt_nominal, softplus/tanh parameters): GeneralTubeMPC.step at B trajectories,
  fixed iteration counts (tol = -1; the general path keeps the reference's four line-search alphas):
  DDP+IFT iterations/s = B * (I_nom + I_aux + 2) / t_step (two IFT passes: ancillary and nominal).
* Receding-horizon nominal MPC (run_nominal.py): nominal_receding over B runs of H steps (tol = 1e-3
  as the reference, early exits on success / collision): iLQR solves/s = sum of steps run / t.
usage: python scripts/bench_callers.py [--batch B] [--steps K] [--H H]"""
import argparse
import dataclasses
import json
import math
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "differentiable-tube-mpc_amd")]
import torch  # noqa: E402

from diff_tube_mpc_strict_pt.core import GeneralTubeMPC  # noqa: E402
from diff_tube_mpc_strict_pt.core.problem import general_setup_from_config, paper_config  # noqa: E402
from diff_tube_mpc_strict_pt.core.receding import nominal_receding, receding_setup_from_config  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=65536)
ap.add_argument("--steps", type=int, default=5)
ap.add_argument("--H", type=int, default=20)
ap.add_argument("--receding-only", action="store_true")
ap.add_argument("--f64", action="store_true", help="the receding legs in f64 too")
a = ap.parse_args()
dev = torch.device("cuda", 0)
B = a.batch
g = torch.Generator().manual_seed(0)
u = torch.rand(B, 3, generator=g, dtype=torch.float64)
x0 = torch.stack([u[:, 0], u[:, 1], u[:, 2] * (math.pi / 2)], 1).float().to(dev)

# ---- general path
cfg = paper_config()
if a.receding_only:
    cfg = None
if cfg is not None:
    cfg["paper_dubins_mode"] = False
    cfg["adaptation"]["adapt_nominal"] = True
    st = general_setup_from_config(cfg)
    st = dataclasses.replace(st, ilqr_nom=dataclasses.replace(st.ilqr_nom, tol=-1.0),
                             ilqr_aux=dataclasses.replace(st.ilqr_aux, tol=-1.0))
    m = GeneralTubeMPC(st, batch=B, device=dev, dtype=torch.float32, disturbance="philox", seed=0)
    for _ in range(2):
        m.reset(x0)
        m.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        m.reset(x0)
        m.step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.steps
    it = st.ilqr_nom.max_iter + st.ilqr_aux.max_iter + 2
    print(json.dumps({"path": "general IFT step (adapt_nominal)", "batch": B, "ms_per_step": dt * 1e3,
                      "ddp_ift_iters_per_s": B * it / dt, "iterations": [st.ilqr_nom.max_iter, st.ilqr_aux.max_iter],
                      "line_search_alphas": len(st.ilqr_nom.line_search_alphas),
                      "healthy": m.healthy_count if hasattr(m, "healthy_count") else None}), flush=True)
    del m
    torch.cuda.empty_cache()

# ---- receding-horizon nominal MPC
problem, cost, icfg = receding_setup_from_config(paper_config())
# the fused solver (receding_fast_kernel, the default) and the generic kernel (DTMPC_FAST=0)
for dt_name in (("f32", "f64") if a.f64 else ("f32",)):
    xd = x0.double() if dt_name == "f64" else x0
    for kern, fast in (("fused", "1"), ("generic", "0")):
        os.environ["DTMPC_FAST"] = fast
        nominal_receding(problem=problem, cost=cost, cfg=icfg, x0=xd[:1024], H=2, check=False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = nominal_receding(problem=problem, cost=cost, cfg=icfg, x0=xd, H=a.H, check=False)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        steps = int(r.h_ran.sum())
        print(json.dumps({"path": "receding nominal MPC (run_nominal.py)", "kernel": kern, "dtype": dt_name,
                          "batch": B, "H": a.H, "seconds": dt, "solves": steps, "ilqr_solves_per_s": steps / dt,
                          "ms_per_receding_step": dt * 1e3 / a.H, "max_iter": icfg.max_iter,
                          "line_search_alphas": len(icfg.line_search_alphas),
                          "success": int((r.success_t >= 0).sum()), "collided": int(r.collided.sum()),
                          "failed": int((r.status != 0).sum())}), flush=True)
os.environ.pop("DTMPC_FAST", None)
