"""Per-phase timing of the solver pieces at the bench size (B = 65,536, f32), each as its own launch:
init rollout only, nominal iLQR (10 it) with 1 / 4 / 7 alphas, ancillary iLQR (20 it, 7 alphas), the
DDP sensitivity, and the fused tube step.  usage: python scripts/phase_bench.py [--batch B]"""
import argparse
import dataclasses
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "differentiable-tube-mpc_amd")]
import torch  # noqa: E402

from bench import bench_setup, initial_states  # noqa: E402
from diff_tube_mpc_strict_pt.core import TubeMPC, dbas_init, ddp_sensitivity, ilqr_solve, tracking_cost  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=65536)
a = ap.parse_args()
B = a.batch
dev = torch.device("cuda", 0)
st = bench_setup("f32")
N = st.problem.horizon
x = initial_states(0, B, dev, torch.float32)
x0 = torch.cat([x, dbas_init(st.problem, x)[:, None]], 1)
V0 = torch.zeros(B, N, 2, device=dev)


def timed(fn, reps=3):
    fn()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts)[len(ts) // 2], out


res = {}
cfg = st.ilqr_nom
for name, c in [("nominal_init_only", dataclasses.replace(cfg, max_iter=0)),
                ("nominal_10it_1alpha", dataclasses.replace(cfg, line_search_alphas=(1.0,))),
                ("nominal_10it_4alpha", dataclasses.replace(cfg, line_search_alphas=cfg.line_search_alphas[:4])),
                ("nominal_10it_7alpha", cfg)]:
    res[name], r = timed(lambda: ilqr_solve(problem=st.problem, cost=st.nominal_cost, cfg=c, x0=x0, V_init=V0,
                                            check=False))
nom = r
ca = tracking_cost(st.theta0)
res["aux_20it_7alpha"], ra = timed(lambda: ilqr_solve(problem=st.problem, cost=ca, cfg=st.ilqr_aux, x0=x0,
                                                      V_init=V0, X_ref=nom.X, U_ref=nom.V, check=False))
res["sensitivity"], _ = timed(lambda: ddp_sensitivity(problem=st.problem, cost=ca, X=ra.X, V=ra.V, X_ref=nom.X,
                                                      U_ref=nom.V, X_bar=nom.X, want_lambda=False, check=False))
mpc = TubeMPC(st, batch=B, device=dev, dtype=torch.float32, disturbance="philox", seed=0)


def tube():
    mpc.reset(x)
    mpc.step()


res["tube_step_total"], _ = timed(tube)
for k, v in res.items():
    print(f"{k:24s} {v:8.3f} ms")
