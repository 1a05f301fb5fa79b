"""Diagnostic: the receding fixture R4 (exact-min, log barrier, gamma/alpha != 0) piece by piece, device vs
oracle (f64): b0, rollout, linearize, iLQR with 1..3 fixed iterations, the receding driver."""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "differentiable-tube-mpc_amd"), os.path.join(REPO, "tests")]

from _common import golden, rel  # noqa: E402
from diff_tube_mpc_strict_pt.core import ddp, nominal_receding  # noqa: E402
from diff_tube_mpc_strict_pt.core.problem import ILQRConfig  # noqa: E402
from diff_tube_mpc_strict_pt.core.receding import receding_setup_from_config  # noqa: E402
from oracle.oracle import Oracle  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "R4"
g = golden(f"receding_{name}")
cfg = json.loads(str(g["config"]))
problem, cost, icfg = receding_setup_from_config(cfg)
print(problem)
print(icfg)
dev = torch.device("cuda:0")
o = Oracle(np.float64)
sp, cc = problem.to_c(), cost.to_c()
N = problem.horizon
x = np.array([[0.0, 0.0, np.pi / 4]])
h, _, _ = o.h_eval(sp, x[:, 0], x[:, 1])
b0o = o.barrier(sp, h)[0]
b0d = ddp.dbas_init(problem, torch.tensor(x, device=dev)).cpu().numpy()
print("b0", b0o, b0d)
xh = np.concatenate([x, b0o[:, None]], 1)
U = np.zeros((1, N, 2))
U[0, :, 0] = problem.u_max[0]
Xo = o.dbas_rollout(sp, xh, U)
Xd = ddp.rollout(problem, torch.tensor(xh, device=dev), torch.tensor(U, device=dev)).cpu().numpy()
print("rollout rel", rel(Xd, Xo))
lo = o.linearize(sp, cc, Xo, U)
ld = [t.cpu().numpy() for t in ddp.linearize(problem, cost, torch.tensor(Xo, device=dev), torch.tensor(U, device=dev))]
for nm, a, b in zip(("A", "B", "lx", "lu"), ld, lo):
    print("linearize", nm, rel(a, np.asarray(b).reshape(a.shape)))
for it in (1, 2, 3, 10):
    c = ILQRConfig(horizon=N, max_iter=it, tol=-1.0, reg=icfg.reg, line_search_alphas=icfg.line_search_alphas)
    Xo2, Vo2, *_ = o.ilqr_solve(sp, cc, c.to_c(), xh, U)
    r = ddp.ilqr_solve(problem=problem, cost=cost, cfg=c, x0=torch.tensor(xh, device=dev), V_init=torch.tensor(U, device=dev))
    print("ilqr it", it, "X rel", rel(r.X.cpu().numpy(), Xo2), "V rel", rel(r.V.cpu().numpy(), Vo2),
          "u0 dev", r.V[0, 0].cpu().numpy(), "u0 or", Vo2[0, 0])
Xo2, Vo2, *_ = o.ilqr_solve(sp, cc, icfg.to_c(), xh, U)
r = ddp.ilqr_solve(problem=problem, cost=cost, cfg=icfg, x0=torch.tensor(xh, device=dev), V_init=torch.tensor(U, device=dev))
print("ilqr tol", icfg.tol, "iters", r.iters.cpu().numpy(), "V rel", rel(r.V.cpu().numpy(), Vo2), "ref u0", g["u_bar"][0])
rr = nominal_receding(problem=problem, cost=cost, cfg=icfg, x0=torch.tensor(x, device=dev), H=int(cfg["system"]["task_horizon_H"]))
print("receding u0 dev", rr.u[0, :3].cpu().numpy(), "ref", g["u_bar"][:3])
import dataclasses  # noqa: E402

for kw in ({}, {"dbas_gamma": 0.0}, {"dbas_alpha": 0.0}, {"barrier_type": "inverse"}, {"obs_aggregation": "smoothmin"},
           {"dbas_gamma": 0.0, "dbas_alpha": 0.0}, {"dbas_gamma": 0.0, "barrier_type": "inverse"}):
    p2 = dataclasses.replace(problem, **kw)
    for it, tol in ((1, -1.0), (2, -1.0), (10, 1e-3)):
        c = ILQRConfig(horizon=N, max_iter=it, tol=tol, reg=icfg.reg, line_search_alphas=icfg.line_search_alphas)
        xh2 = np.concatenate([x, ddp.dbas_init(p2, torch.tensor(x, device=dev)).cpu().numpy()[:, None]], 1)
        r = ddp.ilqr_solve(problem=p2, cost=cost, cfg=c, x0=torch.tensor(xh2, device=dev), V_init=torch.tensor(U, device=dev))
        rr = nominal_receding(problem=p2, cost=cost, cfg=c, x0=torch.tensor(x, device=dev), H=1)
        print(kw, it, tol, "ilqr u0", r.V[0, 0, 1].item(), "receding u0", rr.u[0, 0, 1].item())
