"""Diagnostic (GPU): the receding-horizon driver on the fused solver (csrc/dtmpc_fast.hip receding_fast_kernel)
against the generic kernel (DTMPC_FAST=0) and the oracle (plain build) on the failure-set workload of
tests/test_gpu_receding.py (x0 ~ U[0,1]^2 x U[0, pi/2], paper configuration, H = 20): failure counts, exit
agreement, and for the first runs where they part, the recorded rows side by side.
usage: python scripts/diag_receding.py [B]"""
import json
import math
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "differentiable-tube-mpc_amd"), os.path.join(REPO, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from _common import config, oracles  # noqa: E402
from diff_tube_mpc_strict_pt.core import nominal_receding  # noqa: E402
from diff_tube_mpc_strict_pt.core.receding import receding_setup_from_config  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
problem, cost, icfg = receding_setup_from_config(json.loads(json.dumps(config())))
H, N = 20, problem.horizon
print("spec eps", problem.dbas_eps, "alpha", problem.dbas_alpha, "reg", icfg.reg, "alphas", icfg.line_search_alphas)
g = torch.Generator().manual_seed(0)
u = torch.rand(B, 3, generator=g, dtype=torch.float64)
x0 = torch.stack([u[:, 0], u[:, 1], u[:, 2] * (math.pi / 2)], 1)
for tag, tdt, npdt in (("f64", torch.float64, np.float64), ("f32", torch.float32, np.float32)):
    res = {}
    for name, fast in (("fused", "1"), ("generic", "0")):
        os.environ["DTMPC_FAST"] = fast
        r = nominal_receding(problem=problem, cost=cost, cfg=icfg, x0=x0.to(tdt).cuda(), H=H, check=False)
        torch.cuda.synchronize()
        lg = torch.cat([r.x, r.u, r.b[..., None]], -1).cpu().numpy()
        res[name] = (r.status.cpu().numpy(), r.h_ran.cpu().numpy(), lg)
    os.environ.pop("DTMPC_FAST", None)
    U = np.zeros((B, N, 2), npdt)
    U[:, :, 0] = problem.u_max[0]
    o = oracles(npdt)[0].nominal_receding(problem.to_c(), cost.to_c(), icfg.to_c(), x0.numpy().astype(npdt), H, 0.25, U.copy())
    res["oracle"] = (o[4], o[1], o[0])
    for k, (st, hr, lg) in res.items():
        print(f"[{tag}] {k}: failures {int((st != 0).sum())}, mean h_ran {hr.mean():.2f}")
    for a_, b_ in (("fused", "oracle"), ("generic", "oracle"), ("fused", "generic")):
        ex = (res[a_][1] == res[b_][1]) & ((res[a_][0] != 0) == (res[b_][0] != 0))
        print(f"[{tag}] exits {a_} == {b_}: {ex.mean():.4f}")
    # first runs where fused and oracle part: rows side by side
    shown = 0
    for i in range(B):
        la, lo = res["fused"][2][i], res["oracle"][2][i]
        n = min(res["fused"][1][i], res["oracle"][1][i])
        d = np.abs(la[:n] - lo[:n]).max(1) / (np.abs(lo[:n]).max(1) + 1.0)
        t = int(np.argmax(d > (1e-9 if tag == "f64" else 1e-4))) if (d > (1e-9 if tag == "f64" else 1e-4)).any() else -1
        if t < 0 and res["fused"][1][i] == res["oracle"][1][i] and (res["fused"][0][i] != 0) == (res["oracle"][0][i] != 0):
            continue
        print(f"  traj {i}: h_ran fused {res['fused'][1][i]} generic {res['generic'][1][i]} oracle {res['oracle'][1][i]}; "
              f"status {res['fused'][0][i]} {res['generic'][0][i]} {res['oracle'][0][i]}; first row apart {t}")
        for tt in range(max(0, t - 1), min(max(t, 0) + 2, H)):
            for k in ("fused", "generic", "oracle"):
                print(f"     t={tt} {k:8s} " + " ".join(f"{v: .9g}" for v in res[k][2][i][tt]))
        shown += 1
        if shown >= 4:
            break
