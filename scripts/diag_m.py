"""Fused vs generic receding driver per obstacle count (diagnostic): for M = 1..8 obstacles off the runs' diagonal,
f64, B = 256, print per H the fraction of runs within 1e-9 and the first differing receding step."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "differentiable-tube-mpc_amd")]
from diff_tube_mpc_strict_pt.core import nominal_receding  # noqa: E402
from diff_tube_mpc_strict_pt.core.receding import receding_setup_from_config  # noqa: E402
from _common import config  # noqa: E402

ring = [(8.0, 2.5), (2.5, 8.0), (9.5, 4.5), (4.5, 9.5), (6.5, 1.5), (1.5, 6.5), (9.0, 7.5), (7.5, 9.0)]
order = [int(a) for a in sys.argv[1].split(",")] if len(sys.argv) > 1 else list(range(8))
MS = [int(v) for v in os.environ["DIAG_M"].split(",")] if "DIAG_M" in os.environ else list(range(1, 9))
dt = torch.float64 if os.environ.get("DIAG_F32") != "1" else torch.float32
for m in MS:
    cfg = json.loads(json.dumps(config()))
    cfg["environment"]["obstacles"] = [{"center": list(ring[j]), "radius": 0.8} for j in order[:m]]
    problem, cost, icfg = receding_setup_from_config(cfg)
    B, H = 256, 10
    rng = np.random.default_rng(11)
    x0 = np.stack([rng.uniform(0, 1, B), rng.uniform(0, 1, B), rng.uniform(0, np.pi / 2, B)], 1)
    out = []
    for fast in ("1", "1", "0"):
        os.environ["DTMPC_FAST"] = fast
        r = nominal_receding(problem=problem, cost=cost, cfg=icfg, x0=torch.as_tensor(x0, device="cuda", dtype=dt), H=H,
                             check=False)
        torch.cuda.synchronize()
        out.append(torch.cat([r.x, r.u, r.b[..., None]], -1).double().cpu().numpy())
    del os.environ["DTMPC_FAST"]
    rep = float(np.nanmax(np.abs(out[0] - out[1])))  # the fused driver run twice on the same inputs
    out = [out[0], out[2]]
    d = np.abs(out[0] - out[1]) / (np.abs(out[1]).max(axis=(1, 2), keepdims=True) + 1)
    per_h = d.max(2)  # [B, H]
    bad = per_h > (1e-9 if dt == torch.float64 else 1e-4)
    first = np.where(bad.any(1), bad.argmax(1), -1)
    col = d.reshape(B * H, -1).max(0)
    print(f"M={m} order={order[:m]} repeat-diff {rep:.3e} ok {1 - bad.any(1).mean():.4f} max {d.max():.3e} first-bad-h hist "
          f"{np.bincount(first[first >= 0], minlength=H).tolist()} per-column max {np.array2string(col, precision=2)}",
          flush=True)

# the same obstacle sets through the f64 tube step (tube_fast_kernel vs tube_step_kernel) and the standalone
# batched iLQR (ilqr_fast_kernel vs ilqr_kernel), lanes 1 / 2 / 4
if os.environ.get("DIAG_TUBE") == "1":
    import dataclasses

    from diff_tube_mpc_strict_pt.core import TubeMPC, ilqr_solve
    from diff_tube_mpc_strict_pt.core.problem import ILQRConfig, paper_setup_from_config

    for m in MS:
        cfg = json.loads(json.dumps(config()))
        cfg["environment"]["obstacles"] = [{"center": list(ring[j]), "radius": 0.8} for j in order[:m]]
        st = paper_setup_from_config(cfg)
        B = 512
        rng = np.random.default_rng(21)
        x = np.stack([rng.uniform(0, 1, B), rng.uniform(0, 1, B), rng.uniform(0, np.pi / 2, B)], 1)
        for lanes in ("1", "2", "4"):
            os.environ["DTMPC_TUBE_LANES"] = lanes
            runs = []
            for fast in ("1", "0"):
                os.environ["DTMPC_FAST64"] = fast
                mp = TubeMPC(st, batch=B, device="cuda", dtype=torch.float64, disturbance="philox", seed=5)
                mp.reset(torch.as_tensor(x, device="cuda"))
                mp.step()
                torch.cuda.synchronize()
                runs.append(np.concatenate([mp.Unom.reshape(B, -1).cpu().numpy() if mp.Unom.shape[0] == B else
                                            mp.Unom.reshape(-1, B).T.cpu().numpy(),
                                            mp.Uaux.reshape(B, -1).cpu().numpy() if mp.Uaux.shape[0] == B else
                                            mp.Uaux.reshape(-1, B).T.cpu().numpy()], 1))
            e = np.abs(runs[0] - runs[1]).max(1) / (np.abs(runs[1]).max(1) + 1)
            os.environ["DTMPC_FAST64"] = "1"
            ic = ILQRConfig(horizon=st.problem.horizon, max_iter=10, tol=1e-3,
                            line_search_alphas=st.ilqr_nom.line_search_alphas)
            V0 = np.zeros((B, st.problem.horizon, 2))
            V0[:, :, 0] = 10.0
            rs = []
            for fast in ("1", "0"):
                os.environ["DTMPC_FAST"] = fast
                r = ilqr_solve(problem=st.problem, cost=st.nominal_cost, cfg=ic, x0=torch.as_tensor(np.concatenate([x, np.ones((B, 1))], 1), device="cuda"),
                               V_init=torch.as_tensor(V0, device="cuda"), check=False, lanes=int(lanes))
                torch.cuda.synchronize()
                rs.append(r.V.reshape(B, -1).cpu().numpy())
            del os.environ["DTMPC_FAST"]
            ei = np.abs(rs[0] - rs[1]).max(1) / (np.abs(rs[1]).max(1) + 1)
            print(f"[tube/ilqr f64] M={m} lanes={lanes}: tube plans within 1e-8 {(e <= 1e-8).mean():.4f} (max {e.max():.2e}); "
                  f"ilqr plans within 1e-8 {(ei <= 1e-8).mean():.4f} (max {ei.max():.2e})", flush=True)
