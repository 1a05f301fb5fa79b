"""Bitwise comparison helper: run one batched f32 iLQR solve (bench inputs) + one tube step with the
library in DTMPC_LIBRARY and save the outputs (usage: python scripts/cmp_libs.py OUT.npz)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "differentiable-tube-mpc_amd")]
import numpy as np, torch
from bench import bench_setup, initial_states
from diff_tube_mpc_strict_pt.core import TubeMPC, dbas_init, ilqr_solve
B = 65536
dev = torch.device("cuda", 0)
st = bench_setup("f32")
N = st.problem.horizon
x = initial_states(0, B, dev, torch.float32)
x0 = torch.cat([x, dbas_init(st.problem, x)[:, None]], 1)
r = ilqr_solve(problem=st.problem, cost=st.nominal_cost, cfg=st.ilqr_nom, x0=x0, V_init=torch.zeros(B, N, 2, device=dev), check=False)
mpc = TubeMPC(st, batch=B, device=dev, dtype=torch.float32, disturbance="philox", seed=0)
mpc.reset(x)
out = {"X": r.X.cpu().numpy(), "V": r.V.cpu().numpy(), "st": r.status.cpu().numpy()}
for t in range(3):
    mpc.step()
    torch.cuda.synchronize()
    out[f"theta{t}"] = mpc.theta.cpu().numpy() if hasattr(mpc, "theta") else np.zeros(1)
    out[f"x{t}"] = mpc.x.cpu().numpy()
np.savez(sys.argv[1], **out)
print("saved", sys.argv[1])
