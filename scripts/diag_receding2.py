import json, os, sys
import numpy as np, torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "differentiable-tube-mpc_amd"), os.path.join(REPO, "tests")]
from _common import golden
from diff_tube_mpc_strict_pt.core import nominal_receding
from diff_tube_mpc_strict_pt.core.receding import receding_setup_from_config
g = golden("receding_R4")
cfg = json.loads(str(g["config"]))
problem, cost, icfg = receding_setup_from_config(cfg)
print(cost, icfg)
dev = torch.device("cuda:0")
rr = nominal_receding(problem=problem, cost=cost, cfg=icfg, x0=torch.tensor([[0.0, 0.0, np.pi / 4]], dtype=torch.float64, device=dev), H=2)
print("x", rr.x[0].cpu().numpy(), "u", rr.u[0].cpu().numpy(), "b", rr.b[0].cpu().numpy())
