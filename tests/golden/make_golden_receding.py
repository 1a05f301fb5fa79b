"""Golden vectors for run_nominal.py's receding-horizon nominal MPC (run_nominal.py:204-415), produced
by RUNNING THE REFERENCE on CPU (f64, as the reference runs it).

Usage (container with /root/reference only; never on the GPU box):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_receding.py

Fixture sets  receding_{R1,R2,R3,R4}.npz  (inputs = the config; outputs = the saved arrays + summary)
  R1  configs/dubins.yaml, H = 25 (the paper obstacle field, smooth-min)
  R2  target moved to (0.25, 0.25): the success exit (||x - target|| <= 0.25) fires
  R3  an extra obstacle around the start: the collision exit (true min_i h_i <= 0) fires at t = 0
  R4  exact-min aggregation, log barrier, gamma = 0.4, alpha = 0.05, H = 12
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import PKG, _import_reference  # noqa: E402


def variants(cfg):
    r1 = json.loads(json.dumps(cfg))
    r1["system"]["task_horizon_H"] = 25
    r2 = json.loads(json.dumps(cfg))
    r2["system"]["task_horizon_H"] = 40
    r2["system"]["target"] = [0.25, 0.25, 0.7853981633974483]
    r3 = json.loads(json.dumps(cfg))
    r3["system"]["task_horizon_H"] = 5
    r3["environment"]["obstacles"] = [{"center": [0.2, 0.1], "radius": 0.5}] + r3["environment"]["obstacles"]
    r4 = json.loads(json.dumps(cfg))
    r4["system"]["task_horizon_H"] = 12
    r4["environment"]["obstacle_aggregation"] = "min"
    r4["dbas"].update({"barrier_type": "log", "gamma": 0.4, "alpha": 0.05})
    return {"R1": r1, "R2": r2, "R3": r3, "R4": r4}


def main() -> None:
    sys.dont_write_bytecode = True
    root, cfg = _import_reference()
    import torch

    torch.set_num_threads(1)
    sys.path.insert(0, os.path.join(root, PKG))
    import run_nominal as rn

    for name, c in variants(cfg).items():
        rd = os.path.join(root, "out_receding_" + name)
        res = rn.run_nominal_receding(c, device=torch.device("cpu"), run_dir=rd)
        out = {nm: np.load(os.path.join(rd, nm + ".npy")) for nm in ("x_bar", "u_bar", "b_real")}
        s = res["summary"]
        out["H_ran"] = np.asarray(s["H_ran"])
        out["success"] = np.asarray(bool(s["success"]))
        out["success_t"] = np.asarray(-1 if s["success_t"] is None else s["success_t"])
        out["collided"] = np.asarray(bool(s["collided"]))
        out["final_state"] = np.asarray(s["final_state"])
        out["config"] = np.asarray(json.dumps(c))
        np.savez_compressed(os.path.join(HERE, f"receding_{name}.npz"), **out)
        print(name, s, flush=True)
    print("receding golden vectors written to", HERE)


if __name__ == "__main__":
    main()
