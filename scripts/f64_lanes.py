"""f64 tube step at the bench batch for each lane form of the generic kernel (DTMPC_TUBE_LANES=1|2;
4 runs the generic kernel at two lanes): usage python scripts/f64_lanes.py [--batch B]"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "differentiable-tube-mpc_amd")]
import torch  # noqa: E402

import bench  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=65536)
ap.add_argument("--dtype", default="f64")
a = ap.parse_args()
dev = torch.device("cuda", 0)
for lanes in ("1", "2"):
    os.environ["DTMPC_TUBE_LANES"] = lanes
    r = bench.tube_leg(dev, a.dtype, a.batch, steps=5, warmup=1)
    print(json.dumps({"lanes_env": lanes, **r}), flush=True)
