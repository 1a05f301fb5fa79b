"""The free-running loop of tests/test_gpu_parity.py::test_free_running_loop_f32_theta_bounded (GPU): B = 65,536,
20 warm-started closed-loop steps, theta updated every step under the f32 health policy, run four ways -- fused f32,
generic f32 (DTMPC_FAST=0), fused f64, generic f64 (DTMPC_FAST64=0) -- printing per step the relative theta distance
of each from the fused f64 loop and the healthy fraction.  The shared theta is a batch mean dominated by a few
obstacle-grazing trajectories' large gradients, so its long-run value is as rounding-sensitive as they are; the
question this answers is whether one f32 rounding stays as close to f64 as another valid f32 rounding does.
usage: python scripts/theta_loop.py [steps]"""
import dataclasses
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "differentiable-tube-mpc_amd"), os.path.join(REPO, "tests")]


def main():
    from _common import paper_setup
    from diff_tube_mpc_strict_pt.core import TubeMPC

    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    st = paper_setup()
    st = dataclasses.replace(st, ilqr_nom=dataclasses.replace(st.ilqr_nom, tol=-1.0),
                             ilqr_aux=dataclasses.replace(st.ilqr_aux, tol=-1.0))
    B = 65536
    g = torch.Generator().manual_seed(0)
    u = torch.rand(B, 3, generator=g, dtype=torch.float64)
    x0 = torch.stack([u[:, 0], u[:, 1], u[:, 2] * (np.pi / 2)], 1)

    def loop(dtype, env):
        for k in ("DTMPC_FAST", "DTMPC_FAST64"):
            os.environ.pop(k, None)
        os.environ.update(env)
        m = TubeMPC(st, batch=B, device="cuda", dtype=dtype, disturbance="philox", seed=0, grad_bound=1e6)
        m.reset(x0.to(dtype))
        th, hf = [], []
        for _ in range(steps):
            m.step()
            th.append(m.theta.double().cpu().numpy())
            hf.append(m.healthy_count / B)
        return np.array(th), np.array(hf)

    runs = {"f32 fused": loop(torch.float32, {}), "f32 generic": loop(torch.float32, {"DTMPC_FAST": "0"}),
            "f64 fused": loop(torch.float64, {}), "f64 generic": loop(torch.float64, {"DTMPC_FAST64": "0"})}
    ref = runs["f64 fused"][0]
    rel_d = lambda a, b: (np.abs(a - b) / np.maximum(np.abs(b), 1e-3)).max(1)  # noqa: E731
    for name, (th, hf) in runs.items():
        print(f"{name:12s} distance from f64 fused per step: {[float(f'{v:.2g}') for v in rel_d(th, ref)]}")
        print(f"{'':12s} healthy fraction per step: {[float(f'{v:.4f}') for v in hf]}")
        print(f"{'':12s} theta after {steps} steps: {th[-1].round(4).tolist()}")


if __name__ == "__main__":
    main()
