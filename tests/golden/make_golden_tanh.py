"""Golden vectors for the tanh-box control map and its cost derivatives, by RUNNING THE REFERENCE on CPU.

Usage (container with /root/reference only; never on the GPU box):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_tanh.py

Reference functions exercised (inputs + outputs stored, no reference source text):
  core/control.py:10-35      BoxTanhControl.u, BoxTanhControl.du_dv_diag
  core/cost_derivs.py:16-24  _d2u_dv2_diag
  core/cost_derivs.py:27-55  nominal_cost_derivs   (target cost in the decision variable v)
  core/cost_derivs.py:79-107 auxiliary_cost_derivs (tracking cost in v)
Output: tanh_{f64,f32}.npz next to this script.  Points: B random tapes of N steps (states, v over a
range that reaches tanh saturation, references, weights from configs/dubins.yaml and random ones).
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import _import_reference  # noqa: E402


def main() -> None:
    sys.dont_write_bytecode = True
    _import_reference()
    import torch

    torch.set_num_threads(1)
    from diff_tube_mpc_strict_pt.core import control as rctl
    from diff_tube_mpc_strict_pt.core import cost_derivs as rcd

    rng = np.random.default_rng(7)
    B, N = 6, 5
    for name, dt in (("f64", torch.float64), ("f32", torch.float32)):
        npd = np.float64 if dt == torch.float64 else np.float32
        umin = np.array([-10.0, -np.pi])
        umax = np.array([10.0, np.pi])
        ctrl = rctl.BoxTanhControl(u_min=torch.tensor(umin, dtype=dt), u_max=torch.tensor(umax, dtype=dt))
        X = rng.uniform(-3, 3, (B, N + 1, 4)).astype(npd)
        X[..., 3] = rng.uniform(0, 5, (B, N + 1))
        Vd = rng.uniform(-4, 4, (B, N, 2)).astype(npd)
        Vd[0, 0] = (12.0, -12.0)  # tanh saturated to +-1 in f32
        Vd[0, 1] = (0.0, 1e-6)
        Xr = rng.uniform(-3, 3, (B, N + 1, 3)).astype(npd)
        Ur = rng.uniform(-5, 5, (B, N, 2)).astype(npd)
        Q = np.array([1.0, 1.0, 0.1])
        R = np.array([0.01, 0.01])
        qb = 0.05
        Qa = rng.uniform(0.1, 3.0, 3)
        Ra = rng.uniform(0.001, 0.5, 2)
        qba = 0.3
        target = np.array([4.0, 4.0, 0.0])
        out = {k: np.zeros((B, N, w), npd) for k, w in (("u", 2), ("dudv", 2), ("d2u", 2), ("lx_nom", 4), ("lv_nom", 2),
                                                          ("lvv_nom", 2), ("lx_aux", 4), ("lv_aux", 2), ("lvv_aux", 2))}
        t = lambda a: torch.tensor(a, dtype=dt)  # noqa: E731
        for i in range(B):
            for k in range(N):
                v = t(Vd[i, k])
                out["u"][i, k] = ctrl.u(v).numpy()
                out["dudv"][i, k] = ctrl.du_dv_diag(v).numpy()
                out["d2u"][i, k] = rcd._d2u_dv2_diag(ctrl, v).numpy()
                lx, lv, lxx, lvv, lvx = rcd.nominal_cost_derivs(x_hat=t(X[i, k]), v=v, target=t(target), Q=t(Q), R=t(R),
                                                                qb=t(qb), ctrl=ctrl)
                assert not lvx.any() and torch.equal(lxx, torch.diag(torch.diagonal(lxx)))
                out["lx_nom"][i, k], out["lv_nom"][i, k], out["lvv_nom"][i, k] = lx.numpy(), lv.numpy(), torch.diagonal(lvv).numpy()
                lx, lv, lxx, lvv, lvx = rcd.auxiliary_cost_derivs(x_hat=t(X[i, k]), v=v, x_ref=t(Xr[i, k]), u_ref=t(Ur[i, k]),
                                                                  Q=t(Qa), R=t(Ra), qb=t(qba), ctrl=ctrl)
                assert not lvx.any()
                out["lx_aux"][i, k], out["lv_aux"][i, k], out["lvv_aux"][i, k] = lx.numpy(), lv.numpy(), torch.diagonal(lvv).numpy()
        np.savez(os.path.join(HERE, f"tanh_{name}.npz"), X=X, Vd=Vd, Xr=Xr, Ur=Ur, umin=umin, umax=umax, Q=Q, R=R,
                 qb=np.float64(qb), Qa=Qa, Ra=Ra, qba=np.float64(qba), target=target, **out)
        print("wrote", f"tanh_{name}.npz")


if __name__ == "__main__":
    main()
