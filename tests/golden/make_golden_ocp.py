"""Golden vectors for core/ocp.py `total_cost` (core/ocp.py:63-85) by RUNNING THE REFERENCE on CPU
(never on the GPU box):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_ocp.py

The reference's total_cost is driven with the paper's cost closures -- the nominal stage / terminal
expressions of core/tube_mpc.py:823-832 (weights of configs/dubins.yaml cost_nominal) and the ancillary
tracking ones of core/tube_mpc.py:875-885 (random weights) -- over random tapes.
Output: ocp_{f64,f32}.npz (inputs + reference outputs).
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
    _, cfg = _import_reference()
    import torch

    torch.set_num_threads(1)
    from diff_tube_mpc_strict_pt.core import ocp as rocp

    rng = np.random.default_rng(11)
    B, N = 6, 50
    cn = cfg["cost_nominal"]
    target_np = np.array(cfg["system"]["target"])
    X = rng.uniform(-1, 11, (B, N + 1, 4))
    X[..., 3] = rng.uniform(0, 3, (B, N + 1))
    U = rng.uniform(-10, 10, (B, N, 2))
    Xr = rng.uniform(-1, 11, (B, N + 1, 3))
    Ur = rng.uniform(-10, 10, (B, N, 2))
    Qa_np, Ra_np, qba_np = rng.uniform(0.1, 3, 3), rng.uniform(0.01, 2, 2), 0.4
    for tag, dt in (("f64", torch.float64), ("f32", torch.float32)):
        T = lambda a: torch.tensor(np.asarray(a), dtype=dt)  # noqa: E731
        Qn, Rn, Qfn, qbn, target = T(cn["Q"]), T(cn["R"]), T(cn["Qf"]), T(float(cn["q_b"])), T(target_np)
        Qa, Ra, qba = T(Qa_np), T(Ra_np), T(qba_np)
        Xb, Ub, Xrb, Urb = T(X), T(U), T(Xr), T(Ur)
        k_of = {}

        def stage_nom(xb, ub):  # core/tube_mpc.py:823-827, row by row of the batch
            out = []
            for x_hat_k, u_k in zip(xb, ub):
                dx = x_hat_k[:-1] - target
                bk = x_hat_k[-1]
                out.append((Qn * dx * dx).sum() + (Rn * u_k * u_k).sum() + qbn * (bk * bk))
            return torch.stack(out)

        def term_nom(xb):  # core/tube_mpc.py:829-832
            out = []
            for x_hat_N in xb:
                dxN = x_hat_N[:-1] - target
                bN = x_hat_N[-1]
                out.append((Qfn * dxN * dxN).sum() + qbn * (bN * bN))
            return torch.stack(out)

        def stage_aux(xb, ub):  # core/tube_mpc.py:875-880 (k tracked by call count)
            k = k_of["k"]
            k_of["k"] += 1
            out = []
            for i, (x_hat_k, v_k) in enumerate(zip(xb, ub)):
                dx = x_hat_k[:-1] - Xrb[i, k]
                du = v_k - Urb[i, k]
                bk = x_hat_k[-1]
                out.append((Qa * dx * dx).sum() + (Ra * du * du).sum() + qba * (bk * bk))
            return torch.stack(out)

        def term_aux(xb):  # core/tube_mpc.py:882-885
            out = []
            for i, x_hat_N in enumerate(xb):
                dxN = x_hat_N[:-1] - Xrb[i, N]
                bN = x_hat_N[-1]
                out.append((Qa * dxN * dxN).sum() + qba * (bN * bN))
            return torch.stack(out)

        J_nom = rocp.total_cost(X=Xb, U=Ub, stage_cost=stage_nom, terminal_cost=term_nom, stage_kwargs={},
                                terminal_kwargs={})
        k_of["k"] = 0
        J_aux = rocp.total_cost(X=Xb, U=Ub, stage_cost=stage_aux, terminal_cost=term_aux, stage_kwargs={},
                                terminal_kwargs={})
        J_one = rocp.total_cost(X=Xb[2], U=Ub[2], stage_cost=stage_nom, terminal_cost=term_nom, stage_kwargs={},
                                terminal_kwargs={})
        npd = np.float64 if tag == "f64" else np.float32
        np.savez(os.path.join(HERE, f"ocp_{tag}.npz"), X=X.astype(npd), U=U.astype(npd), Xr=Xr.astype(npd),
                 Ur=Ur.astype(npd), Qn=np.array(cn["Q"]), Rn=np.array(cn["R"]), Qfn=np.array(cn["Qf"]),
                 qbn=np.float64(cn["q_b"]), target=target_np, Qa=Qa_np, Ra=Ra_np, qba=np.float64(qba_np),
                 J_nom=J_nom.numpy(), J_aux=J_aux.numpy(), J_one=J_one.numpy())
        print("wrote", f"ocp_{tag}.npz", J_nom.numpy()[:2], J_aux.numpy()[:2])


if __name__ == "__main__":
    main()
