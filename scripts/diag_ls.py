"""Diagnostic (GPU): where do two libraries' line searches first differ?  One closed-loop step of the paper setup
(f32, fixed iterations, B trajectories at DTMPC_TUBE_LANES) with the decision and candidate-cost records, saved;
``cmp`` prints the first iteration (nominal 0..I_nom-1, then ancillary) whose candidate costs or winners differ.
usage: DTMPC_LIBRARY=... python scripts/diag_ls.py run OUT.npz [B]
       python scripts/diag_ls.py cmp A.npz B.npz"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "differentiable-tube-mpc_amd"), os.path.join(REPO, "tests")]


def run(out, B):
    import dataclasses

    import torch

    from _common import paper_setup
    from diff_tube_mpc_strict_pt.core import TubeMPC

    st = paper_setup()
    it = int(os.environ.get("NOM_ITERS", "0")) or st.ilqr_nom.max_iter
    st = dataclasses.replace(st, ilqr_nom=dataclasses.replace(st.ilqr_nom, tol=-1.0, max_iter=it),
                             ilqr_aux=dataclasses.replace(st.ilqr_aux, tol=-1.0))
    rng = np.random.default_rng(6)
    x = torch.tensor(np.stack([rng.uniform(0, 1, B), rng.uniform(0, 1, B), rng.uniform(0, np.pi / 2, B)], 1),
                     dtype=torch.float32)
    m = TubeMPC(st, batch=B, device="cuda", dtype=torch.float32, disturbance="philox", seed=4,
                record_choices=True, record_costs=True)
    m.reset(x.cuda())
    m.step()
    torch.cuda.synchronize()
    np.savez(out, choices=m.choices.cpu().numpy(), costs=m.costs.cpu().numpy(), Xnom=m.Xnom.cpu().numpy(),
             Unom=m.Unom.cpu().numpy(), Xaux=m.Xaux.cpu().numpy(), Uaux=m.Uaux.cpu().numpy())


def cmp(a, b):
    A, Bz = np.load(a), np.load(b)
    for k in ("Xnom", "Unom"):
        d = np.abs(A[k] - Bz[k])
        if d.max() > 0 or (np.isnan(A[k]) != np.isnan(Bz[k])).any():
            idx = np.argwhere((d > 0) | (np.isnan(A[k]) != np.isnan(Bz[k])))
            print(f"{k} {A[k].shape}: {len(idx)} entries differ; first {idx[:6].tolist()}: A {A[k][tuple(idx[0])]} "
                  f"B {Bz[k][tuple(idx[0])]}")
            rows = sorted(set(idx[:, 0].tolist()))
            trs = sorted(set(idx[:, -1].tolist()))
            print(f"  rows {rows[:10]}, components {sorted(set(idx[:, 1].tolist()))}, trajectories {trs[:40]}")
            print(f"  winners (iteration 0) of those: A {A['choices'][0][trs[:40]].tolist()}")
            t = trs[0]
            print(f"  trajectory {t}: A rows N-1, N {A[k][-2:, :, t].tolist()}  B {Bz[k][-2:, :, t].tolist()}")
            print(f"  all winners (iteration 0) histogram A {np.bincount(A['choices'][0].astype(int) + 1).tolist()}")
    ca, cb = A["costs"], Bz["costs"]
    for it in range(ca.shape[0]):
        da = np.abs(np.nan_to_num(ca[it]) - np.nan_to_num(cb[it]))
        nan_diff = np.isnan(ca[it]) != np.isnan(cb[it])
        ch = A["choices"][it] != Bz["choices"][it]
        if da.max() > 0 or nan_diff.any() or ch.any():
            tr = np.where((da > 0).any(0) | nan_diff.any(0) | ch)[0]
            t = tr[0]
            print(f"iteration {it}: {len(tr)} trajectories differ; first {t}: costs A {ca[it][:, t]} B {cb[it][:, t]} "
                  f"choice {A['choices'][it][t]} {Bz['choices'][it][t]}")
            return
    print("candidate costs and choices bitwise equal;",
          {k: bool(np.array_equal(A[k], Bz[k], equal_nan=True)) for k in ("Xnom", "Unom", "Xaux", "Uaux")})


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 256)
    else:
        cmp(sys.argv[2], sys.argv[3])
