import ctypes as C, json, os, sys
import numpy as np, torch
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "differentiable-tube-mpc_amd"), os.path.join(REPO, "tests")]
from _common import golden
from diff_tube_mpc_strict_pt import _lib
from diff_tube_mpc_strict_pt.core import ddp
from diff_tube_mpc_strict_pt.core.ddp import to_soa, from_soa
from diff_tube_mpc_strict_pt.core.problem import ILQRConfig
from diff_tube_mpc_strict_pt.core.receding import receding_setup_from_config
g = golden("receding_R4")
cfg = json.loads(str(g["config"]))
problem, cost, icfg = receding_setup_from_config(cfg)
dev = torch.device("cuda:0")
N = problem.horizon
for it in (1, 2):
    c = ILQRConfig(horizon=N, max_iter=it, tol=-1.0, reg=icfg.reg, line_search_alphas=icfg.line_search_alphas)
    x = torch.tensor([[0.0, 0.0, np.pi / 4]], dtype=torch.float64, device=dev)
    U = torch.zeros(1, N, 2, dtype=torch.float64, device=dev); U[:, :, 0] = 10.0
    lib = _lib.load()
    B = 1
    work = torch.zeros(lib.dtmpc_receding_workspace_bytes(1, N, B) // 8, dtype=torch.float64, device=dev)
    log = torch.zeros(1, 6, B, dtype=torch.float64, device=dev)
    ints = [torch.zeros(B, dtype=torch.int32, device=dev) for _ in range(4)]
    Us = to_soa(U)
    rc = lib.dtmpc_nominal_receding(1, C.byref(problem.to_c()), C.byref(cost.to_c()), C.byref(c.to_c()), B, 1, 0.25,
                                    x.t().contiguous().data_ptr(), Us.data_ptr(), log.data_ptr(), *[t.data_ptr() for t in ints],
                                    work.data_ptr(), _lib.stream_of(x))
    torch.cuda.synchronize()
    Xw = work[: (N + 1) * 4].view(N + 1, 4).cpu().numpy()
    Kw = work[(N + 1) * 4: (N + 1) * 4 + N * 8].view(N, 8).cpu().numpy()
    kw = work[(N + 1) * 4 + N * 8: (N + 1) * 4 + N * 10].view(N, 2).cpu().numpy()
    b0 = ddp.dbas_init(problem, x)
    xh = torch.cat([x, b0[:, None]], 1)
    U = torch.zeros(1, N, 2, dtype=torch.float64, device=dev); U[:, :, 0] = 10.0
    r = ddp.ilqr_solve(problem=problem, cost=cost, cfg=c, x0=xh, V_init=U)
    X0t = ddp.rollout(problem, xh, U.clone())
    A, Bm, lx, lu = ddp.linearize(problem, cost, X0t, U.clone())
    from oracle.oracle import Oracle
    o = Oracle(np.float64)
    Ao, Bo, lxo, luo = o.linearize(problem.to_c(), cost.to_c(), X0t.cpu().numpy(), U.cpu().numpy())
    d = np.abs(A.cpu().numpy() - Ao)
    print("lin A maxdiff at", np.unravel_index(d.argmax(), d.shape), d.max(), "dev A0", A[0, 0].cpu().numpy(), "or A0", Ao[0, 0])
    print("it", it, "rc", rc, "log", log[0, :, 0].cpu().numpy(), [t.item() for t in ints])
    print(" X diff", np.abs(Xw - r.X[0].cpu().numpy()).max(), "X0", Xw[0], r.X[0, 0].cpu().numpy(), "X1", Xw[1], r.X[0, 1].cpu().numpy())
    print(" K diff", np.abs(Kw - r.K[0].reshape(N, 8).cpu().numpy()).max(), "k diff", np.abs(kw - r.k[0].cpu().numpy()).max())
    print(" K0", Kw[0], r.K[0, 0].reshape(8).cpu().numpy(), "k0", kw[0], r.k[0, 0].cpu().numpy())
    np.savez(f"gpurun_out/diag3_it{it}.npz", X=Xw, K=Kw, k=kw, rX=r.X[0].cpu().numpy(), rK=r.K[0].cpu().numpy(), rk=r.k[0].cpu().numpy())
