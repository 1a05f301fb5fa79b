"""Generate golden vectors by RUNNING THE REFERENCE (lmcggg/differentiable-tube-mpc) on CPU.

Usage (container with /root/reference only; never on the GPU box):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

The reference is copied to /tmp/dtmpc_golden_ref/diff_tube_mpc_strict_pt (its scripts hard-code that
package name and write relative output directories, so it must never run from /root/reference).
Outputs (small .npz data files) go next to this script.  Fixtures are inputs + the reference's
outputs; no reference source text is stored.

Fixture sets
  kat_{f64,f32}.npz      per-function known-answer tests on random points
  ilqr_{f64,f32}.npz     nominal + ancillary iLQR solves, sensitivity, DOC gradient (B = 5 starts)
  closed_loop_{f64,f32}.npz  the reference's own paper-mode loop (_run_dubins_paper), H = 3,
                         injected disturbances, every solver call recorded
  nominal_receding.npz   run_nominal.py's receding-horizon nominal MPC (config #1), H = 2
  config.json            the configuration used (configs/dubins.yaml, device -> cpu)
"""
from __future__ import annotations

import json
import math
import os
import shutil
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
PKG = "diff_tube_mpc_strict_pt"


def _import_reference():
    root = os.path.join(tempfile.gettempdir(), "dtmpc_golden_ref")
    dst = os.path.join(root, PKG)
    if os.path.exists(root):
        shutil.rmtree(root)
    shutil.copytree(REF, dst, ignore=shutil.ignore_patterns("__pycache__", "*.pyc", "*.png", ".git"))
    sys.path.insert(0, root)
    os.chdir(root)
    import yaml

    with open(os.path.join(dst, "configs", "dubins.yaml")) as f:
        cfg = yaml.safe_load(f)
    cfg["device"] = "cpu"
    return root, cfg


def main() -> None:
    sys.dont_write_bytecode = True
    root, cfg = _import_reference()
    import torch

    torch.set_num_threads(1)
    from diff_tube_mpc_strict_pt.core import barrier as rbar
    from diff_tube_mpc_strict_pt.core import cost_derivs as rcd
    from diff_tube_mpc_strict_pt.core import ddp as rddp
    from diff_tube_mpc_strict_pt.core import tube_mpc as rtm
    from diff_tube_mpc_strict_pt.core.control import BoxClampControl
    from diff_tube_mpc_strict_pt.core.systems import dubins as rdub
    from diff_tube_mpc_strict_pt.core.systems import dubins_aug_jac as raj
    from diff_tube_mpc_strict_pt.core.systems import dubins_obstacles as robs

    with open(os.path.join(HERE, "config.json"), "w") as f:
        json.dump(cfg, f, indent=1, sort_keys=True)

    sc = cfg["system"]
    obs = [robs.CircleObstacle(center=tuple(o["center"]), radius=float(o["radius"])) for o in cfg["environment"]["obstacles"]]
    beta = float(cfg["environment"]["obstacle_smoothmin_beta"])
    eps = float(cfg["dbas"]["eps"])
    N = int(sc["horizon_N"])
    dub = rdub.DubinsConfig(dt=float(sc["dt"]), v_max=float(sc["control_bounds"]["v_max"]),
                            omega_max=float(sc["control_bounds"]["omega_max"]),
                            w_low=tuple(sc["disturbance"]["w_low"]), w_high=tuple(sc["disturbance"]["w_high"]),
                            x_target=tuple(sc["target"]))
    alphas = tuple(float(a) for a in sc["line_search_alphas"])

    for dtype, tag in ((torch.float64, "f64"), (torch.float32, "f32")):
        g = torch.Generator().manual_seed(1234)
        # ------------------------------------------------------------------ KATs
        n = 96
        px = torch.rand(n, generator=g, dtype=torch.float64) * 12.0 - 1.0
        py = torch.rand(n, generator=g, dtype=torch.float64) * 12.0 - 1.0
        # put some points close to / inside the obstacles (relaxed barrier branch)
        for j in range(0, 24):
            o = obs[j % len(obs)]
            r = (0.5 + 0.55 * (j / 24.0)) * o.radius
            a = 2 * math.pi * j / 24.0
            px[j] = o.center[0] + r * math.cos(a)
            py[j] = o.center[1] + r * math.sin(a)
        th = torch.rand(n, generator=g, dtype=torch.float64) * 6.0 - 3.0
        bb = torch.rand(n, generator=g, dtype=torch.float64) * 2.0
        uu = torch.stack([torch.rand(n, generator=g, dtype=torch.float64) * 20 - 10,
                          torch.rand(n, generator=g, dtype=torch.float64) * 6.2 - 3.1], 1)
        xh = torch.stack([px, py, th, bb], 1).to(dtype)
        uu = uu.to(dtype)
        zs = torch.cat([torch.linspace(-2.0, 2.0, 41, dtype=torch.float64),
                        torch.tensor([-1e-3, -1e-5, 0.0, 1e-5, 5e-5, 1e-4, 2e-4, 1e-3, 0.05, 0.1, 0.3], dtype=torch.float64)]).to(dtype)
        kat = {"xh": xh.numpy(), "u": uu.numpy(), "z": zs.numpy()}
        kat["dubins_step"] = rdub.dubins_step(xh[:, :3], uu, cfg=dub).numpy()
        hs, gs, hm, gm, h1, g1 = [], [], [], [], [], []
        for i in range(n):
            x3 = xh[i, :3]
            hs.append(robs.h_multi_circle_obstacles(x3, obstacles=obs, beta=beta))
            gs.append(robs.grad_h_multi_circle_obstacles(x3, obstacles=obs, beta=beta))
            hm.append(robs.h_min_circle_obstacles(x3, obstacles=obs))
            gm.append(robs.grad_h_min_circle_obstacles(x3, obstacles=obs))
            h1.append(robs.h_circle_obstacle(x3, obs=obs[0]))
            g1.append(robs.grad_h_circle_obstacle(x3, obs=obs[0]))
        kat["h_smoothmin"] = torch.stack(hs).numpy()
        kat["gh_smoothmin"] = torch.stack(gs).numpy()
        kat["h_min"] = torch.stack(hm).numpy()
        kat["gh_min"] = torch.stack(gm).numpy()
        kat["h_single"] = torch.stack(h1).numpy()
        kat["gh_single"] = torch.stack(g1).numpy()
        for a_name, a_val in (("a0", 0.0), ("a05", 0.05)):
            at = torch.tensor(a_val, dtype=dtype)
            kat[f"B_relaxed_{a_name}"] = rbar.relaxed_inverse_barrier_B_alpha(zs, alpha=at, eps=eps).numpy()
            kat[f"dB_relaxed_{a_name}"] = raj._dB_relaxed_inv_dz(zs, alpha=at, eps=eps).numpy()
        kat["B_log"] = rbar.barrier_B(zs, barrier_type="log", eps=eps).numpy()
        # DBaS step + augmented jacobian for three settings
        settings = {
            "s0": dict(agg="smoothmin", btype="inverse", alpha=0.0, gamma=0.0),
            "s1": dict(agg="min", btype="inverse", alpha=0.05, gamma=0.3),
            "s2": dict(agg="smoothmin", btype="log", alpha=0.0, gamma=-0.5),
        }
        for sname, st in settings.items():
            dbc = rbar.DBaSConfig(barrier_type=st["btype"], alpha=torch.tensor(st["alpha"], dtype=dtype),
                                  gamma=torch.tensor(st["gamma"], dtype=dtype), eps=eps)
            if st["agg"] == "smoothmin":
                h = lambda x_in: robs.h_multi_circle_obstacles(x_in, obstacles=obs, beta=beta)
            else:
                h = lambda x_in: robs.h_min_circle_obstacles(x_in, obstacles=obs)
            f = lambda x, u: rdub.dubins_step(x, u, cfg=dub)
            nxt, A, Bm = [], [], []
            for i in range(n):
                xn, bn = rbar.dbas_step(x_k=xh[i, :3], u_k=uu[i], b_k=xh[i, 3], f=f, h=h, cfg=dbc)
                nxt.append(torch.cat([xn, bn.view(1)]))
                Ai, Bi = raj.dubins_augmented_jacobian(xh[i], uu[i], cfg=dub, obs=obs, db_cfg=dbc, obs_beta=beta,
                                                       obs_agg=st["agg"])
                A.append(Ai)
                Bm.append(Bi)
            kat[f"fhat_{sname}"] = torch.stack(nxt).numpy()
            kat[f"A_{sname}"] = torch.stack(A).numpy()
            kat[f"B_{sname}"] = torch.stack(Bm).numpy()
            kat[f"b0_{sname}"] = torch.stack([rbar.dbas_init_b0(xh[i, :3], h=h, cfg=dbc) for i in range(n)]).numpy()
        np.savez_compressed(os.path.join(HERE, f"kat_{tag}.npz"), **kat)

        # ------------------------------------------------------------------ solver fixtures
        # wiring of core/tube_mpc.py:813-976 (paper mode), built from the reference's own functions
        db_cfg = rbar.DBaSConfig(barrier_type="inverse", alpha=torch.tensor(0.0, dtype=dtype),
                                 gamma=torch.tensor(0.0, dtype=dtype), eps=eps)
        h = lambda x_in: robs.h_multi_circle_obstacles(x_in, obstacles=obs, beta=beta)
        f = lambda x, u: rdub.dubins_step(x, u, cfg=dub)
        ctrl = BoxClampControl(u_min=torch.tensor([float(sc["control_bounds"]["v_min"]), -dub.omega_max], dtype=dtype),
                               u_max=torch.tensor([dub.v_max, dub.omega_max], dtype=dtype))
        target = torch.tensor(dub.x_target, dtype=dtype)
        cn = cfg["cost_nominal"]
        Qn, Rn, Qfn = (torch.tensor(cn[k], dtype=dtype) for k in ("Q", "R", "Qf"))
        qbn = torch.tensor(float(cn["q_b"]), dtype=dtype)
        fjac = lambda xh_, vk: raj.dubins_augmented_jacobian(xh_, vk, cfg=dub, obs=obs, obs_beta=beta,
                                                              obs_agg="smoothmin", db_cfg=db_cfg)

        def f_hat(xk, uk):
            xn, bn = rbar.dbas_step(x_k=xk[:-1], u_k=uk, b_k=xk[-1], f=f, h=h, cfg=db_cfg)
            return torch.cat([xn, bn.view(1)], 0)

        def nominal_solve(x0h, V0, icfg, counter):
            def sc_(x, v, k):
                dx = x[:-1] - target
                return (Qn * dx * dx).sum() + (Rn * v * v).sum() + qbn * (x[-1] * x[-1])

            def tc_(x):
                dx = x[:-1] - target
                return (Qfn * dx * dx).sum() + qbn * (x[-1] * x[-1])

            def sd_(x, v, k):
                if k == 0:
                    counter[0] += 1
                return rcd.nominal_cost_derivs_u(x_hat=x, u=v, target=target, Q=Qn, R=Rn, qb=qbn)

            def td_(x):
                px_, pxx_ = rcd.nominal_terminal_derivs(x_hat_N=x, target=target, Qf=Qfn)
                px_[-1] = 2.0 * qbn * x[-1]
                pxx_[-1, -1] = 2.0 * qbn
                return px_, pxx_

            return rddp.ilqr_solve(x0=x0h, V_init=V0, cfg=icfg, f=f_hat, ctrl=ctrl, f_jac=fjac, stage_cost=sc_,
                                   terminal_cost=tc_, stage_derivs=sd_, terminal_derivs=td_)

        def aux_pieces(Xr, Ur, Qa, Ra, qba):
            def sc_(x, v, k):
                dx = x[:-1] - Xr[k]
                du = v - Ur[k]
                return (Qa * dx * dx).sum() + (Ra * du * du).sum() + qba * (x[-1] * x[-1])

            def tc_(x):
                dx = x[:-1] - Xr[N]
                return (Qa * dx * dx).sum() + qba * (x[-1] * x[-1])

            def sd_(x, v, k):
                return rcd.auxiliary_cost_derivs_u(x_hat=x, u=v, x_ref=Xr[k], u_ref=Ur[k], Q=Qa, R=Ra, qb=qba)

            def td_(x):
                px_, pxx_ = rcd.auxiliary_terminal_derivs(x_hat_N=x, x_ref_N=Xr[N], Qf=Qa)
                px_[-1] = 2.0 * qba * x[-1]
                pxx_[-1, -1] = 2.0 * qba
                return px_, pxx_

            return sc_, tc_, sd_, td_

        fails = []

        def guarded(fn, *a, **kw):
            try:
                return fn(*a, **kw)
            except FloatingPointError as e:  # recorded: the reference raised on this case
                fails.append(str(e))
                raise

        starts = [(0.0, 0.0, math.pi / 4), (1.0, 3.0, 0.3), (3.0, 0.5, 1.2), (2.6, 2.4, 0.9), (0.4, 0.9, 1.5),
                  (1.5, 0.2, 0.6), (0.2, 1.8, 1.0), (5.0, 5.0, 0.5)]
        theta = (1.0, 1.0, 1.0, 1.0, 1.0, 1.0)
        thetas = [theta, (0.7, 1.3, 0.2, 0.5, 2.0, 0.8), (1.0, 1.0, 1.0, 1.0, 1.0, 1.0), (2.0, 0.5, 1.0, 1.5, 0.3, 0.4),
                  (1.0, 1.0, 1.0, 0.1, 0.1, 1.0), (1.0, 1.0, 1.0, 1.0, 1.0, 1.0), (0.5, 0.5, 2.0, 0.8, 1.2, 0.6),
                  (1.0, 1.0, 1.0, 1.0, 1.0, 1.0)]
        # conditioning probe: the reference re-run on inputs perturbed by a few ulps (relative)
        PERT = 1.0 + (1e-14 if dtype == torch.float64 else 3e-7)

        def spread(a, b):
            return float((a - b).abs().max() / max(1.0, float(a.abs().max())))
        out = {k: [] for k in ("x0", "theta", "Vinit_nom", "X_nom_fixed", "V_nom_fixed", "X_nom", "V_nom", "it_nom",
                               "Vinit_aux", "x0_aux", "X_aux_fixed", "V_aux_fixed", "X_aux", "V_aux", "it_aux", "dX", "dV",
                               "dlam", "grad", "cond_nom_fixed", "cond_nom", "cond_aux_fixed", "cond_aux",
                               "cond_sens")}
        def attempt(fn, *a, **kw):
            """(result, None) or (None, message) when the reference raises FloatingPointError"""
            try:
                return fn(*a, **kw), None
            except FloatingPointError as e:
                return None, str(e)

        def sens_of(Xa_, Va_, x_nom, sd_, td_):
            return rddp.ddp_sensitivity(
                X=Xa_, V=Va_, f=f_hat, ctrl=ctrl, f_jac=fjac,
                stage_hess=lambda x, v, k: sd_(x, v, k)[2:],
                terminal_hess=lambda x: td_(x)[1],
                upper_grad_x=lambda x, k: torch.cat([2.0 * (x[:-1] - x_nom[k]), (2.0 * x[-1]).view(1)]),
                upper_grad_u=lambda v, k: torch.zeros_like(v),
                upper_grad_xN=lambda x: torch.cat([2.0 * (x[:-1] - x_nom[N]), (2.0 * x[-1]).view(1)]))

        nanX = torch.full((N + 1, 4), float("nan"), dtype=dtype)
        nanV = torch.full((N, 2), float("nan"), dtype=dtype)
        failures = []
        for si, (s0, th_) in enumerate(zip(starts, thetas)):
            x0 = torch.tensor(s0, dtype=dtype)
            b0 = rbar.dbas_init_b0(x0, h=h, cfg=db_cfg)
            x0h = torch.cat([x0, b0.view(1)])
            gV = torch.Generator().manual_seed(77 + si)
            V0 = (torch.rand(N, 2, generator=gV, dtype=torch.float64) * torch.tensor([4.0, 2.0], dtype=torch.float64)
                  - torch.tensor([1.0, 1.0], dtype=torch.float64)).to(dtype)
            c3 = rddp.ILQRConfig(horizon=N, nx=4, nu=2, max_iter=3, tol=-1.0, line_search_alphas=alphas)
            c10 = rddp.ILQRConfig(horizon=N, nx=4, nu=2, max_iter=10, tol=1e-3, line_search_alphas=alphas)
            cnt = [0]
            rf, ef = attempt(nominal_solve, x0h, V0, c3, [0])
            rn, en = attempt(nominal_solve, x0h, V0, c10, cnt)
            if ef or en:
                failures.append((si, "nominal", ef or en))
            Xf, Vf = rf if rf else (nanX, nanV)
            Xn, Vn = rn if rn else (nanX, nanV)
            pf, _ = attempt(nominal_solve, x0h, V0 * PERT, c3, [0])
            pn, _ = attempt(nominal_solve, x0h, V0 * PERT, c10, [0])
            out["cond_nom_fixed"].append(spread(Xf, pf[0]) if (rf and pf) else float("inf"))
            out["cond_nom"].append(spread(Xn, pn[0]) if (rn and pn) else float("inf"))
            out["x0"].append(x0h.numpy())
            out["theta"].append(np.asarray(th_))
            out["Vinit_nom"].append(V0.numpy())
            out["X_nom_fixed"].append(Xf.numpy())
            out["V_nom_fixed"].append(Vf.numpy())
            out["X_nom"].append(Xn.numpy())
            out["V_nom"].append(Vn.numpy())
            out["it_nom"].append(cnt[0])
            # ancillary: plant start perturbed from the nominal start, tracks the nominal plan
            xa = x0 + torch.tensor([0.03, -0.02, 0.04], dtype=dtype) * (si % 3 - 1)
            ba = rbar.dbas_init_b0(xa, h=h, cfg=db_cfg)
            xah = torch.cat([xa, ba.view(1)])
            Xr, Ur = Xn[:, :-1], Vn
            Qa = torch.tensor(th_[:3], dtype=dtype)
            Ra = torch.tensor(th_[3:5], dtype=dtype)
            qba = torch.tensor(th_[5], dtype=dtype)
            sc_, tc_, sd_, td_ = aux_pieces(Xr, Ur, Qa, Ra, qba)
            Va0 = torch.roll(Vn, shifts=-1, dims=0).clone()
            cnt = [0]

            def sd_count(x, v, k, _sd=sd_, _c=cnt):
                if k == 0:
                    _c[0] += 1
                return _sd(x, v, k)

            res_aux = {}
            for nm, it_, tl_, sdf in (("fixed", 4, -1.0, sd_), ("tol", 20, 1e-3, sd_count)):
                icfg = rddp.ILQRConfig(horizon=N, nx=4, nu=2, max_iter=it_, tol=tl_, line_search_alphas=alphas)
                kw = dict(f=f_hat, ctrl=ctrl, f_jac=fjac, stage_cost=sc_, terminal_cost=tc_, terminal_derivs=td_)
                r_, e_ = (None, "nominal failed") if rn is None else attempt(rddp.ilqr_solve, x0=xah, V_init=Va0, cfg=icfg,
                                                                             stage_derivs=sdf, **kw)
                p_, _ = (None, None) if r_ is None else attempt(rddp.ilqr_solve, x0=xah, V_init=Va0 * PERT, cfg=icfg,
                                                               stage_derivs=sd_, **kw)
                if e_ and rn is not None:
                    failures.append((si, "aux_" + nm, e_))
                res_aux[nm] = (r_ if r_ else (nanX, nanV), spread(r_[0], p_[0]) if (r_ and p_) else float("inf"))
            (Xaf, Vaf), out_c1 = res_aux["fixed"]
            (Xa, Va), out_c2 = res_aux["tol"]
            out["cond_aux_fixed"].append(out_c1)
            out["cond_aux"].append(out_c2)
            out["Vinit_aux"].append(Va0.numpy())
            out["x0_aux"].append(xah.numpy())
            out["X_aux_fixed"].append(Xaf.numpy())
            out["V_aux_fixed"].append(Vaf.numpy())
            out["X_aux"].append(Xa.numpy())
            out["V_aux"].append(Va.numpy())
            out["it_aux"].append(cnt[0])
            # sensitivity with the paper upper loss (core/tube_mpc.py:924-957) + DOC gradient (:963-976)
            x_nom = Xn[:, :-1]
            sens, es = (None, "aux failed") if torch.isnan(Xa).any() else attempt(sens_of, Xa, Va, x_nom, sd_, td_)
            sp_, _ = (None, None) if sens is None else attempt(sens_of, Xa * PERT, Va, x_nom, sd_, td_)
            if sens is None:
                dX, dV, dl = nanX, nanV, nanX
            else:
                dX, dV, dl = sens.delta_X, sens.delta_V, sens.delta_lambda
            out["cond_sens"].append(max(spread(dX, sp_.delta_X), spread(dV, sp_.delta_V)) if (sens and sp_) else float("inf"))
            x_aux, b_aux = Xa[:, :-1], Xa[:, -1]
            L = (x_aux - x_nom).pow(2).sum() + (b_aux.pow(2)).sum()
            dx = x_aux - x_nom
            du = Va - Ur
            gQ = (2.0 * dx[:-1] * dX[:-1, :-1]).sum(dim=0) + 2.0 * dx[-1] * dX[-1, :-1]
            gR = (2.0 * du * dV).sum(dim=0)
            gqb = (2.0 * b_aux[:-1] * dX[:-1, -1]).sum() + 2.0 * b_aux[-1] * dX[-1, -1]
            out["dX"].append(dX.numpy())
            out["dV"].append(dV.numpy())
            out["dlam"].append(dl.numpy())
            out["grad"].append(torch.cat([L.view(1), gQ, gR, gqb.view(1)]).numpy())
        print(f"[{tag}] reference failures (FloatingPointError):", failures, flush=True)
        np.savez_compressed(os.path.join(HERE, f"ilqr_{tag}.npz"), **{k: np.stack([np.asarray(v) for v in vs]) for k, vs in out.items()})

        # ------------------------------------------------------------------ the reference's own loop
        c2 = json.loads(json.dumps(cfg))
        c2["use_float64"] = dtype == torch.float64
        c2["system"]["task_horizon_H"] = 3
        H = 3
        gw = torch.Generator().manual_seed(99)
        w_seq = [(torch.rand(3, generator=gw, dtype=torch.float64) * 0.1 - 0.05).to(dtype) for _ in range(H)]
        rec = {"nom": [], "aux": [], "sens": []}
        orig_ilqr, orig_sens, orig_sd = rtm.ilqr_solve, rtm.ddp_sensitivity, rtm.sample_disturbance
        calls = {"n": 0, "t": 0}

        def rec_ilqr(**kw):
            X, V = orig_ilqr(**kw)
            key = "nom" if kw.get("debug_name") == "iLQR-nominal" else "aux"
            rec[key].append((kw["x0"].clone().numpy(), kw["V_init"].clone().numpy(), X.numpy(), V.numpy()))
            return X, V

        def rec_sens(**kw):
            r = orig_sens(**kw)
            rec["sens"].append((r.delta_X.numpy(), r.delta_V.numpy(), r.delta_lambda.numpy()))
            return r

        def fake_w(x, cfg):
            w = w_seq[calls["t"]]
            calls["t"] += 1
            return w

        rtm.ilqr_solve, rtm.ddp_sensitivity, rtm.sample_disturbance = rec_ilqr, rec_sens, fake_w
        run_dir = os.path.join(root, "out_cl_" + tag)
        try:
            res = rtm.run_closed_loop_experiment(c2, device=torch.device("cpu"), run_dir=run_dir)
        finally:
            rtm.ilqr_solve, rtm.ddp_sensitivity, rtm.sample_disturbance = orig_ilqr, orig_sens, orig_sd
        cl = {"w": np.stack([w.numpy() for w in w_seq])}
        for name in ("x_real", "u_real", "x_bar", "u_bar", "b_real", "loss", "Qa_history", "Ra_history", "qba_history"):
            cl[name] = np.load(os.path.join(run_dir, name + ".npy"))
        for key in ("nom", "aux"):
            for j, nm in enumerate(("x0", "Vinit", "X", "V")):
                cl[f"{key}_{nm}"] = np.stack([r[j] for r in rec[key]])
        for j, nm in enumerate(("dX", "dV", "dlam")):
            cl[f"sens_{nm}"] = np.stack([r[j] for r in rec["sens"]])
        cl["final_loss"] = np.asarray(res["summary"]["final_loss"])
        np.savez_compressed(os.path.join(HERE, f"closed_loop_{tag}.npz"), **cl)
        print(f"[{tag}] closed loop loss:", cl["loss"], flush=True)

    # ------------------------------------------------------------------ run_nominal.py (config #1)
    sys.path.insert(0, os.path.join(root, PKG))
    import run_nominal as rn

    c3 = json.loads(json.dumps(cfg))
    c3["system"]["task_horizon_H"] = 2
    rd = os.path.join(root, "out_nominal")
    res = rn.run_nominal_receding(c3, device=torch.device("cpu"), run_dir=rd)
    nr = {name: np.load(os.path.join(rd, name + ".npy")) for name in ("x_bar", "u_bar", "b_real")}
    nr["H_ran"] = np.asarray(res["summary"]["H_ran"])
    np.savez_compressed(os.path.join(HERE, "nominal_receding.npz"), **nr)
    print("nominal receding:", nr["x_bar"], nr["u_bar"], flush=True)
    print("golden vectors written to", HERE)


if __name__ == "__main__":
    main()
