"""Golden vectors for the GENERAL (softplus/tanh-parameterised, adapt_nominal) IFT path, produced by
RUNNING THE REFERENCE on CPU (core/tube_mpc.py:40-663, core/ift.py:35-92, core/params.py:9-59).

Usage (container with /root/reference only; never on the GPU box):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_general.py

Like make_golden.py the reference runs from a copy under /tmp; only inputs + outputs are stored.

Fixture sets
  general_{A_f64,A_f32,B_f64,C_f64}.npz   the reference's own general closed loop, H = 3 (C: H = 2),
        injected disturbances; every ilqr_solve / ddp_sensitivity / ift_gradient call recorded
        (inputs and outputs), raw theta / theta_bar before every update and at the end.
        A: configs/dubins.yaml with adapt_nominal = true (paper_dubins_mode off)
        B: A + gamma_raw 0.5, alpha_raw -3, nominal_tightening raw -1, grad_clip_norm 5
        C: log barrier in the DBaS dynamics, adapt_nominal = false (general path, ancillary only)
  ift_general_f64.npz   ift_gradient KATs on tapes driven near / into the obstacles (relaxed barrier
        branch, alpha / gamma / tightening gradients), for the ancillary and nominal closure sets.
"""
from __future__ import annotations

import json
import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import _import_reference  # noqa: E402


def variants(cfg):
    a = json.loads(json.dumps(cfg))
    a["paper_dubins_mode"] = False
    a["adaptation"]["adapt_nominal"] = True
    a["system"]["task_horizon_H"] = 3
    b = json.loads(json.dumps(a))
    b["dbas"]["gamma"] = 0.5
    b["dbas"]["alpha"] = -3.0
    b["dbas"]["nominal_tightening"] = -1.0
    b["adaptation"]["grad_clip_norm"] = 5.0
    c = json.loads(json.dumps(a))
    c["dbas"]["barrier_type"] = "log"
    c["adaptation"]["adapt_nominal"] = False
    c["system"]["task_horizon_H"] = 2
    return {"A": a, "B": b, "C": c}


def main() -> None:
    sys.dont_write_bytecode = True
    root, cfg = _import_reference()
    import torch

    torch.set_num_threads(1)
    from diff_tube_mpc_strict_pt.core import barrier as rbar
    from diff_tube_mpc_strict_pt.core import ift as rift
    from diff_tube_mpc_strict_pt.core import tube_mpc as rtm
    from diff_tube_mpc_strict_pt.core.systems import dubins as rdub
    from diff_tube_mpc_strict_pt.core.systems import dubins_obstacles as robs

    runs = [("A", torch.float64), ("A", torch.float32), ("B", torch.float64), ("C", torch.float64)]
    vs = variants(cfg)
    for name, dtype in runs:
        c2 = json.loads(json.dumps(vs[name]))
        c2["use_float64"] = dtype == torch.float64
        tag = f"{name}_{'f64' if dtype == torch.float64 else 'f32'}"
        H = int(c2["system"]["task_horizon_H"])
        gw = torch.Generator().manual_seed(77)
        w_seq = [(torch.rand(3, generator=gw, dtype=torch.float64) * 0.1 - 0.05).to(dtype) for _ in range(H)]
        rec = {"ilqr": [], "sens": [], "ift": [], "theta_snap": []}
        orig = (rtm.ilqr_solve, rtm.ddp_sensitivity, rtm.ift_gradient, rtm.sample_disturbance)
        tcount = {"t": 0}

        def rec_ilqr(**kw):
            X, V = orig[0](**kw)
            rec["ilqr"].append((kw["x0"].detach().clone().numpy(), kw["V_init"].detach().clone().numpy(),
                                X.detach().numpy(), V.detach().numpy()))
            return X, V

        def rec_sens(**kw):
            r = orig[1](**kw)
            rec["sens"].append((r.delta_X.numpy(), r.delta_V.numpy(), r.delta_lambda.numpy()))
            return r

        def rec_ift(**kw):
            # raw parameter values BEFORE this call's update (the tensors are updated in place later)
            snap = [t.detach().clone().numpy().reshape(-1) for t in kw["theta_tensors"]]
            g = orig[2](**kw)
            # a None gradient (parameter unused in the graph, e.g. alpha under the log barrier) is
            # stored as NaN of the parameter's shape
            rec["ift"].append(([np.full(t.shape, np.nan) if x is None else x.detach().numpy()
                                for x, t in zip(g, kw["theta_tensors"])], snap))
            rec["theta_snap"].append(kw["theta_tensors"])
            return g

        def fake_w(x, cfg):
            w = w_seq[tcount["t"]]
            tcount["t"] += 1
            return w

        rtm.ilqr_solve, rtm.ddp_sensitivity, rtm.ift_gradient, rtm.sample_disturbance = rec_ilqr, rec_sens, rec_ift, fake_w
        run_dir = os.path.join(root, "out_general_" + tag)
        try:
            res = rtm.run_closed_loop_experiment(c2, device=torch.device("cpu"), run_dir=run_dir)
        finally:
            rtm.ilqr_solve, rtm.ddp_sensitivity, rtm.ift_gradient, rtm.sample_disturbance = orig
        adapt_nom = bool(c2["adaptation"]["adapt_nominal"])
        out = {"w": np.stack([w.numpy() for w in w_seq]), "config": np.asarray(json.dumps(c2))}
        for nm in ("x_real", "u_real", "x_bar", "u_bar", "b_real", "loss", "Qa_history", "Ra_history", "qba_history"):
            out[nm] = np.load(os.path.join(run_dir, nm + ".npy"))
        il = rec["ilqr"]
        for j, nm in enumerate(("x0", "Vinit", "X", "V")):
            out[f"nom_{nm}"] = np.stack([il[2 * t][j] for t in range(H)])
            out[f"aux_{nm}"] = np.stack([il[2 * t + 1][j] for t in range(H)])
        per = 2 if adapt_nom else 1
        sn = rec["sens"]
        for j, nm in enumerate(("dX", "dV", "dlam")):
            out[f"sens_aux_{nm}"] = np.stack([sn[per * t][j] for t in range(H)])
            if adapt_nom:
                out[f"sens_nom_{nm}"] = np.stack([sn[per * t + 1][j] for t in range(H)])
        ift = rec["ift"]
        # aux grads: Q R Qf qb alpha gamma (+ X_ref, U_ref); nominal: Q R Qf qb alpha gamma tight
        aux_names = ["Q", "R", "Qf", "qb", "alpha", "gamma"] + (["Xref", "Uref"] if adapt_nom else [])
        nom_names = ["Q", "R", "Qf", "qb", "alpha", "gamma", "tight"]
        for i, nm in enumerate(aux_names):
            out[f"gaux_{nm}"] = np.stack([np.asarray(ift[per * t][0][i]) for t in range(H)])
        for i, nm in enumerate(aux_names[:6]):
            out[f"theta_aux_{nm}"] = np.stack([ift[per * t][1][i] for t in range(H)])
        if adapt_nom:
            for i, nm in enumerate(nom_names):
                out[f"gnom_{nm}"] = np.stack([np.asarray(ift[per * t + 1][0][i]) for t in range(H)])
                out[f"theta_nom_{nm}"] = np.stack([ift[per * t + 1][1][i] for t in range(H)])
        # final raw parameters (after the last update)
        last_aux = rec["theta_snap"][per * (H - 1)]
        for i, nm in enumerate(aux_names[:6]):
            out[f"theta_aux_final_{nm}"] = last_aux[i].detach().numpy().reshape(-1)
        if adapt_nom:
            last_nom = rec["theta_snap"][per * (H - 1) + 1]
            for i, nm in enumerate(nom_names):
                out[f"theta_nom_final_{nm}"] = last_nom[i].detach().numpy().reshape(-1)
        out["final_loss"] = np.asarray(res["summary"]["final_loss"])
        np.savez_compressed(os.path.join(HERE, f"general_{tag}.npz"), **out)
        print(f"[{tag}] loss {out['loss']}  x_real[-1] {out['x_real'][-1]}", flush=True)

    # ------------------------------------------------------------------ ift_gradient KATs
    # random tapes near the obstacles; closures exactly as core/tube_mpc.py:461-500 (aux) and
    # :556-585 (nominal), with grad-enabled raw parameters (core/params.py)
    dtype = torch.float64
    sc = cfg["system"]
    obs = [robs.CircleObstacle(center=tuple(o["center"]), radius=float(o["radius"])) for o in cfg["environment"]["obstacles"]]
    beta = float(cfg["environment"]["obstacle_smoothmin_beta"])
    eps = float(cfg["dbas"]["eps"])
    dub = rdub.DubinsConfig(dt=float(sc["dt"]), v_max=10.0, omega_max=math.pi, x_target=tuple(sc["target"]))
    f = lambda x, u: rdub.dubins_step(x, u, cfg=dub)
    h_base = lambda x_in: robs.h_multi_circle_obstacles(x_in, obstacles=obs, beta=beta)
    target = torch.tensor(dub.x_target, dtype=dtype)
    g = torch.Generator().manual_seed(4321)
    N = 12
    cases = 6
    kat = {k: [] for k in ("X", "V", "dX", "dV", "dlam", "Xref", "Uref", "raw_aux", "raw_nom", "btype",
                           "g_aux", "g_nom")}
    for ci in range(cases):
        o = obs[ci % len(obs)]
        # a straight-ish path passing close to (or through) obstacle o
        r0 = 0.6 + 0.25 * ci
        ang = 2 * math.pi * torch.rand(1, generator=g, dtype=dtype).item()
        p0 = torch.tensor([o.center[0] + r0 * math.cos(ang), o.center[1] + r0 * math.sin(ang)], dtype=dtype)
        X = torch.zeros(N + 1, 4, dtype=dtype)
        X[:, 0] = p0[0] + 0.05 * torch.arange(N + 1, dtype=dtype)
        X[:, 1] = p0[1] + 0.03 * torch.arange(N + 1, dtype=dtype) * (1 if ci % 2 else -1)
        X[:, 2] = torch.rand(N + 1, generator=g, dtype=dtype) * 2 - 1
        X[:, 3] = torch.rand(N + 1, generator=g, dtype=dtype) * 3
        V = torch.rand(N, 2, generator=g, dtype=dtype) * 4 - 2
        dX = torch.randn(N + 1, 4, generator=g, dtype=dtype)
        dV = torch.randn(N, 2, generator=g, dtype=dtype)
        dl = torch.randn(N + 1, 4, generator=g, dtype=dtype)
        Xref = X[:, :3] + 0.1 * torch.randn(N + 1, 3, generator=g, dtype=dtype)
        Uref = V + 0.1 * torch.randn(N, 2, generator=g, dtype=dtype)
        btype = "log" if ci == 5 else "inverse"
        # raw parameters: Q R Qf qb alpha gamma (+ tight)
        raw_aux = torch.cat([torch.rand(3, generator=g, dtype=dtype) * 2 - 0.5, torch.rand(2, generator=g, dtype=dtype),
                             torch.rand(3, generator=g, dtype=dtype) * 3, torch.rand(1, generator=g, dtype=dtype),
                             torch.tensor([[-1.0], [0.3], [-4.0], [1.0], [0.5], [-2.0]][ci], dtype=dtype),
                             torch.tensor([[0.0], [0.5], [-0.4], [0.9], [0.2], [-0.7]][ci], dtype=dtype)])
        raw_nom = torch.cat([raw_aux[:6] * 0.7, raw_aux[6:11], torch.tensor([[-1.5], [0.2], [-0.5], [0.0], [0.4], [-3.0]][ci], dtype=dtype)])
        sp = torch.nn.functional.softplus

        def ift_for(raw, nominal):
            ps = [raw[0:3].clone().requires_grad_(True), raw[3:5].clone().requires_grad_(True),
                  raw[5:8].clone().requires_grad_(True), raw[8].clone().requires_grad_(True),
                  raw[9].clone().requires_grad_(True), raw[10].clone().requires_grad_(True)]
            if nominal:
                ps.append(raw[11].clone().requires_grad_(True))
            Xr = Xref.clone().requires_grad_(True)
            Ur = Uref.clone().requires_grad_(True)
            Q, R, Qf, qb = sp(ps[0]), sp(ps[1]), sp(ps[2]), sp(ps[3])
            al = sp(ps[4]) + 1e-6
            ga = torch.tanh(ps[5])
            s = sp(ps[6]) if nominal else None
            h = (lambda xx: h_base(xx) - s) if nominal else h_base
            dbc = rbar.DBaSConfig(barrier_type=btype, alpha=al, gamma=ga, eps=eps)

            def fh(xh, v):
                xn, bn = rbar.dbas_step(x_k=xh[:-1], u_k=v, b_k=xh[-1], f=f, h=h, cfg=dbc)
                return torch.cat([xn, bn.view(1)], dim=0)

            def sc_(xh, v, k):
                d = xh[:-1] - (target if nominal else Xr[k])
                du = v if nominal else v - Ur[k]
                return (Q * d * d).sum() + (R * du * du).sum() + qb * (xh[-1] * xh[-1])

            def tc_(xh):
                d = xh[:-1] - (target if nominal else Xr[N])
                return (Qf * d * d).sum() + qb * (xh[-1] * xh[-1])

            tens = ps + ([] if nominal else [Xr, Ur])
            gr = rift.ift_gradient(inputs=rift.IFTInputs(X=X, V=V, delta_X=dX, delta_V=dV, delta_lambda=dl),
                                   theta_tensors=tens, xi_fn=lambda: X[0].detach(), f_fn=fh, stage_cost_fn=sc_,
                                   terminal_cost_fn=tc_)
            flat = [torch.zeros(t.numel(), dtype=dtype) if gi is None else gi.detach().reshape(-1) for gi, t in zip(gr, tens)]
            return torch.cat(flat).numpy()

        for k_, v_ in (("X", X), ("V", V), ("dX", dX), ("dV", dV), ("dlam", dl), ("Xref", Xref), ("Uref", Uref),
                       ("raw_aux", raw_aux), ("raw_nom", raw_nom)):
            kat[k_].append(v_.numpy())
        kat["btype"].append(1 if btype == "log" else 0)
        kat["g_aux"].append(ift_for(raw_aux, False))
        kat["g_nom"].append(ift_for(raw_nom, True))
    np.savez_compressed(os.path.join(HERE, "ift_general_f64.npz"), **{k: np.stack([np.asarray(v) for v in vs_]) for k, vs_ in kat.items()})
    print("general golden vectors written to", HERE)


if __name__ == "__main__":
    main()
