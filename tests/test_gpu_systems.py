"""The reference's per-function API under its own module names (core.barrier, core.systems.dubins,
core.systems.dubins_obstacles, core.systems.dubins_aug_jac, core.control.BoxClampControl,
core.cost_derivs *_u / *_terminal_derivs), each a HIP kernel of include/dtmpc_systems.h, against the
reference's own outputs on the KAT points (tests/golden/kat_{f64,f32}.npz, written by running the
reference: tests/golden/make_golden.py) at the KAT tolerances.  Clamp / active set and the u-form cost
derivatives have no golden vectors; they are checked against the reference's torch expressions
(core/control.py:61-70, core/cost_derivs.py:58-146) evaluated in the test on the host."""
from __future__ import annotations

import math

import numpy as np
import pytest
import torch

from _common import config, golden

pytestmark = pytest.mark.gpu

DT = {"f64": (np.float64, torch.float64, 1e-12), "f32": (np.float32, torch.float32, 2e-5)}


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("needs a HIP device")
    return torch.device("cuda:0")


def _setup():
    from diff_tube_mpc_strict_pt.core.systems.dubins import DubinsConfig
    from diff_tube_mpc_strict_pt.core.systems.dubins_obstacles import CircleObstacle

    cfg = config()
    sc = cfg["system"]
    dub = DubinsConfig(dt=float(sc["dt"]), v_max=float(sc["control_bounds"]["v_max"]),
                       omega_max=float(sc["control_bounds"]["omega_max"]))
    obs = [CircleObstacle(center=tuple(o["center"]), radius=float(o["radius"])) for o in cfg["environment"]["obstacles"]]
    return dub, obs, float(cfg["environment"]["obstacle_smoothmin_beta"]), float(cfg["dbas"]["eps"])


def _close(a, b, tol):
    a = a.detach().cpu().numpy().astype(np.float64) if isinstance(a, torch.Tensor) else np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    assert a.shape == b.shape, (a.shape, b.shape)
    err = np.abs(a - b) / np.maximum(1.0, np.abs(b))
    assert float(err.max()) <= tol, float(err.max())


@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_dubins_step_and_obstacles_vs_reference_kat(dev, tag):
    from diff_tube_mpc_strict_pt.core.systems import dubins_obstacles as O
    from diff_tube_mpc_strict_pt.core.systems.dubins import dubins_step

    npdt, tdt, tol = DT[tag]
    k = golden(f"kat_{tag}")
    dub, obs, beta, _ = _setup()
    xh = torch.tensor(k["xh"], dtype=tdt, device=dev)
    u = torch.tensor(k["u"], dtype=tdt, device=dev)
    _close(dubins_step(xh[:, :3], u, cfg=dub), k["dubins_step"], tol)
    _close(dubins_step(xh[5, :3], u[5], cfg=dub), k["dubins_step"][5], tol)  # unbatched
    x3 = xh[:, :3]
    _close(O.h_multi_circle_obstacles(x3, obstacles=obs, beta=beta), k["h_smoothmin"], tol)
    _close(O.grad_h_multi_circle_obstacles(x3, obstacles=obs, beta=beta), k["gh_smoothmin"], tol)
    _close(O.h_min_circle_obstacles(x3, obstacles=obs), k["h_min"], tol)
    _close(O.grad_h_min_circle_obstacles(x3, obstacles=obs), k["gh_min"], tol)
    _close(O.h_circle_obstacle(x3, obs=obs[0]), k["h_single"], tol)
    _close(O.grad_h_circle_obstacle(x3, obs=obs[0]), k["gh_single"], tol)
    # unbatched point: scalar h, [3] gradient; no obstacles: h = 1, gradient 0 (dubins_obstacles.py:58-61)
    h7 = O.h_multi_circle_obstacles(x3[7], obstacles=obs, beta=beta)
    assert h7.shape == () and abs(float(h7) - float(k["h_smoothmin"][7])) <= tol * max(1.0, abs(float(h7)))
    assert O.grad_h_min_circle_obstacles(x3[7], obstacles=obs).shape == (3,)
    assert torch.equal(O.h_multi_circle_obstacles(x3, obstacles=[]), torch.ones(96, dtype=tdt, device=dev))
    assert torch.equal(O.grad_h_multi_circle_obstacles(x3[0], obstacles=[]), torch.zeros(3, dtype=tdt, device=dev))


@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_barriers_vs_reference_kat(dev, tag):
    from diff_tube_mpc_strict_pt.core.barrier import barrier_B, relaxed_inverse_barrier_B_alpha
    from diff_tube_mpc_strict_pt.core.systems.dubins_aug_jac import _dB_inv_dz, _dB_relaxed_inv_dz, _B_inv

    npdt, tdt, _ = DT[tag]
    tol = 1e-14 if tag == "f64" else 1e-6
    k = golden(f"kat_{tag}")
    _, _, _, eps = _setup()
    z = torch.tensor(k["z"], dtype=tdt, device=dev)
    for name, alpha in (("a0", 0.0), ("a05", 0.05)):
        B = relaxed_inverse_barrier_B_alpha(z, alpha=torch.tensor(alpha, dtype=tdt), eps=eps).cpu().numpy()
        dB = _dB_relaxed_inv_dz(z, alpha=alpha, eps=eps).cpu().numpy()
        assert np.allclose(B, k[f"B_relaxed_{name}"], rtol=tol, atol=0), name
        assert np.allclose(dB, k[f"dB_relaxed_{name}"], rtol=tol, atol=0), name
    assert np.allclose(barrier_B(z, barrier_type="log", eps=eps).cpu().numpy(), k["B_log"], rtol=tol, atol=tol)
    # the plain inverse barrier and its derivative (core/barrier.py:62-72, dubins_aug_jac.py:22-28)
    zc = np.maximum(k["z"].astype(np.float64), eps)
    assert np.allclose(barrier_B(z, barrier_type="inverse", eps=eps).cpu().numpy(), 1.0 / zc, rtol=1e-6, atol=0)
    assert np.allclose(_B_inv(z, eps).cpu().numpy(), 1.0 / zc, rtol=1e-6, atol=0)
    assert np.allclose(_dB_inv_dz(z, eps).cpu().numpy(), -1.0 / (zc * zc), rtol=1e-6, atol=0)
    with pytest.raises(ValueError, match="alpha"):
        relaxed_inverse_barrier_B_alpha(z, alpha=-0.1)
    with pytest.raises(ValueError, match="barrier_type"):
        barrier_B(z, barrier_type="quadratic")


SETTINGS = {"s0": dict(agg="smoothmin", btype="inverse", alpha=0.0, gamma=0.0),
            "s1": dict(agg="min", btype="inverse", alpha=0.05, gamma=0.3),
            "s2": dict(agg="smoothmin", btype="log", alpha=0.0, gamma=-0.5)}


@pytest.mark.parametrize("setting", ["s0", "s1", "s2"])
@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_dbas_step_and_augmented_jacobian_vs_reference_kat(dev, tag, setting):
    """dbas_step / dbas_init_b0 with the reference's closures (f = dubins_step, h = the aggregation) and
    dubins_augmented_jacobian, three DBaS settings (smooth-min / exact min, inverse / log, gamma != 0)."""
    from diff_tube_mpc_strict_pt.core.barrier import DBaSConfig, dbas_init_b0, dbas_step
    from diff_tube_mpc_strict_pt.core.systems import dubins_obstacles as O
    from diff_tube_mpc_strict_pt.core.systems.dubins import dubins_step
    from diff_tube_mpc_strict_pt.core.systems.dubins_aug_jac import dubins_augmented_jacobian, dubins_f_jac

    npdt, tdt, tol = DT[tag]
    tol = max(tol, 1e-13) if tag == "f64" else 1e-5
    k = golden(f"kat_{tag}")
    dub, obs, beta, eps = _setup()
    st = SETTINGS[setting]
    dbc = DBaSConfig(barrier_type=st["btype"], alpha=torch.tensor(st["alpha"], dtype=tdt),
                     gamma=torch.tensor(st["gamma"], dtype=tdt), eps=eps)
    if st["agg"] == "smoothmin":
        h = lambda x: O.h_multi_circle_obstacles(x, obstacles=obs, beta=beta)  # noqa: E731
    else:
        h = lambda x: O.h_min_circle_obstacles(x, obstacles=obs)  # noqa: E731
    f = lambda x, u: dubins_step(x, u, cfg=dub)  # noqa: E731
    xh = torch.tensor(k["xh"], dtype=tdt, device=dev)
    u = torch.tensor(k["u"], dtype=tdt, device=dev)
    xn, bn = dbas_step(x_k=xh[:, :3], u_k=u, b_k=xh[:, 3], f=f, h=h, cfg=dbc)
    got = torch.cat([xn, bn[:, None]], 1).cpu().numpy()
    assert np.allclose(got, k[f"fhat_{setting}"], rtol=tol, atol=tol)
    b0 = dbas_init_b0(xh[:, :3], h=h, cfg=dbc).cpu().numpy()
    assert np.allclose(b0, k[f"b0_{setting}"], rtol=tol, atol=0)
    A, Bm = dubins_augmented_jacobian(xh, u, cfg=dub, obs=obs, db_cfg=dbc, obs_beta=beta, obs_agg=st["agg"])
    _close(A, k[f"A_{setting}"], tol)
    _close(Bm, k[f"B_{setting}"], tol)
    A1, B1 = dubins_augmented_jacobian(xh[3], u[3], cfg=dub, obs=obs, db_cfg=dbc, obs_beta=beta, obs_agg=st["agg"])
    assert A1.shape == (4, 4) and B1.shape == (4, 2)
    _close(A1, k[f"A_{setting}"][3], tol)
    A3, B3 = dubins_f_jac(xh[3, :3], u[3], cfg=dub)
    _close(A3, k[f"A_{setting}"][3][:3, :3], tol)
    _close(B3, k[f"B_{setting}"][3][:3, :], tol)
    with pytest.raises(ValueError, match="gamma"):
        dbas_step(x_k=xh[:, :3], u_k=u, b_k=xh[:, 3], f=f, h=h, cfg=DBaSConfig(gamma=1.5))


@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_box_clamp_and_active_mask(dev, tag):
    """BoxClampControl.clamp / active_mask (core/control.py:61-70) vs the reference's torch expressions."""
    from diff_tube_mpc_strict_pt.core.control import BoxClampControl
    from diff_tube_mpc_strict_pt.core.systems.dubins import DubinsConfig, clamp_control

    _, tdt, _ = DT[tag]
    lo = torch.tensor([-10.0, -math.pi], dtype=tdt)
    hi = torch.tensor([10.0, math.pi], dtype=tdt)
    box = BoxClampControl(u_min=lo, u_max=hi)
    g = torch.Generator().manual_seed(3)
    u = (torch.rand(500, 2, generator=g, dtype=torch.float64) * 30 - 15).to(tdt)
    u[:10] = torch.stack([lo, hi] * 5)  # exactly at the bounds
    u[10, 0] = lo[0] + 1e-9
    u[11, 1] = hi[1] - 1e-9
    u[12, 0] = float("nan")
    ud = u.to(dev)
    ref = torch.clamp(u, min=lo, max=hi)
    got = box.clamp(ud).cpu()
    assert torch.equal(torch.isnan(got), torch.isnan(ref))
    assert torch.equal(torch.nan_to_num(got), torch.nan_to_num(ref))
    ref_m = (u <= (lo + box.active_tol)) | (u >= (hi - box.active_tol))
    assert torch.equal(box.active_mask(ud).cpu(), ref_m)
    assert box.active_mask(ud[3]).shape == (2,) and box.clamp(ud[3]).shape == (2,)
    dub = DubinsConfig()
    assert torch.equal(clamp_control(ud, cfg=dub).cpu().nan_to_num(), ref.nan_to_num())


@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_cost_derivs_u_form(dev, tag):
    """nominal / auxiliary_cost_derivs_u and *_terminal_derivs (core/cost_derivs.py:58-146) vs the
    reference's expressions in torch on the host, batched and unbatched."""
    from diff_tube_mpc_strict_pt.core import cost_derivs as CD

    _, tdt, _ = DT[tag]
    g = torch.Generator().manual_seed(4)
    n = 64
    xh = (torch.rand(n, 4, generator=g, dtype=torch.float64) * 10 - 2).to(tdt)
    u = (torch.rand(n, 2, generator=g, dtype=torch.float64) * 6 - 3).to(tdt)
    xr = (torch.rand(n, 3, generator=g, dtype=torch.float64) * 10).to(tdt)
    ur = (torch.rand(n, 2, generator=g, dtype=torch.float64) * 4 - 2).to(tdt)
    Q = torch.tensor([1.0, 2.0, 0.5], dtype=tdt)
    R = torch.tensor([0.3, 1.5], dtype=tdt)
    Qf = torch.tensor([100.0, 50.0, 10.0], dtype=tdt)
    qb = torch.tensor(0.7, dtype=tdt)
    tg = torch.tensor([10.0, 10.0, math.pi / 4], dtype=tdt)
    D = lambda t: t.to(dev)  # noqa: E731
    for i in (None, 5):
        sel = (lambda t: t) if i is None else (lambda t: t[i])  # noqa: E731
        lx, lu, lxx, luu, lux = CD.nominal_cost_derivs_u(x_hat=D(sel(xh)), u=D(sel(u)), target=tg, Q=Q, R=R, qb=qb)
        x = sel(xh)
        ref_lx = torch.cat([2.0 * Q * (x[..., :3] - tg), (2.0 * qb * x[..., 3:4])], -1)
        assert torch.equal(lx.cpu(), ref_lx) and torch.equal(lu.cpu(), 2.0 * R * sel(u))
        assert torch.equal(lxx.cpu()[..., :, :], torch.diag(torch.cat([2.0 * Q, (2.0 * qb).view(1)])).expand_as(lxx.cpu()))
        assert torch.equal(luu.cpu(), torch.diag(2.0 * R).expand_as(luu.cpu())) and not lux.any()
        lx, lu, _, _, _ = CD.auxiliary_cost_derivs_u(x_hat=D(sel(xh)), u=D(sel(u)), x_ref=D(sel(xr)), u_ref=D(sel(ur)),
                                                     Q=Q, R=R, qb=qb)
        assert torch.equal(lx.cpu(), torch.cat([2.0 * Q * (x[..., :3] - sel(xr)), 2.0 * qb * x[..., 3:4]], -1))
        assert torch.equal(lu.cpu(), 2.0 * R * (sel(u) - sel(ur)))
        px, pxx = CD.nominal_terminal_derivs(x_hat_N=D(sel(xh)), target=tg, Qf=Qf)
        assert torch.equal(px.cpu(), torch.cat([2.0 * Qf * (x[..., :3] - tg), torch.zeros_like(x[..., :1])], -1))
        assert torch.equal(pxx.cpu()[..., 3, 3], torch.zeros_like(pxx.cpu()[..., 3, 3]))
        px, _ = CD.auxiliary_terminal_derivs(x_hat_N=D(sel(xh)), x_ref_N=D(sel(xr)), Qf=Qf)
        assert torch.equal(px.cpu(), torch.cat([2.0 * Qf * (x[..., :3] - sel(xr)), torch.zeros_like(x[..., :1])], -1))


@pytest.mark.parametrize("setting", ["s0", "s1"])
def test_autograd_through_per_function_api(dev, setting):
    """the reference differentiates its per-function API with autograd
    (core/ddp.py:63-86 _linearize_autograd, core/autodiff.py:9-80).  Here dubins_step, h_*, the barriers and
    BoxClampControl.clamp are autograd Functions whose backward is the library's analytic derivative, so the
    autograd Jacobian of the reference's DBaS closure f_hat(x_hat, u) = [f(x, u), dbas_step b'] equals
    dubins_augmented_jacobian (inverse barrier: the reference's f_jac), dubins_step's Jacobian dubins_f_jac,
    and a second derivative of dubins_step exists.  The entry points with no autograd formula raise instead
    of returning an output cut from the graph."""
    from diff_tube_mpc_strict_pt.core.barrier import DBaSConfig, dbas_step
    from diff_tube_mpc_strict_pt.core.control import BoxClampControl
    from diff_tube_mpc_strict_pt.core.cost_derivs import nominal_cost_derivs_u
    from diff_tube_mpc_strict_pt.core.systems import dubins_obstacles as O
    from diff_tube_mpc_strict_pt.core.systems.dubins import dubins_step
    from diff_tube_mpc_strict_pt.core.systems.dubins_aug_jac import dubins_augmented_jacobian, dubins_f_jac

    tdt = torch.float64
    k = golden("kat_f64")
    dub, obs, beta, eps = _setup()
    st = SETTINGS[setting]
    dbc = DBaSConfig(barrier_type="inverse", alpha=st["alpha"], gamma=st["gamma"], eps=eps)
    if st["agg"] == "smoothmin":
        h = lambda x: O.h_multi_circle_obstacles(x, obstacles=obs, beta=beta)  # noqa: E731
    else:
        h = lambda x: O.h_min_circle_obstacles(x, obstacles=obs)  # noqa: E731
    f = lambda x, u: dubins_step(x, u, cfg=dub)  # noqa: E731

    def fhat(xh, u):
        xn, bn = dbas_step(x_k=xh[:3], u_k=u, b_k=xh[3], f=f, h=h, cfg=dbc)
        return torch.cat([xn, bn.reshape(1)])

    xh_all = torch.tensor(k["xh"], dtype=tdt, device=dev)
    u_all = torch.tensor(k["u"], dtype=tdt, device=dev)
    for i in range(0, 96, 12):
        xh, u = xh_all[i], u_all[i]
        Aa, Ba = torch.autograd.functional.jacobian(fhat, (xh, u))
        A, Bm = dubins_augmented_jacobian(xh, u, cfg=dub, obs=obs, db_cfg=dbc, obs_beta=beta, obs_agg=st["agg"])
        scale = max(1.0, float(A.abs().max()), float(Bm.abs().max()))
        assert float((Aa - A).abs().max()) <= 1e-10 * scale, (i, Aa, A)
        assert float((Ba - Bm).abs().max()) <= 1e-10 * scale, (i, Ba, Bm)
        Ja, Jb = torch.autograd.functional.jacobian(lambda x, v: f(x, v), (xh[:3], u))
        A3, B3 = dubins_f_jac(xh[:3], u, cfg=dub)
        assert torch.allclose(Ja, A3, rtol=0, atol=1e-14) and torch.allclose(Jb, B3, rtol=0, atol=1e-14)
    # a second derivative through dubins_step (autodiff.grad_hess_xu differentiates twice)
    x = xh_all[0, :3].clone().requires_grad_(True)
    u = u_all[0].clone().requires_grad_(True)
    (gx,) = torch.autograd.grad(f(x, u)[0], x, create_graph=True)
    (hxx,) = torch.autograd.grad(gx[2], x)
    ref = -dub.dt * float(u[0]) * math.cos(float(x[2]))  # d2 px' / dtheta2
    assert abs(float(hxx[2]) - ref) <= 1e-14
    # clamp: torch.clamp's gradient rule
    box = BoxClampControl(u_min=(-10.0, -math.pi), u_max=(10.0, math.pi))
    uu = torch.tensor([[-12.0, 0.5], [10.0, 4.0], [3.0, -math.pi]], dtype=tdt, device=dev, requires_grad=True)
    box.clamp(uu).sum().backward()
    assert uu.grad.cpu().tolist() == [[0.0, 1.0], [1.0, 0.0], [1.0, 1.0]]
    # no autograd formula: refuse rather than detach silently
    xg = xh_all[:4].clone().requires_grad_(True)
    with pytest.raises(RuntimeError, match="autograd"):
        dubins_augmented_jacobian(xg, u_all[:4], cfg=dub, obs=obs, db_cfg=dbc, obs_beta=beta, obs_agg=st["agg"])
    with pytest.raises(RuntimeError, match="autograd"):
        nominal_cost_derivs_u(x_hat=xg, u=u_all[:4], target=(10.0, 10.0, 0.7), Q=(1.0, 1.0, 1.0), R=(1.0, 1.0), qb=1.0)
    with torch.no_grad():  # detached use stays allowed
        dubins_augmented_jacobian(xg, u_all[:4], cfg=dub, obs=obs, db_cfg=dbc, obs_beta=beta, obs_agg=st["agg"])


@pytest.mark.parametrize("tag", ["f64", "f32"])
def test_reference_autodiff_exports_on_device(dev, tag):
    """core.compute_jacobian / grad_hess_xu / grad_hess_x (the reference's autograd fallbacks, core/autodiff.py:9-82,
    re-exported in round 5) over the package's differentiable device functions: compute_jacobian of dubins_step at
    the KAT points equals the library's analytic Jacobian (dubins_f_jac, itself checked against the reference's
    KATs), and grad_hess_xu of a quadratic stage cost equals quadratic_cost_derivs_diagonal."""
    from diff_tube_mpc_strict_pt.core import compute_jacobian, grad_hess_x, grad_hess_xu, quadratic_cost_derivs_diagonal
    from diff_tube_mpc_strict_pt.core.systems.dubins import dubins_step
    from diff_tube_mpc_strict_pt.core.systems.dubins_aug_jac import dubins_f_jac

    npdt, tdt, tol = DT[tag]
    k = golden(f"kat_{tag}")
    dub, _, _, _ = _setup()
    xh = torch.tensor(k["xh"], dtype=tdt, device=dev)
    u = torch.tensor(k["u"], dtype=tdt, device=dev)
    A, Bm = dubins_f_jac(xh[:, :3], u, cfg=dub)
    for i in range(min(8, xh.shape[0])):
        Ja, Jb = compute_jacobian(lambda x, uu: dubins_step(x, uu, cfg=dub), xh[i, :3], u[i])
        assert Ja.device == dev
        _close(Ja, A[i].cpu().numpy(), tol)
        _close(Jb, Bm[i].cpu().numpy(), tol)
    Q = torch.tensor([1.0, 2.0, 0.5, 3.0], dtype=tdt, device=dev)
    R = torch.tensor([0.1, 0.2], dtype=tdt, device=dev)
    xr = torch.tensor([10.0, 10.0, 0.7, 0.0], dtype=tdt, device=dev)
    ref = quadratic_cost_derivs_diagonal(xh[0], u[0], Q, R, xr)
    auto = grad_hess_xu(lambda x, uu, kk: (Q * (x - xr) ** 2).sum() + (R * uu ** 2).sum(), xh[0], u[0], 0)
    for a, r in zip(auto, ref):
        _close(a, r.cpu().numpy(), tol)
    gx, Hx = grad_hess_x(lambda x: (Q * (x - xr) ** 2).sum(), xh[0])
    _close(gx, ref[0].cpu().numpy(), tol)
    _close(Hx, ref[2].cpu().numpy(), tol)
