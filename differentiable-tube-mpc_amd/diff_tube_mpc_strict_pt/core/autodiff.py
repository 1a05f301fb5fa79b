"""Autograd derivatives of user closures: the reference's fallbacks (core/autodiff.py:9-82), kept for API parity.

The reference uses these when a caller gives ilqr_solve a cost or dynamics closure without analytic derivatives.
This package never needs them on its hot path: its solver evaluates the typed problem's analytic derivatives on
the device (csrc/dtmpc_fast.hip, csrc/dtmpc_systems.hip), and a closure it cannot evaluate on the device is
refused (core/closures.py).  They are here for code written against the reference's ``core`` package: the same
signatures and results, computed with torch.autograd on whatever device the inputs live on -- e.g. over the
package's differentiable per-function entry points (``dubins_step``, the barriers, ``h_*``, the box clamp:
autograd Functions whose backward is the library's analytic derivative).
"""
from __future__ import annotations

from typing import Callable, Tuple

import torch
from torch import Tensor


def grad_hess_xu(cost_fn: Callable[[Tensor, Tensor, int], Tensor], x: Tensor, u: Tensor,
                 k: int) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor]:
    """(l_x, l_u, l_xx, l_uu, l_ux) of a scalar stage cost l(x, u, k) (core/autodiff.py:9-43): gradient and
    Hessian over z = [x, u] by autograd (exact, no finite differences).  l_ux is the [nu, nx] block."""
    nx, nu = x.numel(), u.numel()

    def l_of_z(z: Tensor) -> Tensor:
        return cost_fn(z[:nx], z[nx:], k)

    z = torch.cat([x.detach().reshape(-1), u.detach().reshape(-1)]).requires_grad_(True)
    g = torch.autograd.grad(l_of_z(z), z, create_graph=True)[0]
    H = torch.autograd.functional.hessian(l_of_z, z, create_graph=True)
    return g[:nx], g[nx:], H[:nx, :nx], H[nx:, nx:], H[nx:, :nx]


def grad_hess_x(term_cost_fn: Callable[[Tensor], Tensor], xN: Tensor) -> Tuple[Tensor, Tensor]:
    """(phi_x, phi_xx) of a scalar terminal cost phi(x_N) (core/autodiff.py:46-63)."""
    xr = xN.detach().requires_grad_(True)
    g = torch.autograd.grad(term_cost_fn(xr), xr, create_graph=True)[0]
    H = torch.autograd.functional.hessian(term_cost_fn, xr, create_graph=True)
    return g, H


def compute_jacobian(f: Callable[[Tensor, Tensor], Tensor], x: Tensor, u: Tensor) -> Tuple[Tensor, Tensor]:
    """(df/dx, df/du) of dynamics f(x, u) by autograd (core/autodiff.py:66-82)."""
    xr = x.detach().clone().requires_grad_(True)
    ur = u.detach().clone().requires_grad_(True)
    A = torch.autograd.functional.jacobian(lambda xx: f(xx, ur), xr)
    B = torch.autograd.functional.jacobian(lambda uu: f(xr, uu), ur)
    return A, B
