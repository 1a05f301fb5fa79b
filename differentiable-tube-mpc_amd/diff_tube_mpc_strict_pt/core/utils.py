"""Small linear-algebra and cost helpers of the reference's ``core.utils`` (core/utils.py:15-91), for API parity.

None of them is on this package's hot path -- the solver's 2 x 2 Q_uu solve (pivoted LU, as torch.linalg.solve)
and its diagonal cost derivatives run inside the fused kernels (csrc/dtmpc_fast.hip riccati_pk, backward) -- but
code written against the reference's ``core`` imports them.  Same signatures and results, on the inputs' device.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
from torch import Tensor


def solve_psd(A: Tensor, b: Tensor, reg: float = 1e-6) -> Tensor:
    """x with A x = b for a positive semi-definite A (core/utils.py:15-40): Cholesky, and on failure the
    regularised A + reg I by LU.  b [n] or [n, m]."""
    L, info = torch.linalg.cholesky_ex(A)
    vec = b.ndim == 1
    rhs = b.unsqueeze(-1) if vec else b
    if int(info) == 0:
        x = torch.cholesky_solve(rhs, L)
    else:
        x = torch.linalg.solve(regularize_matrix(A, reg), rhs)
    return x.squeeze(-1) if vec else x


def regularize_matrix(H: Tensor, reg: float = 1e-6) -> Tensor:
    """H + reg I (core/utils.py:43-54)."""
    n = H.shape[-1]
    return H + reg * torch.eye(n, device=H.device, dtype=H.dtype)


def quadratic_cost_derivs_diagonal(x: Tensor, u: Tensor, Q: Tensor, R: Tensor, x_ref: Optional[Tensor] = None,
                                   u_ref: Optional[Tensor] = None) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor]:
    """Derivatives of ||x - x_ref||_Q^2 + ||u - u_ref||_R^2 with diagonal Q [nx], R [nu] (core/utils.py:57-91):
    (l_x, l_u, l_xx, l_uu, l_ux) = (2 Q dx, 2 R du, diag 2Q, diag 2R, 0 [nu, nx])."""
    dx = x if x_ref is None else x - x_ref
    du = u if u_ref is None else u - u_ref
    return (2.0 * Q * dx, 2.0 * R * du, torch.diag(2.0 * Q), torch.diag(2.0 * R),
            torch.zeros(u.numel(), x.numel(), device=x.device, dtype=x.dtype))
