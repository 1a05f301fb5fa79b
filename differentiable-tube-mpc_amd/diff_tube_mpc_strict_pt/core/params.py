"""Raw (unconstrained) adaptive parameters of the general path -- core/params.py:9-59.

The reference keeps each parameter as a separate grad-enabled tensor; the HIP path keeps one raw
[12] vector per parameter set (include/dtmpc.h, DTMPC_P_* layout) shared by the batch and
differentiated in closed form.  These classes are the host-side view with the reference's field
names and transforms (softplus weights, alpha = softplus + 1e-6, gamma = tanh, tight = softplus).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Sequence

import torch
from torch import Tensor

from .. import _abi

__all__ = ["NominalTheta", "AuxiliaryTheta", "theta_from_raw"]


def _pos(x: Tensor) -> Tensor:
    return torch.nn.functional.softplus(x)


@dataclass
class _ThetaBase:
    Q_raw: Tensor
    R_raw: Tensor
    Qf_raw: Tensor
    qb_raw: Tensor
    alpha_raw: Tensor
    gamma_raw: Tensor

    def Q(self) -> Tensor:
        return _pos(self.Q_raw)

    def R(self) -> Tensor:
        return _pos(self.R_raw)

    def Qf(self) -> Tensor:
        return _pos(self.Qf_raw)

    def qb(self) -> Tensor:
        return _pos(self.qb_raw)

    def alpha(self) -> Tensor:
        return _pos(self.alpha_raw) + 1e-6

    def gamma(self) -> Tensor:
        return torch.tanh(self.gamma_raw)

    def _raw(self, tight: Tensor) -> Tensor:
        parts = [self.Q_raw.reshape(3), self.R_raw.reshape(2), self.Qf_raw.reshape(3), self.qb_raw.reshape(1),
                 self.alpha_raw.reshape(1), self.gamma_raw.reshape(1), tight.reshape(1)]
        return torch.cat([p.detach().to(parts[0].dtype) for p in parts])


@dataclass
class AuxiliaryTheta(_ThetaBase):
    """core/params.py:41-59"""

    def tensors(self) -> list:
        return [self.Q_raw, self.R_raw, self.Qf_raw, self.qb_raw, self.alpha_raw, self.gamma_raw]

    def raw(self) -> Tensor:
        """[12] raw vector (DTMPC_P_* layout, tight slot 0)."""
        return self._raw(torch.zeros((), dtype=self.Q_raw.dtype, device=self.Q_raw.device))


@dataclass
class NominalTheta(_ThetaBase):
    """core/params.py:14-38"""

    tight_raw: Tensor = None

    def tight(self) -> Tensor:
        return _pos(self.tight_raw)

    def tensors(self) -> list:
        return [self.Q_raw, self.R_raw, self.Qf_raw, self.qb_raw, self.alpha_raw, self.gamma_raw, self.tight_raw]

    def raw(self) -> Tensor:
        return self._raw(self.tight_raw)


def theta_from_raw(raw: Sequence[float] | Tensor, nominal: bool, *, dtype=torch.float64, device="cpu"):
    """Split a [12] raw vector into the reference's parameter objects."""
    r = torch.as_tensor(raw, dtype=dtype, device=device).reshape(_abi.P_COUNT)
    kw = dict(Q_raw=r[0:3].clone(), R_raw=r[3:5].clone(), Qf_raw=r[5:8].clone(), qb_raw=r[8].clone(),
              alpha_raw=r[9].clone(), gamma_raw=r[10].clone())
    return NominalTheta(**kw, tight_raw=r[11].clone()) if nominal else AuxiliaryTheta(**kw)
