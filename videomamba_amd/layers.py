"""Small building blocks: RMSNorm module (mamba-ssm ``RMSNorm`` surface), DropPath,
``to_2tuple`` and ``trunc_normal_`` (the timm helpers the reference imports at
``models/videomamba/videomamba.py:12-15``).  ``trunc_normal_`` consumes the RNG exactly as
timm's does, so a seeded build reproduces the reference's initial weights."""

from __future__ import annotations

import math
import warnings
from typing import Optional

import torch
import torch.nn as nn
from torch import Tensor

from . import kernels as K


class RMSNorm(nn.Module):
    """RMSNorm with the mamba-ssm module surface (``weight``, ``bias=None``, ``eps``);
    ``forward(x, residual=None, prenorm=False, residual_in_fp32=False)`` runs the fused
    add+norm HIP kernel."""

    def __init__(self, hidden_size: int, eps: float = 1e-5, dropout_p: float = 0.0,
                 device=None, dtype=None):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(hidden_size, device=device, dtype=dtype))
        self.register_parameter("bias", None)

    def forward(self, x: Tensor, residual: Optional[Tensor] = None, prenorm: bool = False,
                residual_in_fp32: bool = False):
        return K._norm(x, self.weight, self.bias, residual, prenorm, residual_in_fp32, self.eps,
                       True, owner=self)


class DropPath(nn.Module):
    """Stochastic depth (identity in eval mode, which is the only mode the HIP path runs)."""

    def __init__(self, drop_prob: float = 0.0):
        super().__init__()
        self.drop_prob = drop_prob

    def forward(self, x: Tensor) -> Tensor:
        if self.drop_prob == 0.0 or not self.training:
            return x
        keep = 1.0 - self.drop_prob
        mask = x.new_empty((x.shape[0],) + (1,) * (x.ndim - 1)).bernoulli_(keep)
        return x * mask / keep


def to_2tuple(v):
    return tuple(v) if isinstance(v, (tuple, list)) else (v, v)


def trunc_normal_(tensor: Tensor, mean: float = 0.0, std: float = 1.0, a: float = -2.0,
                  b: float = 2.0) -> Tensor:
    """Truncated normal init by inverse-CDF sampling (timm ``trunc_normal_``)."""
    def cdf(v):
        return 0.5 * (1.0 + math.erf(v / math.sqrt(2.0)))

    if mean < a - 2 * std or mean > b + 2 * std:
        warnings.warn("mean is more than 2 std from [a, b] in trunc_normal_", stacklevel=2)
    with torch.no_grad():
        lo, hi = cdf((a - mean) / std), cdf((b - mean) / std)
        tensor.uniform_(2 * lo - 1, 2 * hi - 1)
        tensor.erfinv_()
        tensor.mul_(std * math.sqrt(2.0))
        tensor.add_(mean)
        tensor.clamp_(min=a, max=b)
    return tensor


_warned_grad = False


def warn_if_grad(*tensors: Optional[Tensor]) -> None:
    """The HIP path is forward-only; say so once when autograd would expect a graph."""
    global _warned_grad
    if _warned_grad or not torch.is_grad_enabled():
        return
    if any(t is not None and t.requires_grad for t in tensors):
        _warned_grad = True
        warnings.warn("VideoMamba's HIP kernels are forward-only: outputs are computed "
                      "without autograd (wrap inference in torch.no_grad()).", stacklevel=3)


def round_up(n: int, m: int = 8) -> int:
    return ((n + m - 1) // m) * m
