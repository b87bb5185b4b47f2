"""Bidirectional refiner block (``models/refiner_backbone.py:13-135`` surface).

Two independent unidirectional blocks: the forward block scans the sequence as given,
the backward block scans it reversed in time — for 4-D input (B, T, N, C) the frame order
is reversed while the within-frame token order is kept — and a sigmoid gate mixes the two
before a Linear.  Only the forward block's streaming state is returned.
"""

from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch
import torch.nn as nn
from torch import Tensor

from .videomamba import Block, create_block

LayerState = Tuple[Tensor, Tensor]


class BiMambaRefinerBlock(nn.Module):
    """Bidirectional wrapper around two independent unidirectional VideoMamba blocks."""

    def __init__(self, dim: int, ssm_cfg: Optional[Dict[str, object]] = None, **block_kwargs):
        super().__init__()
        layer_idx = block_kwargs.pop("layer_idx", None)
        self.block_fwd = create_block(d_model=dim, ssm_cfg=ssm_cfg, layer_idx=layer_idx,
                                      bimamba=False, **block_kwargs)
        bwd_idx = None if layer_idx is None else int(layer_idx) + 1_000_000
        self.block_bwd = create_block(d_model=dim, ssm_cfg=ssm_cfg, layer_idx=bwd_idx,
                                      bimamba=False, **block_kwargs)
        self.fusion_gate = nn.Sequential(nn.Linear(dim * 2, dim), nn.Sigmoid())
        self.out_proj = nn.Linear(dim, dim)

    @staticmethod
    def _pack_tokens(x: Tensor):
        if x.ndim == 3:
            return x, None
        if x.ndim == 4:
            b, t, n, c = x.shape
            return x.reshape(b, t * n, c), (b, t, n)
        raise ValueError("Expected x to be [B, L, C] or [B, T, N, C].")

    @staticmethod
    def _unpack_tokens(x: Tensor, packed_shape):
        if packed_shape is None:
            return x
        b, t, n = packed_shape
        return x.reshape(b, t, n, x.shape[-1])

    @staticmethod
    def _flip_time(x: Tensor, packed_shape) -> Tensor:
        if packed_shape is None:
            return torch.flip(x, dims=[1])
        b, t, n = packed_shape
        return torch.flip(x.reshape(b, t, n, x.shape[-1]), dims=[1]).reshape(b, t * n, x.shape[-1])

    @staticmethod
    def _ensure_state(block: Block, state: Optional[LayerState], batch_size: int, device):
        if state is not None:
            return state
        return block.mixer.allocate_state(batch_size=batch_size, device=device)

    def allocate_state(self, batch_size: int, dtype=None, device=None):
        return (self.block_fwd.mixer.allocate_state(batch_size=batch_size, dtype=dtype, device=device),
                self.block_bwd.mixer.allocate_state(batch_size=batch_size, dtype=dtype, device=device))

    def forward(self, x: Tensor, state_fwd: Optional[LayerState] = None,
                state_bwd_init: Optional[LayerState] = None, use_checkpoint: bool = False):
        seq, packed = self._pack_tokens(x)
        bsz = seq.shape[0]
        st_f = self._ensure_state(self.block_fwd, state_fwd, bsz, seq.device)
        out_f, _, new_f = self.block_fwd(seq, state=st_f, return_state=True,
                                         use_checkpoint=use_checkpoint)
        st_b = self._ensure_state(self.block_bwd, state_bwd_init, bsz, seq.device)
        out_b_rev, _, _ = self.block_bwd(self._flip_time(seq, packed), state=st_b,
                                         return_state=True, use_checkpoint=use_checkpoint)
        out_b = self._flip_time(out_b_rev, packed)
        with torch.no_grad():
            gate = self.fusion_gate(torch.cat([out_f, out_b], dim=-1))
            out = self.out_proj(gate * out_f + (1.0 - gate) * out_b)
        return self._unpack_tokens(out, packed), new_f
