"""Bidirectional refiner block (``models/refiner_backbone.py:13-135`` surface).

Two independent unidirectional blocks: the forward block scans the sequence as given,
the backward block scans it reversed in time — for 4-D input (B, T, N, C) the frame order
is reversed while the within-frame token order is kept — and a sigmoid gate mixes the two
before a Linear.  Only the forward block's streaming state is returned.

The two directions run as one paired pipeline over a (2B, Lp, C) buffer (rows [0, B)
forward, [B, 2B) backward) with no flipped copies of the sequence:

    norm (HIP, per direction; the backward one reads its input rows in flipped order)
    -> in_proj / conv / x_proj / dt_proj per direction into the halves of shared buffers
    -> ONE scan launch for both directions (vm_selective_scan_bidir_fwd: the backward rows
       use their own A / D / dt bias and store each step's output at its un-flipped row)
    -> out_proj per direction into the two column halves of the gate's (n, 2C) input
    -> fusion gate + out_proj (torch, as the reference).

The reference's flipped copies of the input and of the backward output
(``refiner_backbone.py:121``, ``:128``) are folded into the norm's load and the scan's store.

Configurations the paired kernels do not take (d_state != 16, forward / backward mixers of
different geometry, widths the fused norm rejects, odd bf16 x_dbl rows, unaligned input)
run the reference's composition instead — the forward block, the backward block on a
flipped copy, the flip back and the gate — on the same per-block HIP kernels.
"""

from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch
import torch.nn as nn
from torch import Tensor

from . import kernels as K
from .layers import round_up, warn_if_grad
from .mamba_simple import _linear_into
from .videomamba import Block, _norm_kind, create_block

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
        K.require_gpu(seq, what="BiMambaRefinerBlock")
        warn_if_grad(seq, self.block_fwd.mixer.in_proj.weight)
        st_f = self._ensure_state(self.block_fwd, state_fwd, bsz, seq.device)
        st_b = self._ensure_state(self.block_bwd, state_bwd_init, bsz, seq.device)
        frame = 1 if packed is None else packed[2]
        with torch.no_grad():
            if self._paired_ok(seq):
                out, new_f = self._forward_paired(seq, frame, st_f, st_b)
            else:
                out, new_f = self._forward_blocks(seq, packed, st_f, st_b)
        return self._unpack_tokens(out, packed), new_f

    def _paired_ok(self, seq: Tensor) -> bool:
        """The one-launch paired pipeline's preconditions (else :meth:`_forward_blocks`):
        equal mixer geometry, 16 states (the paired scan's scalar B/C rows), a width the
        fused norm takes (C % 4 == 0, C <= 2048) with a 16-byte aligned input, and B|C rows
        of x_dbl on 4-byte boundaries."""
        mf, mb = self.block_fwd.mixer, self.block_bwd.mixer
        if any(getattr(mf, a) != getattr(mb, a) for a in ("d_inner", "d_state", "dt_rank", "d_conv")):
            return False
        C = seq.shape[-1]
        es = seq.element_size() if self.block_fwd.fused_add_norm else \
            self.block_fwd.norm.weight.element_size()
        return (mf.d_state == 16 and C % 4 == 0 and 4 <= C <= 2048
                and ((mf.dt_rank + 2 * mf.d_state) * es) % 4 == 0
                and (not seq.is_contiguous() or seq.data_ptr() % 16 == 0))

    def _forward_blocks(self, seq: Tensor, packed, st_f: LayerState, st_b: LayerState):
        """The reference's composition (``refiner_backbone.py:98-135``) on the per-block
        HIP path: forward block, backward block over the time-flipped sequence (frame order
        flipped for 4-D input, ``:61-68``), flip back, sigmoid gate, Linear."""
        def flip(t: Tensor) -> Tensor:
            if packed is None:
                return torch.flip(t, dims=[1])
            b, tt, n = packed
            return torch.flip(t.reshape(b, tt, n, t.shape[-1]), dims=[1]).reshape(b, tt * n, -1)

        out_f, _, new_f = self.block_fwd(seq, state=st_f, return_state=True)
        out_b_rev, _, _ = self.block_bwd(flip(seq), state=st_b, return_state=True)
        out_b = flip(out_b_rev)
        gate = self.fusion_gate(torch.cat([out_f, out_b], dim=-1))
        return self.out_proj(gate * out_f + (1.0 - gate) * out_b), new_f

    def _forward_paired(self, seq: Tensor, frame: int, st_f: LayerState, st_b: LayerState):
        bf, bb = self.block_fwd, self.block_bwd
        mf, mb = bf.mixer, bb.mixer
        B, L, C = seq.shape
        Dm, N, R, W = mf.d_inner, mf.d_state, mf.dt_rank, mf.d_conv
        for blk, (cs, ss) in ((bf, st_f), (bb, st_b)):
            blk.mixer._check_state(cs, W, "conv_state", B)
            blk.mixer._check_state(ss, N, "ssm_state", B)
        if L == 0:
            return seq.new_empty((B, 0, C)), (st_f[0].clone(), st_f[1])
        Lp = round_up(L)
        n = B * Lp
        E = R + 2 * N
        x_in = (seq if bf.fused_add_norm else seq.to(bf.norm.weight.dtype)).contiguous()
        dev, hdt = seq.device, x_in.dtype

        # add + norm of both directions (residual is None in a standalone block); the
        # backward half reads its rows in flipped frame order
        hn = torch.empty((2 * B, Lp, C), dtype=hdt, device=dev)
        for half, blk, rev in ((0, bf, 0), (1, bb, frame)):
            K.norm_pool(x_in, None, L, K.f32_cached(blk.norm, blk.norm.weight, "w"),
                        K.f32_cached(blk.norm, blk.norm.bias, "b"), blk.norm.eps,
                        _norm_kind(blk.norm), head=0, groups=1, group_rows=L,
                        out=hn[half * B:(half + 1) * B], rev_frame=rev)
        if Lp > L:
            hn[:, L:] = 0

        # mixer fronts into the halves of the paired buffers
        xz = torch.empty((2 * n, 2 * Dm), dtype=hdt, device=dev)
        u = torch.empty((2 * n, Dm), dtype=hdt, device=dev)
        x_dbl = torch.empty((2 * n, E), dtype=hdt, device=dev)
        dt = torch.empty((2 * n, Dm), dtype=hdt, device=dev)
        half = lambda t, i: t[i * n:(i + 1) * n]  # noqa: E731
        conv_new = torch.empty((B, Dm, W), dtype=st_f[0].dtype, device=dev)
        mf._tm_front(hn[:B], L, st_f[0], conv_new,
                     bufs=tuple(half(t, 0) for t in (xz, u, x_dbl, dt)))
        mb._tm_front(hn[B:], L, st_b[0], None,
                     bufs=tuple(half(t, 1) for t in (xz, u, x_dbl, dt)))

        # one scan for both directions; both ssm states update in place (the reference's
        # aliasing), the backward one through a buffer of the forward one's layout if needed
        A_f, D_f, bias_f, _, _ = mf._fp32_params()
        A_b, D_b, bias_b, _, _ = mb._fp32_params()
        ssm_f, ssm_b = st_f[1], st_b[1]
        hb = ssm_b
        if ssm_b.dtype != ssm_f.dtype or ssm_b.stride() != ssm_f.stride():
            hb = torch.empty_strided(ssm_f.shape, ssm_f.stride(), dtype=ssm_f.dtype,
                                     device=dev).copy_(ssm_b)
        y = torch.empty_like(u)
        s_u, s_xz, s_bc = (Lp * Dm, 1, Dm), (Lp * 2 * Dm, 1, 2 * Dm), (Lp * E, 1, E)
        hs = (ssm_f.stride(0), ssm_f.stride(1))
        K.scan_raw(u, s_u, dt, s_u, A_f, x_dbl[:, R:R + N], s_bc, x_dbl[:, R + N:], s_bc, D_f,
                   xz[:, Dm:], s_xz, bias_f, True, ssm_f, hs, ssm_f, hs, y, s_u, Lp, 2 * B, Dm,
                   L, N, K.dtype_code(hdt), torch.cuda.current_stream(dev).cuda_stream,
                   pair=(B, A_b, D_b, bias_b, hb, hb, frame))
        if hb is not ssm_b:
            ssm_b.copy_(hb)

        # out_proj of each direction straight into the gate's concatenated input
        cat = torch.empty((n, 2 * C), dtype=hdt, device=dev)
        _linear_into(half(y, 0), mf.out_proj.weight, mf.out_proj.bias, cat[:, :C], clips=B)
        _linear_into(half(y, 1), mb.out_proj.weight, mb.out_proj.bias, cat[:, C:], clips=B)
        out_f, out_b = cat[:, :C], cat[:, C:]
        gate = self.fusion_gate(cat)
        out = self.out_proj(gate * out_f + (1.0 - gate) * out_b).view(B, Lp, C)
        if Lp > L:
            out = out[:, :L].contiguous()
        return out, (conv_new, ssm_f)
