"""HIP-graph replay of the stateful streaming chunk (the B=1 latency path).

A streaming chunk of VideoMamba-M issues ~230 kernel launches (patch embed, then per
layer add+norm, in_proj, conv, x_proj, dt_proj, scan, out_proj, ...).  At B=1 every kernel
is short, so host launch latency leaves the GPU idle between them (profiles: 5.8 ms wall
for 4.4 ms of kernels).  ``StreamingChunkGraph`` captures the whole chunk forward once per
chunk kind (first chunk with CLS, continuation chunk without) into a ``torch.cuda.CUDAGraph``
(a hipGraph on ROCm) and replays it:

* the clip chunk, the temporal-position slice and the per-layer ``(conv_state, ssm_state)``
  live in static device buffers owned by the runner;
* ``run(x, temporal_pos_offset)`` copies the chunk and its temporal-embedding slice into
  the static buffers (two device copies), replays the graph, and returns the outputs the
  eager ``model(x, ssm_state=..., temporal_pos_offset=...)`` would return minus the state
  container — views of static buffers, valid until the next ``run``;
* the state advances in place (the ssm state is updated in place by the scan as in the
  eager path; the conv windows live in two stacked buffers used in turn — a chunk reads
  the current one and its conv kernels write the next, so no copy carries them over: each
  chunk kind is captured once per buffer parity),
  so consecutive ``run`` calls stream exactly like the eager loop with carried state.

Semantics are the eager path's (same kernels, same rounding points); tests check replay
against eager chunk by chunk.  Masks and keep_temporal pooling are not graph-captured
(use the eager forward for those).

Lifetimes.  A graph replays raw device pointers, so everything it touches is pinned for
its lifetime: the runner owns the scan's scratch workspace (no shared cache can grow and
free it under the graph), and it records every parameter's (data_ptr, version) at
capture (and holds references to them).  When the model's parameters change
(``load_state_dict``, an in-place edit, a ``.to()``), the next ``run`` drops the stale
graphs and captures again, so a replay never reads weight caches that the eager path has
since replaced; replacing Parameter objects outright needs ``invalidate()``.
"""

from __future__ import annotations

import operator
from typing import Dict, List, Optional, Tuple

import torch
from torch import Tensor

from . import kernels as K

_VERSION = operator.attrgetter("_version")

__all__ = ["StreamingChunkGraph", "chunk_workspace_bytes"]


def chunk_workspace_bytes(model, batch: int, tt: int, gh: int, gw: int) -> Tuple[int, int]:
    """(scratch bytes, sync bytes) one streaming chunk of ``tt`` temporal tokens on a
    ``gh`` x ``gw`` grid needs, over BOTH chunk kinds: the first chunk scans
    L = tt*gh*gw + 1 tokens (CLS row), continuation chunks L - 1, and the scan's cost model
    may pick a larger segment count (more scratch) for the shorter one.  The max over the
    scan, the conv_proj forms and the pooling sums of every mixer."""
    C = model.embed_dim
    need, sync_need = 0, 0
    for L in (tt * gh * gw + 1, tt * gh * gw):
        Lp = (L + 7) // 8 * 8
        need = max(need, K.norm_pool_workspace_bytes(batch, 1, L, C),
                   K.norm_pool_workspace_bytes(batch, tt, gh * gw, C))
        for mx in model._mixers():
            E = mx.dt_rank + 2 * mx.d_state
            need = max(need, K.scan_workspace_bytes(batch, mx.d_inner, L, mx.d_state))
            if mx.d_inner % 64 == 0:
                need = max(need, K.conv_proj_cm_workspace_bytes(batch, Lp, mx.d_inner, E),
                           K.conv_proj_workspace_bytes(batch, Lp, mx.d_inner, E))
            sync_need = max(sync_need, K.scan_sync_bytes(batch, mx.d_inner, L, mx.d_state))
    return need, sync_need


class StreamingChunkGraph:
    def __init__(self, model, batch: int, frames: int, height: int = 224, width: int = 224,
                 dtype: Optional[torch.dtype] = None, device=None):
        self.model = model
        p = model.patch_embed.proj.weight
        self.dtype = p.dtype if dtype is None else dtype
        self.device = p.device if device is None else torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("StreamingChunkGraph requires the model on a HIP device")
        self.batch, self.frames = batch, frames
        self.tt = model._validate_temporal_length(frames)
        self.static_x = torch.zeros(batch, 3, frames, height, width, dtype=self.dtype,
                                    device=self.device)
        self.static_tpos = torch.zeros(1, self.tt, model.embed_dim, dtype=self.dtype,
                                       device=self.device)
        # per-layer conv states as views of two stacked buffers used in turn: a chunk reads
        # _conv[_cur] and its conv kernels write _conv[1 - _cur] (a copy back cost a 4 us
        # launch per chunk); the ssm states are updated in place
        st = model.allocate_state(batch, dtype=self.dtype, device=self.device)
        conv = torch.stack([c for c, _ in st])
        self._conv = (conv, torch.zeros_like(conv))
        self._ssm = [s for _, s in st]
        self._cur = 0
        self._graphs: Dict[Tuple[bool, int], Tuple[torch.cuda.CUDAGraph, object]] = {}
        self._pool = None
        self._param_key = None
        self._plist = None
        self._tpos_offset = None  # temporal offset whose embedding slice static_tpos holds
        self._ws = None  # scan scratch owned by the captured graphs
        self._sync = None  # the one-launch scan's sync buffer (zeroed once; replays keep it valid)
        self._cnt = None  # vm_linear_add_norm_fwd hand-off counters (zeroed, left zeroed)

    # ------------------------------------------------------------------ state
    def _state_at(self, parity: int) -> List[Tuple[Tensor, Tensor]]:
        conv = self._conv[parity]
        return [(conv[i], s) for i, s in enumerate(self._ssm)]

    @property
    def state(self) -> List[Tuple[Tensor, Tensor]]:
        """The carried per-layer (conv_state, ssm_state): views of the runner's static
        buffers, current until the next run() (which moves the conv states to the other
        buffer of the pair)."""
        return self._state_at(self._cur)

    def reset_state(self) -> None:
        for c, s in self.state:
            c.zero_()
            s.zero_()

    def load_state(self, state) -> None:
        for (c, s), (c2, s2) in zip(self.state, state):
            c.copy_(c2)
            s.copy_(s2)

    # ------------------------------------------------------------------ capture / replay
    def _body(self, has_cls: bool, parity: int):
        m = self.model
        offset = 0 if has_cls else 1  # only has_cls matters inside; tpos comes from the buffer
        pool = None
        if m.add_pool_norm:
            gh, gw = m._spatial_token_grid(self.static_x.shape[-2], self.static_x.shape[-1])
            pool = (False, self.tt, gh * gw)
        feats, x_pool, _ = m._encode(self.static_x, None, self._state_at(parity), offset,
                                     tpos=self.static_tpos, pool=pool,
                                     conv_out=self._conv[1 - parity])
        if pool is None:
            return (feats,)
        return (feats[:, 1:] if has_cls else feats), x_pool

    def _params_key(self):
        # the parameter list is walked once (the module-tree walk was ~0.4 ms of every
        # run); held references keep the captured tensors' memory alive, and a load /
        # in-place edit / .to() shows as a version or data_ptr change on them
        if self._plist is None:
            self._plist = list(self.model.parameters()) + list(self.model.buffers())
        # two C-level maps instead of a generator of pairs: ~35 % less host time per chunk
        return (tuple(map(_VERSION, self._plist)), tuple(map(Tensor.data_ptr, self._plist)))

    def invalidate(self) -> None:
        """Drop the captured graphs and re-scan the parameters: call after replacing
        Parameter objects (``module.weight = nn.Parameter(...)``); loads, in-place edits
        and ``.to()`` are detected on their own."""
        self._graphs.clear()
        self._pool = None
        self._plist = None
        self._param_key = None
        self._tpos_offset = None

    def _workspace(self) -> Tensor:
        """Kernel scratch (segmented scan, conv_proj partials, pooling sums) sized for the
        largest consumer of either chunk kind; allocated once per capture set, owned by this
        runner (with the one-launch scan's sync buffer)."""
        m = self.model
        gh, gw = m._spatial_token_grid(self.static_x.shape[-2], self.static_x.shape[-1])
        need, sync_need = chunk_workspace_bytes(m, self.batch, self.tt, gh, gw)
        if self._ws is None or self._ws.numel() < max(need, 1):
            self._ws = torch.empty(max(need, 1), dtype=torch.uint8, device=self.device)
        # the one-launch scan's sync buffer: zeroed once, left valid for the next by every replay
        if self._sync is None or self._sync.numel() < max(sync_need, 1):
            self._sync = torch.zeros(max(sync_need, 4096), dtype=torch.uint8, device=self.device)
        Lp = (self.tt * gh * gw + 1 + 7) // 8 * 8
        cnt_need = K.linear_add_norm_counter_bytes(self.batch * Lp)
        if self._cnt is None or self._cnt.numel() < max(cnt_need, 1):
            self._cnt = torch.zeros(max(cnt_need, 4096), dtype=torch.uint8, device=self.device)
        return self._ws

    def check(self) -> None:
        """Raise if a replayed one-launch scan ever timed out on a block hand-off, or a
        replayed fused out_proj + add + RMSNorm on a row-block hand-off (their outputs were
        NaN); synchronises with the queued replays.  See K.check_scan_sync and
        K.check_linear_add_norm."""
        if self._sync is not None and K.scan_sync_status(self._sync):
            K.clear_scan_sync_error(self._sync)
            raise RuntimeError("StreamingChunkGraph: a replayed one-launch scan timed out on a "
                               "block hand-off; the affected outputs were NaN")
        if self._cnt is not None and K.linear_add_norm_status(self._cnt):
            self._cnt.zero_()  # whole buffer: late producers may have left counts behind
            raise RuntimeError("StreamingChunkGraph: a replayed fused out_proj + add + RMSNorm "
                               "timed out on a row-block hand-off; the affected rows were NaN")

    def _capture(self, has_cls: bool, parity: int):
        # the warm-up passes advance the ssm states in place and write the other conv
        # buffer: keep the current states to restore them
        saved = [(c.clone(), s.clone()) for c, s in self._state_at(parity)]
        ws = self._workspace()
        side = torch.cuda.Stream(self.device)
        side.wait_stream(torch.cuda.current_stream(self.device))
        with torch.no_grad(), torch.cuda.stream(side), K.scratch_override(ws), \
                K.sync_override(self._sync), K.counter_override(self._cnt):
            for _ in range(2):  # warm caches (fp32 params, padded weights) and GEMM plans
                self._body(has_cls, parity)
        torch.cuda.current_stream(self.device).wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.no_grad(), torch.cuda.graph(g, pool=self._pool), K.scratch_override(ws), \
                K.sync_override(self._sync), K.counter_override(self._cnt):
            outs = self._body(has_cls, parity)
        self._pool = g.pool()
        for (c, s), (c2, s2) in zip(self._state_at(parity), saved):
            c.copy_(c2)
            s.copy_(s2)
        self._graphs[(has_cls, parity)] = (g, outs)

    def run(self, x: Tensor, temporal_pos_offset: int = 0):
        """One chunk: (x_vis, x_pool) with ``add_pool_norm``, else x_vis — as the eager
        forward with a full carried state, minus the returned state (see ``state``)."""
        if tuple(x.shape) != tuple(self.static_x.shape):
            raise ValueError(f"chunk shape {tuple(x.shape)} != captured "
                             f"{tuple(self.static_x.shape)}")
        m = self.model
        has_cls = temporal_pos_offset <= 0
        if m.add_pool_norm:
            m._check_pool(has_cls)
        # the input copy goes first, so the device runs it while the host checks the
        # parameters (~25 us of host time per chunk)
        self.static_x.copy_(x)
        key = self._params_key()
        if key != self._param_key:  # parameters changed since capture: capture again
            self._graphs.clear()
            self._pool = None
            self._param_key = key
            self._tpos_offset = None
        if temporal_pos_offset != self._tpos_offset:  # the slice only changes with the offset
            tpos = m._get_temporal_pos_embedding(self.tt, offset=temporal_pos_offset,
                                                 dtype=self.dtype, device=self.device)
            self.static_tpos.copy_(tpos)
            self._tpos_offset = temporal_pos_offset
        key = (has_cls, self._cur)
        if key not in self._graphs:
            self._capture(*key)
        g, outs = self._graphs[key]
        g.replay()
        self._cur = 1 - self._cur  # the conv kernels wrote the other buffer
        return outs[0] if len(outs) == 1 else outs
