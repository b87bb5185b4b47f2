"""Host-side operator shims over the HIP C ABI, mirroring the reference's kernel seams.

Public functions keep the call shapes the reference uses for its third-party kernels
(``models/videomamba/mamba_simple.py:11-14``, ``videomamba.py:11``):

* ``selective_scan_fn``      <- mamba_ssm ``selective_scan_fn`` (+ ``initial_state``)
* ``selective_state_update`` <- mamba_ssm Triton ``selective_state_update``
* ``causal_conv1d_fn`` / ``causal_conv1d_update`` <- causal-conv1d
* ``rms_norm_fn`` / ``layer_norm_fn`` <- mamba_ssm Triton layer norm

plus ``patch_embed`` (PatchEmbed Conv3d + positional adds).  Every function runs the HIP
kernels of ``libvideomamba_hip.so`` on the tensors' device and current stream; CPU
tensors raise ``RuntimeError`` (as the reference does at ``mamba_simple.py:304-308``),
and a missing library raises — there is no fallback path.

The ``*_raw`` launchers take explicit element strides and are what the model uses for
its padded channel-major layouts.
"""

from __future__ import annotations

import threading
import weakref
from typing import Optional, Tuple

import torch
from torch import Tensor

from . import _lib, options

_DT = {torch.float32: _lib.VM_DTYPE_F32, torch.bfloat16: _lib.VM_DTYPE_BF16}


def dtype_code(dt: torch.dtype) -> int:
    try:
        return _DT[dt]
    except KeyError:
        raise TypeError(f"unsupported dtype {dt}: the HIP kernels take float32 or bfloat16")


def require_gpu(*tensors: Optional[Tensor], what: str = "VideoMamba") -> None:
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise RuntimeError(
                f"{what} requires CUDA tensors in this package because its HIP kernels "
                "(libvideomamba_hip, gfx950) are GPU-only; move the model and inputs to the "
                "ROCm device (.cuda())."
            )


def _stream(t: Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _p(t: Optional[Tensor]):
    return None if t is None else t.data_ptr()


def f32c(t: Optional[Tensor]) -> Optional[Tensor]:
    """fp32 contiguous view/copy of a small parameter (A, D, biases, weights)."""
    if t is None:
        return None
    t = t.detach()
    if t.dtype != torch.float32:
        t = t.float()
    return t.contiguous()


def f32_cached(owner, t: Optional[Tensor], slot: str) -> Optional[Tensor]:
    """fp32 contiguous copy of a small parameter cached on ``owner`` (a module) and
    refreshed when the parameter changes (data pointer, version, dtype or device)."""
    if t is None:
        return None
    key = (t.data_ptr(), t._version, t.dtype, t.device)
    cache = owner.__dict__.setdefault("_vm_f32_cache", {})
    hit = cache.get(slot)
    if hit is None or hit[0] != key:
        with torch.no_grad():
            hit = (key, f32c(t))
        cache[slot] = hit
    return hit[1]


def _lastdim_contig(t: Optional[Tensor]) -> Optional[Tensor]:
    if t is None:
        return None
    return t if (t.stride(-1) == 1 or t.shape[-1] <= 1) else t.contiguous()


def _channel_contig(t: Optional[Tensor]) -> Optional[Tensor]:
    """(b, d, l) view with unit stride on d (token-major storage)."""
    if t is None:
        return None
    if t.stride(1) == 1 or t.shape[1] <= 1:
        return t
    return t.transpose(1, 2).contiguous().transpose(1, 2)


# --------------------------------------------------------------------------- raw launchers
class _Slot(threading.local):
    """A per-host-thread override slot.  The sub-batch forward issues its streams from one
    host thread each (videomamba._issue_phase_locked): an override entered on one thread (a
    graph capture's scratch, sync and counter buffers) must never reach a launch issued by
    another thread onto another stream, which would then share those buffers unordered."""

    value = None


_WORKSPACE = {}
_WS_OVERRIDE = _Slot()


class scratch_override:
    """Within the block every kernel that needs scratch (the segmented token-major scan,
    the channel-major conv_proj's x_proj partials) uses ``buf`` (a uint8 device tensor owned
    by the caller) instead of the per-stream cache — how a captured HIP graph keeps its
    scratch alive and fixed for its lifetime (graphs.StreamingChunkGraph).  Consumers run
    one after another on one stream, so they share the buffer from offset 0."""

    def __init__(self, buf: Tensor):
        self.buf = buf

    def __enter__(self):
        self.prev = _WS_OVERRIDE.value
        _WS_OVERRIDE.value = self.buf
        return self.buf

    def __exit__(self, *exc):
        _WS_OVERRIDE.value = self.prev
        return False


def scratch(device: torch.device, stream: int, nbytes: int) -> Optional[Tensor]:
    """Kernel scratch, one buffer per (device, stream), grown and never shrunk (or the
    caller's buffer inside ``scratch_override``).  When it grows, the old buffer is released
    back to the caching allocator on that same stream, so work already queued there
    finishes first.  Captured HIP graphs own their scratch (graphs.StreamingChunkGraph) and
    never reach this cache."""
    if nbytes <= 0:
        return None
    ov = _WS_OVERRIDE.value
    if ov is not None:
        if ov.numel() < nbytes:
            raise RuntimeError(f"scratch_override buffer too small: {ov.numel()} < {nbytes}")
        return ov
    key = (device.type, device.index, stream)
    buf = _WORKSPACE.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.empty(nbytes, dtype=torch.uint8, device=device)
        _WORKSPACE[key] = buf
    return buf


_SYNC = {}
_SYNC_OVERRIDE = _Slot()
_SYNC_SEEN = weakref.WeakValueDictionary()  # id -> caller-owned sync buffer (sync_override)


class sync_override:
    """Within the block the one-launch segmented scan uses ``buf`` (a zero-filled uint8
    device tensor owned by the caller, e.g. a captured graph) as its sync buffer instead of
    the per-stream one.  The library leaves the buffer zeroed after every launch."""

    def __init__(self, buf: Tensor):
        self.buf = buf

    def __enter__(self):
        self.prev = _SYNC_OVERRIDE.value
        _SYNC_OVERRIDE.value = self.buf
        _SYNC_SEEN[id(self.buf)] = self.buf
        return self.buf

    def __exit__(self, *exc):
        _SYNC_OVERRIDE.value = self.prev
        return False


def sync_buffer(device: torch.device, stream: int, nbytes: int) -> Optional[Tensor]:
    """The one-launch scan's sync buffer: zero-filled when allocated, left valid for the next
    launch by every launch (epoch-tagged hand-off granules, ABI v9), one per (device, stream)
    so no two concurrent launches share it; grown (a new zeroed buffer) when a shape needs
    more."""
    if nbytes <= 0:
        return None
    ov = _SYNC_OVERRIDE.value
    if ov is not None:
        return ov if ov.numel() >= nbytes else None
    key = (device.type, device.index, stream)
    buf = _SYNC.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.zeros(max(nbytes, 4096), dtype=torch.uint8, device=device)
        _SYNC[key] = buf
    return buf


SYNC_HEADER_BYTES = 16  # error word, epoch, start count, pad (ABI v9)
SYNC_ERROR_BYTES = 4  # the error word alone


def scan_sync_status(buf: Tensor) -> int:
    """0 when no one-launch scan that used ``buf`` (a sync buffer, device or host copy)
    timed out waiting for an earlier block, 1 when one did (its outputs are NaN).  Reads
    the header through ``vm_selective_scan_sync_status``; a device buffer is copied to the
    host first (this synchronises with the work queued on it)."""
    head = buf.detach().reshape(-1)[:SYNC_HEADER_BYTES].to(torch.uint8)
    head = head.cpu().contiguous() if head.is_cuda else head.contiguous()
    rc = int(_lib.load().vm_selective_scan_sync_status(head.data_ptr(), head.numel()))
    if rc < 0:
        _lib.check(rc, "vm_selective_scan_sync_status")
    return rc


def clear_scan_sync_error(buf: Tensor) -> None:
    """Re-arm a sync buffer after a reported timeout: zero its error word (header word 0)
    only.  The epoch (word 1) must keep growing — granules of earlier launches never match a
    later launch's tag only because every launch uses a higher one (ABI v9)."""
    buf.reshape(-1)[:SYNC_ERROR_BYTES].zero_()


def check_scan_sync(clear: bool = True) -> None:
    """Raise RuntimeError if any sync buffer this process has used (the per-stream ones and
    those passed through :class:`sync_override`, e.g. a captured graph's) recorded a
    timed-out block hand-off.  ``clear`` re-arms the buffers' error words first.  The
    kernels never hang and never write plausible wrong values on a timeout (the affected
    outputs are NaN); this turns the event into an exception."""
    bad = 0
    for buf in list(_SYNC.values()) + list(_SYNC_SEEN.values()):
        if scan_sync_status(buf):
            bad += 1
            if clear:
                clear_scan_sync_error(buf)
    if bad:
        raise RuntimeError(f"one-launch selective scan: {bad} sync buffer(s) recorded a "
                           "timed-out block hand-off; the affected outputs are NaN")


def scan_sync_bytes(batch: int, dim: int, seqlen: int, dstate: int,
                    segments: Optional[int] = None) -> int:
    seg = options.get().scan_segments if segments is None else segments
    return int(_lib.load().vm_selective_scan_sync_bytes(batch, dim, seqlen, dstate, seg))


def scan_workspace_bytes(batch: int, dim: int, seqlen: int, dstate: int,
                         segments: Optional[int] = None) -> int:
    seg = options.get().scan_segments if segments is None else segments
    return int(_lib.load().vm_selective_scan_workspace_bytes(batch, dim, seqlen, dstate, seg))


def scan_raw(u, u_s, delta, dl_s, A32, B, b_s, C, c_s, D32, z, z_s, bias32, softplus,
             h0, h0_s, h_last, hl_s, out, o_s, out_len, batch, dim, seqlen, dstate, dtype,
             stream, workspace: Optional[Tensor] = None, pair=None):
    """Strides are (batch, channel|state, step) element strides; either every
    u/delta/z/out channel stride is 1 (token-major) or every step stride is 1.
    ``workspace`` (a uint8 device buffer) replaces the per-stream scratch cache.
    ``pair`` = (split, A32_bwd, D32_bwd, bias32_bwd, h0_bwd, h_last_bwd, frame_len) runs
    ``vm_selective_scan_bidir_fwd``: rows >= split are the flipped backward direction."""
    lib = _lib.load()
    seg = int(options.get().scan_segments)
    ws_bytes = 0
    ws = None
    sync, sync_bytes = None, 0
    if u_s[1] == 1:
        ws_bytes = scan_workspace_bytes(batch, dim, seqlen, dstate, seg)
        if workspace is not None:
            if workspace.numel() < ws_bytes:
                raise ValueError(f"scan workspace too small: {workspace.numel()} < {ws_bytes}")
            ws = workspace
        else:
            ws = scratch(u.device, int(stream), ws_bytes)
        if options.get().scan_one_launch:
            sync_bytes = scan_sync_bytes(batch, dim, seqlen, dstate, seg)
            sync = sync_buffer(u.device, int(stream), sync_bytes)
            if sync is None:
                sync_bytes = 0
    args = (_p(u), u_s[0], u_s[1], u_s[2], _p(delta), dl_s[0], dl_s[1], dl_s[2], _p(A32),
            _p(B), b_s[0], b_s[1], b_s[2], _p(C), c_s[0], c_s[1], c_s[2],
            _p(D32), _p(z), z_s[0], z_s[1], z_s[2], _p(bias32), int(softplus),
            _p(h0), dtype_code(h0.dtype) if h0 is not None else 0, h0_s[0], h0_s[1],
            _p(h_last), dtype_code(h_last.dtype) if h_last is not None else 0, hl_s[0],
            hl_s[1], _p(out), o_s[0], o_s[1], o_s[2], out_len, batch, dim, seqlen, dstate, dtype)
    if pair is None:
        rc = lib.vm_selective_scan_fwd(*args, seg, _p(ws), ws_bytes, _p(sync), sync_bytes,
                                       stream)
        _lib.check(rc, "vm_selective_scan_fwd")
        return
    split, a_b, d_b, bias_b, h0_b, hl_b, frame = pair
    rc = lib.vm_selective_scan_bidir_fwd(*args, split, _p(a_b), _p(d_b), _p(bias_b), _p(h0_b),
                                         _p(hl_b), frame, seg, _p(ws), ws_bytes, _p(sync),
                                         sync_bytes, stream)
    _lib.check(rc, "vm_selective_scan_bidir_fwd")


def scan_chunk_steps(batch: int, dim: int, seqlen: int, dstate: int, segments: int = -1) -> int:
    """Steps per segment the token-major scan runs for this shape (0: the single pass);
    ``segments`` -1 = ``options.scan_segments`` (``vm_selective_scan_chunk_steps``)."""
    seg = int(options.get().scan_segments) if segments < 0 else segments
    return int(_lib.load().vm_selective_scan_chunk_steps(batch, dim, seqlen, dstate, seg))


SCAN_DTPROJ_MAX_SEGMENT = 64  # the segmented dt_proj-in-scan form (ABI v11)
_SCAN_CHUNK_SEGS_PER_BLOCK = 8  # segments per workgroup of the chunked scan (kChW)
_CU_COUNT = {}


def _cu_count(device) -> int:
    idx = torch.device(device).index
    idx = torch.cuda.current_device() if idx is None else idx
    if idx not in _CU_COUNT:
        _CU_COUNT[idx] = int(torch.cuda.get_device_properties(idx).multi_processor_count)
    return _CU_COUNT[idx]


def scan_dtproj_segmented_pays(batch: int, dim: int, seqlen: int, dstate: int, device,
                               segments: int = -1) -> bool:
    """Whether the mixer should fold dt_proj into the SEGMENTED scan for this shape: segments
    of at most 64 steps, and a grid that fits the chip at one workgroup per CU.  Each wave's
    dt block lives in LDS (119 KB per workgroup), which admits one workgroup per CU; where
    the plain chunked scan would stack several per CU the folded form measured slower than
    it saves in conv_proj (B = 4 M-16f: 138.6 vs 111.2 us per scan against ~19 us of dt
    rows; B = 1 / 2 with 252-workgroup grids: +1.9 / +1.5 us per scan against 4.7 / ~9 us;
    profiles/r04v_scan_segments_dtp.jsonl)."""
    steps = scan_chunk_steps(batch, dim, seqlen, dstate, segments)
    if not 0 < steps <= SCAN_DTPROJ_MAX_SEGMENT:
        return False
    segs = -(-seqlen // steps)
    nblk = -(-segs // _SCAN_CHUNK_SEGS_PER_BLOCK)
    return batch * (-(-dim // 64)) * nblk <= _cu_count(device)


def scan_dtproj_raw(u, u_s, dtl, dtl_s, dt_rank, wdt_pad, A32, B, b_s, C, c_s, D32, z, z_s,
                    bias32, h0, h0_s, h_last, hl_s, out, o_s, out_len, batch, dim, seqlen,
                    dstate, stream, workspace: Optional[Tensor] = None):
    """``vm_selective_scan_dtproj_fwd``: the token-major scan with dt_proj folded in —
    delta = bf16(dt_low @ W_dt^T) on the matrix cores, then softplus(delta + bias) as
    selective_scan_fn.  ``dtl`` = the x_dbl rows (dt_low = their first ``dt_rank`` columns),
    ``dtl_s`` = (batch, row) element strides; ``wdt_pad`` = the zero-padded (D, 32|64) bf16
    W_dt.  bf16 only, z and softplus on.  Single pass at chip-filling batches; below that
    the segmented form (segments of at most 64 steps) computes each segment's dt exactly as
    conv_proj's dt_proj would (ABI v11), with the scratch / sync buffers of ``scan_raw``."""
    lib = _lib.load()
    seg = int(options.get().scan_segments)
    ws_bytes = scan_workspace_bytes(batch, dim, seqlen, dstate, seg)
    ws, sync, sync_bytes = None, None, 0
    if ws_bytes:
        if workspace is not None:
            if workspace.numel() < ws_bytes:
                raise ValueError(f"scan workspace too small: {workspace.numel()} < {ws_bytes}")
            ws = workspace
        else:
            ws = scratch(u.device, int(stream), ws_bytes)
        if options.get().scan_one_launch:
            sync_bytes = scan_sync_bytes(batch, dim, seqlen, dstate, seg)
            sync = sync_buffer(u.device, int(stream), sync_bytes)
            if sync is None:
                sync_bytes = 0
    rc = lib.vm_selective_scan_dtproj_fwd(
        _p(u), u_s[0], u_s[1], u_s[2], _p(dtl), dtl_s[0], dtl_s[1], int(dt_rank),
        _p(wdt_pad), wdt_pad.stride(0), _p(A32),
        _p(B), b_s[0], b_s[1], b_s[2], _p(C), c_s[0], c_s[1], c_s[2],
        _p(D32), _p(z), z_s[0], z_s[1], z_s[2], _p(bias32), 1,
        _p(h0), dtype_code(h0.dtype) if h0 is not None else 0, h0_s[0], h0_s[1],
        _p(h_last), dtype_code(h_last.dtype) if h_last is not None else 0, hl_s[0], hl_s[1],
        _p(out), o_s[0], o_s[1], o_s[2], out_len, batch, dim, seqlen, dstate,
        dtype_code(u.dtype), seg, _p(ws), ws_bytes, _p(sync), sync_bytes, stream)
    _lib.check(rc, "vm_selective_scan_dtproj_fwd")


def conv_raw(x, x_s, w32, b32, cs_in, csi_s, cs_out, cso_s, out, o_s, out_len, batch, dim,
             seqlen, width, silu, dtype, stream):
    """x_s / o_s: (batch, channel, step) element strides (unit step or unit channel)."""
    lib = _lib.load()
    rc = lib.vm_causal_conv1d_fwd(
        _p(x), x_s[0], x_s[1], x_s[2], _p(w32), _p(b32),
        _p(cs_in), dtype_code(cs_in.dtype) if cs_in is not None else 0, csi_s[0], csi_s[1],
        _p(cs_out), dtype_code(cs_out.dtype) if cs_out is not None else 0, cso_s[0], cso_s[1],
        _p(out), o_s[0], o_s[1], o_s[2], out_len, batch, dim, seqlen, width, int(silu), dtype,
        stream)
    _lib.check(rc, "vm_causal_conv1d_fwd")


def conv_proj_raw(xz, xz_s, cw32, cb32, cs_in, csi_s, cs_out, cso_s, wx_pad, e, wdt_pad, r,
                  u, u_s, xdbl, xd_s, dt, dt_s, out_len, batch, dim, seqlen, width, stream,
                  dt_bias32=None, dt_softplus=False):
    """Fused token-major conv1d + SiLU -> x_proj -> dt_proj (bf16).  *_s = (batch, step)
    element strides of the token-major buffers; wx_pad (e_pad, D) / wdt_pad (D, r_pad) are
    zero-padded copies of the projection weights.  dt_softplus: `dt` receives the scan's
    activated step softplus(dt + dt_bias32) instead (the scan then runs without them).
    dt=None skips dt_proj (conv + x_proj only; wdt_pad may be None)."""
    lib = _lib.load()
    nbytes = int(lib.vm_conv_proj_workspace_bytes(batch, out_len, dim, e))
    ws = scratch(xz.device, int(stream), nbytes)
    rc = lib.vm_conv_proj_fwd(
        _p(xz), xz_s[0], xz_s[1], _p(cw32), _p(cb32),
        _p(cs_in), dtype_code(cs_in.dtype) if cs_in is not None else 0, csi_s[0], csi_s[1],
        _p(cs_out), dtype_code(cs_out.dtype) if cs_out is not None else 0, cso_s[0], cso_s[1],
        _p(wx_pad), e, wx_pad.shape[0], _p(wdt_pad), r,
        wdt_pad.shape[1] if wdt_pad is not None else 0,
        _p(u), u_s[0], u_s[1], _p(xdbl), xd_s[0], xd_s[1], _p(dt),
        dt_s[0] if dt is not None else 0, dt_s[1] if dt is not None else 0,
        _p(dt_bias32), int(dt_softplus), out_len, batch, dim, seqlen, width, dtype_code(u.dtype),
        _p(ws), nbytes, stream)
    _lib.check(rc, "vm_conv_proj_fwd")


def in_proj_conv_proj_fits(k: int, batch: int, out_len: int, dim: int, e: int, e_pad: int,
                           r_pad: int, width: int, has_dt: bool) -> bool:
    """Whether ``vm_in_proj_conv_proj_fwd`` takes this shape (pure host query)."""
    return bool(_lib.load().vm_in_proj_conv_proj_fits(k, batch, out_len, dim, e, e_pad, r_pad,
                                                      width, int(has_dt)))


def in_proj_conv_proj_raw(hn, w_in, z, cw32, cb32, cs_in, csi_s, cs_out, cso_s, wx_pad, e,
                          wdt_pad, r, u, xdbl, dt, out_len, batch, dim, seqlen, width, stream):
    """in_proj + conv1d + SiLU -> x_proj [-> dt_proj] in two launches (bf16, small batches,
    token-major): hn (n, k), w_in (2 dim, k); z (n, dim) receives in_proj's z half (any row
    stride, e.g. the right half of an (n, 2 dim) xz), u (n, dim), xdbl (n, e), dt (n, dim) or
    None (the scan computes dt).  Bit-identical to ``linear`` + :func:`conv_proj_raw`.
    Scratch for the x_proj partials comes from :func:`scratch`."""
    lib = _lib.load()
    nbytes = int(lib.vm_in_proj_conv_proj_workspace_bytes(batch, out_len, dim, e))
    ws = scratch(hn.device, int(stream), nbytes)
    rc = lib.vm_in_proj_conv_proj_fwd(
        _p(hn), hn.stride(0), _p(w_in), w_in.stride(0), hn.shape[1], _p(z), z.stride(0),
        _p(cw32), _p(cb32),
        _p(cs_in), dtype_code(cs_in.dtype) if cs_in is not None else 0, csi_s[0], csi_s[1],
        _p(cs_out), dtype_code(cs_out.dtype) if cs_out is not None else 0, cso_s[0], cso_s[1],
        _p(wx_pad), e, wx_pad.shape[0], _p(wdt_pad if dt is not None else None), r,
        wdt_pad.shape[1] if (wdt_pad is not None and dt is not None) else 0,
        _p(u), u.stride(0), _p(xdbl), xdbl.stride(0), _p(dt),
        dt.stride(0) if dt is not None else 0, out_len, batch, dim, seqlen, width,
        _p(ws), nbytes, stream)
    _lib.check(rc, "vm_in_proj_conv_proj_fwd")


def conv_proj_fits(batch: int, out_len: int, seqlen: int, dim: int, e: int, r_pad: int,
                   xz_s, u_sl: int, cs_in: Optional[Tensor], width: int) -> bool:
    """Whether ``vm_conv_proj_fwd`` accepts this token-major shape (``vm_conv_proj_fits``):
    the wide form (batch > 8) addresses its operands through 31-bit buffer offsets, so very
    long sequences go to the unfused conv + projection path instead of raising."""
    csi = (cs_in.stride(0), cs_in.stride(1)) if cs_in is not None else (0, 0)
    return bool(_lib.load().vm_conv_proj_fits(
        batch, out_len, seqlen, dim, e, r_pad, 0, xz_s[0], xz_s[1], int(cs_in is not None),
        dtype_code(cs_in.dtype) if cs_in is not None else 0, csi[0], csi[1], width, u_sl))


def conv_proj_workspace_bytes(batch: int, out_len: int, dim: int, e: int) -> int:
    return int(_lib.load().vm_conv_proj_workspace_bytes(batch, out_len, dim, e))


def conv_proj_cm_workspace_bytes(batch: int, out_len: int, dim: int, e: int) -> int:
    return int(_lib.load().vm_conv_proj_cm_workspace_bytes(batch, out_len, dim, e))


def conv_proj_cm_raw(xz, x_sd, cw32, cb32, cs_in, csi_s, cs_out, cso_s, wx_pad, e, wdt_pad, r,
                     u, u_sd, xdbl, xd_sd, dt, dt_sd, out_len, batch, dim, seqlen, width,
                     stream):
    """Channel-major conv1d + SiLU -> x_proj -> dt_proj (bf16, small batches): rows are
    channels (x = the first ``dim`` rows of xz), columns the batch * out_len tokens;
    ``*_sd`` are row strides.  Scratch for the split-K x_proj partials comes from
    :func:`scratch`."""
    lib = _lib.load()
    nbytes = conv_proj_cm_workspace_bytes(batch, out_len, dim, e)
    ws = scratch(xz.device, int(stream), nbytes)
    rc = lib.vm_conv_proj_cm_fwd(
        _p(xz), x_sd, _p(cw32), _p(cb32),
        _p(cs_in), dtype_code(cs_in.dtype) if cs_in is not None else 0, csi_s[0], csi_s[1],
        _p(cs_out), dtype_code(cs_out.dtype) if cs_out is not None else 0, cso_s[0], cso_s[1],
        _p(wx_pad), e, wx_pad.shape[0], _p(wdt_pad), r, wdt_pad.shape[1],
        _p(u), u_sd, _p(xdbl), xd_sd, _p(dt), dt_sd, out_len, batch, dim, seqlen, width,
        _p(ws), nbytes, stream)
    _lib.check(rc, "vm_conv_proj_cm_fwd")


def add_norm_raw(x, residual, w32, b32, out, residual_out, rows, cols, eps, is_rms, stream):
    lib = _lib.load()
    rc = lib.vm_add_norm_fwd(
        _p(x), dtype_code(x.dtype), _p(residual),
        dtype_code(residual.dtype) if residual is not None else 0,
        _p(w32), _p(b32), _p(out), dtype_code(out.dtype), _p(residual_out),
        dtype_code(residual_out.dtype) if residual_out is not None else 0,
        rows, cols, float(eps), int(is_rms), stream)
    _lib.check(rc, "vm_add_norm_fwd")


LINEAR_FORMS = {"auto": 0, "dma": 1, "persistent": 2}


def linear(x: Tensor, w: Tensor, b32: Optional[Tensor] = None,
           out: Optional[Tensor] = None, form: str = "auto") -> Tensor:
    """``x @ w.T (+ b)`` on the HIP GEMM (``vm_linear_fwd_form``): x (m, k), w (n, k) bf16
    with unit column stride; ``out`` (m, n) may be a column-sliced view.  ``form`` names the
    kernel ("dma": 128-row LDS-DMA tiles, "persistent": the 256-row persistent kernel,
    "auto": by shape); every form gives the same bits."""
    m, k = x.shape
    n = w.shape[0]
    if out is None:
        out = torch.empty((m, n), dtype=x.dtype, device=x.device)
    rc = _lib.load().vm_linear_fwd_form(_p(x), x.stride(0), _p(w), w.stride(0), _p(b32),
                                        _p(out), out.stride(0), m, n, k, dtype_code(x.dtype),
                                        LINEAR_FORMS[form], _stream(x))
    _lib.check(rc, "vm_linear_fwd")
    return out


_CNT = {}
_CNT_OVERRIDE = _Slot()
_CNT_SEEN = weakref.WeakValueDictionary()  # id -> caller-owned counter buffer (counter_override)


class counter_override:
    """Within the block ``vm_linear_add_norm_fwd`` takes its hand-off counters from ``buf``
    (a zero-filled uint8 device tensor owned by the caller, e.g. a captured graph) instead
    of the per-stream buffer.  The kernel leaves the counters zeroed."""

    def __init__(self, buf: Tensor):
        self.buf = buf

    def __enter__(self):
        self.prev = _CNT_OVERRIDE.value
        _CNT_OVERRIDE.value = self.buf
        _CNT_SEEN[id(self.buf)] = self.buf
        return self.buf

    def __exit__(self, *exc):
        _CNT_OVERRIDE.value = self.prev
        return False


def counter_buffer(device: torch.device, stream: int, nbytes: int) -> Tensor:
    ov = _CNT_OVERRIDE.value
    if ov is not None:
        if ov.numel() < nbytes:
            raise RuntimeError(f"counter_override buffer too small: {ov.numel()} < {nbytes}")
        return ov
    key = (device.type, device.index, stream)
    buf = _CNT.get(key)
    if buf is None or buf.numel() < nbytes:
        buf = torch.zeros(max(nbytes, 4096), dtype=torch.uint8, device=device)
        _CNT[key] = buf
    return buf


def linear_add_norm_counter_bytes(m: int) -> int:
    return int(_lib.load().vm_linear_add_norm_counter_bytes(m))


def linear_add_norm_status(buf: Tensor) -> int:
    """0 when no ``vm_linear_add_norm_fwd`` launch that used the counter buffer ``buf``
    timed out waiting for a row block's producers, else non-zero (that launch's normalised
    rows are NaN).  Reads the error word (word 0); a device buffer is copied to the host,
    which synchronises with the work queued on it."""
    w = buf.detach().reshape(-1)[:4].to(torch.uint8)
    w = w.cpu() if w.is_cuda else w
    return int.from_bytes(bytes(w.tolist()), "little")


def check_linear_add_norm(clear: bool = True) -> None:
    """Raise RuntimeError if any counter buffer this process has used (the per-stream ones
    and those passed through :class:`counter_override`) recorded a timed-out hand-off of the
    fused out_proj + add + RMSNorm.  With ``clear`` every such buffer is re-zeroed whole, not
    just its error word: a timed-out poller resets its block's counter while late producers
    may still add to it, which would leave a stale count that lets a later launch pass its
    poll early.  The status read synchronises first, so every producer has finished."""
    bad = 0
    for buf in list(_CNT.values()) + list(_CNT_SEEN.values()):
        if linear_add_norm_status(buf):
            bad += 1
            if clear:
                buf.zero_()
    if bad:
        raise RuntimeError(f"fused out_proj + add + RMSNorm: {bad} counter buffer(s) recorded a "
                           "timed-out row-block hand-off; the affected rows are NaN")


def linear_add_norm(x: Tensor, w: Tensor, residual: Tensor, norm_w32: Tensor, eps: float,
                    hn: Tensor, h: Optional[Tensor] = None) -> Tensor:
    """The mixer's out_proj fused with the next block's residual add + RMSNorm
    (``vm_linear_add_norm_fwd``): h = bf16(x @ w^T); residual += h (fp32, in place);
    hn = bf16(rmsnorm(residual) * norm_w) — bit-identical to ``linear`` followed by
    ``vm_add_norm_fwd``.  x (m, k), w (n, k) bf16; residual (m, n) fp32; hn (m, n) bf16.
    Returns h (the block output, a new (m, n) bf16 tensor unless given)."""
    m, k = x.shape
    n = w.shape[0]
    if h is None:
        h = torch.empty((m, n), dtype=x.dtype, device=x.device)
    nbytes = linear_add_norm_counter_bytes(m)
    cnt = counter_buffer(x.device, _stream(x), nbytes)
    rc = _lib.load().vm_linear_add_norm_fwd(
        _p(x), x.stride(0), _p(w), w.stride(0), _p(h), h.stride(0), _p(residual),
        residual.stride(0), _p(norm_w32), float(eps), _p(hn), hn.stride(0), m, n, k, _p(cnt),
        cnt.numel(), _stream(x))
    _lib.check(rc, "vm_linear_add_norm_fwd")
    return h


POOL_MODES = {"avg": 0, "cls+avg": 1, "cls_cat_avg": 2, "cls": 3}


def norm_pool_workspace_bytes(batch: int, groups: int, max_group_rows: int, cols: int) -> int:
    return int(_lib.load().vm_norm_pool_workspace_bytes(batch, groups, max_group_rows, cols))


def norm_pool(h: Tensor, residual: Optional[Tensor], rows: int, w32: Tensor,
              b32: Optional[Tensor], eps: float, is_rms: bool, *, head: int, groups: int,
              group_rows: int = 0, bounds: Optional[Tensor] = None, max_group_rows: int = 0,
              sums: bool = False, out: Optional[Tensor] = None,
              rev_frame: int = 0) -> Tuple[Tensor, Optional[Tensor]]:
    """Final add + norm of rows [0, rows) of the padded (B, Lp, C) ``h`` (+ ``residual``)
    into a contiguous (B, rows, C) tensor; with ``sums`` also the per-group fp32 column
    sums for :func:`pool_finish` (returned workspace, valid until the next scratch user
    on this stream).  Groups: ``groups`` x ``group_rows`` rows after ``head`` rows, or
    int32 ``bounds`` (B, groups+1).  ``out`` may be a (B, >= rows, C) buffer with contiguous
    rows; ``rev_frame`` > 0 reads the grouped rows in reversed frame order."""
    Bsz, Lp, C = h.shape
    if out is None:
        out = torch.empty((Bsz, rows, C), dtype=h.dtype, device=h.device)
    if bounds is None:
        max_group_rows = group_rows
    ws, nbytes = None, 0
    if sums:
        nbytes = norm_pool_workspace_bytes(Bsz, groups, max_group_rows, C)
        ws = scratch(h.device, _stream(h), nbytes)
    if residual is not None and residual.stride() != h.stride():
        raise ValueError("residual must share h's padded layout")
    rc = _lib.load().vm_norm_pool_fwd(
        _p(h), dtype_code(h.dtype), _p(residual),
        dtype_code(residual.dtype) if residual is not None else 0, h.stride(0),
        _p(w32), _p(b32), float(eps), int(is_rms), _p(out), dtype_code(out.dtype),
        out.stride(0), Bsz, rows, C, head, groups, group_rows, _p(bounds), max_group_rows,
        int(rev_frame), _p(ws), nbytes, _stream(h))
    _lib.check(rc, "vm_norm_pool_fwd")
    return out, ws


def pool_finish(ws: Optional[Tensor], feats: Tensor, *, mode: str, keep_temporal: bool,
                groups: int, group_rows: int = 0, bounds: Optional[Tensor] = None,
                max_group_rows: int = 0, has_cls: bool, lnw32: Optional[Tensor],
                lnb32: Optional[Tensor], ln_eps: float) -> Tensor:
    """Pool tail over :func:`norm_pool`'s sums: means (per group with ``keep_temporal``),
    the CLS add / concat of ``mode`` (CLS = row 0 of ``feats``) and the pool LayerNorm."""
    Bsz, _, C = feats.shape
    if bounds is None:
        max_group_rows = group_rows
    navg = groups if keep_temporal else 1
    prow = {"cls": 1, "cls_cat_avg": 1 + navg}.get(mode, navg)
    x_pool = torch.empty((Bsz, prow, C), dtype=feats.dtype, device=feats.device)
    rc = _lib.load().vm_pool_finish_fwd(
        _p(ws), Bsz, groups, group_rows, _p(bounds), max(1, max_group_rows),
        _p(feats) if has_cls else None, dtype_code(feats.dtype), feats.stride(0),
        POOL_MODES[mode], int(keep_temporal), _p(lnw32), _p(lnb32), float(ln_eps),
        _p(x_pool), dtype_code(x_pool.dtype), C, _stream(feats))
    _lib.check(rc, "vm_pool_finish_fwd")
    return x_pool


# --------------------------------------------------------------------------- selective scan
def selective_scan_fn(u: Tensor, delta: Tensor, A: Tensor, B: Tensor, C: Tensor,
                      D: Optional[Tensor] = None, z: Optional[Tensor] = None,
                      delta_bias: Optional[Tensor] = None, delta_softplus: bool = False,
                      return_last_state: bool = False, initial_state: Optional[Tensor] = None,
                      *, last_state_out: Optional[Tensor] = None):
    """mamba-ssm ``selective_scan_fn`` with the ``initial_state`` extension the reference
    probes for (``mamba_simple.py:17-22``, ``:138-152``).

    u, delta, z: (b, d, l); A: (d, n) real; B, C: (b, n, l) (input-dependent); D,
    delta_bias: (d,).  Returns ``out`` (u.dtype) or ``(out, last_state)``; last_state is a
    new fp32 (b, d, n) tensor unless ``last_state_out`` is given, in which case it is
    written there (in its dtype; may be ``initial_state`` itself) and returned.
    """
    require_gpu(u, delta, A, B, C, D, z, delta_bias, initial_state, what="selective_scan_fn")
    if A.is_complex():
        raise NotImplementedError("complex A is not supported")
    if B.dim() != 3 or C.dim() != 3:
        raise NotImplementedError("selective_scan_fn supports input-dependent B/C of shape "
                                  "(batch, dstate, seqlen) only (the reference's usage)")
    batch, dim, seqlen = u.shape
    dstate = A.shape[1]
    dt = dtype_code(u.dtype)
    if seqlen == 0 or batch == 0 or dim == 0:  # nothing to scan: the state passes through
        out = u.new_empty((batch, dim, seqlen))
        if not return_last_state:
            return out
        h = (initial_state.float() if initial_state is not None else
             torch.zeros((batch, dim, dstate), dtype=torch.float32, device=u.device))
        if last_state_out is not None:
            last_state_out.copy_(h)
            h = last_state_out
        return out, h
    # Layout follows u: token-major views (unit channel stride, e.g. a transposed
    # (b, l, d) tensor) take the channel-per-lane kernels, anything else is made
    # step-contiguous for the time-parallel kernels.
    tm = dim > 1 and u.stride(1) == 1
    conv = _channel_contig if tm else _lastdim_contig
    u = conv(u)
    delta = conv(delta.to(u.dtype))
    z = conv(None if z is None else z.to(u.dtype))
    B = B.to(u.dtype)
    C = C.to(u.dtype)
    if not tm:
        B = _lastdim_contig(B)
        C = _lastdim_contig(C)
    if tm:
        out = torch.empty((batch, seqlen, dim), dtype=u.dtype, device=u.device).transpose(1, 2)
    else:
        out = torch.empty((batch, dim, seqlen), dtype=u.dtype, device=u.device)
    h0 = None
    if initial_state is not None:
        h0 = _lastdim_contig(initial_state)
    hl = None
    if return_last_state:
        hl = last_state_out if last_state_out is not None else torch.empty(
            (batch, dim, dstate), dtype=torch.float32, device=u.device)
        if hl.stride(-1) != 1:
            raise ValueError("last_state_out must have unit stride on the state axis")
    s3 = lambda t: (t.stride(0), t.stride(1), t.stride(2))  # noqa: E731
    scan_raw(u, s3(u), delta, s3(delta), f32c(A), B, s3(B), C, s3(C),
             f32c(D), z, s3(z) if z is not None else (0, 0, 0),
             f32c(delta_bias), delta_softplus,
             h0, (h0.stride(0), h0.stride(1)) if h0 is not None else (0, 0),
             hl, (hl.stride(0), hl.stride(1)) if hl is not None else (0, 0),
             out, s3(out), seqlen, batch, dim, seqlen, dstate, dt, _stream(u))
    return (out, hl) if return_last_state else out


def selective_state_update(state: Tensor, x: Tensor, dt: Tensor, A: Tensor, B: Tensor,
                           C: Tensor, D: Optional[Tensor] = None, z: Optional[Tensor] = None,
                           dt_bias: Optional[Tensor] = None, dt_softplus: bool = False) -> Tensor:
    """One-token scan step; ``state`` (b, d, n) updated in place (its dtype).  x, dt, z:
    (b, d); B, C: (b, n).  Returns out (b, d) in x.dtype."""
    require_gpu(state, x, dt, A, B, C, D, z, dt_bias, what="selective_state_update")
    batch, dim = x.shape
    dstate = A.shape[1]
    if state.stride(-1) != 1:
        raise ValueError("state must have unit stride on the state axis")
    x = _lastdim_contig(x)
    dt_ = _lastdim_contig(dt.to(x.dtype))
    B = _lastdim_contig(B.to(x.dtype))
    C = _lastdim_contig(C.to(x.dtype))
    z = _lastdim_contig(None if z is None else z.to(x.dtype))
    out = torch.empty((batch, dim), dtype=x.dtype, device=x.device)
    lib = _lib.load()
    rc = lib.vm_selective_state_update(
        _p(state), dtype_code(state.dtype), state.stride(0), state.stride(1),
        _p(x), x.stride(0), _p(dt_), dt_.stride(0), _p(f32c(A)), _p(B), B.stride(0),
        _p(C), C.stride(0), _p(f32c(D)), _p(z), z.stride(0) if z is not None else 0,
        _p(f32c(dt_bias)), int(dt_softplus), _p(out), out.stride(0),
        batch, dim, dstate, dtype_code(x.dtype), _stream(x))
    _lib.check(rc, "vm_selective_state_update")
    return out


# --------------------------------------------------------------------------- causal conv1d
def causal_conv1d_fn(x: Tensor, weight: Tensor, bias: Optional[Tensor] = None,
                     activation: Optional[str] = None, *, conv_state: Optional[Tensor] = None,
                     return_conv_state: bool = False):
    """causal-conv1d ``causal_conv1d_fn(x, weight, bias, activation)``; x: (b, d, l),
    weight: (d, w).  With ``conv_state`` (b, d, w) the conv runs over
    ``cat([conv_state, x])`` and keeps the last l outputs (``mamba_simple.py:382-390``).
    ``return_conv_state`` also returns the last w raw inputs (new tensor)."""
    require_gpu(x, weight, bias, conv_state, what="causal_conv1d_fn")
    if activation not in (None, "silu", "swish"):
        raise NotImplementedError(f"activation {activation!r}")
    if weight.dim() == 3:
        weight = weight.reshape(weight.shape[0], weight.shape[-1])
    batch, dim, seqlen = x.shape
    width = weight.shape[1]
    tm = dim > 1 and x.stride(1) == 1  # token-major view: keep the layout
    if tm:
        out = torch.empty((batch, seqlen, dim), dtype=x.dtype, device=x.device).transpose(1, 2)
    else:
        x = _lastdim_contig(x)
        out = torch.empty((batch, dim, seqlen), dtype=x.dtype, device=x.device)
    cs_in = _lastdim_contig(conv_state)
    cs_out = None
    if return_conv_state:
        cs_dtype = conv_state.dtype if conv_state is not None else x.dtype
        cs_out = torch.empty((batch, dim, width), dtype=cs_dtype, device=x.device)
    conv_raw(x, (x.stride(0), x.stride(1), x.stride(2)), f32c(weight), f32c(bias),
             cs_in, (cs_in.stride(0), cs_in.stride(1)) if cs_in is not None else (0, 0),
             cs_out, (cs_out.stride(0), cs_out.stride(1)) if cs_out is not None else (0, 0),
             out, (out.stride(0), out.stride(1), out.stride(2)), seqlen, batch, dim, seqlen, width,
             activation is not None, dtype_code(x.dtype), _stream(x))
    return (out, cs_out) if return_conv_state else out


def causal_conv1d_update(x: Tensor, conv_state: Tensor, weight: Tensor,
                         bias: Optional[Tensor] = None, activation: Optional[str] = None) -> Tensor:
    """causal-conv1d ``causal_conv1d_update`` for one token: x (b, d); ``conv_state``
    (b, d, w) is shifted in place."""
    require_gpu(x, conv_state, weight, bias, what="causal_conv1d_update")
    if weight.dim() == 3:
        weight = weight.reshape(weight.shape[0], weight.shape[-1])
    batch, dim = x.shape
    width = weight.shape[1]
    if conv_state.stride(-1) != 1:
        raise ValueError("conv_state must have unit stride on the width axis")
    x = _lastdim_contig(x)
    out = torch.empty((batch, dim), dtype=x.dtype, device=x.device)
    lib = _lib.load()
    rc = lib.vm_causal_conv1d_update(
        _p(x), x.stride(0), _p(conv_state), dtype_code(conv_state.dtype), conv_state.stride(0),
        conv_state.stride(1), _p(f32c(weight)), _p(f32c(bias)), _p(out), out.stride(0),
        batch, dim, width, int(activation in ("silu", "swish")), dtype_code(x.dtype), _stream(x))
    _lib.check(rc, "vm_causal_conv1d_update")
    return out


# --------------------------------------------------------------------------- norms
def _norm(x, weight, bias, residual, prenorm, residual_in_fp32, eps, is_rms, out=None,
          residual_out=None, owner=None):
    require_gpu(x, weight, bias, residual, what="rms_norm_fn/layer_norm_fn")
    shape = x.shape
    cols = shape[-1]
    x2 = x.reshape(-1, cols)
    if not x2.is_contiguous():
        x2 = x2.contiguous()
    r2 = None
    if residual is not None:
        r2 = residual.reshape(-1, cols)
        if not r2.is_contiguous():
            r2 = r2.contiguous()
    rows = x2.shape[0]
    y = out if out is not None else torch.empty(shape, dtype=x.dtype, device=x.device)
    ro = None
    if prenorm:
        if residual_out is not None:
            ro = residual_out
        else:
            rdt = residual.dtype if residual is not None else (
                torch.float32 if residual_in_fp32 else x.dtype)
            ro = torch.empty(shape, dtype=rdt, device=x.device)
    if owner is not None:
        w32, b32 = f32_cached(owner, weight, "w"), f32_cached(owner, bias, "b")
    else:
        w32, b32 = f32c(weight), f32c(bias)
    add_norm_raw(x2, r2, w32, b32, y, ro, rows, cols, eps, is_rms, _stream(x))
    return (y, ro) if prenorm else y


def rms_norm_fn(x: Tensor, weight: Tensor, bias: Optional[Tensor], residual: Optional[Tensor] = None,
                prenorm: bool = False, residual_in_fp32: bool = False, eps: float = 1e-6, **_):
    """mamba-ssm ``rms_norm_fn``: returns y, or (y, residual_out) with ``prenorm``."""
    return _norm(x, weight, bias, residual, prenorm, residual_in_fp32, eps, True)


def layer_norm_fn(x: Tensor, weight: Tensor, bias: Optional[Tensor], residual: Optional[Tensor] = None,
                  prenorm: bool = False, residual_in_fp32: bool = False, eps: float = 1e-6,
                  is_rms_norm: bool = False, **_):
    """mamba-ssm ``layer_norm_fn`` (LayerNorm unless ``is_rms_norm``)."""
    return _norm(x, weight, bias, residual, prenorm, residual_in_fp32, eps, is_rms_norm)


# --------------------------------------------------------------------------- patch embed
def patch_embed(video: Tensor, weight: Tensor, bias: Tensor, spos: Tensor, tpos: Tensor,
                out: Tensor, row0: int, out_batch_stride: int, cls: Optional[Tensor] = None,
                cls_pos: Optional[Tensor] = None, pad_rows: int = 0,
                bias32: Optional[Tensor] = None) -> None:
    """Conv3d tubelet embed + bias + spatial/temporal positional adds, written as token
    rows into ``out`` (token j of batch b at ``out[b*out_batch_stride + (row0+j)*C]``).
    ``cls`` / ``cls_pos`` (C values each): rows [0, row0) of every batch = cls + cls_pos in
    the model dtype; ``pad_rows`` zero rows after the tokens (ABI v12, same launch).
    ``bias32``: the bias already in fp32 (a cached copy), else converted here."""
    require_gpu(video, weight, bias, spos, tpos, out, what="patch_embed")
    Bsz, cin, T, H, W = video.shape
    C, _, kt, Ph, Pw = weight.shape
    dt = dtype_code(weight.dtype)
    video = video.to(weight.dtype).contiguous()
    if (cls is None) != (cls_pos is None):
        raise ValueError("patch_embed: pass cls and cls_pos together")
    if cls is not None:
        cls = cls.reshape(-1).to(weight.dtype).contiguous()
        cls_pos = cls_pos.reshape(-1).to(weight.dtype).contiguous()
        if cls.numel() != C or cls_pos.numel() != C:
            raise ValueError(f"patch_embed: cls / cls_pos need {C} values")
    lib = _lib.load()
    rc = lib.vm_patch_embed_fwd(
        _p(video), _p(weight.contiguous()), _p(bias32 if bias32 is not None else f32c(bias)),
        _p(spos.to(weight.dtype).contiguous()),
        _p(tpos.to(weight.dtype).contiguous()), _p(out), out_batch_stride, row0,
        Bsz, cin, T, H, W, kt, Ph, Pw, C, dt, _p(cls), _p(cls_pos), int(pad_rows),
        _stream(video))
    _lib.check(rc, "vm_patch_embed_fwd")
