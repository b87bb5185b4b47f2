"""Mamba mixer on the HIP kernels (``models/videomamba/mamba_simple.py:175-590`` surface).

Construction, parameter names / shapes and initialisation follow the reference exactly
(so state_dicts interchange and a seeded build gives the same weights).  The forward
replaces the reference's kernel calls with this package's HIP kernels and a layout
chosen for them:

    hn (B, Lp, C) token-major, Lp = round_up(L, 8), rows >= L zero
    xz = W_in @ hn^T            -> (2D, B*Lp)   channel-major, batch-interleaved rows
    u  = silu(conv1d(x [+ conv_state]))  HIP  (D, B*Lp), padded columns written 0
    x_dbl = W_x @ u             -> (R+2N, B*Lp) (dt_low, B, C rows)
    dt = W_dt @ dt_low          -> (D, B*Lp)
    y  = selective_scan(u, dt, A, B, C, D, z, dt_bias, softplus)  HIP, fp32 state
    out = y^T @ W_out^T         -> (B*Lp, C)

For batches that fill the chip (>= ~1.25 channel-group waves per SIMD) the mixer runs
token-major instead — every buffer (B*Lp, channels), every projection a plain
``F.linear`` — so the scan can take the channel-per-lane kernel (vm_scan_seq.hip):

    xz = hn @ W_in^T (B*Lp, 2D);  u = conv(x) (B*Lp, D);  x_dbl = u @ W_x^T (B*Lp, R+2N)
    dt = x_dbl[:, :R] @ W_dt^T (B*Lp, D);  y = scan(...) (B*Lp, D);  out = y @ W_out^T

Rounding points match the reference slow path (xz, u, x_dbl, dt, y, out in the model
dtype).  The GEMMs are plain library GEMMs (hipBLASLt via torch.matmul) on this layout;
no transpose copies are materialised.  The scan runs once per chunk — never per token —
and keeps the state in fp32 internally.  State semantics:

* ``state=(conv, ssm), return_state=True``: conv over ``[conv_state | x]``; the new
  conv state is a fresh tensor (last d_conv raw inputs); the ssm state is updated in
  place and returned (the reference's fallback aliases it the same way).
* ``ssm_state=t`` alone (legacy): conv restarts from zeros, ``t`` updated in place.
* ``inference_params``: prefill (offset 0) fills the cache; offset > 0 runs ``step``.
"""

from __future__ import annotations

import contextlib
import math
import os
from typing import Any, List, MutableMapping, Optional, Protocol, Tuple, Union

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch import Tensor

from . import kernels as K
from . import options
from . import phase_lock as _phase
from .gemm_tuning import tuned
from .layers import round_up, warn_if_grad

_SMALL_GEMM_K = (192, 384, 576, 768, 1152, 1536)  # vm_linear_fwd's unrolled K-step counts


def _small_gemm_ok(x: Tensor, w: Tensor, b: Optional[Tensor], out: Optional[Tensor] = None,
                   clips: Optional[int] = None) -> bool:
    """Whether a bf16 projection runs on the HIP GEMM (vm_linear_fwd) instead of the library.

    ``options.projection_gemm == "hip"`` (default): whenever the HIP GEMM takes the shape
    (bf16, no bias, K in its unrolled set, 16-byte rows; x past 2 GB only on the persistent
    form, n a multiple of 192 or 256).  Its two kernel forms compute every output element as
    the same MFMA chain in K order, so a row's bits never depend on the row count: a chunked
    stream equals the one-pass forward at every batch (C4 at 72 clips was 1.4e-4 on the
    library GEMM, whose kernel choice depends on M), and at the bench batch the persistent
    form outruns the library.
    ``"library"``: the round-3 rule — the HIP GEMM for mixers of at most
    ``row_invariant_gemm_clips`` clips (C5, 16 x 64-frame chunks vs one 1,024-frame pass:
    6.2e-4 relative on the library, 0.0 here; scripts/diag/c5_invariance.py) and for one
    clip's narrow projections; hipBLASLt otherwise."""
    o = options.get()
    ok16 = lambda t: t.data_ptr() % 16 == 0 and t.stride(0) % 8 == 0 and t.stride(1) == 1  # noqa: E731
    if not (x.shape[0] > 0 and b is None and x.dtype == torch.bfloat16
            and w.dtype == torch.bfloat16 and x.is_cuda and x.shape[1] in _SMALL_GEMM_K
            and w.shape[0] % 8 == 0 and ok16(x) and ok16(w) and (out is None or ok16(out))):
        return False
    small_x = x.shape[0] * x.stride(0) * 2 < (1 << 31)
    if o.projection_gemm == "hip":
        return small_x or w.shape[0] % 192 == 0 or w.shape[0] % 256 == 0
    if not small_x:
        return False
    if clips is not None and 0 < clips <= o.row_invariant_gemm_clips:
        return True
    return x.shape[0] <= o.small_gemm_rows and w.shape[0] <= o.small_gemm_max_n


def _linear(x: Tensor, w: Tensor, b: Optional[Tensor] = None,
            clips: Optional[int] = None) -> Tensor:
    """A projection GEMM of the mixer: the HIP GEMM where :func:`_small_gemm_ok` says so,
    else the library GEMM with the shipped tuning results."""
    if _small_gemm_ok(x, w, b, clips=clips):
        return K.linear(x, w)
    with tuned():
        return F.linear(x, w, b)


def _linear_into(x: Tensor, w: Tensor, b: Optional[Tensor], out: Tensor,
                 clips: Optional[int] = None) -> Tensor:
    """:func:`_linear` into a preallocated buffer with unit column stride (a half of the
    bidirectional refiner's paired buffers)."""
    if _small_gemm_ok(x, w, b, out, clips=clips):
        return K.linear(x, w, out=out)
    with tuned():
        if b is None:
            return torch.mm(x, w.t(), out=out)
        return torch.addmm(b.to(out.dtype), x, w.t(), out=out)


_Z_STREAMS = {}

# Measurement hook (bench.py's roofline.in_step): while a list is installed here, every
# token-major scan launch is bracketed by two timing events on its own launch stream, so the
# scan's duration inside a real step (beside the other sub-batch stream's kernels) can be
# read without a profiler.  None (the default) records nothing.
_SCAN_EVENTS: List[Optional[list]] = [None]


@contextlib.contextmanager
def scan_event_log():
    """Collect (start, end, batch) timing events around every token-major scan launch in
    the block, from every issuing thread (list.append is atomic)."""
    log: list = []
    prev, _SCAN_EVENTS[0] = _SCAN_EVENTS[0], log
    try:
        yield log
    finally:
        _SCAN_EVENTS[0] = prev


def _scan_event(log: Optional[list]):
    if log is None:
        return None
    e = torch.cuda.Event(enable_timing=True)
    e.record()
    return e


def _z_stream(device: torch.device) -> torch.cuda.Stream:
    """The side stream the small-batch mixer runs in_proj's z half on (one per device)."""
    key = (device.type, device.index)
    s = _Z_STREAMS.get(key)
    if s is None:
        s = _Z_STREAMS[key] = torch.cuda.Stream(device)
    return s


def _matmul(a: Tensor, b: Tensor) -> Tensor:
    with tuned():
        return torch.matmul(a, b)


_CUDA_ERROR = ("VideoMamba requires CUDA tensors in this package because its HIP "
               "kernels (libvideomamba_hip, gfx950) are GPU-only.")


def mixer_layout(batch: int, d_inner: int, device: torch.device) -> str:
    """"tm" (token-major: every buffer (B*Lp, channels), channel-per-lane scan; time-
    segmented two-pass form below a chip-filling batch) at every batch size; "cm"
    (channel-major buffers, time-parallel scan) only when ``options.mixer_layout`` asks.
    Token-major runs every token with arithmetic that does not depend on the sequence
    length, so chunked streaming matches the full sequence within the north star's 1e-4 at
    every batch (the channel-major time-parallel scan missed it at M-32f B=1: 1.1e-4,
    scripts/diag/chunk_invariance.py); at B=1 it costs ~0.2 ms of chunk latency against the
    channel-major path with library x_proj / dt_proj GEMMs (scripts/diag/b1_layouts.py)."""
    forced = options.get().mixer_layout
    if forced != "auto":
        return forced
    return "tm"


class InferenceParamsLike(Protocol):
    seqlen_offset: int
    key_value_memory_dict: MutableMapping[int, Tuple[Tensor, Tensor]]


class Mamba(nn.Module):
    def __init__(self, d_model: int, d_state: int = 16, d_conv: int = 4, expand: int = 2,
                 dt_rank: Union[int, str] = "auto", dt_min: float = 0.001,
                 dt_max: float = 0.1, dt_init: str = "random", dt_scale: float = 1.0,
                 dt_init_floor: float = 1e-4, conv_bias: bool = True, bias: bool = False,
                 use_fast_path: bool = True, layer_idx: Optional[int] = None,
                 bimamba: bool = True, device=None, dtype=None, **_: Any):
        fk = {k: v for k, v in (("device", device), ("dtype", dtype)) if v is not None}
        super().__init__()
        self.d_model = d_model
        self.d_state = d_state
        self.d_conv = d_conv
        self.expand = expand
        self.d_inner = int(expand * d_model)
        self.dt_rank = math.ceil(d_model / 16) if dt_rank == "auto" else int(dt_rank)
        self.bimamba = bool(bimamba)  # API compatibility; the mixer scans one direction
        if os.getenv("VIDEOMAMBA_DISABLE_FUSED", "").lower() in {"1", "true", "yes", "y", "on"}:
            use_fast_path = False
        # Both settings run the same fused HIP path; the flag is kept for API parity.
        self.use_fast_path = use_fast_path
        self.layer_idx = layer_idx

        self.in_proj = nn.Linear(d_model, self.d_inner * 2, bias=bias, **fk)
        self.conv1d = nn.Conv1d(self.d_inner, self.d_inner, kernel_size=d_conv,
                                groups=self.d_inner, padding=d_conv - 1, bias=conv_bias, **fk)
        self.activation = "silu"
        self.act = nn.SiLU()
        self.x_proj = nn.Linear(self.d_inner, self.dt_rank + 2 * d_state, bias=False, **fk)
        self.dt_proj = nn.Linear(self.dt_rank, self.d_inner, bias=True, **fk)

        # dt_proj init: variance-preserving weights; bias = softplus^-1(U[dt_min, dt_max])
        std = self.dt_rank ** -0.5 * dt_scale
        if dt_init == "constant":
            nn.init.constant_(self.dt_proj.weight, std)
        elif dt_init == "random":
            nn.init.uniform_(self.dt_proj.weight, -std, std)
        else:
            raise NotImplementedError
        dt = torch.exp(torch.rand(self.d_inner, **fk) * (math.log(dt_max) - math.log(dt_min))
                       + math.log(dt_min)).clamp(min=dt_init_floor)
        with torch.no_grad():
            self.dt_proj.bias.copy_(dt + torch.log(-torch.expm1(-dt)))
        self.dt_proj.bias._no_reinit = True

        # S4D-real A, kept as log in fp32; D skip in fp32
        a = torch.arange(1, d_state + 1, dtype=torch.float32, device=device)
        self.A_log = nn.Parameter(torch.log(a).unsqueeze(0).repeat(self.d_inner, 1).contiguous())
        self.A_log._no_weight_decay = True
        self.D = nn.Parameter(torch.ones(self.d_inner, device=device))
        self.D._no_weight_decay = True
        self.out_proj = nn.Linear(self.d_inner, d_model, bias=bias, **fk)
        self._pcache_key = None
        self._pcache = None

    # ------------------------------------------------------------------ params (fp32)
    def _fp32_params(self):
        """A = -exp(A_log), D, dt bias, conv weight/bias as fp32 contiguous (cached per
        parameter version so bf16 models convert once, not per call)."""
        srcs = (self.A_log, self.D, self.dt_proj.bias, self.conv1d.weight, self.conv1d.bias)
        key = tuple(None if p is None else (p.data_ptr(), p._version, p.dtype, p.device)
                    for p in srcs)
        if key != self._pcache_key:
            with torch.no_grad():
                A = (-torch.exp(self.A_log.float())).contiguous()
                Dv = K.f32c(self.D)
                bias = K.f32c(self.dt_proj.bias)
                w = K.f32c(self.conv1d.weight.reshape(self.d_inner, self.d_conv))
                cb = K.f32c(self.conv1d.bias)
            self._pcache = (A, Dv, bias, w, cb)
            self._pcache_key = key
        return self._pcache

    def _padded_proj_weights(self):
        """x_proj / dt_proj weights zero-padded for the fused conv_proj kernel:
        W_x -> (round_up(R+2N, 16), D), W_dt -> (D, 32 or 64); cached per version."""
        srcs = (self.x_proj.weight, self.dt_proj.weight)
        key = tuple((p.data_ptr(), p._version, p.dtype, p.device) for p in srcs)
        if key != getattr(self, "_wpad_key", None):
            with torch.no_grad():
                wx, wdt = self.x_proj.weight, self.dt_proj.weight
                e, r = wx.shape[0], wdt.shape[1]
                wx_pad = wx.new_zeros(((e + 15) // 16 * 16, wx.shape[1]))
                wx_pad[:e] = wx
                wdt_pad = wdt.new_zeros((wdt.shape[0], 32 if r <= 32 else 64))
                wdt_pad[:, :r] = wdt
            self._wpad = (wx_pad.contiguous(), wdt_pad.contiguous())
            self._wpad_key = key
        return self._wpad

    def _fused_conv_proj_ok(self, hn: Tensor, seqlen: int, conv_state_in: Optional[Tensor] = None,
                            tm: bool = True) -> bool:
        """The fused conv + x_proj (+ dt_proj) kernel applies: bf16, its shape limits and,
        token-major (``tm``), buffer extents its 31-bit offsets cover (vm_conv_proj_fits: a
        very long sequence at batch > 8 takes the unfused conv + projection path)."""
        E = self.dt_rank + 2 * self.d_state
        if not (hn.dtype == torch.bfloat16 and seqlen >= 1 and self.d_inner % 64 == 0
                and self.d_conv <= 4 and E <= 128 and self.dt_rank <= 64
                and self.x_proj.bias is None and self.dt_proj.weight.dtype == torch.bfloat16
                and options.get().fused_conv_proj):
            return False
        if not tm:
            return True
        Bsz, Lp = hn.shape[0], hn.shape[1]
        Dm = self.d_inner
        return K.conv_proj_fits(Bsz, Lp, seqlen, Dm, E, 32 if self.dt_rank <= 32 else 64,
                                (Lp * 2 * Dm, 2 * Dm), Dm, conv_state_in, self.d_conv)

    # ------------------------------------------------------------------ core
    def _forward_padded(self, hn: Tensor, seqlen: int, *, conv_state_in: Optional[Tensor] = None,
                        conv_state_out: Optional[Tensor] = None, h0: Optional[Tensor] = None,
                        h_last: Optional[Tensor] = None, next_norm=None) -> Tensor:
        """hn: (B, Lp, C) contiguous, rows >= seqlen zero.  Returns (B, Lp, C) with rows
        >= seqlen zero.  States are read/written by the kernels (see module doc).
        ``next_norm`` (videomamba.NextNorm): fuse the next block's add + RMSNorm into
        out_proj when it runs on the HIP GEMM (sets ``next_norm.done``)."""
        if mixer_layout(hn.shape[0], self.d_inner, hn.device) == "tm":
            return self._forward_padded_tm(hn, seqlen, conv_state_in, conv_state_out, h0, h_last,
                                           next_norm)
        Bsz, Lp, C = hn.shape
        Dm, N, R, W = self.d_inner, self.d_state, self.dt_rank, self.d_conv
        n = Bsz * Lp
        dt_code = K.dtype_code(hn.dtype)
        stream = torch.cuda.current_stream(hn.device).cuda_stream
        A, Dv, dbias, cw, cb = self._fp32_params()
        rows = (Lp, n)  # (batch stride, channel stride) of a (ch, B*Lp) buffer
        rows3 = (Lp, n, 1)  # + step stride

        xz = _matmul(self.in_proj.weight, hn.view(n, C).t())  # (2D, B*Lp)
        if self.in_proj.bias is not None:
            xz += self.in_proj.bias.to(xz.dtype)[:, None]
        x, z = xz[:Dm], xz[Dm:]
        u = torch.empty((Dm, n), dtype=hn.dtype, device=hn.device)
        csi_s = ((conv_state_in.stride(0), conv_state_in.stride(1))
                 if conv_state_in is not None else (0, 0))
        cso_s = ((conv_state_out.stride(0), conv_state_out.stride(1))
                 if conv_state_out is not None else (0, 0))
        if self._fused_conv_proj_ok(hn, seqlen, tm=False):
            # conv + silu -> x_proj -> dt_proj with a fixed reduction order
            # (vm_conv_proj_cm.hip): faster than the latency-bound library GEMMs at small
            # batch, and chunk-invariant (every token's bits independent of L)
            wx_pad, wdt_pad = self._padded_proj_weights()
            E = R + 2 * N
            x_dbl = torch.empty((E, n), dtype=hn.dtype, device=hn.device)
            dt = torch.empty((Dm, n), dtype=hn.dtype, device=hn.device)
            K.conv_proj_cm_raw(xz, n, cw, cb, conv_state_in, csi_s, conv_state_out, cso_s,
                               wx_pad, E, wdt_pad, R, u, n, x_dbl, n, dt, n, Lp, Bsz, Dm,
                               seqlen, W, stream)
        else:
            K.conv_raw(x, rows3, cw, cb, conv_state_in, csi_s, conv_state_out, cso_s,
                       u, rows3, Lp, Bsz, Dm, seqlen, W, True, dt_code, stream)
            x_dbl = _matmul(self.x_proj.weight, u)  # (R+2N, B*Lp)
            dt = _matmul(self.dt_proj.weight, x_dbl[:R])  # (D, B*Lp), bias added in scan
        y = torch.empty_like(u)
        K.scan_raw(u, rows3, dt, rows3, A, x_dbl[R:R + N], rows3, x_dbl[R + N:], rows3, Dv,
                   z, rows3, dbias, True,
                   h0, (h0.stride(0), h0.stride(1)) if h0 is not None else (0, 0),
                   h_last, (h_last.stride(0), h_last.stride(1)) if h_last is not None else (0, 0),
                   y, rows3, Lp, Bsz, Dm, seqlen, N, dt_code, stream)
        out = _matmul(y.t(), self.out_proj.weight.t())  # (B*Lp, C)
        if self.out_proj.bias is not None:
            out += self.out_proj.bias.to(out.dtype)
        return out.view(Bsz, Lp, C)

    def _dtp_ok(self, hn: Tensor, seqlen: int, conv_state_in: Optional[Tensor] = None) -> bool:
        """Fold dt_proj into the scan (vm_selective_scan_dtproj_fwd, conv_proj then writes no
        dt rows): bf16 fused conv_proj path, 16 states, dt_rank a multiple of 4, and
          * a segmented scan (streaming batches) of at most 64 steps per segment whose grid
            fits the chip at one workgroup per CU (K.scan_dtproj_segmented_pays; "on": any
            grid): each segment
            computes its dt exactly as conv_proj's dt_proj would (ABI v11), so the bits are the
            ones conv_proj writes otherwise — the choice never changes a result, and chunked
            == full stays exact whichever form a chunk length selects; or
          * the single-pass scan (D % 128 == 0) above the split-K batch (> 8 clips; "on":
            at any batch), whose 16-step MFMA dt blocks are its own arithmetic — below 9
            clips a short sequence's single pass keeps conv_proj's dt for the same
            invariance."""
        mode = options.get().scan_dt_proj
        Bsz = hn.shape[0]
        if mode == "off":
            return False
        if not (self._fused_conv_proj_ok(hn, seqlen, conv_state_in) and self.d_state == 16
                and self.dt_rank <= 64 and self.dt_rank % 4 == 0):
            return False
        steps = K.scan_chunk_steps(Bsz, self.d_inner, seqlen, self.d_state)
        if steps > 0:
            if mode == "on":
                return steps <= K.SCAN_DTPROJ_MAX_SEGMENT
            return K.scan_dtproj_segmented_pays(Bsz, self.d_inner, seqlen, self.d_state,
                                                hn.device)
        if mode == "auto" and Bsz <= 8:
            return False
        return self.d_inner % 128 == 0

    def _tm_front(self, hn, seqlen, conv_state_in, conv_state_out, bufs=None, want_dt=True):
        """in_proj -> conv + silu -> x_proj -> dt_proj of the token-major form: (xz, u,
        x_dbl, dt), each (B*Lp, channels).  ``bufs`` = preallocated (xz, u, x_dbl, dt) (the
        refiner's paired buffers); otherwise they are allocated here.  ``want_dt=False``
        (fused conv_proj only) skips dt_proj: dt is None, the scan computes it."""
        Bsz, Lp, C = hn.shape
        Dm, N, R, W = self.d_inner, self.d_state, self.dt_rank, self.d_conv
        n = Bsz * Lp
        E = R + 2 * N
        dt_code = K.dtype_code(hn.dtype)
        stream = torch.cuda.current_stream(hn.device).cuda_stream
        _, _, _, cw, cb = self._fp32_params()
        s_u, s_xz = (Lp * Dm, 1, Dm), (Lp * 2 * Dm, 1, 2 * Dm)
        z_side = None
        if bufs is None and self._in_proj_conv_ok(hn, seqlen, want_dt):
            # in_proj with the conv + SiLU and the x_proj split partials in its epilogue
            # (vm_in_proj_conv_proj_fwd): x stays in the GEMM's LDS tiles; bit-identical to
            # the in_proj + conv_proj pair below
            wx_pad, wdt_pad = self._padded_proj_weights()
            xz = torch.empty((n, 2 * Dm), dtype=hn.dtype, device=hn.device)  # z half written
            u = torch.empty((n, Dm), dtype=hn.dtype, device=hn.device)
            x_dbl = torch.empty((n, E), dtype=hn.dtype, device=hn.device)
            dt = torch.empty((n, Dm), dtype=hn.dtype, device=hn.device) if want_dt else None
            csi_s = ((conv_state_in.stride(0), conv_state_in.stride(1))
                     if conv_state_in is not None else (0, 0))
            cso_s = ((conv_state_out.stride(0), conv_state_out.stride(1))
                     if conv_state_out is not None else (0, 0))
            K.in_proj_conv_proj_raw(hn.view(n, C), self.in_proj.weight, xz[:, Dm:], cw, cb,
                                    conv_state_in, csi_s, conv_state_out, cso_s, wx_pad, E,
                                    wdt_pad, R, u, x_dbl, dt, Lp, Bsz, Dm, seqlen, W, stream)
            return xz, u, x_dbl, dt
        if bufs is None and self._split_in_proj_ok(hn, Bsz):
            # in_proj as two launches: x (what conv_proj needs) here, z (what only the scan's
            # gate reads) on a side stream, so it runs beside conv_proj; the current stream
            # waits for it before returning.  Every row of either half is the same MFMA
            # chain as in the one-launch GEMM (the HIP GEMM's rows do not depend on n).
            h2 = hn.view(n, C)
            w = self.in_proj.weight
            xz = torch.empty((n, 2 * Dm), dtype=hn.dtype, device=hn.device)
            K.linear(h2, w[:Dm], out=xz[:, :Dm])
            cur = torch.cuda.current_stream(hn.device)
            z_side = _z_stream(hn.device)
            z_side.wait_stream(cur)
            with torch.cuda.stream(z_side):
                K.linear(h2, w[Dm:], out=xz[:, Dm:])
            u = torch.empty((n, Dm), dtype=hn.dtype, device=hn.device)
            x_dbl = dt = None
        elif bufs is None:
            xz = _linear(hn.view(n, C), self.in_proj.weight, self.in_proj.bias,
                         clips=Bsz)  # (n, 2D)
            u = torch.empty((n, Dm), dtype=hn.dtype, device=hn.device)
            x_dbl = dt = None
        else:
            xz, u, x_dbl, dt = bufs
            _linear_into(hn.view(n, C), self.in_proj.weight, self.in_proj.bias, xz, clips=Bsz)
        csi_s = ((conv_state_in.stride(0), conv_state_in.stride(1))
                 if conv_state_in is not None else (0, 0))
        cso_s = ((conv_state_out.stride(0), conv_state_out.stride(1))
                 if conv_state_out is not None else (0, 0))
        if self._fused_conv_proj_ok(hn, seqlen, conv_state_in):
            # conv + silu -> x_proj -> dt_proj in one kernel (vm_conv_proj.hip).  The scan
            # keeps the delta activation softplus(dt + bias): moved into conv_proj's dt
            # epilogue it measured a wash at B = 336 (scan -222 us, conv_proj +385 us per
            # layer, profiles/r01f_delta_placement.txt)
            wx_pad, wdt_pad = self._padded_proj_weights()
            if x_dbl is None:
                x_dbl = torch.empty((n, E), dtype=hn.dtype, device=hn.device)
                dt = torch.empty((n, Dm), dtype=hn.dtype, device=hn.device) if want_dt else None
            K.conv_proj_raw(xz, s_xz[::2], cw, cb, conv_state_in, csi_s, conv_state_out, cso_s,
                            wx_pad, E, wdt_pad if want_dt else None, R, u, s_u[::2], x_dbl,
                            (Lp * E, E), dt if want_dt else None, s_u[::2], Lp, Bsz, Dm, seqlen,
                            W, stream)
        else:
            K.conv_raw(xz, s_xz, cw, cb, conv_state_in, csi_s, conv_state_out, cso_s,
                       u, s_u, Lp, Bsz, Dm, seqlen, W, True, dt_code, stream)
            if x_dbl is None:
                x_dbl = _linear(u, self.x_proj.weight)  # (n, R+2N)
                dt = _linear(x_dbl[:, :R], self.dt_proj.weight)  # (n, D); bias in the scan
            else:
                _linear_into(u, self.x_proj.weight, None, x_dbl)
                _linear_into(x_dbl[:, :R], self.dt_proj.weight, None, dt)
        if z_side is not None:  # the z half is complete before anything after this reads xz
            torch.cuda.current_stream(hn.device).wait_stream(z_side)
        return xz, u, x_dbl, dt

    def _in_proj_conv_ok(self, hn: Tensor, seqlen: int, want_dt: bool) -> bool:
        """in_proj runs with the conv and the x_proj partials in its epilogue
        (``options.in_proj_conv_clips``): streaming batches whose in_proj would take the
        row-tile HIP GEMM, the fused conv_proj path (bf16, its shape limits) and the shapes
        ``vm_in_proj_conv_proj_fwd`` takes (in_proj K in the GEMM's set, d_inner % 128 == 0,
        a chunk of at least 56 padded tokens)."""
        o = options.get()
        Bsz, Lp, C = hn.shape
        if (Bsz > o.in_proj_conv_clips or o.projection_gemm != "hip" or o.in_proj_z_stream
                or self.in_proj.bias is not None or not self._fused_conv_proj_ok(hn, seqlen)):
            return False
        w = self.in_proj.weight
        if not _small_gemm_ok(hn.view(Bsz * Lp, C), w, None, clips=Bsz):
            return False
        wx_pad, wdt_pad = self._padded_proj_weights()
        E = self.dt_rank + 2 * self.d_state
        return K.in_proj_conv_proj_fits(C, Bsz, Lp, self.d_inner, E, wx_pad.shape[0],
                                        wdt_pad.shape[1], self.d_conv, want_dt)

    def _split_in_proj_ok(self, hn: Tensor, clips: int) -> bool:
        """in_proj runs as x / z halves on two streams (``options.in_proj_z_stream``) at
        streaming batches (``clips <= options.in_proj_split_clips``), where every kernel of
        the layer is latency-bound and conv_proj can share the CUs with the z half; the HIP
        GEMM must take both halves (bf16, no bias; n = d_inner per half)."""
        o = options.get()
        if not o.in_proj_z_stream or clips > o.in_proj_split_clips or self.in_proj.bias is not None:
            return False
        n = hn.shape[0] * hn.shape[1]
        w = self.in_proj.weight
        return (_small_gemm_ok(hn.view(n, hn.shape[2]), w[:self.d_inner], None, clips=clips)
                and (self.d_inner * w.stride(0) * w.element_size()) % 16 == 0)

    def _forward_padded_tm(self, hn, seqlen, conv_state_in, conv_state_out, h0, h_last,
                           next_norm=None):
        """Token-major form of :meth:`_forward_padded` (same math, same rounding points)."""
        Bsz, Lp, C = hn.shape
        Dm, N, R = self.d_inner, self.d_state, self.dt_rank
        E = R + 2 * N
        dt_code = K.dtype_code(hn.dtype)
        stream = torch.cuda.current_stream(hn.device).cuda_stream
        A, Dv, dbias, _, _ = self._fp32_params()
        s_u, s_xz, s_bc = (Lp * Dm, 1, Dm), (Lp * 2 * Dm, 1, 2 * Dm), (Lp * E, 1, E)
        dtp = self._dtp_ok(hn, seqlen, conv_state_in)
        xz, u, x_dbl, dt = self._tm_front(hn, seqlen, conv_state_in, conv_state_out,
                                          want_dt=not dtp)
        _phase.pre_done(self.layer_idx)  # sub-batch streams: the next part's pre phase may go
        y = torch.empty_like(u)
        h0_s = (h0.stride(0), h0.stride(1)) if h0 is not None else (0, 0)
        hl_s = (h_last.stride(0), h_last.stride(1)) if h_last is not None else (0, 0)
        log = _SCAN_EVENTS[0]
        ev0 = _scan_event(log)
        if dtp:  # dt_proj inside the scan: no dt rows written or read
            _, wdt_pad = self._padded_proj_weights()
            K.scan_dtproj_raw(u, s_u, x_dbl, (Lp * E, E), R, wdt_pad, A, x_dbl[:, R:R + N],
                              s_bc, x_dbl[:, R + N:], s_bc, Dv, xz[:, Dm:], s_xz, dbias,
                              h0, h0_s, h_last, hl_s, y, s_u, Lp, Bsz, Dm, seqlen, N, stream)
        else:
            K.scan_raw(u, s_u, dt, s_u, A, x_dbl[:, R:R + N], s_bc, x_dbl[:, R + N:], s_bc, Dv,
                       xz[:, Dm:], s_xz, dbias, True, h0, h0_s, h_last, hl_s,
                       y, s_u, Lp, Bsz, Dm, seqlen, N, dt_code, stream)
        if log is not None:
            log.append((ev0, _scan_event(log), Bsz))
        if (next_norm is not None and next_norm.residual is not None
                and _small_gemm_ok(y, self.out_proj.weight, self.out_proj.bias, clips=Bsz)):
            # out_proj + the next block's residual add + RMSNorm in one kernel
            out = K.linear_add_norm(y, self.out_proj.weight, next_norm.residual.view(-1, C),
                                    next_norm.w32, next_norm.eps, next_norm.hn.view(-1, C))
            next_norm.done = True
            return out.view(Bsz, Lp, C)
        out = _linear(y, self.out_proj.weight, self.out_proj.bias, clips=Bsz)  # (n, C)
        return out.view(Bsz, Lp, C)

    def _check_state(self, t: Tensor, last: int, what: str, batch: int) -> Tensor:
        want = (batch, self.d_inner, last)
        if tuple(t.shape) != want:
            raise ValueError(f"{what} shape mismatch: expected {want}, got {tuple(t.shape)}.")
        if t.stride(-1) != 1:
            raise ValueError(f"{what} must have unit stride on its last axis")
        return t

    def forward_padded(self, hn: Tensor, seqlen: int, *, ssm_state: Optional[Tensor] = None,
                       state: Optional[Tuple[Tensor, Tensor]] = None,
                       return_state: bool = False, conv_out: Optional[Tensor] = None,
                       next_norm=None):
        """Model-internal entry on the padded layout (no inference_params).  Same state
        semantics as :meth:`forward`; ``conv_out`` (B, D, d_conv) receives the new conv
        state instead of a fresh tensor (the graph runner's batched state buffers)."""
        conv_state = None
        if state is not None:
            conv_state, ssm_state = state
        Bsz = hn.shape[0]
        if conv_state is not None:
            self._check_state(conv_state, self.d_conv, "conv_state", Bsz)
        if ssm_state is not None:
            self._check_state(ssm_state, self.d_state, "ssm_state", Bsz)
        use_inplace = ssm_state is not None and state is None and not return_state
        cs_out = None
        if return_state and conv_out is not None:
            cs_out = self._check_state(conv_out, self.d_conv, "conv_out", Bsz)
        elif return_state:
            cs_dtype = conv_state.dtype if conv_state is not None else hn.dtype
            cs_out = torch.empty((Bsz, self.d_inner, self.d_conv), dtype=cs_dtype,
                                 device=hn.device)
        h_last = None
        if return_state or use_inplace:
            h_last = ssm_state if ssm_state is not None else torch.empty(
                (Bsz, self.d_inner, self.d_state), dtype=torch.float32, device=hn.device)
        out = self._forward_padded(hn, seqlen, conv_state_in=conv_state, conv_state_out=cs_out,
                                   h0=ssm_state, h_last=h_last, next_norm=next_norm)
        if return_state:
            return out, (cs_out, h_last)
        return out

    def forward(self, hidden_states: Tensor, inference_params: Optional[InferenceParamsLike] = None,
                ssm_state: Optional[Tensor] = None, state: Optional[Tuple[Tensor, Tensor]] = None,
                return_state: bool = False):
        """hidden_states: (B, L, D) -> (B, L, D) [, (conv_state, ssm_state)]."""
        if state is not None and ssm_state is not None:
            raise ValueError("Pass either state or ssm_state, not both.")
        if inference_params is not None and state is not None:
            raise ValueError("state is not supported with inference_params.")
        if not hidden_states.is_cuda:
            raise RuntimeError(_CUDA_ERROR)
        warn_if_grad(hidden_states, self.in_proj.weight)
        with torch.no_grad():
            return self._forward(hidden_states, inference_params, ssm_state, state, return_state)

    def _forward(self, hs, inference_params, ssm_state, state, return_state):
        batch, seqlen, dm = hs.shape
        Lp = round_up(max(seqlen, 1))
        if Lp == seqlen and hs.is_contiguous():
            hp = hs
        else:
            hp = torch.zeros((batch, Lp, dm), dtype=hs.dtype, device=hs.device)
            hp[:, :seqlen] = hs

        def trim(o):
            return o if Lp == seqlen else o[:, :seqlen].contiguous()

        if inference_params is not None:
            conv_state, cache_state = self._get_states_from_cache(inference_params, batch)
            if ssm_state is None:
                ssm_state = cache_state
            if inference_params.seqlen_offset > 0:
                out, _, _ = self.step(hs, conv_state, ssm_state)
                return out
            # prefill: conv restarts from zeros, the cache receives the last d_conv raw
            # inputs and the final ssm state (in place); return_state is ignored.
            self._check_state(ssm_state, self.d_state, "ssm_state", batch)
            out = self._forward_padded(hp, seqlen, conv_state_out=conv_state, h0=ssm_state,
                                       h_last=ssm_state)
            return trim(out)
        res = self.forward_padded(hp, seqlen, ssm_state=ssm_state, state=state,
                                  return_state=return_state)
        if return_state:
            return trim(res[0]), res[1]
        return trim(res)

    def step(self, hidden_states: Tensor, conv_state: Tensor, ssm_state: Tensor):
        """One-token decode (``mamba_simple.py:453-497``); states updated in place."""
        if not hidden_states.is_cuda:
            raise RuntimeError(_CUDA_ERROR)
        assert hidden_states.shape[1] == 1, "Only support decoding with 1 token at a time for now"
        with torch.no_grad():
            A, Dv, dbias, cw, cb = self._fp32_params()
            xz = self.in_proj(hidden_states.squeeze(1))  # (B, 2D)
            x, z = xz.chunk(2, dim=-1)
            x = K.causal_conv1d_update(x, conv_state, cw, cb, self.activation)
            x_db = self.x_proj(x)
            dt, Bm, Cm = torch.split(x_db, [self.dt_rank, self.d_state, self.d_state], dim=-1)
            dt = F.linear(dt, self.dt_proj.weight)  # bias is added inside the step kernel
            y = K.selective_state_update(ssm_state, x, dt, A, Bm, Cm, Dv, z=z, dt_bias=dbias,
                                         dt_softplus=True)
            out = self.out_proj(y)
        return out.unsqueeze(1), conv_state, ssm_state

    # ------------------------------------------------------------------ state allocation
    def _zeros_states(self, batch_size, conv_dtype, ssm_dtype, device):
        conv = torch.zeros(batch_size, self.d_inner, self.d_conv, device=device, dtype=conv_dtype)
        ssm = torch.zeros(batch_size, self.d_inner, self.d_state, device=device, dtype=ssm_dtype)
        return conv, ssm

    def allocate_inference_cache(self, batch_size: int, max_seqlen: int, dtype=None, **kwargs):
        return self._zeros_states(batch_size, self.conv1d.weight.dtype if dtype is None else dtype,
                                  self.dt_proj.weight.dtype if dtype is None else dtype,
                                  self.out_proj.weight.device)

    def allocate_state(self, batch_size: int, dtype=None, device=None):
        """Zero (conv_state, ssm_state) for chunked streaming."""
        return self._zeros_states(batch_size, self.conv1d.weight.dtype if dtype is None else dtype,
                                  self.dt_proj.weight.dtype if dtype is None else dtype,
                                  self.out_proj.weight.device if device is None else device)

    def _get_states_from_cache(self, inference_params: InferenceParamsLike, batch_size: int,
                               initialize_states: bool = False):
        assert self.layer_idx is not None
        cache = inference_params.key_value_memory_dict
        entry = cache.get(self.layer_idx)
        if entry is None or entry[0].shape[0] != batch_size or entry[1].shape[0] != batch_size:
            entry = self._zeros_states(batch_size, self.conv1d.weight.dtype,
                                       self.dt_proj.weight.dtype, self.conv1d.weight.device)
            cache[self.layer_idx] = entry
        elif initialize_states:
            entry[0].zero_()
            entry[1].zero_()
        return entry
