"""Host-side selection knobs of the HIP path — the only configuration channel there is.

The C library reads no environment: every choice it makes beyond the operands' shapes
and layouts arrives as an explicit ABI argument (today: the token-major scan's segment
count).  Above it, the Python host picks the mixer layout and a few paths from this one
documented options object; tests and sweeps change them with :func:`override`.

    mixer_layout     "auto" (default) | "tm" | "cm".  "auto": token-major at every batch
                     (single-pass or chunked scan); "cm" forces the channel-major layout
                     (time-parallel scan); see mamba_simple.mixer_layout.
    scan_segments    0 (default) = the library's cost model; > 0 forces the token-major
                     scan's time-segment count (vm_selective_scan_fwd ``segments``).
    fused_conv_proj  True (default): bf16 token-major mixers run conv1d + x_proj + dt_proj
                     as one kernel (vm_conv_proj_fwd); False: conv kernel + library GEMMs.
    gemm_tuning      "on" (default): the mixer's projection GEMMs use the shipped TunableOp
                     results (gemm_tuning.py), enabled only around those calls; "off": the
                     library heuristic; "tune": record new shapes (slow, offline).
                     Initialised from ``VM_GEMM_TUNING`` when that is set (the tuning
                     script's switch); nothing else is read from the environment.
    scan_one_launch  True (default): a segmented token-major scan whose grid fits one
                     workgroup per CU runs as one launch (blocks hand their aggregates on
                     through a zeroed sync buffer, vm_selective_scan_fwd ``sync``); False:
                     the two-launch form (identical results).
    scan_dt_proj     "auto" (default): the bf16 token-major mixer folds dt_proj into the scan
                     (vm_selective_scan_dtproj_fwd) and conv_proj skips its dt rows when the
                     scan is segmented with <= 64-step segments on a grid of at most one
                     workgroup per CU (streaming batches 1-2 at M-16f; dt in conv_proj's own
                     arithmetic, ABI v11) or single-pass above 8 clips; "on": also on larger
                     segmented grids and single-pass at <= 8 clips (tests); "off": conv_proj
                     writes dt.
    projection_gemm  "hip" (default): the mixer's bf16 in_proj / out_proj run on the HIP GEMM
                     (vm_linear_fwd: the LDS-DMA tile kernel for small row counts, the
                     persistent 256-row kernel from 1.5 tiles per CU up; bit-identical forms)
                     at every batch, so every row is computed the same way whatever the
                     row count — chunked streaming == the one-pass forward bit for bit at any
                     batch; "library": the round-3 rule below (hipBLASLt above 8 clips).
    row_invariant_gemm_clips
                     ("library" mode) mixers holding at most this many clips (default 8)
                     run in_proj / out_proj on the HIP GEMM at every token count, whose rows
                     do not depend on the row count — chunked streaming == the one-pass
                     forward bit for bit; 0: only the small_gemm_* rule below.
    fuse_out_norm    False (default): True makes a mixer whose out_proj runs on the HIP GEMM
                     (bf16 fused RMSNorm blocks) also run the next block's residual add +
                     RMSNorm (vm_linear_add_norm_fwd; bit-identical to the separate kernels:
                     the one-launch LDS-DMA form at small row counts, the persistent tile
                     GEMM's per-row-block norm pass at chip-filling ones).  Measured slower
                     at both ends: B = 1 16.5-17.3 vs 13.1-13.8 us per layer,
                     B = 448 4.14 vs 3.37-3.55 ms per layer (the step 492 vs 441 ms), so it
                     is off by default.
    batch_streams    2 (default): a forward over at least ``batch_stream_min_clips`` clips runs
                     as this many sub-batches, each on its own HIP stream, so one part's
                     VALU-bound scan overlaps another part's MFMA / HBM-bound kernels; every
                     kernel's rows are independent of the batch, so the outputs and states
                     are bit-identical to the one-stream forward.  1 = one stream.
                     Measured on M-16f (scripts/diag/batch_streams_sweep.py): B = 448 in two
                     parts 424-425 vs 432-436 ms per step; three or four parts, or two parts
                     of B = 224 / 112, are slower than one stream.
    batch_stream_lock
                     True (default) orders the parts' layer "pre" phases in a ring (add +
                     norm, in_proj, conv_proj; phase_lock.py).  Each part's layers are issued
                     from its own host thread, with cross-stream event waits, so one part's
                     scan runs beside another part's pre phase and no two pre phases overlap.
                     B = 896: 0.3-1.1 % faster per step, same bits (809.8-810.2 vs
                     817.8-818.7 ms in one process; 820.6-823.3 vs 823.4-830.7 ms across
                     processes).  False lets the streams run free.
    batch_stream_min_clips
                     the smallest batch that is split (default 224: parts of >= 112 clips).
                     With the phase lock, B = 224 split in two runs 217.2 vs 221.0-222.8 ms
                     per step on one stream; B = 112 split runs 143.0-143.3 vs 113.1-113.6 ms,
                     so smaller batches stay whole (profiles/r05zzu_small_split_lock_ab.jsonl;
                     448 before the lock, when B = 224 split was slower).
    batch_stream_min_work
                     ... and at least this many clip-channels (B x d_inner; default 224 x 1152,
                     VideoMamba-M's 224 clips), so a narrower model needs more clips for each
                     part's scan grid to fill the chip: VideoMamba-Ti (d_inner 384) splits from
                     672 clips.  C2 (Ti-8f, 512 clips) on one stream: 13.65-13.67 M
                     video-tokens/s against 13.51-13.53 M as two locked streams
                     (profiles/r05zzw_c2_streams_ab.jsonl).
    in_proj_z_stream False (default): True makes the mixer at streaming batches (at most
                     ``in_proj_split_clips`` clips, default 8) run in_proj as two launches,
                     the x half on the current stream and the z half (read only by the scan's
                     gate) on a side stream beside conv_proj; bit-identical (the HIP GEMM's
                     rows do not depend on the column count).  Measured slower: the B = 1
                     graph replay 2.97-2.99 vs 2.56-2.58 ms (each cross-stream edge of the
                     replayed graph costs more than the z half's ~6 us), so it is off.
    in_proj_conv_clips
                     Mixers of at most this many clips (default 2; 0 turns it off) run in_proj
                     with the depthwise conv + SiLU and the x_proj split partials in its
                     epilogue (``vm_in_proj_conv_proj_fwd``, vm_inproj_conv.hip): x never
                     reaches HBM and conv_proj's per-tile W_x stream is gone.  Bit-identical
                     to in_proj + conv_proj (the split-K form's arithmetic), so the choice
                     never changes a result.
    small_gemm_rows  ("library" mode) in_proj / out_proj with at most this many token rows (one clip's
                     chunk) run on the HIP small-M GEMM (vm_linear_fwd, bf16); larger ones,
                     or 0, on the library.  Default 4096 (B = 1 at M-16f: 3144 rows).
    small_gemm_max_n ... and at most this many output columns (default 1024: out_proj;
                     in_proj's N = 2 * d_inner stays on the library GEMM).

Options are process-global (not thread-local): the model is driven from one host thread,
and the sub-batch issue threads of ``batch_stream_lock`` read the caller's options.
"""

from __future__ import annotations

import contextlib
import dataclasses
import os
from typing import Iterator

__all__ = ["Options", "get", "override"]

_LAYOUTS = ("auto", "tm", "cm")
_TUNING = ("on", "off", "tune")


@dataclasses.dataclass
class Options:
    mixer_layout: str = "auto"
    scan_segments: int = 0
    fused_conv_proj: bool = True
    scan_one_launch: bool = True
    scan_dt_proj: str = "auto"
    gemm_tuning: str = "on"
    projection_gemm: str = "hip"
    row_invariant_gemm_clips: int = 8
    fuse_out_norm: bool = False
    batch_streams: int = 2
    batch_stream_lock: bool = True
    in_proj_z_stream: bool = False
    in_proj_split_clips: int = 8
    in_proj_conv_clips: int = 2
    batch_stream_min_clips: int = 224
    batch_stream_min_work: int = 224 * 1152
    small_gemm_rows: int = 4096
    small_gemm_max_n: int = 1024

    def validate(self) -> None:
        if self.mixer_layout not in _LAYOUTS:
            raise ValueError(f"mixer_layout must be one of {_LAYOUTS}, got {self.mixer_layout!r}")
        if int(self.scan_segments) < 0:
            raise ValueError("scan_segments must be >= 0")
        if int(self.batch_streams) < 1:
            raise ValueError("batch_streams must be >= 1")
        if int(self.small_gemm_rows) < 0:
            raise ValueError("small_gemm_rows must be >= 0")
        if self.scan_dt_proj not in ("auto", "on", "off"):
            raise ValueError(f"scan_dt_proj must be auto / on / off, got {self.scan_dt_proj!r}")
        if self.projection_gemm not in ("hip", "library"):
            raise ValueError(f"projection_gemm must be hip / library, got {self.projection_gemm!r}")
        if self.gemm_tuning not in _TUNING:
            raise ValueError(f"gemm_tuning must be one of {_TUNING}, got {self.gemm_tuning!r}")


def _initial() -> Options:
    o = Options()
    env = os.environ.get("VM_GEMM_TUNING", "").strip().lower()
    if env in ("0", "off", "false", "no"):
        o.gemm_tuning = "off"
    elif env == "tune":
        o.gemm_tuning = "tune"
    return o


_OPTS = _initial()


def get() -> Options:
    """The live options object (read by the mixer on every call)."""
    return _OPTS


@contextlib.contextmanager
def override(**changes) -> Iterator[Options]:
    """Temporarily change options: ``with override(mixer_layout="tm"): ...``."""
    global _OPTS
    old = _OPTS
    new = dataclasses.replace(old, **changes)
    new.validate()
    _OPTS = new
    try:
        yield new
    finally:
        _OPTS = old
