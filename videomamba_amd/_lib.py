"""ctypes binding of ``libvideomamba_hip.so`` (the C ABI in ``include/videomamba_hip.h``).

The library is built in-tree (``make -C videomamba_amd/csrc`` or
``__graft_entry__.build()``).  There is no fallback: if the library is missing or fails
to load, every kernel entry point raises.  ``torch`` is imported first so that the HIP
runtime the library links against (soname ``libamdhip64.so.7``) resolves to the one
PyTorch already loaded — one runtime, one set of streams.
"""

from __future__ import annotations

import ctypes
import os
from ctypes import c_float, c_int, c_longlong, c_void_p

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

LIB_NAME = "libvideomamba_hip.so"
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)

VM_DTYPE_F32 = 0
VM_DTYPE_BF16 = 1
ABI_VERSION = 14

_P = c_void_p
_LL = c_longlong
_I = c_int

_SIGNATURES = {
    "vm_abi_version": ([], _I),
    "vm_last_error": ([], ctypes.c_char_p),
    "vm_selective_scan_fwd": (
        [_P, _LL, _LL, _LL,       # u (sb, sd, sl)
         _P, _LL, _LL, _LL,       # delta
         _P,                      # A
         _P, _LL, _LL, _LL,       # B (sb, sn, sl)
         _P, _LL, _LL, _LL,       # C
         _P, _P, _LL, _LL, _LL,   # D, z
         _P, _I,                  # delta_bias, softplus
         _P, _I, _LL, _LL,        # h0
         _P, _I, _LL, _LL,        # h_last
         _P, _LL, _LL, _LL, _I,   # out, out_len
         _I, _I, _I, _I, _I,      # batch, dim, seqlen, dstate, dtype
         _I, _P, _LL,             # segments, workspace, workspace_bytes
         _P, _LL,                 # sync, sync_bytes
         _P], _I),
    "vm_selective_scan_bidir_fwd": (
        [_P, _LL, _LL, _LL, _P, _LL, _LL, _LL, _P, _P, _LL, _LL, _LL, _P, _LL, _LL, _LL,
         _P, _P, _LL, _LL, _LL, _P, _I, _P, _I, _LL, _LL, _P, _I, _LL, _LL,
         _P, _LL, _LL, _LL, _I, _I, _I, _I, _I, _I,
         _I, _P, _P, _P, _P, _P, _I,              # split, A/D/bias/h0/h_last bwd, frame_len
         _I, _P, _LL, _P, _LL, _P], _I),
    "vm_selective_scan_dtproj_fwd": (
        [_P, _LL, _LL, _LL,       # u (sb, sd, sl)
         _P, _LL, _LL, _I,        # dt_low (sb, sl), dt_rank
         _P, _I,                  # W_dt padded, its leading dimension
         _P,                      # A
         _P, _LL, _LL, _LL,       # B (sb, sn, sl)
         _P, _LL, _LL, _LL,       # C
         _P, _P, _LL, _LL, _LL,   # D, z
         _P, _I,                  # delta_bias, softplus
         _P, _I, _LL, _LL,        # h0
         _P, _I, _LL, _LL,        # h_last
         _P, _LL, _LL, _LL, _I,   # out, out_len
         _I, _I, _I, _I, _I,      # batch, dim, seqlen, dstate, dtype
         _I, _P, _LL, _P, _LL,    # segments, workspace, sync (ABI v11)
         _P], _I),
    "vm_selective_scan_chunk_steps": ([_I, _I, _I, _I, _I], _I),
    "vm_selective_scan_workspace_bytes": ([_I, _I, _I, _I, _I], _LL),
    "vm_selective_scan_sync_bytes": ([_I, _I, _I, _I, _I], _LL),
    "vm_selective_scan_sync_status": ([_P, _LL], _I),
    "vm_selective_state_update": (
        [_P, _I, _LL, _LL, _P, _LL, _P, _LL, _P, _P, _LL, _P, _LL, _P, _P, _LL, _P, _I,
         _P, _LL, _I, _I, _I, _I, _P], _I),
    "vm_causal_conv1d_fwd": (
        [_P, _LL, _LL, _LL, _P, _P, _P, _I, _LL, _LL, _P, _I, _LL, _LL, _P, _LL, _LL, _LL, _I,
         _I, _I, _I, _I, _I, _I, _P], _I),
    "vm_conv_proj_fwd": (
        [_P, _LL, _LL, _P, _P,                    # xz, conv weight / bias
         _P, _I, _LL, _LL, _P, _I, _LL, _LL,      # conv state in / out
         _P, _I, _I, _P, _I, _I,                  # W_x pad, e, e_pad, W_dt pad, r, r_pad
         _P, _LL, _LL, _P, _LL, _LL, _P, _LL, _LL,  # u, x_dbl, dt
         _P, _I,                                  # dt bias, dt softplus
         _I, _I, _I, _I, _I, _I,                  # out_len, batch, dim, seqlen, width, dtype
         _P, _LL, _P], _I),                       # workspace, bytes, stream
    "vm_conv_proj_workspace_bytes": ([_I, _I, _I, _I], _LL),
    "vm_conv_proj_fits": (
        [_I, _I, _I, _I, _I, _I, _I,              # batch, out_len, seqlen, dim, e, r_pad, softplus
         _LL, _LL, _I, _I, _LL, _LL, _I, _LL], _I),  # xz strides, conv state in, width, u_sl
    "vm_in_proj_conv_proj_fwd": (
        [_P, _LL, _P, _LL, _I,                    # hn, ldh, w_in, ldw, k
         _P, _LL, _P, _P,                         # z, ldz, conv weight / bias
         _P, _I, _LL, _LL, _P, _I, _LL, _LL,      # conv state in / out
         _P, _I, _I, _P, _I, _I,                  # W_x pad, e, e_pad, W_dt pad, r, r_pad
         _P, _LL, _P, _LL, _P, _LL,               # u, x_dbl, dt (row strides)
         _I, _I, _I, _I, _I,                      # out_len, batch, dim, seqlen, width
         _P, _LL, _P], _I),                       # workspace, bytes, stream
    "vm_in_proj_conv_proj_workspace_bytes": ([_I, _I, _I, _I], _LL),
    "vm_in_proj_conv_proj_fits": ([_I, _I, _I, _I, _I, _I, _I, _I, _I], _I),
    "vm_conv_proj_cm_fwd": (
        [_P, _LL, _P, _P,                         # xz (row stride), conv weight / bias
         _P, _I, _LL, _LL, _P, _I, _LL, _LL,      # conv state in / out
         _P, _I, _I, _P, _I, _I,                  # W_x pad, e, e_pad, W_dt pad, r, r_pad
         _P, _LL, _P, _LL, _P, _LL,               # u, x_dbl, dt (row strides)
         _I, _I, _I, _I, _I,                      # out_len, batch, dim, seqlen, width
         _P, _LL, _P], _I),
    "vm_conv_proj_cm_workspace_bytes": ([_I, _I, _I, _I], _LL),
    "vm_causal_conv1d_update": (
        [_P, _LL, _P, _I, _LL, _LL, _P, _P, _P, _LL, _I, _I, _I, _I, _I, _P], _I),
    "vm_add_norm_fwd": (
        [_P, _I, _P, _I, _P, _P, _P, _I, _P, _I, _LL, _I, c_float, _I, _P], _I),
    "vm_norm_pool_workspace_bytes": ([_I, _I, _I, _I], _LL),
    "vm_norm_pool_fwd": (
        [_P, _I, _P, _I, _LL,                     # x, residual, batch stride
         _P, _P, c_float, _I,                     # weight, bias, eps, is_rms
         _P, _I, _LL, _I, _I, _I,                 # out, dtype, batch stride, batch, rows, cols
         _I, _I, _I, _P, _I, _I,                  # head, groups, rows, bounds, max, rev_frame
         _P, _LL, _P], _I),
    "vm_pool_finish_fwd": (
        [_P, _I, _I, _I, _P, _I,                  # workspace, batch, groups, rows, bounds, max
         _P, _I, _LL, _I, _I,                     # cls, dtype, stride, mode, keep_temporal
         _P, _P, c_float, _P, _I, _I, _P], _I),   # LN w / b / eps, x_pool, dtype, cols
    "vm_linear_fwd": ([_P, _LL, _P, _LL, _P, _P, _LL, _I, _I, _I, _I, _P], _I),
    "vm_linear_fwd_form": ([_P, _LL, _P, _LL, _P, _P, _LL, _I, _I, _I, _I, _I, _P], _I),
    "vm_linear_add_norm_fwd": (
        [_P, _LL, _P, _LL,                        # x, ldx, w, ldw
         _P, _LL, _P, _LL,                        # h (out), ldo, residual (fp32), ldr
         _P, c_float, _P, _LL,                    # norm weight, eps, hn, ldh
         _I, _I, _I, _P, _LL, _P], _I),           # m, n, k, counters, bytes, stream
    "vm_linear_add_norm_counter_bytes": ([_I], _LL),
    "vm_patch_embed_fwd": (
        [_P, _P, _P, _P, _P, _P, _LL, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I, _I,
         _P, _P, _I, _P], _I),
}

EXPORTED = tuple(_SIGNATURES)

_lib = None
_load_error: str | None = None


def load():
    """Load (once) and return the CDLL; raises RuntimeError with the reason on failure."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    if _load_error is not None:
        raise RuntimeError(_load_error)
    if not os.path.exists(LIB_PATH):
        _load_error = (f"{LIB_NAME} not found at {LIB_PATH}: build it with "
                       "`make -C videomamba_amd/csrc` (hipcc --offload-arch=gfx950)")
        raise RuntimeError(_load_error)
    try:
        lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
    except OSError as exc:
        _load_error = f"failed to load {LIB_PATH}: {exc}"
        raise RuntimeError(_load_error) from exc
    for name, (args, res) in _SIGNATURES.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = res
    ver = lib.vm_abi_version()
    if ver != ABI_VERSION:
        _load_error = f"{LIB_NAME} ABI version {ver} != expected {ABI_VERSION}"
        raise RuntimeError(_load_error)
    _lib = lib
    return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = _lib.vm_last_error().decode(errors="replace") if _lib is not None else ""
        raise RuntimeError(f"{what} failed (rc={rc}): {msg}")
