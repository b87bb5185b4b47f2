"""Chunked token-major scan time vs forced segment count (M-16f mixer geometry, bf16,
stateful, delta softplus, z gate), HIP events over back-to-back launches.  Used to fit the
segment cost model in vm_scan_seq.hip::choose_segments.
    python scripts/diag/scan_segments_sweep.py  (env CASES="B:L,..." SEGS="0 50 100 ...")
DTP=1: the dt_proj-inside form (vm_selective_scan_dtproj_fwd, segments of <= 64 steps)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from videomamba_amd import kernels as K  # noqa: E402
from videomamba_amd import options  # noqa: E402
from videomamba_amd.mamba_simple import Mamba  # noqa: E402

dev = "cuda"
torch.manual_seed(0)
m = Mamba(d_model=576, d_state=16, d_conv=4, expand=2, layer_idx=0).to(dev, torch.bfloat16)
Dm, E, R, N = m.d_inner, m.dt_rank + 2 * m.d_state, m.dt_rank, m.d_state
A, Dv, dbias, _, _ = m._fp32_params()
st = torch.cuda.current_stream().cuda_stream
DTP = os.environ.get("DTP", "0") == "1"
wdt_pad = m._padded_proj_weights()[1] if DTP else None


def timeit(fn, reps=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


cases = [tuple(int(v) for v in c.split(":")) for c in
         os.environ.get("CASES", "1:3137,2:3137,4:3137,8:3137,1:12545").split(",")]
segs = [int(s) for s in os.environ.get("SEGS", "0 50 75 100 150 200 300 400").split()]
for B, L in cases:
    Lp = (L + 7) // 8 * 8
    n = B * Lp
    u = (0.5 * torch.randn(n, Dm, device=dev)).to(torch.bfloat16)
    dt = (0.5 * torch.randn(n, Dm, device=dev) - 1.0).to(torch.bfloat16)
    xz = torch.randn(n, 2 * Dm, device=dev).to(torch.bfloat16)
    xd = torch.randn(n, E, device=dev).to(torch.bfloat16)
    y = torch.empty_like(u)
    h = torch.zeros(B, Dm, N, device=dev)
    s_u, s_xz, s_bc = (Lp * Dm, 1, Dm), (Lp * 2 * Dm, 1, 2 * Dm), (Lp * E, 1, E)
    row = {"B": B, "L": L, "dtp": DTP}
    for S in segs:
        if S > (L + 7) // 8:
            continue
        if DTP and not 0 < K.scan_chunk_steps(B, Dm, L, N, S) <= K.SCAN_DTPROJ_MAX_SEGMENT:
            continue
        with options.override(scan_segments=S):
            if DTP:
                fn = lambda: K.scan_dtproj_raw(  # noqa: E731
                    u, s_u, xd, (Lp * E, E), R, wdt_pad, A, xd[:, R:R + N], s_bc, xd[:, R + N:],
                    s_bc, Dv, xz[:, Dm:], s_xz, dbias, h, (Dm * N, N), h, (Dm * N, N), y, s_u,
                    Lp, B, Dm, L, N, st)
                row[f"S{S}"] = round(timeit(fn), 2)
                continue
            fn = lambda: K.scan_raw(u, s_u, dt, s_u, A, xd[:, R:R + N], s_bc, xd[:, R + N:],  # noqa: E731
                                    s_bc, Dv, xz[:, Dm:], s_xz, dbias, True, h, (Dm * N, N), h,
                                    (Dm * N, N), y, s_u, Lp, B, Dm, L, N, 1, st)
            row[f"S{S}"] = round(timeit(fn), 2)
    print(json.dumps(row), flush=True)
