"""Per-kernel timing of the token-major mixer middle and scan at small batches (M-16f
geometry), HIP events over back-to-back launches."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from videomamba_amd import kernels as K  # noqa: E402
from videomamba_amd.mamba_simple import Mamba  # noqa: E402

dev = "cuda"
torch.manual_seed(0)
m = Mamba(d_model=576, d_state=16, d_conv=4, expand=2, layer_idx=0).to(dev, torch.bfloat16)
Dm, E, R, W, N = m.d_inner, m.dt_rank + 2 * m.d_state, m.dt_rank, m.d_conv, m.d_state
A, Dv, dbias, cw, cb = m._fp32_params()
wx_pad, wdt_pad = m._padded_proj_weights()
st = torch.cuda.current_stream().cuda_stream
L = 3137
Lp = (L + 7) // 8 * 8


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


for B in [int(b) for b in os.environ.get("BATCHES", "1 2 4 8 16").split()]:
    n = B * Lp
    xz = torch.randn(n, 2 * Dm, device=dev).to(torch.bfloat16)
    u = torch.empty(n, Dm, device=dev, dtype=torch.bfloat16)
    xd = torch.empty(n, E, device=dev, dtype=torch.bfloat16)
    dt = torch.empty(n, Dm, device=dev, dtype=torch.bfloat16)
    y = torch.empty_like(u)
    h = torch.zeros(B, Dm, N, device=dev)
    s_u, s_xz, s_bc = (Lp * Dm, 1, Dm), (Lp * 2 * Dm, 1, 2 * Dm), (Lp * E, 1, E)
    cp = lambda: K.conv_proj_raw(xz, s_xz[::2], cw, cb, None, (0, 0), None, (0, 0), wx_pad, E,  # noqa: E731
                                 wdt_pad, R, u, s_u[::2], xd, (Lp * E, E), dt, s_u[::2], Lp, B,
                                 Dm, L, W, st)
    sc = lambda: K.scan_raw(u, s_u, dt, s_u, A, xd[:, R:R + N], s_bc, xd[:, R + N:], s_bc, Dv,  # noqa: E731
                            xz[:, Dm:], s_xz, dbias, True, h, (Dm * N, N), h, (Dm * N, N), y, s_u,
                            Lp, B, Dm, L, N, 1, st)
    print(json.dumps({"B": B, "conv_proj_us": round(timeit(cp), 2), "scan_us": round(timeit(sc), 2)}),
          flush=True)
