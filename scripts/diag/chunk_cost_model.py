"""Fixed vs per-step cost of the chunked (segmented) token-major scan at B=1, D=1152:
time (HIP events, 30 launches) over sequence lengths and forced segment counts.
    python scripts/diag/chunk_cost_model.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from videomamba_amd import kernels as K  # noqa: E402
from videomamba_amd.layers import round_up  # noqa: E402


def run(L, S, B=1, D=1152, N=16, R=36, reps=30):
    dev = torch.device("cuda", 0)
    Lp = round_up(L)
    n = B * Lp
    bf = torch.bfloat16
    A = -torch.arange(1, N + 1, device=dev, dtype=torch.float32).repeat(D, 1).contiguous()
    Dv = torch.ones(D, device=dev)
    bias = torch.full((D,), -4.0, device=dev)
    h = torch.zeros(B, D, N, device=dev, dtype=bf)
    u = torch.randn(n, D, device=dev).to(bf)
    dt = (0.5 * torch.randn(n, D, device=dev) - 4.0).to(bf)
    xz = torch.randn(n, 2 * D, device=dev).to(bf)
    xdbl = torch.randn(n, R + 2 * N, device=dev).to(bf)
    y = torch.empty_like(u)
    s_u, s_z, s_bc = (Lp * D, 1, D), (Lp * 2 * D, 1, 2 * D), (Lp * (R + 2 * N), 1, R + 2 * N)
    ws = torch.empty(max(1, K.scan_workspace_bytes(B, D, L, N, S)), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream
    from videomamba_amd import options

    def launch():
        K.scan_raw(u, s_u, dt, s_u, A, xdbl[:, R:], s_bc, xdbl[:, R + N:], s_bc, Dv, xz[:, D:], s_z,
                   bias, True, h, (h.stride(0), h.stride(1)), h, (h.stride(0), h.stride(1)), y, s_u,
                   Lp, B, D, L, N, 1, stream, workspace=ws)

    with options.override(scan_segments=S):
        for _ in range(3):
            launch()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            launch()
        e1.record()
        torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


for L, S in [(3137, 100), (1600, 50), (800, 25), (3137, 50), (1600, 100), (800, 100), (400, 50),
             (3137, 200), (3137, 25)]:
    print(json.dumps({"L": L, "S": S, "T": -(-L // S), "us": round(run(L, S), 2)}), flush=True)
