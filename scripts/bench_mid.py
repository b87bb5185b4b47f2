"""Microbenchmark of the token-major mixer middle at VideoMamba-M geometry (bf16):
fused conv+x_proj+dt_proj kernel vs conv kernel + two library GEMMs.
    python scripts/bench_mid.py --batches 32 224
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from videomamba_amd import kernels as K  # noqa: E402
from videomamba_amd.layers import round_up  # noqa: E402


def timeit(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


ap = argparse.ArgumentParser()
ap.add_argument("--batches", type=int, nargs="+", default=[32, 224])
ap.add_argument("--reps", type=int, default=10)
a = ap.parse_args()
dev = torch.device("cuda", 0)
D, N, R, L, W = 1152, 16, 36, 3137, 4
E = R + 2 * N
Lp = round_up(L)
bf = torch.bfloat16
g = torch.Generator(device=dev).manual_seed(0)
cw = torch.randn(D, W, device=dev, generator=g) * 0.3
cb = torch.randn(D, device=dev, generator=g) * 0.1
wx = (torch.randn(E, D, device=dev, generator=g) * 0.03).to(bf)
wdt = (torch.randn(D, R, device=dev, generator=g) * 0.1).to(bf)
wx_pad = torch.zeros(80, D, device=dev, dtype=bf)
wx_pad[:E] = wx
wdt_pad = torch.zeros(D, 64, device=dev, dtype=bf)
wdt_pad[:, :R] = wdt
stream = torch.cuda.current_stream(dev).cuda_stream
for B in a.batches:
    n = B * Lp
    xz = torch.randn(n, 2 * D, device=dev, generator=g).to(bf)
    u = torch.empty(n, D, device=dev, dtype=bf)
    u2 = torch.empty_like(u)
    xdbl = torch.empty(n, E, device=dev, dtype=bf)
    dt = torch.empty(n, D, device=dev, dtype=bf)

    def fused():
        K.conv_proj_raw(xz, (Lp * 2 * D, 2 * D), cw, cb, None, (0, 0), None, (0, 0), wx_pad, E,
                        wdt_pad, R, u, (Lp * D, D), xdbl, (Lp * E, E), dt, (Lp * D, D), Lp, B, D,
                        L, W, stream)

    def conv_only():
        K.conv_raw(xz, (Lp * 2 * D, 1, 2 * D), cw, cb, None, (0, 0), None, (0, 0), u2,
                   (Lp * D, 1, D), Lp, B, D, L, W, True, 1, stream)

    def unfused():
        conv_only()
        xd = F.linear(u2, wx)
        F.linear(xd[:, :R], wdt)

    t_f, t_c, t_u = timeit(fused, a.reps), timeit(conv_only, a.reps), timeit(unfused, a.reps)
    fused()
    unfused()
    xd_ref = F.linear(u2, wx)
    dt_ref = F.linear(xd_ref[:, :R], wdt)
    rel = lambda x, y: ((x.float() - y.float()).norm() / y.float().norm()).item()  # noqa: E731
    hbm = n * (3 * D * 2 + E * 2)
    print(json.dumps({"B": B, "fused_us": round(t_f, 1), "conv_us": round(t_c, 1),
                      "unfused_us": round(t_u, 1), "fused_GBps": round(hbm / t_f / 1e3, 1),
                      "rel_u": rel(u, u2), "rel_xdbl": rel(xdbl, xd_ref),
                      "rel_dt": rel(dt, dt_ref)}), flush=True)
