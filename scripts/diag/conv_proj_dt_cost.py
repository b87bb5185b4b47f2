"""B=1 fused conv_proj (conv + x_proj [+ dt_proj]) with and without its dt rows: what moving
dt_proj into the chunked scan would save at the streaming-chunk shape (VideoMamba-M, L=3137).
    python scripts/diag/conv_proj_dt_cost.py"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from bench import _event_us  # noqa: E402
from videomamba_amd import kernels as K  # noqa: E402
from videomamba_amd.layers import round_up  # noqa: E402
from videomamba_amd.mamba_simple import Mamba  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
mx = Mamba(d_model=576, layer_idx=0).to(dev, torch.bfloat16).eval()
Dm, N, R, W = mx.d_inner, mx.d_state, mx.dt_rank, mx.d_conv
E = R + 2 * N
out = {}
for B in (1, 2, 4):
    L = 3137
    Lp = round_up(L)
    n = B * Lp
    xz = torch.randn(n, 2 * Dm, device=dev, dtype=torch.bfloat16)
    u = torch.empty(n, Dm, device=dev, dtype=torch.bfloat16)
    dt = torch.empty(n, Dm, device=dev, dtype=torch.bfloat16)
    xdbl = torch.empty(n, E, device=dev, dtype=torch.bfloat16)
    cs_in = torch.randn(B, Dm, W, device=dev, dtype=torch.bfloat16)
    cs_out = torch.empty(B, Dm, W, device=dev, dtype=torch.bfloat16)
    _, _, _, cw, cb = mx._fp32_params()
    wx_pad, wdt_pad = mx._padded_proj_weights()
    stream = torch.cuda.current_stream(dev).cuda_stream

    def run(with_dt):
        K.conv_proj_raw(xz, (Lp * 2 * Dm, 2 * Dm), cw, cb, cs_in, (cs_in.stride(0), cs_in.stride(1)),
                        cs_out, (cs_out.stride(0), cs_out.stride(1)), wx_pad, E,
                        wdt_pad if with_dt else None, R, u, (Lp * Dm, Dm), xdbl, (Lp * E, E),
                        dt if with_dt else None, (Lp * Dm, Dm), Lp, B, Dm, L, W, stream)
    out[f"B{B}_with_dt_us"] = round(_event_us(lambda: run(True), 50), 2)
    out[f"B{B}_no_dt_us"] = round(_event_us(lambda: run(False), 50), 2)
print(json.dumps(out), flush=True)
