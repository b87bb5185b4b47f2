"""Which kernels make C5's chunked stream differ from the one-pass 1,024-frame forward?
Per-chunk relative L2 (16 x chunk64, fp32 carried state, bf16 model) under host options
that make parts of the path row-invariant:
  default          library in/out_proj GEMMs (M-dependent kernel choice), segmented scan
  gemm_inv         in_proj / out_proj on vm_linear_fwd at every M (row order fixed)
  scan1            the single-pass scan (no segment composition)
  gemm_inv+scan1   both
    python scripts/diag/c5_invariance.py [--frames 1024]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from videomamba_amd import options  # noqa: E402
from videomamba_amd.videomamba import PretrainVideoMamba  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=1024)
ap.add_argument("--variants", nargs="+", default=["default", "gemm_inv", "scan1", "gemm_inv+scan1"])
a = ap.parse_args()

VARIANTS = {"default": {}, "gemm_inv": dict(small_gemm_rows=1 << 30, small_gemm_max_n=1 << 20),
            "scan1": dict(scan_segments=1),
            "gemm_inv+scan1": dict(small_gemm_rows=1 << 30, small_gemm_max_n=1 << 20,
                                   scan_segments=1)}
DEV = "cuda"
torch.manual_seed(0)
model = PretrainVideoMamba(depth=32, embed_dim=576, num_frames=a.frames, add_pool_norm=False)
with torch.no_grad():
    model.temporal_pos_embedding.normal_(0, 0.02)
model = model.to(DEV).to(torch.bfloat16).eval()
g = torch.Generator(device=DEV).manual_seed(6)
x = torch.randn(1, 3, a.frames, 224, 224, device=DEV, generator=g).to(torch.bfloat16)
nch = a.frames // 64
rel = lambda p, q: ((p.float() - q.float()).norm() / q.float().norm()).item()  # noqa: E731
for name in a.variants:
    t0 = time.time()
    with options.override(**VARIANTS[name]), torch.no_grad():
        full = model(x)
        st = model.allocate_state(1, dtype=torch.float32)
        rs = []
        for c in range(nch):
            out, st = model(x[:, :, 64 * c:64 * (c + 1)], ssm_state=st, temporal_pos_offset=64 * c)
            lo = 0 if c == 0 else 1 + 12544 * c
            rs.append(rel(out, full[:, lo:1 + 12544 * (c + 1)]))
    torch.cuda.synchronize()
    print(json.dumps({"variant": name, "worst": max(rs), "per_chunk": [f"{r:.2e}" for r in rs],
                      "s": round(time.time() - t0, 1)}), flush=True)
