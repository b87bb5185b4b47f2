"""Repeatability at a chip-filling batch (the bench's kernel forms): the persistent HIP GEMM
at the in_proj / out_proj shapes, and whole VideoMamba-M forwards (depth 32, 16 frames),
each repeated and compared bitwise.  Prints one JSON line.

    python scripts/diag/determinism_b72.py [--batch 72] [--gemm-reps 30] [--model-reps 3]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from videomamba_amd import kernels as K  # noqa: E402
from videomamba_amd.videomamba import PretrainVideoMamba  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=72)
    ap.add_argument("--gemm-reps", type=int, default=30)
    ap.add_argument("--model-reps", type=int, default=3)
    ap.add_argument("--shapes", default="in_proj,out_proj")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    out = {"batch": a.batch}
    g = torch.Generator(device=dev).manual_seed(0)
    m = a.batch * 3144
    shapes = {"in_proj": (2304, 576), "out_proj": (576, 1152)}
    for tag in a.shapes.split(","):
        n, k = shapes[tag]
        x = torch.randn(m, k, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(n, k, device=dev, generator=g) * k ** -0.5).to(torch.bfloat16)
        r0 = K.linear(x, w, form="persistent")
        bad, rows = 0, set()
        for _ in range(a.gemm_reps):
            r = K.linear(x, w, form="persistent")
            if not torch.equal(r, r0):
                bad += 1
                rows.update((r != r0).any(1).nonzero().flatten()[:8].tolist())
        out[tag + "_mismatch_runs"] = bad
        out[tag + "_rows"] = sorted(rows)[:16]
        del x, w, r0
    if a.model_reps <= 0:
        print(json.dumps(out), flush=True)
        return
    torch.manual_seed(0)
    model = PretrainVideoMamba(depth=32, embed_dim=576, num_frames=16, add_pool_norm=False)
    model = model.to(dev, torch.bfloat16).eval()
    x = torch.randn(a.batch, 3, 16, 224, 224, device=dev, generator=g).to(torch.bfloat16)
    with torch.no_grad():
        f0 = model(x)
        res = []
        for _ in range(a.model_reps):
            f = model(x)
            d = (f != f0).any(-1)
            res.append({"equal": bool(torch.equal(f, f0)), "clips": int(d.any(1).sum()),
                        "tokens": int(d.any(0).sum())})
    out["model_runs"] = res
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
