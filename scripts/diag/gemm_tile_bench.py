"""Projection GEMMs at the bench batch: hipBLASLt (TunableOp-tuned F.linear, what the mixer
ran above 8 clips through round 3), the 128-row LDS-DMA HIP kernel and the persistent
256-row HIP kernel (vm_gemm_tile.hip).  Interleaved rounds in one process, HIP events on
the launch stream, random bf16 operands; prints one JSON line per (shape, form) with the
median ms and PFLOP/s, and checks the two HIP forms bit for bit.

    python scripts/diag/gemm_tile_bench.py [--batch 448] [--rounds 5] [--reps 20]
"""
import argparse
import json
import os
import statistics
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from videomamba_amd import kernels as K  # noqa: E402
from videomamba_amd.gemm_tuning import tuned  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=448)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--forms", default="lib,dma,persistent")
    a = ap.parse_args()
    dev = torch.device("cuda")
    m = a.batch * 3144
    shapes = {"in_proj": (2304, 576), "out_proj": (576, 1152)}
    forms = a.forms.split(",")
    for name, (n, k) in shapes.items():
        x = (torch.rand(m, k, device=dev) * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(n, k, device=dev) * 2 - 1) * k ** -0.5).to(torch.bfloat16)
        out = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
        # the LDS-DMA form addresses x through one 31-bit buffer: time it on row slabs
        slab = max(256, ((1 << 31) - 1) // (2 * k) // 256 * 256)
        fns = {"lib": lambda: _lib_mm(x, w, out),
               "dma": lambda: [K.linear(x[r:r + slab], w, out=out[r:r + slab], form="dma")
                               for r in range(0, m, slab)],
               "persistent": lambda: K.linear(x, w, out=out, form="persistent")}
        if "dma" in forms and "persistent" in forms:
            pre = min(m, 200000)
            a1 = K.linear(x[:pre], w, form="dma")
            a2 = K.linear(x, w, form="persistent")[:pre]
            torch.cuda.synchronize()
            print(json.dumps({"shape": name, "bitwise_dma_vs_persistent": bool(torch.equal(a1, a2))}),
                  flush=True)
            del a1, a2
        times = {f: [] for f in forms}
        for f in forms:
            for _ in range(3):
                fns[f]()
        torch.cuda.synchronize()
        for _ in range(a.rounds):
            for f in forms:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(a.reps):
                    fns[f]()
                e1.record()
                torch.cuda.synchronize()
                times[f].append(e0.elapsed_time(e1) / a.reps)
        flops = 2.0 * m * n * k
        for f in forms:
            med = statistics.median(times[f])
            print(json.dumps({"shape": name, "m": m, "n": n, "k": k, "form": f,
                              "ms_median": round(med, 4), "ms_min": round(min(times[f]), 4),
                              "pflops": round(flops / med / 1e12, 4)}), flush=True)
        del x, w, out


def _lib_mm(x, w, out):
    with tuned():
        torch.mm(x, w.t(), out=out)


if __name__ == "__main__":
    main()
