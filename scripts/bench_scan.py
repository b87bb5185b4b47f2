"""Scan-kernel microbenchmark at VideoMamba-M geometry (D=1152, L=3137, N=16, bf16,
stateful); prints one JSON line per batch.
    python scripts/bench_scan.py --batches 1 4 8 --layout cm
    python scripts/bench_scan.py --batches 1 --layout tm --segments 8
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import scan_roofline  # noqa: E402
from videomamba_amd import options  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batches", type=int, nargs="+", default=[1, 4, 8])
ap.add_argument("--reps", type=int, default=30)
ap.add_argument("--layout", default="tm", choices=["tm", "cm"])
ap.add_argument("--segments", type=int, default=0, help="token-major segment count (0 = auto)")
ap.add_argument("--dtp", action="store_true",
                help="the dt_proj-in-scan kernel (vm_selective_scan_dtproj_fwd) the bench runs")
a = ap.parse_args()
dev = torch.device("cuda", 0)
with options.override(scan_segments=a.segments):
    for B in a.batches:
        r = scan_roofline(B, a.reps, dev, a.layout, dtp=a.dtp)
        r["segments"] = a.segments
        r["us_per_clip_layer"] = round(r["avg_us"] / B, 2)
        print(json.dumps(r), flush=True)
