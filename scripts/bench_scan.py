"""Scan-kernel microbenchmark at VideoMamba-M geometry (D=1152, L=3137, N=16, bf16,
stateful) for the variant selected by VM_SCAN_VARIANT; prints one JSON line per batch.
    VM_SCAN_VARIANT=3 python scripts/bench_scan.py --batches 1 4 8 --layout cm
    VM_SCAN_SEGMENTS=8 python scripts/bench_scan.py --batches 1 --layout tm
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import scan_roofline  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batches", type=int, nargs="+", default=[1, 4, 8])
ap.add_argument("--reps", type=int, default=30)
ap.add_argument("--layout", default="tm", choices=["tm", "cm"])
a = ap.parse_args()
dev = torch.device("cuda", 0)
for B in a.batches:
    r = scan_roofline(B, a.reps, dev, a.layout)
    r["variant"] = int(os.environ.get("VM_SCAN_VARIANT", "0"))
    r["segments_env"] = os.environ.get("VM_SCAN_SEGMENTS", "")
    r["us_per_clip_layer"] = round(r["avg_us"] / B, 2)
    print(json.dumps(r), flush=True)
