"""Chunked token-major scan, one launch (sync flags) vs two launches, at M-16f geometry:
python scripts/diag/scan_one_launch.py  (HIP events over back-to-back launches)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from bench import scan_roofline  # noqa: E402
from videomamba_amd import options  # noqa: E402

dev = torch.device("cuda", 0)
for B in (1, 2, 4):
    row = {"B": B}
    for one in (False, True, False, True):
        with options.override(scan_one_launch=one):
            r = scan_roofline(B, 30, dev, "tm")
        row.setdefault("one_launch_us" if one else "two_launch_us", []).append(r["avg_us"])
    print(json.dumps(row), flush=True)
