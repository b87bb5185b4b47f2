"""Cross-calibrate the CPU baseline: the oracle's fp32 B=1 forward (oracle/videomamba_oracle.py,
the timed leg of bench.py's cpu_baseline) on N threads against the reference's own CPU path
measured in the survey container (8 threads, Ti-8f 3.32 s/clip, M-16f 24.9 s/clip).
Writes one JSON line; the committed result is profiles/r02_cpu_calibration.json.
    python scripts/cpu_calibration.py --threads 8
"""
import argparse
import json
import os
import platform
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import CONFIGS, _oracle_clip_seconds  # noqa: E402

REFERENCE_8T = {"ti8": 3.32, "m16": 24.9}  # s/clip, BASELINE.md "Reference CPU path" table

ap = argparse.ArgumentParser()
ap.add_argument("--threads", type=int, default=8)
ap.add_argument("--configs", nargs="+", default=["ti8", "m16"])
a = ap.parse_args()
torch.set_num_threads(a.threads)
out = {"threads": a.threads, "host": platform.processor() or platform.machine(),
       "cpu_count": os.cpu_count(), "torch": torch.__version__, "configs": {}}
for name in a.configs:
    s = _oracle_clip_seconds(CONFIGS[name])
    ref = REFERENCE_8T[name]
    out["configs"][name] = {"oracle_s_per_clip": round(s, 3), "reference_s_per_clip": ref,
                            "oracle_over_reference": round(s / ref, 3)}
    print(json.dumps({name: out["configs"][name]}), flush=True)
print(json.dumps(out))
