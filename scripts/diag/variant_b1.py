"""Per-stage B = 1 layer timings (bench.b1_kernel_rooflines: each stage of one VideoMamba-M
layer at the one-clip chunk shape, HIP events) of a probe build or the product:
    python scripts/diag/variant_b1.py <variant|product>"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
name = sys.argv[1]
if name != "product":
    import videomamba_amd._lib as L
    L.LIB_PATH = os.path.join(ROOT, "tools", "probes", "var", name, "libvideomamba_hip.so")
import torch  # noqa: E402
from bench import b1_kernel_rooflines  # noqa: E402

r = b1_kernel_rooflines(torch.device("cuda", 0), reps=100)
print(json.dumps({"variant": name, **{k: v["us"] for k, v in r.items() if isinstance(v, dict)},
                  "sum": r["layer_us_sum"]}), flush=True)
