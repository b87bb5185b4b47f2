"""Scan timing of probe variants (scripts/diag/build_variant.py) against the product build:
    python scripts/diag/variant_scan.py <variant|product> [batches...]
One JSON line per batch (scan_roofline at the M-16f shape, token-major layout)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
name = sys.argv[1]
if name != "product":
    import videomamba_amd._lib as L
    L.LIB_PATH = os.path.join(ROOT, "tools", "probes", "var", name, "libvideomamba_hip.so")
    abi = [a for a in sys.argv[2:] if a.startswith("--abi=")]
    if abi:  # an older build (same entry points) for a same-box A/B
        L.ABI_VERSION = int(abi[0].split("=")[1])
        sys.argv = [a for a in sys.argv if not a.startswith("--abi=")]
import torch  # noqa: E402
from bench import scan_roofline  # noqa: E402

dev = torch.device("cuda", 0)
args = sys.argv[2:]
dtp = "--dtp" in args
for B in [int(b) for b in ([a for a in args if a != "--dtp"] or ["1", "336"])]:
    r = scan_roofline(B, 30, dev, "tm", dtp=dtp)
    print(json.dumps({"variant": name, "dtp": dtp, "B": B, "kernel": r["kernel"],
                      "avg_us": r["avg_us"], "frac": r["frac"]}), flush=True)
