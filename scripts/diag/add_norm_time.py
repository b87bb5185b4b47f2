"""vm_add_norm_fwd at the bench shape (448 clips x 3144 rows x 576, bf16 x + fp32 residual in
place, bf16 out), HIP events; a probe variant by name:
    python scripts/diag/add_norm_time.py <variant|product>"""
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
from bench import _event_us  # noqa: E402
from videomamba_amd import kernels as K  # noqa: E402

dev = torch.device("cuda", 0)
out = {"variant": name}
for tag, rows in (("b448", 448 * 3144), ("b1", 3144)):
    cols = 576
    x = torch.randn(rows, cols, device=dev).to(torch.bfloat16)
    r = torch.randn(rows, cols, device=dev)
    w = torch.ones(cols, device=dev)
    o = torch.empty(rows, cols, device=dev, dtype=torch.bfloat16)
    st = torch.cuda.current_stream().cuda_stream
    us = _event_us(lambda: K.add_norm_raw(x, r, w, None, o, r, rows, cols, 1e-5, True, st), 20)
    out[tag + "_us"] = round(us, 2)
    out[tag + "_TBps"] = round(rows * cols * 12 / us / 1e6, 2)
print(json.dumps(out), flush=True)
