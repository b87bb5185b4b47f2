"""vm_linear_fwd timing at the B=1 chunk projection shapes for a probe variant:
python scripts/diag/variant_linear.py <variant|product>"""
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
import torch.nn.functional as F  # noqa: E402
from bench import _event_us  # noqa: E402
from videomamba_amd import kernels as K  # noqa: E402

dev = torch.device("cuda", 0)
out = {"variant": name}
for tag, m, n, k in [("in_proj", 3144, 2304, 576), ("out_proj", 3144, 576, 1152),
                     ("in_proj_b2", 6288, 2304, 576), ("out_proj_b2", 6288, 576, 1152)]:
    x = torch.randn(m, k, device=dev).to(torch.bfloat16)
    w = torch.randn(n, k, device=dev).to(torch.bfloat16)
    out[tag + "_hip_us"] = round(_event_us(lambda: K.linear(x, w), 50), 2)
    ref = (x.float() @ w.float().t())
    err = ((K.linear(x, w).float() - ref).abs().max() / ref.abs().max()).item()
    out[tag + "_maxrel"] = float(f"{err:.2e}")
    out[tag + "_lib_us"] = round(_event_us(lambda: F.linear(x, w), 50), 2)
print(json.dumps(out), flush=True)
