"""Persistent-GEMM timing at the bench's B = 448 projection shapes for a probe variant
(scripts/diag/build_variant.py), HIP events, with an exact integer checksum of the output
so variants that must be bit-identical can be compared across processes:
    python scripts/diag/variant_gemm448.py <variant|product>"""
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
m = 448 * 3144
out = {"variant": name}
for tag, n, k in (("in_proj", 2304, 576), ("out_proj", 576, 1152)):
    g = torch.Generator(device=dev).manual_seed(n + k)
    x = (torch.rand(m, k, device=dev, generator=g) * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(n, k, device=dev, generator=g) * 2 - 1) * k ** -0.5).to(torch.bfloat16)
    o = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
    fn = lambda: K.linear(x, w, out=o, form="persistent")  # noqa: E731
    out[tag + "_us"] = round(_event_us(fn, 10), 1)
    out[tag + "_pflops"] = round(2.0 * m * n * k / out[tag + "_us"] / 1e9, 3)
    out[tag + "_checksum"] = int(o.view(torch.int16).to(torch.int64).sum().item())
    del x, o
    torch.cuda.empty_cache()
print(json.dumps(out), flush=True)
