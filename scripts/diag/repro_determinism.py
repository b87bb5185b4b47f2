"""Repeatability of the B <= 8 streaming-batch kernels for a probe variant (or the product):
the HIP GEMM (vm_linear_fwd) at the in_proj / out_proj shapes, the one-launch chunked scan,
and a depth-1 VideoMamba-M bf16 forward at B = 2, each run repeatedly and compared bitwise.
    python scripts/diag/repro_determinism.py <variant|product>"""
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
from bench import scan_roofline  # noqa: F401,E402
from videomamba_amd import kernels as K  # noqa: E402
from videomamba_amd.videomamba import PretrainVideoMamba  # noqa: E402

dev = torch.device("cuda", 0)
out = {"variant": name}
g = torch.Generator(device=dev).manual_seed(0)
for tag, m, n, k in [("in_proj", 6288, 2304, 576), ("out_proj", 6288, 576, 1152)]:
    x = torch.randn(m, k, device=dev, generator=g).to(torch.bfloat16)
    w = torch.randn(n, k, device=dev, generator=g).to(torch.bfloat16)
    r0 = K.linear(x, w)
    bad = sum(int(not torch.equal(K.linear(x, w), r0)) for _ in range(20))
    ref = x.float() @ w.float().t()
    out[tag + "_mismatch_runs"] = bad
    out[tag + "_maxrel"] = float(f"{((r0.float() - ref).abs().max() / ref.abs().max()).item():.2e}")
torch.manual_seed(1)
model = PretrainVideoMamba(depth=1, embed_dim=576, num_frames=16, pool_type="avg")
model = model.to(dev, torch.bfloat16).eval()
x = torch.randn(2, 3, 16, 224, 224, device=dev, dtype=torch.bfloat16)
with torch.no_grad():
    f0 = model.forward_features(x)
    fb = [int(not torch.equal(model.forward_features(x), f0)) for _ in range(10)]
    xv = [int(not torch.equal(model(x)[0], f0[:, 1:])) for _ in range(10)]
out["forward_features_mismatch_runs"] = sum(fb)
out["forward_vs_features_mismatch_runs"] = sum(xv)
print(json.dumps(out), flush=True)
