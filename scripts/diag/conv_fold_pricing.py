"""VERDICT r5 #2 pricing: what folding the depthwise conv + SiLU into the persistent in_proj's
epilogue (x-half tiles write u, x_proj then reads u) would cost and save at the bench's
per-launch batch.  One process per library (product or a build_variant.py probe), HIP
events on the launch stream, VideoMamba-M mixer front shapes, random operands:

  in_proj_us      persistent in_proj (M = B x 3144, N 2304, K 576): product vs tg_convpx
                  (the x tiles' conv + SiLU priced in the epilogue)
  front_us        the mixer's token-major front as the model runs it above the streaming
                  batches: in_proj then conv_proj (conv + SiLU -> u, x_proj -> x_dbl)
  xproj_from_u_us x_proj as a GEMM that reads u (what replaces conv_proj after the fold),
                  timed as F.linear(u, W_x) on hipBLASLt (N = 68)
  conv_proj_us    front_us - in_proj_us

    python scripts/diag/conv_fold_pricing.py <variant|product> [batch]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
name = sys.argv[1]
B = int(sys.argv[2]) if len(sys.argv) > 2 else 448
if name != "product":
    import videomamba_amd._lib as L
    L.LIB_PATH = os.path.join(ROOT, "tools", "probes", os.environ.get("VARIANT_DIR", "var"), name,
                              "libvideomamba_hip.so")
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402
from bench import _event_us  # noqa: E402
from videomamba_amd import kernels as K  # noqa: E402
from videomamba_amd.mamba_simple import Mamba  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
Lp, C = 3144, 576
mx = Mamba(d_model=C, layer_idx=0).to(dev).to(torch.bfloat16).eval()
m = B * Lp
g = torch.Generator(device=dev).manual_seed(1)
hn = torch.randn(B, Lp, C, device=dev, generator=g).to(torch.bfloat16)
out = {"variant": name, "batch": B}
xz = torch.empty(m, 2 * mx.d_inner, device=dev, dtype=torch.bfloat16)
with torch.no_grad():
    out["in_proj_us"] = round(_event_us(
        lambda: K.linear(hn.view(m, C), mx.in_proj.weight, out=xz, form="persistent"), 10), 1)
    out["front_us"] = round(_event_us(
        lambda: mx._tm_front(hn, 3137, None, None, want_dt=False), 10), 1)
    out["conv_proj_us"] = round(out["front_us"] - out["in_proj_us"], 1)
    del xz
    u = torch.randn(m, mx.d_inner, device=dev, generator=g).to(torch.bfloat16)
    wx = mx.x_proj.weight.detach().to(torch.bfloat16)
    F.linear(u, wx)
    out["xproj_from_u_us"] = round(_event_us(lambda: F.linear(u, wx), 10), 1)
print(json.dumps(out), flush=True)
