"""conv_proj timing at the B=1 chunk shape (M layer, L=3137) for probe variants
(scripts/diag/build_variant.py): python scripts/diag/variant_conv.py <variant|product>"""
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
from videomamba_amd.mamba_simple import Mamba  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
mx = Mamba(d_model=576, layer_idx=0).to(dev, torch.bfloat16)
Dm, N, R, W = mx.d_inner, mx.d_state, mx.dt_rank, mx.d_conv
E = R + 2 * N
out = {"variant": name}
for B in [int(b) for b in (sys.argv[2:] or ["1"])]:
    L = 3137
    Lp = 3144
    n = B * Lp
    bf = torch.bfloat16
    xz = torch.randn(n, 2 * Dm, device=dev, dtype=bf)
    u = torch.empty(n, Dm, device=dev, dtype=bf)
    dt = torch.empty(n, Dm, device=dev, dtype=bf)
    xd = torch.empty(n, E, device=dev, dtype=bf)
    cs_in = torch.randn(B, Dm, W, device=dev, dtype=bf)
    cs_out = torch.empty(B, Dm, W, device=dev, dtype=bf)
    _, _, _, cw, cb = mx._fp32_params()
    wx_pad, wdt_pad = mx._padded_proj_weights()
    st = torch.cuda.current_stream(dev).cuda_stream
    us = _event_us(lambda: K.conv_proj_raw(
        xz, (Lp * 2 * Dm, 2 * Dm), cw, cb, cs_in, (cs_in.stride(0), cs_in.stride(1)), cs_out,
        (cs_out.stride(0), cs_out.stride(1)), wx_pad, E, wdt_pad, R, u, (Lp * Dm, Dm), xd,
        (Lp * E, E), dt, (Lp * Dm, Dm), Lp, B, Dm, L, W, st), 50)
    out[f"B{B}_us"] = round(us, 2)
    # without dt rows (the dt_proj-in-scan mixer's call, the bench's above 8 clips)
    us = _event_us(lambda: K.conv_proj_raw(
        xz, (Lp * 2 * Dm, 2 * Dm), cw, cb, cs_in, (cs_in.stride(0), cs_in.stride(1)), cs_out,
        (cs_out.stride(0), cs_out.stride(1)), wx_pad, E, None, R, u, (Lp * Dm, Dm), xd,
        (Lp * E, E), None, None, Lp, B, Dm, L, W, st), 50)
    out[f"B{B}_nodt_us"] = round(us, 2)
print(json.dumps(out), flush=True)
