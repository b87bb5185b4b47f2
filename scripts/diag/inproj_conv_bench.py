"""B = 1 M-16f layer front timed from HIP graphs (20 calls per graph, 10 replays, HIP events):
in_proj (vm_linear_fwd) + conv_proj (vm_conv_proj_fwd, no dt) against vm_in_proj_conv_proj_fwd
(+ its reduce).  python scripts/diag/inproj_conv_bench.py <variant|product> [batch]
Variants from scripts/diag/build_variant.py with VARIANT_DIR=ab."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
name = sys.argv[1]
if name != "product":
    import videomamba_amd._lib as L
    L.LIB_PATH = os.path.join(ROOT, "tools", "probes", "ab", name, "libvideomamba_hip.so")
import torch  # noqa: E402
from videomamba_amd import kernels as K  # noqa: E402
from videomamba_amd.mamba_simple import Mamba  # noqa: E402

B = int(sys.argv[2]) if len(sys.argv) > 2 else 1
dev = "cuda"
torch.manual_seed(0)
m = Mamba(d_model=576, layer_idx=0).to(dev, torch.bfloat16)
C, Dm, E, R, W = 576, m.d_inner, m.dt_rank + 2 * m.d_state, m.dt_rank, m.d_conv
_, _, _, cw, cb = m._fp32_params()
wx_pad, wdt_pad = m._padded_proj_weights()
L, Lp = 3137, 3144
n = B * Lp
hn = torch.randn(n, C, device=dev).to(torch.bfloat16)
cs = torch.randn(B, Dm, W, device=dev).to(torch.bfloat16)
cso = torch.empty(B, Dm, W, device=dev, dtype=torch.bfloat16)
xz = torch.empty(n, 2 * Dm, device=dev, dtype=torch.bfloat16)
u = torch.empty(n, Dm, device=dev, dtype=torch.bfloat16)
xd = torch.empty(n, E, device=dev, dtype=torch.bfloat16)
ws = torch.empty(1 << 26, dtype=torch.uint8, device=dev)


def two():
    st = torch.cuda.current_stream().cuda_stream
    K.linear(hn, m.in_proj.weight, out=xz)
    K.conv_proj_raw(xz, (Lp * 2 * Dm, 2 * Dm), cw, cb, cs, (Dm * W, W), cso, (Dm * W, W),
                    wx_pad, E, None, R, u, (Lp * Dm, Dm), xd, (Lp * E, E), None, (Lp * Dm, Dm),
                    Lp, B, Dm, L, W, st)


def inproj():
    K.linear(hn, m.in_proj.weight, out=xz)


def fused():
    st = torch.cuda.current_stream().cuda_stream
    K.in_proj_conv_proj_raw(hn, m.in_proj.weight, xz[:, Dm:], cw, cb, cs, (Dm * W, W), cso,
                            (Dm * W, W), wx_pad, E, wdt_pad, R, u, xd, None, Lp, B, Dm, L, W, st)


def timed(fn, calls=20, reps=10):
    with K.scratch_override(ws):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(3):
                fn()
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(calls):
                fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (calls * reps)


res = {"variant": name, "B": B}
for k, fn in (("in_proj_us", inproj), ("in_proj_plus_conv_proj_us", two), ("fused_us", fused)):
    res[k] = round(timed(fn), 2)
print(json.dumps(res), flush=True)
