"""Final norm + pooling tail (vm_norm_pool_fwd with sums, then vm_pool_finish_fwd) at the
M-16f geometry (CLS + 16 frames x 196 tokens, 576 channels, bf16 rows, fp32 residual,
cls+avg), HIP events over graph-replayed launches, and a fingerprint of x_pool:
    python scripts/diag/pool_ab.py [--lib=VARIANT] [--batch=N]
Run once per library (chosen at import); equal fingerprints = same bits."""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
LIB = [a.split("=", 1)[1] for a in sys.argv if a.startswith("--lib=")]
if LIB:  # a probe variant (scripts/diag/build_variant.py)
    import videomamba_amd._lib as L
    L.LIB_PATH = os.path.join(ROOT, "tools", "probes", "var", LIB[0], "libvideomamba_hip.so")
import torch  # noqa: E402
from videomamba_amd import kernels as K  # noqa: E402

B = int(([a.split("=", 1)[1] for a in sys.argv if a.startswith("--batch=")] or ["1"])[0])
dev = torch.device("cuda", 0)
C, T, HW = 576, 16, 196
rows = 1 + T * HW
Lp = (rows + 7) // 8 * 8
g = torch.Generator(device=dev).manual_seed(3)
h = torch.randn(B, Lp, C, device=dev, generator=g).to(torch.bfloat16)
res = torch.randn(B, Lp, C, device=dev, generator=g)
w32 = torch.rand(C, device=dev, generator=g) + 0.5
lnw = torch.rand(C, device=dev, generator=g) + 0.5
lnb = torch.randn(C, device=dev, generator=g) * 0.1
feats = torch.empty(B, rows, C, device=dev, dtype=torch.bfloat16)
box = {}


def run():
    _, ws = K.norm_pool(h, res, rows, w32, None, 1e-5, True, head=1, groups=T, group_rows=HW,
                        sums=True, out=feats)
    box["xp"] = K.pool_finish(ws, feats, mode="cls+avg", keep_temporal=False, groups=T,
                              group_rows=HW, has_cls=True, lnw32=lnw, lnb32=lnb, ln_eps=1e-5)


run()
torch.cuda.synchronize()
fp = hashlib.sha1(box["xp"].float().cpu().numpy().tobytes()).hexdigest()[:16]
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    run()
torch.cuda.current_stream().wait_stream(s)
graph = torch.cuda.CUDAGraph()
with torch.cuda.graph(graph):
    for _ in range(10):
        run()
us = []
for _ in range(5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    graph.replay()
    e1.record()
    torch.cuda.synchronize()
    us.append(round(e0.elapsed_time(e1) * 1e3 / 10, 1))
print(json.dumps({"lib": LIB[0] if LIB else "product", "batch": B, "norm_pool_finish_us": us,
                  "fingerprint": fp}), flush=True)
