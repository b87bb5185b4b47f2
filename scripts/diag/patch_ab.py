"""Patch-embed launch time at the bench's per-launch batch (448 clips of 3x16x224^2 bf16,
VideoMamba-M embed 576), HIP events, and an output fingerprint to compare libraries by.
    python scripts/diag/patch_ab.py [--lib=VARIANT] [--batch=N]
Run once per library (the library is chosen at import); equal fingerprints = same bits."""
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
from bench import _event_us  # noqa: E402
from videomamba_amd import kernels as K  # noqa: E402

B = int(([a.split("=", 1)[1] for a in sys.argv if a.startswith("--batch=")] or ["448"])[0])
dev = torch.device("cuda", 0)
C, T, HW, P = 576, 16, 224, 16
g = torch.Generator(device=dev).manual_seed(7)
video = torch.randn(B, 3, T, HW, HW, device=dev, generator=g).to(torch.bfloat16)
w = (torch.randn(C, 3, 1, P, P, device=dev, generator=g) * 0.02).to(torch.bfloat16)
bias = torch.randn(C, device=dev, generator=g).to(torch.bfloat16)
ntok = (HW // P) ** 2
spos = torch.randn(ntok, C, device=dev, generator=g).to(torch.bfloat16)
tpos = torch.randn(T, C, device=dev, generator=g).to(torch.bfloat16)
cls = torch.randn(C, device=dev, generator=g).to(torch.bfloat16)
cls_pos = torch.randn(C, device=dev, generator=g).to(torch.bfloat16)
L_rows = 1 + T * ntok + 7
out = torch.empty(B, L_rows, C, device=dev, dtype=torch.bfloat16)


def run():
    K.patch_embed(video, w, bias, spos, tpos, out, 1, L_rows * C, cls=cls, cls_pos=cls_pos,
                  pad_rows=7)


run()
torch.cuda.synchronize()
fp = hashlib.sha1(out.view(torch.int16).cpu().numpy().tobytes()).hexdigest()[:16]
us = [round(_event_us(run, 10), 1) for _ in range(5)]
# the same launches replayed from a HIP graph (the fp32 bias cached): no host work between
# them, so small batches time the kernel, not the wrapper
b32 = bias.float()


def run32():
    K.patch_embed(video, w, bias, spos, tpos, out, 1, L_rows * C, cls=cls, cls_pos=cls_pos,
                  pad_rows=7, bias32=b32)


s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    run32()
torch.cuda.current_stream().wait_stream(s)
graph = torch.cuda.CUDAGraph()
with torch.cuda.graph(graph):
    for _ in range(20):
        run32()
gus = []
for _ in range(5):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    graph.replay()
    e1.record()
    torch.cuda.synchronize()
    gus.append(round(e0.elapsed_time(e1) * 1e3 / 20, 1))
print(json.dumps({"lib": LIB[0] if LIB else "product", "batch": B, "patch_us": us,
                  "graph_us": gus, "fingerprint": fp}), flush=True)
