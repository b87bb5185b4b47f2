"""Per-kernel cost of a dependent chain of tiny kernels replayed from a captured graph
(the floor under every kernel of the B=1 chunk), plus the B=1 chunk graph replay.
Run under different HIP runtime settings to compare."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
x = torch.zeros(64, device="cuda")
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    for _ in range(3):
        x.add_(1)
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=s):
        for _ in range(400):
            x.add_(1)
torch.cuda.synchronize()
for _ in range(5):
    g.replay()
torch.cuda.synchronize()
ts = []
for _ in range(20):
    t0 = time.perf_counter()
    g.replay()
    torch.cuda.synchronize()
    ts.append(time.perf_counter() - t0)
ts.sort()
print(f"tiny-kernel chain: {ts[10] / 400 * 1e6:.2f} us per kernel (graph of 400)", flush=True)
