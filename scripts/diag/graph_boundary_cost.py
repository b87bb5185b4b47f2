"""Per-kernel fixed cost inside a replayed HIP graph: N dependent tiny kernels (one-element
in-place adds) captured in one graph, replay time / N; and the same for N kernels of a
chunk-like grid (256 workgroups x 512 threads doing nothing but one store).
    python scripts/diag/graph_boundary_cost.py"""
import json
import time

import torch

dev = torch.device("cuda", 0)
out = {}
for n in (50, 200):
    x = torch.zeros(1, device=dev)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            x.add_(1)
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g):
        for _ in range(n):
            x.add_(1)
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(30):
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    out[f"tiny_x{n}_us_per_kernel"] = round(ts[len(ts) // 2] / n * 1e6, 2)
    # a chip-wide grid: 256 x 512 threads, each writes one element
    y = torch.zeros(256 * 512, device=dev)
    g2 = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        y.add_(1)
    torch.cuda.current_stream().wait_stream(s)
    with torch.cuda.graph(g2):
        for _ in range(n):
            y.add_(1)
    for _ in range(5):
        g2.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(30):
        t0 = time.perf_counter()
        g2.replay()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    ts.sort()
    out[f"wide_x{n}_us_per_kernel"] = round(ts[len(ts) // 2] / n * 1e6, 2)
print(json.dumps(out), flush=True)
