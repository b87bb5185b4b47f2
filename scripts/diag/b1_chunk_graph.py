"""B=1 M-16f stateful chunks replayed from the captured HIP graph (the bench's chunk_p50
path), for rocprofv3 kernel stats: python scripts/diag/b1_chunk_graph.py [replays]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from videomamba_amd.graphs import StreamingChunkGraph  # noqa: E402
from videomamba_amd.videomamba import PretrainVideoMamba  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
batch = 1
for kv in list(sys.argv[2:]):  # lib=<path>: a probe build of the library (A/B); batch=<clips>
    if kv.startswith("batch="):
        batch = int(kv[6:])
        sys.argv.remove(kv)
    if kv.startswith("lib="):
        import videomamba_amd._lib as L
        L.LIB_PATH = os.path.abspath(kv[4:])
        sys.argv.remove(kv)
if len(sys.argv) > 2:  # option overrides, e.g. small_gemm_max_n=4096
    from videomamba_amd import options
    for kv in sys.argv[2:]:
        k, v = kv.split("=")
        t = type(getattr(options.get(), k))
        val = v.lower() in ("1", "true", "yes", "on") if t is bool else t(v)
        options._OPTS = options.dataclasses.replace(options.get(), **{k: val})
torch.manual_seed(0)
model = PretrainVideoMamba(depth=32, embed_dim=576, num_frames=16).cuda().to(torch.bfloat16).eval()
x = torch.randn(batch, 3, 16, 224, 224, device="cuda").to(torch.bfloat16)
runner = StreamingChunkGraph(model, batch=batch, frames=16)
with torch.no_grad():
    for _ in range(2):  # captures both conv-state buffer parities
        runner.run(x, temporal_pos_offset=0)
    torch.cuda.synchronize()
    lat = []
    for _ in range(n):
        t0 = time.perf_counter()
        runner.run(x, temporal_pos_offset=0)
        torch.cuda.synchronize()
        lat.append((time.perf_counter() - t0) * 1e3)
    g, _ = runner._graphs[(True, runner._cur)]
    rep = []
    for _ in range(n):
        t0 = time.perf_counter()
        g.replay()
        torch.cuda.synchronize()
        rep.append((time.perf_counter() - t0) * 1e3)
    key = []
    for _ in range(n):
        t0 = time.perf_counter()
        runner._params_key()
        key.append((time.perf_counter() - t0) * 1e3)
lat.sort()
rep.sort()
key.sort()
print(f"{sys.argv[2:]} graph replays {n}: run() p50 {lat[n // 2]:.3f} ms  min {lat[0]:.3f} ms; "
      f"replay-only p50 {rep[n // 2]:.3f} ms; params-key p50 {key[n // 2]:.3f} ms")
