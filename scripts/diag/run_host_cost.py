"""Where StreamingChunkGraph.run()'s time goes beyond the bare replay (B=1 M-16f chunk):
host time of each step of run() and the synchronised wall time of the pieces.
python scripts/diag/run_host_cost.py [n]"""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from videomamba_amd.graphs import StreamingChunkGraph  # noqa: E402
from videomamba_amd.videomamba import PretrainVideoMamba  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100
torch.manual_seed(0)
model = PretrainVideoMamba(depth=32, embed_dim=576, num_frames=16).cuda().to(torch.bfloat16).eval()
x = torch.randn(1, 3, 16, 224, 224, device="cuda").to(torch.bfloat16)
runner = StreamingChunkGraph(model, batch=1, frames=16)


def p50(fn, sync=True):
    lat = []
    for i in range(n + 3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        if sync:
            torch.cuda.synchronize()
        if i >= 3:
            lat.append((time.perf_counter() - t0) * 1e6)
    return statistics.median(lat)


with torch.no_grad():
    for _ in range(2):
        runner.run(x, temporal_pos_offset=0)
    torch.cuda.synchronize()
    g, _ = runner._graphs[(True, runner._cur)]
    res = {
        "run_us": p50(lambda: runner.run(x, temporal_pos_offset=0)),
        "run_host_us": p50(lambda: runner.run(x, temporal_pos_offset=0), sync=False),
        "replay_us": p50(g.replay),
        "replay_host_us": p50(g.replay, sync=False),
        "copy_replay_us": p50(lambda: (runner.static_x.copy_(x), g.replay())),
        "copy_us": p50(lambda: runner.static_x.copy_(x)),
        "copy_host_us": p50(lambda: runner.static_x.copy_(x), sync=False),
        "params_key_host_us": p50(runner._params_key, sync=False),
        "sync_only_us": p50(lambda: None),
    }
print({k: round(v, 1) for k, v in res.items()})
