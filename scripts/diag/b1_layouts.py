"""B=1 M-16f stateful chunk latency (hipGraph replay) under host options."""
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from videomamba_amd import options  # noqa: E402
from videomamba_amd.graphs import StreamingChunkGraph  # noqa: E402
from videomamba_amd.videomamba import PretrainVideoMamba  # noqa: E402

dev = "cuda"
torch.manual_seed(0)
model = PretrainVideoMamba(depth=32, embed_dim=576, num_frames=16).to(dev).to(torch.bfloat16).eval()
x = torch.randn(1, 3, 16, 224, 224, device=dev).to(torch.bfloat16)
configs = [dict(mixer_layout="cm", fused_conv_proj=False), dict(mixer_layout="cm"),
           dict(mixer_layout="tm")] + [dict(mixer_layout="tm", scan_segments=s) for s in (48, 64, 96)]
for kw in configs:
    with options.override(**kw), torch.no_grad():
        runner = StreamingChunkGraph(model, batch=1, frames=16)
        lat = []
        for i in range(23):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            runner.run(x, temporal_pos_offset=0)
            torch.cuda.synchronize()
            if i >= 3:
                lat.append((time.perf_counter() - t0) * 1e3)
    print(json.dumps({"opts": kw, "p50_ms": round(statistics.median(lat), 3)}), flush=True)
