"""Sub-batch streams with / without a priority difference (the first half's stream at high
priority), B = 896 M-16f stateful chunk, interleaved rounds:
    python scripts/diag/stream_priority.py"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from videomamba_amd import videomamba as V  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = V.PretrainVideoMamba(depth=32, embed_dim=576, num_frames=16, pool_type="cls+avg")
model = model.to(device=dev, dtype=torch.bfloat16).eval()
B = 896
g = torch.Generator(device=dev).manual_seed(1000)
x = torch.randn(B, 3, 16, 224, 224, device=dev, generator=g).to(torch.bfloat16)
st = model.allocate_state(B, dtype=torch.bfloat16, device=dev)
key = (dev.type, dev.index)
plain = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
lo, hi = torch.cuda.Stream.priority_range() if hasattr(torch.cuda.Stream, "priority_range") else (0, -1)
prio = [torch.cuda.Stream(dev, priority=-1), torch.cuda.Stream(dev, priority=0)]
with torch.no_grad():
    for mode, ss in (("plain", plain), ("prio", prio)):
        V._SIDE_STREAMS.by_device = {key: ss}  # this thread's side streams
        model(x, ssm_state=st, temporal_pos_offset=0)
    for r in range(3):
        for mode, ss in (("plain", plain), ("prio", prio)):
            V._SIDE_STREAMS.by_device = {key: ss}  # this thread's side streams
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                model(x, ssm_state=st, temporal_pos_offset=0)
            torch.cuda.synchronize()
            print(json.dumps({"round": r, "mode": mode, "ms_per_step": round((time.perf_counter() - t0) / 3 * 1e3, 2)}), flush=True)
