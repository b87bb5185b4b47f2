"""options.batch_streams sweep on the bench's model (VideoMamba-M 16x224^2 bf16, one stateful
chunk per step): ms per step for each batch and sub-batch stream count, interleaved rounds.
    python scripts/diag/batch_streams_sweep.py [batches...] [--streams 1,2,3,4] [--rounds 2]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from videomamba_amd import options  # noqa: E402
from videomamba_amd.videomamba import PretrainVideoMamba  # noqa: E402

args = [a for a in sys.argv[1:]]
streams = [1, 2, 3, 4]
rounds = 2
if "--streams" in args:
    i = args.index("--streams")
    streams = [int(v) for v in args[i + 1].split(",")]
    del args[i:i + 2]
if "--rounds" in args:
    i = args.index("--rounds")
    rounds = int(args[i + 1])
    del args[i:i + 2]
batches = [int(a) for a in args] or [448, 224, 112]
dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = PretrainVideoMamba(depth=32, embed_dim=576, num_frames=16, pool_type="cls+avg")
model = model.to(device=dev, dtype=torch.bfloat16).eval()
with torch.no_grad():
    for B in batches:
        g = torch.Generator(device=dev).manual_seed(1000)
        x = torch.randn(B, 3, 16, 224, 224, device=dev, generator=g).to(torch.bfloat16)
        st = model.allocate_state(B, dtype=torch.bfloat16, device=dev)
        for n in streams:  # warm every mode (workspaces per stream)
            with options.override(batch_streams=n, batch_stream_min_clips=2, batch_stream_min_work=0):
                model(x, ssm_state=st, temporal_pos_offset=0)
        for r in range(rounds):
            for n in streams:
                with options.override(batch_streams=n, batch_stream_min_clips=2, batch_stream_min_work=0):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for _ in range(3):
                        model(x, ssm_state=st, temporal_pos_offset=0)
                    torch.cuda.synchronize()
                ms = (time.perf_counter() - t0) / 3 * 1e3
                print(json.dumps({"B": B, "streams": n, "round": r, "ms_per_step": round(ms, 2),
                                  "us_per_clip": round(ms * 1e3 / B, 1)}), flush=True)
        del x, st
        torch.cuda.empty_cache()
