"""Does running the B = 448 bench step as two concurrent half batches on two HIP streams beat
one stream?  (Round 1 measured -16 % with that round's kernels; the kernel mix changed since:
the scan is VALU-issue-bound, the add + norm HBM-bound, the projections MFMA-bound.)
    python scripts/diag/two_streams.py [--rounds 3]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from videomamba_amd.videomamba import PretrainVideoMamba  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = PretrainVideoMamba(depth=32, embed_dim=576, num_frames=16, pool_type="cls+avg")
model = model.to(device=dev, dtype=torch.bfloat16).eval()
B = 448
g = torch.Generator(device=dev).manual_seed(1000)
x = torch.randn(B, 3, 16, 224, 224, device=dev, generator=g).to(torch.bfloat16)
st = model.allocate_state(B, dtype=torch.bfloat16, device=dev)
half = B // 2
xa, xb = x[:half].contiguous(), x[half:].contiguous()
sa = model.allocate_state(half, dtype=torch.bfloat16, device=dev)
sb = model.allocate_state(half, dtype=torch.bfloat16, device=dev)
s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)


def one():
    return model(x, ssm_state=st, temporal_pos_offset=0)


def two():
    cur = torch.cuda.current_stream(dev)
    s1.wait_stream(cur)
    s2.wait_stream(cur)
    with torch.cuda.stream(s1):
        oa = model(xa, ssm_state=sa, temporal_pos_offset=0)
    with torch.cuda.stream(s2):
        ob = model(xb, ssm_state=sb, temporal_pos_offset=0)
    cur.wait_stream(s1)
    cur.wait_stream(s2)
    return oa, ob


rounds = int(sys.argv[sys.argv.index("--rounds") + 1]) if "--rounds" in sys.argv else 3
with torch.no_grad():
    for fn in (one, two):
        fn()
    torch.cuda.synchronize()
    for r in range(rounds):
        for name, fn in (("one_stream", one), ("two_streams", two)):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / 3 * 1e3
            print(json.dumps({"round": r, "mode": name, "ms_per_step": round(ms, 2)}), flush=True)
    o1 = one()[1]
    oa, ob = two()
    print(json.dumps({"pool_bitwise_equal": bool(torch.equal(o1, torch.cat([oa[1], ob[1]])))}), flush=True)
