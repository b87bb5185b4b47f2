"""Which ops break chunked == full at B=1?  M-32f bf16, 2 x 16-frame chunks (fp32 state)
vs one 32-frame pass, under several host options; prints relative L2 differences."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from videomamba_amd import options  # noqa: E402
from videomamba_amd.videomamba import PretrainVideoMamba  # noqa: E402

dev = "cuda"
torch.manual_seed(0)
frames = int(os.environ.get("FRAMES", "32"))
model = PretrainVideoMamba(depth=32, embed_dim=576, num_frames=frames, add_pool_norm=False)
with torch.no_grad():
    model.temporal_pos_embedding.normal_(0, 0.02)
model = model.to(dev).to(torch.bfloat16).eval()
g = torch.Generator(device=dev).manual_seed(4)
x = torch.randn(1, 3, frames, 224, 224, device=dev, generator=g).to(torch.bfloat16)
h = frames // 2
rel = lambda a, b: ((a.float() - b.float()).norm() / b.float().norm()).item()  # noqa: E731
for kw in (dict(), dict(gemm_tuning="off"), dict(mixer_layout="tm", scan_segments=1),
           dict(mixer_layout="tm", scan_segments=1, gemm_tuning="off"),
           dict(mixer_layout="tm"), dict(mixer_layout="tm", fused_conv_proj=False, scan_segments=1)):
    with options.override(**kw), torch.no_grad():
        full = model(x)
        st = model.allocate_state(1, dtype=torch.float32)
        c1, st = model(x[:, :, :h], ssm_state=st, temporal_pos_offset=0)
        c2, st = model(x[:, :, h:], ssm_state=st, temporal_pos_offset=h)
    s = torch.cat([c1, c2], 1)
    print(json.dumps({"opts": kw, "rel": rel(s, full), "rel_chunk2": rel(c2, full[:, c1.shape[1]:]),
                      "bitexact": bool(torch.equal(s, full))}), flush=True)
