"""Eager B=1 M-16f stateful chunks under one mixer layout (for rocprofv3 kernel stats)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from videomamba_amd import options  # noqa: E402
from videomamba_amd.videomamba import PretrainVideoMamba  # noqa: E402

lay = sys.argv[1] if len(sys.argv) > 1 else "auto"
torch.manual_seed(0)
model = PretrainVideoMamba(depth=32, embed_dim=576, num_frames=16).cuda().to(torch.bfloat16).eval()
x = torch.randn(1, 3, 16, 224, 224, device="cuda").to(torch.bfloat16)
st = model.allocate_state(1, dtype=torch.bfloat16)
with options.override(mixer_layout=lay), torch.no_grad():
    for _ in range(10):
        model(x, ssm_state=st, temporal_pos_offset=0)
torch.cuda.synchronize()
print("done", lay)
