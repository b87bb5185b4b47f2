"""M-16f bf16 chunked (2 x 8 frames, fp32 state) vs full, B=1, under host options."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from videomamba_amd import options  # noqa: E402
from videomamba_amd.videomamba import PretrainVideoMamba  # noqa: E402

torch.manual_seed(0)
model = PretrainVideoMamba(depth=32, embed_dim=576, num_frames=16, add_pool_norm=False).cuda().eval()
x = torch.randn(1, 3, 16, 224, 224, device="cuda")
mb = model.to(torch.bfloat16)
xb = x.to(torch.bfloat16)
rel = lambda a, b: ((a.float() - b.float()).norm() / b.float().norm()).item()  # noqa: E731
res = {}
for name, kw in (("cm_fused", dict(mixer_layout="cm")),
                 ("cm_lib", dict(mixer_layout="cm", fused_conv_proj=False)),
                 ("tm", dict(mixer_layout="tm"))):
    with options.override(**kw), torch.no_grad():
        full = mb(xb)
        st = mb.allocate_state(1, dtype=torch.float32)
        c1, st = mb(xb[:, :, :8], ssm_state=st, temporal_pos_offset=0)
        c2, st = mb(xb[:, :, 8:], ssm_state=st, temporal_pos_offset=8)
    s = torch.cat([c1, c2], 1)
    res[name] = full
    print(json.dumps({"opts": name, "rel": rel(s, full), "rel_c1": rel(c1, full[:, :c1.shape[1]]),
                      "rel_c2": rel(c2, full[:, c1.shape[1]:])}), flush=True)
print(json.dumps({"cm_fused_vs_lib": rel(res["cm_fused"], res["cm_lib"]),
                  "cm_fused_vs_tm": rel(res["cm_fused"], res["tm"]),
                  "cm_lib_vs_tm": rel(res["cm_lib"], res["tm"])}), flush=True)
