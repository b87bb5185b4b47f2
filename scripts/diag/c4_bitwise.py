"""Where does C4's chunked stream (2 x 16-frame chunks, fp32 state) leave the one-pass
32-frame forward at a chip-filling batch?  Runs VideoMamba-M 32f at B clips with depth
1, 2, 4 and 32 and prints, per depth, the relative L2 gap, the count of differing
elements, and the first differing token in each chunk's rows (CLS = token 0).

    python scripts/diag/c4_bitwise.py [--batch 72] [--depths 1,2,4,32]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from videomamba_amd.videomamba import PretrainVideoMamba  # noqa: E402

DEV = "cuda"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=72)
    ap.add_argument("--depths", default="1,2,4,32")
    a = ap.parse_args()
    g = torch.Generator(device=DEV).manual_seed(4)
    x = torch.randn(a.batch, 3, 32, 224, 224, device=DEV, generator=g).to(torch.bfloat16)
    for depth in [int(v) for v in a.depths.split(",")]:
        torch.manual_seed(0)
        model = PretrainVideoMamba(depth=depth, embed_dim=576, num_frames=32, add_pool_norm=False)
        with torch.no_grad():
            model.temporal_pos_embedding.normal_(0, 0.02)
        model = model.to(DEV).to(torch.bfloat16).eval()
        with torch.no_grad():
            full = model(x)
            st = model.allocate_state(a.batch, dtype=torch.float32)
            c1, st = model(x[:, :, :16], ssm_state=st, temporal_pos_offset=0)
            c2, st = model(x[:, :, 16:], ssm_state=st, temporal_pos_offset=16)
        s = torch.cat([c1, c2], 1)
        diff = (s != full).any(-1)  # (B, tokens)
        rel = ((s.float() - full.float()).norm() / full.float().norm()).item()
        n1 = c1.shape[1]
        tok = diff.any(0).nonzero().flatten().tolist()
        first1 = next((t for t in tok if t < n1), None)
        first2 = next((t - n1 for t in tok if t >= n1), None)
        print(json.dumps({"depth": depth, "batch": a.batch, "rel": rel,
                          "differing_elements": int((s != full).sum()),
                          "differing_tokens": len(tok), "clips_differing": int(diff.any(1).sum()),
                          "first_token_chunk1": first1, "first_token_chunk2": first2,
                          "tokens": [n1, c2.shape[1]]}), flush=True)
        del model, full, c1, c2, s, st
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
