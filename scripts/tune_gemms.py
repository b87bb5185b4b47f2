"""Record TunableOp results for the mixer GEMM shapes of the B=1 streaming chunk
(token-major in_proj / out_proj at L = 3137 and 3136 rows, padded) into
gpurun_out/tunableop_gfx950.csv, starting from the shipped results file.
    python scripts/tune_gemms.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from videomamba_amd import options  # noqa: E402
from videomamba_amd.gemm_tuning import RESULTS  # noqa: E402
from videomamba_amd.videomamba import PretrainVideoMamba  # noqa: E402

out = os.path.join("gpurun_out", "tunableop_gfx950.csv")
os.makedirs("gpurun_out", exist_ok=True)
tun = torch.cuda.tunable
tun.set_filename(out, insert_device_ordinal=False)
tun.read_file(RESULTS)
dev = torch.device("cuda", 0)
model = PretrainVideoMamba(depth=1, embed_dim=576, num_frames=16,
                           add_pool_norm=False).to(dev, torch.bfloat16).eval()
with torch.no_grad(), options.override(gemm_tuning="tune"):
    for B in [int(b) for b in os.environ.get("BATCHES", "1").split(",")]:
        x = torch.randn(B, 3, 16, 224, 224, device=dev, dtype=torch.bfloat16)
        st = model.allocate_state(B, dtype=torch.bfloat16, device=dev)
        model(x, ssm_state=st, temporal_pos_offset=0)   # L = 3137 (CLS chunk)
        model(x, ssm_state=st, temporal_pos_offset=16)  # L = 3136 (continuation)
        print("tuned batch", B, flush=True)
with open(out, "w") as f:  # the results-file format tunable.read_file takes
    for k, v in tun.get_validators():
        f.write(f"Validator,{k},{v}\n")
    for r in tun.get_results():
        f.write(",".join(str(x) for x in r) + "\n")
print(open(out).read())
