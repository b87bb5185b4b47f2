"""Step-by-step check of vm_conv_proj_cm_fwd on the GPU (progress printed per step)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from videomamba_amd import kernels as K  # noqa: E402
from videomamba_amd.mamba_simple import Mamba  # noqa: E402

dev = "cuda"
for (Bsz, L, d_model) in [(1, 70, 64), (2, 301, 96), (1, 3137, 576)]:
    t0 = time.time()
    m = Mamba(d_model=d_model, d_state=16, d_conv=4, expand=2, layer_idx=0).to(dev, torch.bfloat16)
    Dm, E, R, W = m.d_inner, m.dt_rank + 2 * m.d_state, m.dt_rank, m.d_conv
    _, _, _, cw, cb = m._fp32_params()
    wx_pad, wdt_pad = m._padded_proj_weights()
    Lp = (L + 7) // 8 * 8
    n = Bsz * Lp
    xz = torch.randn(2 * Dm, n, device=dev).to(torch.bfloat16)
    u = torch.empty(Dm, n, device=dev, dtype=torch.bfloat16)
    xd = torch.empty(E, n, device=dev, dtype=torch.bfloat16)
    dt = torch.empty(Dm, n, device=dev, dtype=torch.bfloat16)
    print("launch", Bsz, L, d_model, "ws", K.conv_proj_cm_workspace_bytes(Bsz, Lp, Dm, E), flush=True)
    K.conv_proj_cm_raw(xz, n, cw, cb, None, (0, 0), None, (0, 0), wx_pad, E, wdt_pad, R, u, n,
                       xd, n, dt, n, Lp, Bsz, Dm, L, W, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    print("ok", Bsz, L, d_model, round(time.time() - t0, 2), "s", u.float().abs().sum().item(),
          dt.float().abs().sum().item(), flush=True)
    with torch.no_grad():
        y = m(torch.randn(Bsz, L, d_model, device=dev).to(torch.bfloat16))
    torch.cuda.synchronize()
    print("mixer ok", y.float().abs().sum().item(), flush=True)
