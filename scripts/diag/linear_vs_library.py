"""vm_linear_fwd (row-invariant HIP GEMM) against the library GEMM (torch F.linear with the
shipped TunableOp results) for the mixer's projections at one clip's token counts:
in_proj (K 576 -> N 2304) and out_proj (K 1152 -> N 576), M = B=1 chunk rows.
HIP-event time per call on the current stream; also whether each output row's bits are
independent of M (the first M0 rows of a long call vs a short call on the same rows).
    python scripts/diag/linear_vs_library.py
"""
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from videomamba_amd import kernels as K  # noqa: E402
from videomamba_amd.gemm_tuning import tuned  # noqa: E402


def ev_us(fn, reps=30):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def lib_linear(x, w):
    with tuned():
        return F.linear(x, w)


dev = "cuda"
torch.manual_seed(0)
shapes = {"in_proj": (576, 2304), "out_proj": (1152, 576)}
Ms = [3144, 6280, 12552, 25096, 50184, 100360, 200712]
for name, (k, n) in shapes.items():
    w = (0.05 * torch.randn(n, k, device=dev)).to(torch.bfloat16)
    xbig = torch.randn(max(Ms), k, device=dev).to(torch.bfloat16)
    ref_hip = K.linear(xbig, w)
    ref_lib = lib_linear(xbig, w)
    for m in Ms:
        x = xbig[:m]
        t_hip = ev_us(lambda: K.linear(x, w))
        t_lib = ev_us(lambda: lib_linear(x, w))
        inv_hip = torch.equal(K.linear(x, w), ref_hip[:m])
        inv_lib = torch.equal(lib_linear(x, w), ref_lib[:m])
        tf = 2 * m * n * k / 1e6
        print(json.dumps({"gemm": name, "M": m, "N": n, "K": k, "hip_us": round(t_hip, 2),
                          "lib_us": round(t_lib, 2), "hip_tflops": round(tf / t_hip, 1),
                          "lib_tflops": round(tf / t_lib, 1), "hip_rows_invariant": inv_hip,
                          "lib_rows_invariant": inv_lib}), flush=True)
