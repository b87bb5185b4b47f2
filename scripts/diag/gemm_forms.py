"""GEMM forms for the B = 448 projections (in_proj M x 576 -> 2304, out_proj
M x 1152 -> 576, M = 448 * 3144): torch.mm against w.t() (the product), against a
pre-transposed weight, the transposed product (w @ x^T), rocBLAS instead of hipBLASLt.
    python scripts/diag/gemm_forms.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402
from bench import _event_us  # noqa: E402
from videomamba_amd import kernels as VK  # noqa: E402
from videomamba_amd.gemm_tuning import tuned  # noqa: E402

dev = torch.device("cuda", 0)
M = 448 * 3144
bf = torch.bfloat16
for name, K, N in (("in_proj", 576, 2304), ("out_proj", 1152, 576)):
    x = torch.randn(M, K, device=dev, dtype=bf)
    w = torch.randn(N, K, device=dev, dtype=bf) * 0.05
    out = torch.empty(M, N, device=dev, dtype=bf)
    wt = w.t().contiguous()
    flop = 2.0 * M * N * K
    res = {"gemm": name}
    forms = {
        "mm_wT": lambda: torch.mm(x, w.t(), out=out),
        "mm_wt_contig": lambda: torch.mm(x, wt, out=out),
    }
    for lib in ("cublaslt", "cublas"):
        try:
            torch.backends.cuda.preferred_blas_library(lib)
        except Exception as e:  # noqa: BLE001
            res[lib] = repr(e)[:80]
            continue
        for fname, fn in forms.items():
            us = _event_us(fn, 10)
            res[f"{lib}:{fname}_us"] = round(us, 1)
            res[f"{lib}:{fname}_tflops"] = round(flop / us / 1e6, 1)
    torch.backends.cuda.preferred_blas_library("cublaslt")
    with tuned():
        us = _event_us(lambda: torch.mm(x, w.t(), out=out), 10)
    res["tuned_mm_us"] = round(us, 1)
    # the HIP LDS-DMA GEMM (vm_gemm.hip) over row slabs that keep its 31-bit offsets
    slab = (1 << 30) // (K * 2) // 128 * 128
    def hip():
        for r0 in range(0, M, slab):
            VK.linear(x[r0:r0 + slab], w, out=out[r0:r0 + slab])
    us = _event_us(hip, 10)
    res["hip_dma_us"] = round(us, 1)
    res["hip_dma_tflops"] = round(flop / us / 1e6, 1)
    # halves of M (two launches): does a smaller M pick another tile?
    h = M // 2
    us = _event_us(lambda: (torch.mm(x[:h], w.t(), out=out[:h]), torch.mm(x[h:], w.t(), out=out[h:])), 10)
    res["two_halves_us"] = round(us, 1)
    print(json.dumps(res), flush=True)
    del x, w, out, wt
    torch.cuda.empty_cache()
