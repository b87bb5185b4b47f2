"""A/B of the channel-major x_proj -> dt_proj: fused kernel vs the two library GEMMs, at
M-16f (D=1152, R=36, N=16) for a few batch sizes; also checks the fused outputs against
the GEMM path (same bf16 rounding points; fp32 accumulation order differs).

    python scripts/xdt_cm_ab.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from videomamba_amd import kernels as K  # noqa: E402
from videomamba_amd.gemm_tuning import enable_tuned_gemms  # noqa: E402


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    enable_tuned_gemms()
    dev, bf = "cuda", torch.bfloat16
    D, R, N = 1152, 36, 16
    E = R + 2 * N
    g = torch.Generator(device=dev).manual_seed(3)
    wx = (0.03 * torch.randn(E, D, device=dev, generator=g)).to(bf)
    wdt = (0.1 * torch.randn(D, R, device=dev, generator=g)).to(bf)
    wx_pad = torch.zeros(80, D, device=dev, dtype=bf)
    wx_pad[:E] = wx
    wdt_pad = torch.zeros(D, 64, device=dev, dtype=bf)
    wdt_pad[:, :R] = wdt
    stream = torch.cuda.current_stream().cuda_stream
    for B in (1, 2, 4, 8):
        n = B * 3144
        u = torch.randn(D, n, device=dev, generator=g).to(bf)
        xd = torch.empty(E, n, device=dev, dtype=bf)
        dt = torch.empty(D, n, device=dev, dtype=bf)

        def fused():
            K.xdt_proj_cm_raw(u, n, wx_pad, E, wdt_pad, R, xd, n, dt, n, n, D, stream)

        def lib():
            x_dbl = torch.matmul(wx, u)
            return x_dbl, torch.matmul(wdt, x_dbl[:R])

        tf, tl = timeit(fused), timeit(lib)
        fused()
        x_ref, dt_ref = lib()
        torch.cuda.synchronize()
        ex = ((xd.float() - x_ref.float()).abs().max() / x_ref.float().abs().max()).item()
        ed = ((dt.float() - dt_ref.float()).abs().max() / dt_ref.float().abs().max()).item()
        print(f"B={B} n={n}: fused {tf:7.1f} us  library GEMMs {tl:7.1f} us  "
              f"max rel diff x_dbl {ex:.2e} dt {ed:.2e}", flush=True)


if __name__ == "__main__":
    main()
