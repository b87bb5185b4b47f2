"""out_proj + add + RMSNorm: library GEMM (TunableOp-selected) + vm_add_norm_fwd against the
fused vm_out_proj_add_norm_fwd, at the bench shape (M: N = 576, K = 1152, B clips of
Lp = 3144 rows).  Prints agreement and per-call times (HIP events, 10 reps)."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from videomamba_amd import kernels as K  # noqa: E402
from videomamba_amd.gemm_tuning import enable_tuned_gemms  # noqa: E402

dev = torch.device("cuda", 0)
enable_tuned_gemms()
B = int(sys.argv[1]) if len(sys.argv) > 1 else 336
N, Kd, Lp = (int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])) if len(sys.argv) > 4 else (576, 1152, 3144)
rows = B * Lp
g = torch.Generator(device=dev).manual_seed(0)
bf = torch.bfloat16
y = torch.randn(rows, Kd, device=dev, generator=g).to(bf)
W = (torch.randn(N, Kd, device=dev, generator=g) / Kd ** 0.5).to(bf)
res = torch.randn(rows, N, device=dev, generator=g)
nw = 1.0 + 0.1 * torch.randn(N, device=dev, generator=g)
st = torch.cuda.current_stream().cuda_stream
out_a, out_b = torch.empty(rows, N, device=dev, dtype=bf), torch.empty(rows, N, device=dev, dtype=bf)
ro_a, ro_b = torch.empty_like(res), torch.empty_like(res)


def unfused():
    h = F.linear(y, W)
    K.add_norm_raw(h, res, nw, None, out_a, ro_a, rows, N, 1e-5, True, st)


def fused():
    K.out_norm_raw(y, Kd, W, res, nw, None, out_b, ro_b, rows, 1e-5, True, st)


unfused()
fused()
torch.cuda.synchronize()
rel = lambda a, b: ((a.float() - b.float()).norm() / b.float().norm()).item()  # noqa: E731
print(f"rows={rows} N={N} K={Kd}: rel(out) {rel(out_b, out_a):.2e}  rel(res_out) {rel(ro_b, ro_a):.2e}  "
      f"max|d out| {(out_b.float() - out_a.float()).abs().max().item():.3e}", flush=True)


def tm(fn, reps=10):
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


for name, fn, epi in [("library GEMM + add_norm", unfused, "1"), ("fused, LDS row epilogue", fused, "1"),
                      ("fused, direct epilogue", fused, "0"), ("fused, GEMM only (probe)", fused, "2"),
                      ("library GEMM + add_norm", unfused, "1"), ("fused, LDS row epilogue", fused, "1")]:
    os.environ["VM_OUT_NORM_EPI"] = epi
    us = tm(fn)
    flops = 2.0 * rows * N * Kd
    print(f"{name:26s} {us:9.1f} us  ({flops / us / 1e6:7.1f} TFLOP/s GEMM-equivalent)", flush=True)
