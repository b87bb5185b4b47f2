"""Time the M-16f projection GEMMs at the bench shape (B=336 -> M = 336*3144 rows) with the
shipped TunableOp results and with the library heuristic, in TFLOP/s against the gfx950
dense bf16 MFMA peak.

    python scripts/gemm_probe.py [batch]
"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PEAK = 2516.6  # TFLOP/s, dense bf16, MI355X_MICROARCH.md


def bench(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    batch = int(sys.argv[1]) if len(sys.argv) > 1 else 336
    mode = sys.argv[2] if len(sys.argv) > 2 else "tuned"
    if mode == "tuned":
        from videomamba_amd.gemm_tuning import enable_tuned_gemms
        print("tunableop:", enable_tuned_gemms())
    dev = "cuda"
    C, D = 576, 1152
    M = batch * 3144
    bf = torch.bfloat16
    hn = torch.randn(M, C, device=dev, dtype=bf)
    y = torch.randn(M, D, device=dev, dtype=bf)
    w_in = torch.randn(2 * D, C, device=dev, dtype=bf) * 0.02
    w_out = torch.randn(C, D, device=dev, dtype=bf) * 0.02
    for name, fn, flop in (
            ("in_proj  (M,576)x(576,2304)", lambda: F.linear(hn, w_in), 2 * M * C * 2 * D),
            ("out_proj (M,1152)x(1152,576)", lambda: F.linear(y, w_out), 2 * M * D * C)):
        ms = bench(fn)
        tf = flop / ms / 1e9
        print(f"{mode:6s} B={batch} {name}: {ms * 1e3:8.1f} us  {tf:7.1f} TFLOP/s  "
              f"{tf / PEAK:.3f} of peak", flush=True)


if __name__ == "__main__":
    main()
