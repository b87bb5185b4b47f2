"""Scan-kernel ablation at the bench shape (M-16f, token-major, B clips): the same launch
with softplus off (delta pre-activated by its producer), without the z gate, and both —
prices the per-step non-state work.  Prints one line per form."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from videomamba_amd import kernels as K  # noqa: E402
from videomamba_amd.layers import round_up  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 336
dev = torch.device("cuda", 0)
D, N, L, R = 1152, 16, 3137, 36
Lp = round_up(L)
n = B * Lp
g = torch.Generator(device=dev).manual_seed(1)
bf = torch.bfloat16
A = -torch.arange(1, N + 1, device=dev, dtype=torch.float32).repeat(D, 1).contiguous()
Dv = torch.ones(D, device=dev)
bias = torch.full((D,), -4.0, device=dev)
h = torch.zeros(B, D, N, device=dev, dtype=bf)
u = torch.randn(n, D, device=dev, generator=g).to(bf)
dt = (0.5 * torch.randn(n, D, device=dev, generator=g) - 4.0).to(bf)
xz = torch.randn(n, 2 * D, device=dev, generator=g).to(bf)
xdbl = torch.randn(n, R + 2 * N, device=dev, generator=g).to(bf)
z, Bm, Cm = xz[:, D:], xdbl[:, R:], xdbl[:, R + N:]
y = torch.empty_like(u)
delta = torch.nn.functional.softplus(dt.float() - 4.0).to(bf)  # pre-activated form
s_u, s_z, s_bc = (Lp * D, 1, D), (Lp * 2 * D, 1, 2 * D), (Lp * (R + 2 * N), 1, R + 2 * N)
stream = torch.cuda.current_stream(dev).cuda_stream


def run(sp, zz, reps=20):
    def launch():
        K.scan_raw(u, s_u, dt if sp else delta, s_u, A, Bm, s_bc, Cm, s_bc, Dv, zz, s_z, bias if sp else None, sp,
                   h, (h.stride(0), h.stride(1)), h, (h.stride(0), h.stride(1)), y, s_u, Lp,
                   B, D, L, N, 1, stream)
    for _ in range(5):
        launch()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        launch()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


algo = B * D * L * 8 + 4 * B * N * L + 4 * D * N + 8 * D + 4 * B * D * N
for name, sp, zz in [("softplus+z (model today)", True, z), ("pre-activated delta, z", False, z),
                     ("softplus, no z", True, None), ("pre-activated, no z", False, None),
                     ("softplus+z (again)", True, z)]:
    us = run(sp, zz)
    print(f"{name:28s} B={B} {us:9.1f} us  {us / B:6.2f} us/clip-layer  frac {algo / us / 1e3 / 8000:.4f}",
          flush=True)
