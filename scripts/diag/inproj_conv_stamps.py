"""Phase stamps of vm_in_proj_conv_proj_fwd's x tiles (probe build ic_stamp of
scripts/diag/build_variant.py, VARIANT_DIR=ab): s_memrealtime (100 MHz) at the kernel start,
after the K loop, after the LDS x tile, before / after the conv, after u + the x_proj MFMAs,
after the partial staging — per workgroup, B = 1 M-16f.  Prints the per-phase medians and
the start / end spread."""
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import videomamba_amd._lib as L  # noqa: E402
L.LIB_PATH = os.path.join(ROOT, "tools", "probes", "ab", "ic_stamp", "libvideomamba_hip.so")
import torch  # noqa: E402
from videomamba_amd import kernels as K  # noqa: E402
from videomamba_amd.mamba_simple import Mamba  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
dev = "cuda"
torch.manual_seed(0)
m = Mamba(d_model=576, layer_idx=0).to(dev, torch.bfloat16)
C, Dm, E, R, W = 576, m.d_inner, m.dt_rank + 2 * m.d_state, m.dt_rank, m.d_conv
_, _, _, cw, cb = m._fp32_params()
wx_pad, wdt_pad = m._padded_proj_weights()
Lp = 3144
n = B * Lp
hn = torch.randn(n, C, device=dev).to(torch.bfloat16)
cs = torch.randn(B, Dm, W, device=dev).to(torch.bfloat16)
cso = torch.empty(B, Dm, W, device=dev, dtype=torch.bfloat16)
xz = torch.empty(n, 2 * Dm, device=dev, dtype=torch.bfloat16)
u = torch.empty(n, Dm, device=dev, dtype=torch.bfloat16)
xd = torch.empty(n, E, device=dev, dtype=torch.bfloat16)


def call():
    K.in_proj_conv_proj_raw(hn, m.in_proj.weight, xz[:, Dm:], cw, cb, cs, (Dm * W, W), cso,
                            (Dm * W, W), wx_pad, E, wdt_pad, R, u, xd, None, Lp, B, Dm, 3137, W,
                            torch.cuda.current_stream().cuda_stream)


lib = L.load()
lib.vm_ic_stamps.argtypes = [ctypes.c_void_p]
for _ in range(5):
    call()
torch.cuda.synchronize()
res = []
for rep in range(3):
    call()
    torch.cuda.synchronize()
    buf = (ctypes.c_ulonglong * (4096 * 8))()
    assert lib.vm_ic_stamps(buf) == 0
    nxr, nsp = -(-n // 112), Dm // 128
    nx, nz = nxr * nsp, -(-n // 128) * nsp
    st = [[buf[w * 8 + p] for p in range(8)] for w in range(nx + nz)]
    t0 = min(s[0] for s in st)
    xs = st[:nx]
    ph = {f"p{p}_p{p + 1}": statistics.median((s[p + 1] - s[p]) * 10e-3 for s in xs) for p in range(6)}
    ph["x_start_max"] = max((s[0] - t0) * 10e-3 for s in xs)
    ph["x_end_median"] = statistics.median((s[6] - t0) * 10e-3 for s in xs)
    ph["x_end_max"] = max((s[6] - t0) * 10e-3 for s in xs)
    ph["z_start_median"] = statistics.median((s[0] - t0) * 10e-3 for s in st[nx:])
    ph["z_end_median"] = statistics.median((s[1] - t0) * 10e-3 for s in st[nx:])
    ph["z_end_max"] = max((s[1] - t0) * 10e-3 for s in st[nx:])
    ph["x_gemm_p0_p1_max"] = max((s[1] - s[0]) * 10e-3 for s in xs)
    res.append({k: round(v, 2) for k, v in ph.items()})
for r in res:
    print(json.dumps(r))
