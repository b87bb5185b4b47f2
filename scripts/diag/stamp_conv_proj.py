"""Phase timeline of the fused small-batch conv_proj at the B=1 M-16f chunk shape, from the
cp_stamp probe variant (scripts/diag/build_variant.py cp_stamp): per workgroup s_memrealtime
stamps (100 MHz) at entry (0), conv done (1), x_proj partials ready (2), x_dbl summed (3),
dt tile in LDS (4), stores drained (5).  python scripts/diag/stamp_conv_proj.py"""
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import videomamba_amd._lib as L  # noqa: E402
WAVES = "--waves" in sys.argv  # cp_stampw: per-wave stamps [wg][16][8]
L.LIB_PATH = os.path.join(ROOT, "tools", "probes", "var", "cp_stampw" if WAVES else "cp_stamp",
                          "libvideomamba_hip.so")
import numpy as np  # noqa: E402
import torch  # noqa: E402
from bench import _event_us  # noqa: E402
from videomamba_amd import kernels as K  # noqa: E402
from videomamba_amd.layers import round_up  # noqa: E402
from videomamba_amd.mamba_simple import Mamba  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
C, L_ = 576, 3137
Lp = round_up(L_)
bf = torch.bfloat16
mx = Mamba(d_model=C, layer_idx=0).to(dev, bf).eval()
Dm, N, R, W = mx.d_inner, mx.d_state, mx.dt_rank, mx.d_conv
E = R + 2 * N
stream = torch.cuda.current_stream(dev).cuda_stream
xz = torch.randn(Lp, 2 * Dm, device=dev, dtype=bf)
u = torch.empty(Lp, Dm, device=dev, dtype=bf)
dt = torch.empty(Lp, Dm, device=dev, dtype=bf)
xdbl = torch.empty(Lp, E, device=dev, dtype=bf)
cs_in = torch.randn(1, Dm, W, device=dev, dtype=bf)
cs_out = torch.empty(1, Dm, W, device=dev, dtype=bf)
_, _, _, cw, cb = mx._fp32_params()
wx_pad, wdt_pad = mx._padded_proj_weights()


def run():
    K.conv_proj_raw(xz, (Lp * 2 * Dm, 2 * Dm), cw, cb, cs_in, (cs_in.stride(0), cs_in.stride(1)),
                    cs_out, (cs_out.stride(0), cs_out.stride(1)), wx_pad, E, wdt_pad, R, u,
                    (Lp * Dm, Dm), xdbl, (Lp * E, E), dt, (Lp * Dm, Dm), Lp, 1, Dm, L_, W, stream)


us = _event_us(run, 50)
lib = L.load()
lib.vm_dbg_read_stamps.argtypes = [ctypes.c_void_p]
res = []
if WAVES:
    run()
    torch.cuda.synchronize()
    nwg = (Lp + 15) // 16
    buf = np.zeros(2048 * 16 * 8, dtype=np.uint64)
    assert lib.vm_dbg_read_stamps(buf.ctypes.data) == 0
    st = buf.reshape(2048, 16, 8)[:nwg, :9, :].astype(np.int64)
    rel = (st - st[:, :, 0].min()) * 10e-3
    d = rel[:, :, 1:] - rel[:, :, :-1]  # [wg][wave][7] phase durations
    print(json.dumps({"event_us_avg": round(us, 2),
                      "phase_median_us": [round(float(np.median(d[:, :, k])), 2) for k in range(7)],
                      "phase_p90_us": [round(float(np.percentile(d[:, :, k], 90)), 2) for k in range(7)],
                      "wave_skew_at_barrier_us": round(float(np.median(rel[:, :, 6].max(1) - rel[:, :, 6].min(1))), 2),
                      "wave_start_skew_us": round(float(np.median(rel[:, :, 0].max(1) - rel[:, :, 0].min(1))), 2)}))
    sys.exit(0)
for rep in range(5):
    run()
    torch.cuda.synchronize()
    buf = np.zeros(4096 * 8, dtype=np.uint64)
    assert lib.vm_dbg_read_stamps(buf.ctypes.data) == 0
    nwg = (Lp + 15) // 16
    st = buf[: nwg * 8].reshape(nwg, 8)[:, :6].astype(np.int64)
    t0 = st[:, 0].min()
    rel = (st - t0) * 10e-3  # us
    res.append({
        "wg": nwg, "event_us_avg": round(us, 2),
        "start_spread_us": round(float(rel[:, 0].max()), 2),
        "last_end_us": round(float(rel[:, 5].max()), 2),
        "phase_median_us": [round(float(np.median(rel[:, k + 1] - rel[:, k])), 2) for k in range(5)],
        "phase_max_us": [round(float(np.max(rel[:, k + 1] - rel[:, k])), 2) for k in range(5)],
    })
for r in res:
    print(json.dumps(r), flush=True)
