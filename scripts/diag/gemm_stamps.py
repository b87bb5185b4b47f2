"""Phase timestamps of the persistent GEMM (probe build tg_stamp, scripts/diag/build_variant.py):
one steady-state iteration of workgroup 0, waves 0 (leader) and 4 (one barrier behind),
s_memtime at phase start (0), after the waits (1), after the first barrier (2), after the
MFMA issue (3) and after the second barrier (4).  Prints per-phase segment lengths in
cycles and their medians.
    python scripts/diag/gemm_stamps.py [in_proj|out_proj]
"""
import ctypes
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import videomamba_amd._lib as L  # noqa: E402

L.LIB_PATH = os.path.join(ROOT, "tools", "probes", "var", "tg_stamp", "libvideomamba_hip.so")
import torch  # noqa: E402
from videomamba_amd import kernels as K  # noqa: E402

shape = sys.argv[1] if len(sys.argv) > 1 else "in_proj"
n, k = {"in_proj": (2304, 576), "out_proj": (576, 1152)}[shape]
m = 448 * 3144
x = (torch.rand(m, k, device="cuda") * 2 - 1).to(torch.bfloat16)
w = ((torch.rand(n, k, device="cuda") * 2 - 1) * k ** -0.5).to(torch.bfloat16)
for _ in range(3):
    K.linear(x, w, form="persistent")
torch.cuda.synchronize()
lib = ctypes.CDLL(L.LIB_PATH)
buf = (ctypes.c_ulonglong * 1024)()
assert lib.vm_tile_stamps(buf) == 0
st = list(buf)
nph = 72
out = {"shape": shape}
for wv, name in ((0, "leader"), (1, "lagger")):
    seg = {"issue_read_wait": [], "barrier1": [], "mfma_issue": [], "barrier2": [], "to_next": []}
    for ph in range(nph):
        b = (wv * nph + ph) * 5
        t = st[b:b + 5]
        if 0 in t:
            continue
        seg["issue_read_wait"].append(t[1] - t[0])
        seg["barrier1"].append(t[2] - t[1])
        seg["mfma_issue"].append(t[3] - t[2])
        seg["barrier2"].append(t[4] - t[3])
        if ph + 1 < nph and st[b + 5] != 0:
            seg["to_next"].append(st[b + 5] - t[4])
    total = (st[(wv * nph + nph - 1) * 5 + 4] - st[wv * nph * 5]) / nph
    out[name] = {k2: round(statistics.median(v), 1) for k2, v in seg.items() if v}
    out[name]["phase_mean"] = round(total, 1)
    out[name]["per_phase_P"] = [[st[(wv * nph + ph) * 5 + 4] - st[(wv * nph + ph) * 5]
                                 for ph in range(P, nph, 4)][:6] for P in range(4)]
print(json.dumps(out), flush=True)
