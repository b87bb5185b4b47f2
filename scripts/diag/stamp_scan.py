"""Phase timeline of the one-launch chunked scan at B=1 (M-16f chunk shape) from the
sc_stamp probe variant (scripts/diag/build_variant.py sc_stamp): per workgroup
s_memrealtime stamps (100 MHz): entry (0), start-up loads landed (1), PASS 1 done (2),
aggregate published (3), preceding flags seen (4), entry state composed (5), PASS 2 done
and drained (6).  python scripts/diag/stamp_scan.py [batch]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import videomamba_amd._lib as L  # noqa: E402
L.LIB_PATH = os.path.join(ROOT, "tools", "probes", "var", "sc_stamp", "libvideomamba_hip.so")
if not os.path.exists(L.LIB_PATH):  # a build pushed to the GPU box (VARIANT_DIR=ab)
    L.LIB_PATH = os.path.join(ROOT, "tools", "probes", "ab", "sc_stamp", "libvideomamba_hip.so")
import numpy as np  # noqa: E402
import torch  # noqa: E402
from bench import scan_roofline  # noqa: E402

dev = torch.device("cuda", 0)
B = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 1
r = scan_roofline(B, 20, dev, "tm", dtp="--nodtp" not in sys.argv)  # leaves the last launch's stamps in the array
torch.cuda.synchronize()
lib = L.load()
lib.vm_dbg_read_stamps.argtypes = [ctypes.c_void_p]
buf = np.zeros(4096 * 8, dtype=np.uint64)
assert lib.vm_dbg_read_stamps(buf.ctypes.data) == 0
st8 = buf.reshape(4096, 8).astype(np.int64)
dtb = st8[:, 7]  # DTP: the dt block written (after stamp 1)
st = st8[:, :7]
live = st[:, 0] > 0
st = st[live]
t0 = st[:, 0].min()
rel = (st - t0) * 10e-3
dtrel = (dtb[live] - t0) * 10e-3
nblk = st.shape[0]
print(json.dumps({
    "B": B, "event_us_avg": r["avg_us"], "workgroups": int(nblk),
    "start_spread_us": round(float(rel[:, 0].max()), 2),
    "last_end_us": round(float(rel[:, 6].max()), 2),
    "phase_median_us": [round(float(np.median(rel[:, k + 1] - rel[:, k])), 2) for k in range(6)],
    "phase_max_us": [round(float(np.max(rel[:, k + 1] - rel[:, k])), 2) for k in range(6)],
    "stamp_median_us": [round(float(np.median(rel[:, k])), 2) for k in range(7)],
    "stamp_max_us": [round(float(np.max(rel[:, k])), 2) for k in range(7)],
    "dt_block_median_us": round(float(np.median(dtrel - rel[:, 1])), 2) if (dtb[live] > 0).all() else None,
}), flush=True)
