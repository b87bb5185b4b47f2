"""Per-wave phase timeline of the one-launch chunked scan (sc_stampw probe build):
stamps 0 start-up wait passed, 1 dt block ready, 2 PASS 1 loop done, 3 composed + published.
python scripts/diag/stamp_scan_waves.py [batch]"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import videomamba_amd._lib as L  # noqa: E402
L.LIB_PATH = os.path.join(ROOT, "tools", "probes", "var", "sc_stampw", "libvideomamba_hip.so")
if not os.path.exists(L.LIB_PATH):  # a build pushed to the GPU box (VARIANT_DIR=ab)
    L.LIB_PATH = os.path.join(ROOT, "tools", "probes", "ab", "sc_stampw", "libvideomamba_hip.so")
import numpy as np  # noqa: E402
import torch  # noqa: E402
from bench import scan_roofline  # noqa: E402

dev = torch.device("cuda", 0)
B = int(sys.argv[1]) if len(sys.argv) > 1 else 1
r = scan_roofline(B, 20, dev, "tm", dtp=True)
torch.cuda.synchronize()
lib = L.load()
lib.vm_dbg_read_stamps.argtypes = [ctypes.c_void_p]
buf = np.zeros(4096 * 8 * 4, dtype=np.uint64)
assert lib.vm_dbg_read_stamps(buf.ctypes.data) == 0
st = buf.reshape(4096, 8, 4).astype(np.int64)
live = st[:, 0, 0] > 0
st = st[live]
t0 = st[:, :, 0].min()
rel = (st - t0) * 10e-3  # us
out = {"B": B, "workgroups": int(st.shape[0]), "event_us_avg": r["avg_us"]}
for k, name in enumerate(["startup_done", "dt_ready", "pass1_done", "published"]):
    out[name + "_median"] = round(float(np.median(rel[:, :, k])), 2)
    out[name + "_max"] = round(float(np.max(rel[:, :, k])), 2)
d = rel[:, :, 1] - rel[:, :, 0]
out["dt_block_median"] = round(float(np.median(d)), 2)
p1 = rel[:, :, 2] - rel[:, :, 1]
out["pass1_loop_median"] = round(float(np.median(p1)), 2)
out["pass1_loop_max"] = round(float(np.max(p1)), 2)
sk = rel[:, :, 2].max(axis=1) - rel[:, :, 2].min(axis=1)
out["pass1_done_skew_in_block_median"] = round(float(np.median(sk)), 2)
out["pass1_done_skew_in_block_max"] = round(float(np.max(sk)), 2)
cp = rel[:, 0, 3] - rel[:, :, 2].max(axis=1)
out["compose_after_last_wave_median"] = round(float(np.median(cp)), 2)
print(json.dumps(out), flush=True)
