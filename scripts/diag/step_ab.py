"""One library's B-clip M-16f stateful-chunk step time (the bench's forward, default
sub-batch streams), for A/B across probe builds run in alternating processes:
    python scripts/diag/step_ab.py [--lib=VARIANT] [--batch=896] [--reps=3] [--lock=0|1] [--opt=name=value]
Prints ms per step and a fingerprint of the pooled features (equal = same bits)."""
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
LIB = [a.split("=", 1)[1] for a in sys.argv if a.startswith("--lib=")]
if LIB:  # a probe variant (scripts/diag/build_variant.py)
    import videomamba_amd._lib as L
    L.LIB_PATH = os.path.join(ROOT, "tools", "probes", os.environ.get("VARIANT_DIR", "var"), LIB[0],
                              "libvideomamba_hip.so")
import torch  # noqa: E402
from videomamba_amd import options  # noqa: E402
from videomamba_amd.videomamba import PretrainVideoMamba  # noqa: E402


def arg(name, default):
    v = [a.split("=", 1)[1] for a in sys.argv if a.startswith(f"--{name}=")]
    return int(v[0]) if v else default


B, reps, lock = arg("batch", 896), arg("reps", 3), arg("lock", -1)
_kw = {} if lock < 0 else {"batch_stream_lock": bool(lock)}
for a in sys.argv:  # --opt=name=value (bool / int options)
    if a.startswith("--opt="):
        k, v = a[6:].split("=", 1)
        _kw[k] = v.lower() in ("true", "on") if v.lower() in ("true", "false", "on", "off") else int(v)
_ctx = options.override(**_kw) if _kw else None
if _ctx is not None:
    _ctx.__enter__()  # (held in _ctx: a collected generator would restore the options)
dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = PretrainVideoMamba(depth=32, embed_dim=576, num_frames=16, pool_type="cls+avg")
model = model.to(device=dev, dtype=torch.bfloat16).eval()
g = torch.Generator(device=dev).manual_seed(1000)
x = torch.randn(B, 3, 16, 224, 224, device=dev, generator=g).to(torch.bfloat16)
with torch.no_grad():
    st = model.allocate_state(B, dtype=torch.bfloat16, device=dev)
    out = model(x, ssm_state=st, temporal_pos_offset=0)[1]
    fp = hashlib.sha1(out.float().cpu().numpy().tobytes()).hexdigest()[:16]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        model(x, ssm_state=st, temporal_pos_offset=0)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / reps * 1e3
print(json.dumps({"lib": LIB[0] if LIB else "product", "batch": B,
                  "batch_stream_lock": options.get().batch_stream_lock,
                  "fuse_out_norm": options.get().fuse_out_norm,
                  "batch_streams": options.get().batch_streams,
                  "min_clips": options.get().batch_stream_min_clips, "ms_per_step": round(ms, 2),
                  "fingerprint": fp}), flush=True)
