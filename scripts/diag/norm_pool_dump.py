"""Final norm + pooling (vm_norm_pool_fwd + vm_pool_finish_fwd through kernels.norm_pool /
pool_finish) on fixed random bf16 inputs, saved for a bitwise comparison between library
builds, and timed at the B = 1 chunk shape:
    python scripts/diag/norm_pool_dump.py <variant|product> <out.pt>"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
name = sys.argv[1]
if name != "product":
    import videomamba_amd._lib as L
    L.LIB_PATH = os.path.join(ROOT, "tools", "probes", "var", name, "libvideomamba_hip.so")
import torch  # noqa: E402
from bench import _event_us  # noqa: E402
from videomamba_amd import kernels as K  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
res = {}
times = {}
for tag, (B, L, C, head, groups, gr, res_on, rms) in {
        "m16_b1": (1, 3137, 576, 1, 1, 3136, True, True),
        "m16_b3_frames": (3, 3137, 576, 1, 16, 196, True, True),
        "ti_ln": (2, 1569, 192, 1, 8, 196, False, False),
        "noncls_1024": (2, 784, 1024, 0, 4, 196, True, True)}.items():
    Lp = (L + 7) // 8 * 8
    h = torch.randn(B, Lp, C, device=dev, generator=g).to(torch.bfloat16)
    r = torch.randn(B, Lp, C, device=dev, generator=g) if res_on else None
    w = torch.randn(C, device=dev, generator=g)
    bb = None if rms else torch.randn(C, device=dev, generator=g)
    run = lambda: K.norm_pool(h, r, L, w, bb, 1e-5, rms, head=head, groups=groups,  # noqa: E731
                              group_rows=gr, max_group_rows=gr, sums=True)
    feats, ws = run()
    nb = K.norm_pool_workspace_bytes(B, groups, gr, C)
    res[tag] = (feats.clone(), ws.reshape(-1)[:nb].clone())
    times[tag + "_us"] = round(_event_us(run, 50), 2)
torch.save(res, sys.argv[2])
print(json.dumps({"variant": name, **times}), flush=True)
