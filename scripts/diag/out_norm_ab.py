"""out_proj + the next block's add + RMSNorm: one launch (vm_linear_add_norm_fwd) against
out_proj then vm_add_norm_fwd, HIP events, interleaved rounds.
    python scripts/diag/out_norm_ab.py [--model]
Kernel level at the bench's B = 448 out_proj (1,408,512 x 576, K 1152) and at B = 1 / 2;
with --model also the bench's C3 step (VideoMamba-M 16x224^2 bf16, B = 448, stateful
chunk) with options.fuse_out_norm off / on, outputs compared bit for bit."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
LIB = [a.split("=", 1)[1] for a in sys.argv if a.startswith("--lib=")]
if LIB:  # a probe variant (scripts/diag/build_variant.py)
    import videomamba_amd._lib as L
    L.LIB_PATH = os.path.join(ROOT, "tools", "probes", "var", LIB[0], "libvideomamba_hip.so")
import torch  # noqa: E402
from bench import _event_us  # noqa: E402
from videomamba_amd import kernels as K  # noqa: E402
from videomamba_amd import options  # noqa: E402

dev = torch.device("cuda", 0)
st = torch.cuda.current_stream().cuda_stream
n, k = 576, 1152
SHAPES = (("b448", 448 * 3144), ("b2", 2 * 3144), ("b1", 3144))
if "--b448" in sys.argv:
    SHAPES = SHAPES[:1]
for tag, m in SHAPES:
    torch.manual_seed(0)
    x = torch.randn(m, k, device=dev).to(torch.bfloat16)
    w = (torch.randn(n, k, device=dev) / k ** 0.5).to(torch.bfloat16)
    res = torch.randn(m, n, device=dev)
    nw = torch.rand(n, device=dev) + 0.5
    h = torch.empty(m, n, device=dev, dtype=torch.bfloat16)
    hn = torch.empty(m, n, device=dev, dtype=torch.bfloat16)

    def sep():
        K.linear(x, w, out=h)
        K.add_norm_raw(h, res, nw, None, hn, res, m, n, 1e-5, True, st)

    def fused():
        K.linear_add_norm(x, w, res, nw, 1e-5, hn, h=h)

    reps = 10 if tag == "b448" else 50
    a, b = [], []
    for _ in range(3):
        a.append(_event_us(sep, reps))
        b.append(_event_us(fused, reps))
    print(json.dumps({"lib": LIB[0] if LIB else "product", "tag": tag, "m": m, "separate_us": [round(v, 1) for v in a],
                      "fused_us": [round(v, 1) for v in b]}), flush=True)
    del x, res, h, hn
    torch.cuda.empty_cache()

if "--model" in sys.argv:
    from videomamba_amd.videomamba import PretrainVideoMamba
    torch.manual_seed(0)
    model = PretrainVideoMamba(depth=32, embed_dim=576, num_frames=16, pool_type="cls+avg")
    model = model.to(device=dev, dtype=torch.bfloat16).eval()
    B = 448
    g = torch.Generator(device=dev).manual_seed(1000)
    xv = torch.randn(B, 3, 16, 224, 224, device=dev, generator=g).to(torch.bfloat16)
    state = model.allocate_state(B, dtype=torch.bfloat16, device=dev)
    outs = {}
    with torch.no_grad():
        for r in range(3):
            for fuse in (False, True):
                with options.override(fuse_out_norm=fuse):
                    model(xv, ssm_state=state, temporal_pos_offset=0)
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for _ in range(3):
                        out = model(xv, ssm_state=state, temporal_pos_offset=0)
                    torch.cuda.synchronize()
                    ms = (time.perf_counter() - t0) / 3 * 1e3
                outs[fuse] = out[1].float().clone()
                print(json.dumps({"model": "m16_b448", "round": r, "fuse_out_norm": fuse,
                                  "ms_per_step": round(ms, 2)}), flush=True)
    print(json.dumps({"model_pool_bitwise_equal": bool(torch.equal(outs[False], outs[True]))}),
          flush=True)
