"""Sub-batch streams with their layers phase-locked by cross-stream events, B = 896 M-16f
stateful chunk, against the product's free-running streams.
Each half issues its layers from its own host thread.  The "pre" phase of a layer is its
add + norm, in_proj and conv_proj; the scan and out_proj follow it.
  - free:      threads, no cross-stream waits (the control for the threading itself);
  - oneway:    half B's pre(l) waits for half A's pre(l), so B's pre meets A's scan;
  - alternate: oneway, and half A's pre(l + 1) also waits for half B's pre(l), so the two
               halves' pre phases never overlap and each scan meets the other's pre;
  - alternate_post: alternate with the previous layer's out_proj inside the locked phase
               (out_proj(l - 1) + pre(l)), so no two GEMMs of the halves overlap;
  - alt_inproj: alternate with the locked phase ending after in_proj (conv_proj outside);
  - alt_op:    alternate, and each half's out_proj(l) waits for the other half's next
               in_proj, so out_proj meets conv_proj rather than in_proj;
  - alt_nonorm: alternate with the add + norm outside the locked phase (it runs when its
               own half gets there; the lock starts at in_proj).
"product" is the model's own forward (since round 5 with options.batch_stream_lock).
    python scripts/diag/phase_lock_streams.py"""
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from videomamba_amd import videomamba as V  # noqa: E402
from videomamba_amd import mamba_simple as MS  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
model = V.PretrainVideoMamba(depth=32, embed_dim=576, num_frames=16, pool_type="cls+avg")
model = model.to(device=dev, dtype=torch.bfloat16).eval()
depth = len(model.layers)
B = int(([a.split('=', 1)[1] for a in sys.argv if a.startswith('--batch=')] or ['896'])[0])
g = torch.Generator(device=dev).manual_seed(1000)
x = torch.randn(B, 3, 16, 224, 224, device=dev, generator=g).to(torch.bfloat16)
for i, layer in enumerate(model.layers):
    layer.mixer._phase_idx = i

tls = threading.local()
state = {}


def hook(kind, idx):
    part = getattr(tls, "part", None)
    mode = state.get("mode")
    if part is None or mode in (None, "free"):
        return
    ev, rec = state["ev"], state["rec"]
    cur = torch.cuda.current_stream(dev)
    if kind == "pre_done_early" and mode == "alt_op":  # in_proj(idx) issued
        state["ev2"][part][idx].record(cur)
        state["rec2"][part][idx].set()
        return
    if kind == "post_start" and mode == "alt_op":  # out_proj(idx) waits the other's in_proj
        o, j = (1, idx) if part == 0 else (0, idx + 1)
        if j < depth:
            state["rec2"][o][j].wait()
            cur.wait_event(state["ev2"][o][j])
        return
    if kind in ("pre_done", "pre_done_early"):
        # alt_inproj: the locked phase ends after in_proj (conv_proj outside it)
        if (kind == "pre_done_early") != (mode == "alt_inproj"):
            return
        ev[part][idx].record(cur)
        rec[part][idx].set()
    elif kind in ("pre_start", "mixer_start") and (kind == "mixer_start") != (mode == "alt_nonorm"):
        return  # alt_nonorm: the locked phase starts after the add + norm, at the mixer
    if kind in ("pre_start", "mixer_start", "post_start"):
        # alternate_post: a layer's locked phase starts at the previous layer's out_proj
        # (post_start of idx - 1 is the phase start of idx); layer 0's at its add + norm
        if mode == "alternate_post":
            if kind == "post_start":
                idx += 1
                if idx >= depth:
                    return
            elif idx != 0:
                return
        elif kind == "post_start":
            return
        if part == 1:
            rec[0][idx].wait()
            cur.wait_event(ev[0][idx])
        elif mode in ("alternate", "alternate_post", "alt_inproj", "alt_op", "alt_nonorm") and idx >= 1:
            rec[1][idx - 1].wait()
            cur.wait_event(ev[1][idx - 1])


_front = MS.Mamba._tm_front


def tm_front(self, *a, **k):
    r = _front(self, *a, **k)
    tls.layer = self._phase_idx
    hook("pre_done", self._phase_idx)
    return r


MS.Mamba._tm_front = tm_front
_scan = MS.K.scan_dtproj_raw


def scan_dtproj_raw(*a, **k):
    r = _scan(*a, **k)
    hook("post_start", tls.layer)
    return r


MS.K.scan_dtproj_raw = scan_dtproj_raw
_cp = MS.K.conv_proj_raw


def conv_proj_raw(*a, **k):
    hook("pre_done_early", tls.layer)
    return _cp(*a, **k)


MS.K.conv_proj_raw = conv_proj_raw
_fp = V.Block.forward_padded


def block_fp(self, *a, **k):
    tls.layer = self.mixer._phase_idx
    hook("pre_start", self.mixer._phase_idx)
    return _fp(self, *a, **k)


V.Block.forward_padded = block_fp
_mfp = MS.Mamba.forward_padded


def mixer_fp(self, *a, **k):
    hook("mixer_start", self._phase_idx)
    return _mfp(self, *a, **k)


MS.Mamba.forward_padded = mixer_fp


def threaded(st, mode):
    """The _encode_streams split with each half issued from its own host thread."""
    state["mode"] = mode
    state["ev"] = [[torch.cuda.Event() for _ in range(depth)] for _ in range(2)]
    state["rec"] = [[threading.Event() for _ in range(depth)] for _ in range(2)]
    state["ev2"] = [[torch.cuda.Event() for _ in range(depth)] for _ in range(2)]
    state["rec2"] = [[threading.Event() for _ in range(depth)] for _ in range(2)]
    cut = [0, B // 2, B]
    cur = torch.cuda.current_stream(dev)
    streams = V._side_streams(dev, 2)
    model._prepare_param_caches()
    m0 = model.layers[0].mixer
    conv_new = torch.empty((depth, B, m0.d_inner, m0.d_conv), dtype=st[0][0].dtype, device=dev)
    L = 1 + 16 * 196
    feats = torch.empty((B, L, model.embed_dim), dtype=torch.bfloat16, device=dev)
    outs = [None, None]

    def run(i):
        tls.part = i
        a, b = cut[i], cut[i + 1]
        s = streams[i]
        with torch.cuda.stream(s):
            outs[i] = model._encode(x[a:b], None, [(t[0][a:b], t[1][a:b]) for t in st], 0,
                                    pool=(False, 16, 196), conv_out=conv_new[:, a:b],
                                    feats_out=feats[a:b], split=False)
        tls.part = None

    for s in streams:
        s.wait_stream(cur)
    th = [threading.Thread(target=run, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for s in streams:
        cur.wait_stream(s)
    return torch.cat([o[1] for o in outs], 0)


with torch.no_grad():
    ref_state = model.allocate_state(B, dtype=torch.bfloat16, device=dev)
    ref = model(x, ssm_state=ref_state, temporal_pos_offset=0)[1].float()
    for mode in ("alternate", "alt_nonorm"):
        fresh = model.allocate_state(B, dtype=torch.bfloat16, device=dev)
        out = threaded(fresh, mode).float()
        print(json.dumps({"mode": mode, "pool_bitwise_equal_product": bool(torch.equal(out, ref))}),
              flush=True)
        del fresh
    st = model.allocate_state(B, dtype=torch.bfloat16, device=dev)
    for r in range(3):
        for mode in ("product", "alt_nonorm"):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(3):
                if mode == "product":
                    model(x, ssm_state=st, temporal_pos_offset=0)
                else:
                    threaded(st, mode)
            torch.cuda.synchronize()
            print(json.dumps({"round": r, "mode": mode,
                              "ms_per_step": round((time.perf_counter() - t0) / 3 * 1e3, 2)}),
                  flush=True)
