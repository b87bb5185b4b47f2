"""Generate golden fixtures from the REFERENCE model code (run in the dev container).

    python tests/golden/gen_golden.py [scan|mixer|model|refiner ...]   # writes tests/golden/*.npz

This script imports ``/root/reference/models/videomamba/{mamba_simple,videomamba}.py``
as-is (read-only, nothing is copied) with ``_standins.py`` registered for the absent
third-party packages, and records inputs / parameters / outputs as small ``.npz``
fixtures.  Only the fixtures are committed and travel to the GPU box; this script
refuses to run without ``/root/reference``.

Routing of the scan: ``mamba_simple.selective_scan_fn`` is rebound to the reference's
own ``_selective_scan_ref`` (``mamba_simple.py:30-106``) and
``_SELECTIVE_SCAN_HAS_INITIAL_STATE`` is set, so the stateful path
(``mamba_simple.py:138-152``) also runs reference scan arithmetic.  The reference's
CUDA guard (``mamba_simple.py:304-308``) is bypassed for the duration of each call.
"""

from __future__ import annotations

import contextlib
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"


def _import_reference():
    if not os.path.isdir(REF):
        raise SystemExit("gen_golden.py needs /root/reference (dev container only)")
    sys.path.insert(0, HERE)
    import _standins  # noqa: E402

    _standins.install()
    sys.path.insert(0, REF)
    import models.videomamba.mamba_simple as ms  # noqa: E402
    import models.videomamba.videomamba as vm  # noqa: E402
    import models.refiner_backbone as rb  # noqa: E402

    ms.selective_scan_fn = ms._selective_scan_ref
    ms._SELECTIVE_SCAN_HAS_INITIAL_STATE = True
    return ms, vm, rb


@contextlib.contextmanager
def _pretend_cuda():
    orig = torch.Tensor.is_cuda
    torch.Tensor.is_cuda = property(lambda self: True)
    try:
        yield
    finally:
        torch.Tensor.is_cuda = orig


def _np(t):
    if isinstance(t, torch.Tensor):
        return t.detach().float().cpu().numpy() if t.is_floating_point() else t.detach().cpu().numpy()
    return np.asarray(t)


def _save(name, arrays, meta):
    path = os.path.join(HERE, name)
    arrays = {k: _np(v) for k, v in arrays.items()}
    arrays["__meta__"] = np.frombuffer(json.dumps(meta).encode(), dtype=np.uint8)
    np.savez_compressed(path, **arrays)
    print(f"wrote {name}: {sum(a.nbytes for a in arrays.values()) / 1024:.1f} KiB raw")


# --------------------------------------------------------------------------- scan
def gen_scan(ms):
    """``_selective_scan_ref`` on seeded inputs: the scan's own known answers."""
    cases = [
        # name, B, D, L, N, dtype, use_D, use_z, softplus+bias, h0
        ("s_fp32_basic", 2, 24, 37, 16, torch.float32, True, True, True, False),
        ("s_fp32_h0", 2, 24, 37, 16, torch.float32, True, True, True, True),
        ("s_bf16_h0", 2, 24, 37, 16, torch.bfloat16, True, True, True, True),
        ("s_fp32_L1", 3, 16, 1, 16, torch.float32, True, True, True, True),
        ("s_fp32_long", 1, 32, 257, 16, torch.float32, True, True, True, True),
        ("s_bf16_long", 2, 32, 1000, 16, torch.bfloat16, True, True, True, False),
        ("s_fp32_plain", 2, 16, 20, 16, torch.float32, False, False, False, False),
        ("s_fp32_n8", 2, 16, 33, 8, torch.float32, True, True, True, True),
        ("s_fp32_n4", 1, 16, 9, 4, torch.float32, True, False, True, True),
    ]
    out = {}
    meta = {}
    for i, (name, B, D, L, N, dt, useD, usez, sp, h0) in enumerate(cases):
        g = torch.Generator().manual_seed(1000 + i)
        u = torch.randn(B, D, L, generator=g).to(dt)
        delta = 0.5 * torch.randn(B, D, L, generator=g) - 1.0
        if not sp:  # without softplus the raw delta must already be a positive step
            delta = 0.05 + 0.3 * delta.abs()
        delta = delta.to(dt)
        A = -torch.exp(torch.log(torch.arange(1, N + 1, dtype=torch.float32)).repeat(D, 1)
                       + 0.1 * torch.randn(D, N, generator=g))
        Bm = torch.randn(B, N, L, generator=g).to(dt)
        Cm = torch.randn(B, N, L, generator=g).to(dt)
        Dv = torch.randn(D, generator=g) if useD else None
        z = torch.randn(B, D, L, generator=g).to(dt) if usez else None
        bias = (0.1 * torch.randn(D, generator=g)) if sp else None
        init = torch.randn(B, D, N, generator=g) if h0 else None
        y, last = ms._selective_scan_ref(u, delta, A, Bm, Cm, D=Dv, z=z, delta_bias=bias,
                                         delta_softplus=sp, initial_state=init,
                                         return_last_state=True)
        arrs = dict(u=u, delta=delta, A=A, B=Bm, C=Cm, out=y, last_state=last)
        if Dv is not None:
            arrs["D"] = Dv
        if z is not None:
            arrs["z"] = z
        if bias is not None:
            arrs["delta_bias"] = bias
        if init is not None:
            arrs["initial_state"] = init
        for k, v in arrs.items():
            out[f"{name}/{k}"] = v
        meta[name] = dict(dtype=str(dt).replace("torch.", ""), softplus=sp)
    _save("scan_cases.npz", out, meta)


# --------------------------------------------------------------------------- mixer
def gen_mixer(ms):
    """``Mamba`` (slow path) full vs chunked with state, as ``scripts/check_streaming_state.py``."""
    out = {}
    meta = {}
    cases = [
        # name, d_model, d_state, d_conv, B, L, split, dtype
        ("m_fp32_n8", 16, 8, 4, 2, 12, 5, torch.float32),
        ("m_fp32_n16", 32, 16, 4, 2, 21, 9, torch.float32),
        ("m_fp32_short", 16, 16, 4, 1, 7, 2, torch.float32),
        ("m_bf16_n16", 32, 16, 4, 2, 21, 9, torch.bfloat16),
        ("m_fp32_dconv2", 8, 4, 2, 2, 6, 3, torch.float32),
    ]
    for i, (name, dm, ds, dc, B, L, split, dt) in enumerate(cases):
        torch.manual_seed(2000 + i)
        m = ms.Mamba(d_model=dm, d_state=ds, d_conv=dc, expand=2, use_fast_path=False,
                     layer_idx=0).to(dt).eval()
        x = torch.randn(B, L, dm).to(dt)
        with torch.no_grad(), _pretend_cuda():
            full = m(x)
            o1, st1 = m(x[:, :split], return_state=True)
            st1 = (st1[0].clone(), st1[1].clone())
            o2, st2 = m(x[:, split:], state=(st1[0].clone(), st1[1].clone()),
                        return_state=True)
            # legacy ssm-only in-place path (conv restarts from zeros)
            ssm_only = torch.zeros(B, m.d_inner, ds, dtype=dt)
            o_inplace = m(x, ssm_state=ssm_only)
        arrs = dict(x=x, full=full, out1=o1, conv_state1=st1[0], ssm_state1=st1[1],
                    out2=o2, conv_state2=st2[0], ssm_state2=st2[1], out_inplace=o_inplace,
                    ssm_inplace=ssm_only)
        for k, v in m.state_dict().items():
            arrs[f"param.{k}"] = v
        for k, v in arrs.items():
            out[f"{name}/{k}"] = v
        meta[name] = dict(d_model=dm, d_state=ds, d_conv=dc, split=split,
                          dtype=str(dt).replace("torch.", ""))
    _save("mixer_cases.npz", out, meta)


# --------------------------------------------------------------------------- model
def _tiny(vm, **kw):
    base = dict(img_size=8, patch_size=4, depth=2, embed_dim=16, channels=3,
                ssm_cfg={"use_fast_path": False}, fused_add_norm=False, rms_norm=False,
                residual_in_fp32=False, kernel_size=1, num_frames=4)
    base.update(kw)
    return vm.PretrainVideoMamba(**base)


def gen_model(vm):
    """Tiny PretrainVideoMamba models: full forward, pooling variants, 2-chunk streaming."""
    out = {}
    meta = {}
    cases = [
        # name, model kwargs, input (B, T, H, W), dtype
        ("t_ln", dict(), (2, 4, 8, 8), torch.float32),
        ("t_rms", dict(img_size=32, patch_size=16, depth=3, embed_dim=32, fused_add_norm=True,
                       rms_norm=True, residual_in_fp32=True, num_frames=4), (2, 4, 32, 32),
         torch.float32),
        ("t_rms_bf16", dict(img_size=32, patch_size=16, depth=3, embed_dim=32,
                            fused_add_norm=True, rms_norm=True, residual_in_fp32=True,
                            num_frames=4), (1, 4, 32, 32), torch.bfloat16),
        ("t_tubelet2", dict(img_size=16, patch_size=8, depth=2, embed_dim=16, kernel_size=2,
                            num_frames=8, fused_add_norm=True, rms_norm=True,
                            residual_in_fp32=True), (1, 8, 16, 16), torch.float32),
        # rectangular patches, PatchEmbed(patch_size=(ph, pw)) (videomamba.py:340-364)
        ("t_rect", dict(img_size=16, patch_size=(8, 4), depth=2, embed_dim=16,
                        fused_add_norm=True, rms_norm=True, residual_in_fp32=True,
                        num_frames=4), (2, 4, 16, 16), torch.float32),
        ("t_rect_bf16", dict(img_size=32, patch_size=(16, 8), depth=2, embed_dim=32,
                             fused_add_norm=True, rms_norm=True, residual_in_fp32=True,
                             num_frames=4), (1, 4, 32, 32), torch.bfloat16),
    ]
    for i, (name, kw, (B, T, H, W), dt) in enumerate(cases):
        torch.manual_seed(3000 + i)
        model = _tiny(vm, **kw).eval()
        with torch.no_grad():
            model.temporal_pos_embedding.copy_(0.02 * torch.randn_like(model.temporal_pos_embedding))
            model.cls_token.copy_(0.02 * torch.randn_like(model.cls_token))
        model = model.to(dt)
        x = torch.randn(B, 3, T, H, W).to(dt)
        k = model.patch_embed.tubelet_size
        half = T // 2
        arrs = dict(x=x)
        with torch.no_grad(), _pretend_cuda():
            for pool in ("cls+avg", "cls", "cls_cat_avg", "avg"):
                model.pool_type = pool
                xv, xp = model(x)
                arrs[f"x_vis"] = xv
                arrs[f"pool[{pool}]"] = xp
                _, xpt = model(x, keep_temporal=True) if pool != "cls" else (None, xp)
                arrs[f"pool_kt[{pool}]"] = xpt
            model.pool_type = "cls+avg"
            feats = model.forward_features(x)
            arrs["features"] = feats
            # masked forward: drop the same count of tokens per sample (keep CLS)
            Ltot = 1 + (T // k) * model.patch_embed.num_patches
            g = torch.Generator().manual_seed(7 + i)
            mask = torch.zeros(B, Ltot, dtype=torch.bool)
            for b in range(B):
                drop = torch.randperm(Ltot - 1, generator=g)[: (Ltot - 1) // 3] + 1
                mask[b, drop] = True
            xv_m, xp_m = model(x, mask=mask)
            arrs["mask"] = mask
            arrs["x_vis_masked"] = xv_m
            arrs["pool_masked"] = xp_m
            # streaming: two chunks with full (conv, ssm) state, add_pool_norm=False semantics
            model.add_pool_norm = False
            full = model(x)
            state = model.allocate_state(B, dtype=dt)
            c1, state = model(x[:, :, :half], ssm_state=state, temporal_pos_offset=0)
            st1 = [(a.clone(), b2.clone()) for a, b2 in state]
            c2, state2 = model(x[:, :, half:], ssm_state=[(a.clone(), b2.clone()) for a, b2 in st1],
                               temporal_pos_offset=half // k)
            model.add_pool_norm = True
            # continuation chunk with avg pooling and the pool norm
            model.pool_type = "avg"
            st_tmp = [(a.clone(), b2.clone()) for a, b2 in st1]
            xv2, xp2, _ = model(x[:, :, half:], ssm_state=st_tmp, temporal_pos_offset=half // k)
            model.pool_type = "cls+avg"
        arrs.update(full_noPool=full, chunk1=c1, chunk2=c2, x_vis_chunk2_avg=xv2,
                    pool_chunk2_avg=xp2)
        for li, (cs, ss) in enumerate(st1):
            arrs[f"state1.{li}.conv"] = cs
            arrs[f"state1.{li}.ssm"] = ss
        for li, (cs, ss) in enumerate(state2):
            arrs[f"state2.{li}.conv"] = cs
            arrs[f"state2.{li}.ssm"] = ss
        for kk, v in model.state_dict().items():
            arrs[f"param.{kk}"] = v
        for kk, v in arrs.items():
            out[f"{name}/{kk}"] = v
        mk = dict(kw)
        mk.pop("ssm_cfg", None)
        meta[name] = dict(model=mk, input=[B, 3, T, H, W], dtype=str(dt).replace("torch.", ""),
                          half=half)
    _save("model_cases.npz", out, meta)


# --------------------------------------------------------------------------- refiner
def gen_refiner(rb):
    """``BiMambaRefinerBlock.forward`` (``models/refiner_backbone.py:98-135``): 3-D and 4-D
    input (frame-order flip for 4-D), with and without a carried forward state, fused
    RMSNorm and plain LayerNorm blocks, fp32 and bf16."""
    out = {}
    meta = {}
    cases = [
        # name, dim, block kwargs, x shape, dtype, carried forward state
        ("r_3d", 16, dict(), (2, 9, 16), torch.float32, False),
        ("r_4d_state", 16, dict(), (2, 3, 5, 16), torch.float32, True),
        ("r_4d_ln", 16, dict(rms_norm=False, fused_add_norm=False, residual_in_fp32=False),
         (1, 4, 3, 16), torch.float32, True),
        ("r_4d_bf16", 32, dict(), (1, 4, 6, 32), torch.bfloat16, True),
    ]
    for i, (name, dim, kw, shape, dt, carried) in enumerate(cases):
        torch.manual_seed(4000 + i)
        blk = rb.BiMambaRefinerBlock(dim, ssm_cfg={"use_fast_path": False}, layer_idx=0,
                                     **kw).to(dt).eval()
        x = torch.randn(*shape).to(dt)
        arrs = dict(x=x)
        st_f = None
        if carried:
            (cs, ss), _ = blk.allocate_state(shape[0], dtype=dt)
            cs.copy_(0.5 * torch.randn_like(cs.float()).to(dt))
            ss.copy_(0.5 * torch.randn_like(ss.float()).to(dt))
            arrs.update(state_fwd_conv=cs.clone(), state_fwd_ssm=ss.clone())
            st_f = (cs, ss)
        with torch.no_grad(), _pretend_cuda():
            y, (nc, nss) = blk(x, state_fwd=st_f)
        arrs.update(out=y, new_conv=nc, new_ssm=nss)
        for k, v in blk.state_dict().items():
            arrs[f"param.{k}"] = v
        for k, v in arrs.items():
            out[f"{name}/{k}"] = v
        meta[name] = dict(dim=dim, block=kw, shape=list(shape), carried=carried,
                          dtype=str(dt).replace("torch.", ""))
    _save("refiner_cases.npz", out, meta)


def main():
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    ms, vm, rb = _import_reference()
    only = set(sys.argv[1:])
    if not only or "scan" in only:
        gen_scan(ms)
    if not only or "mixer" in only:
        gen_mixer(ms)
    if not only or "model" in only:
        gen_model(vm)
    if not only or "refiner" in only:
        gen_refiner(rb)


if __name__ == "__main__":
    main()
