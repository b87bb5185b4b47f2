"""Pin the oracle: CPU restatement vs fixtures recorded from the reference model code.

Tolerances: fp32 cases 2e-5 (different accumulation order from the reference's einsum);
bf16 cases compare values that went through identical bf16 rounding points, so they are
held to one bf16 ulp-ish (2e-2 abs/rel) to absorb the occasional rounding-boundary flip.
"""

import numpy as np
import pytest
import torch

from conftest import load_golden
from oracle import videomamba_oracle as orc


def _t(npz, key, dtype=torch.float32):
    return torch.from_numpy(npz[key].copy()).to(dtype)


def _tol(dtype):
    return (2e-5, 2e-5) if dtype == "float32" else (2e-2, 2e-2)


SCAN, SCAN_META = load_golden("scan_cases.npz")


@pytest.mark.parametrize("name", sorted(SCAN_META))
def test_oracle_scan_matches_reference(name):
    meta = SCAN_META[name]
    dt = torch.bfloat16 if meta["dtype"] == "bfloat16" else torch.float32
    g = lambda k, d=dt: _t(SCAN, f"{name}/{k}", d)  # noqa: E731
    has = lambda k: f"{name}/{k}" in SCAN.files  # noqa: E731
    y, last = orc.selective_scan(
        g("u"), g("delta"), g("A", torch.float32), g("B"), g("C"),
        D=g("D", torch.float32) if has("D") else None,
        z=g("z") if has("z") else None,
        delta_bias=g("delta_bias", torch.float32) if has("delta_bias") else None,
        delta_softplus=meta["softplus"],
        initial_state=g("initial_state", torch.float32) if has("initial_state") else None,
        return_last_state=True)
    rtol, atol = _tol(meta["dtype"])
    torch.testing.assert_close(y.float(), g("out", torch.float32), rtol=rtol, atol=atol)
    torch.testing.assert_close(last, g("last_state", torch.float32), rtol=2e-5, atol=2e-5)


MIX, MIX_META = load_golden("mixer_cases.npz")


@pytest.mark.parametrize("name", sorted(MIX_META))
def test_oracle_mixer_matches_reference(name):
    meta = MIX_META[name]
    dt = torch.bfloat16 if meta["dtype"] == "bfloat16" else torch.float32
    p = {k: v.to(dt) for k, v in orc.params_from_npz(MIX, name + "/").items()}
    x = _t(MIX, f"{name}/x", dt)
    split = meta["split"]
    kw = dict(d_state=meta["d_state"], d_conv=meta["d_conv"])
    rtol, atol = _tol(meta["dtype"])
    chk = lambda a, k: torch.testing.assert_close(  # noqa: E731
        a.float(), _t(MIX, f"{name}/{k}"), rtol=rtol, atol=atol)
    chk(orc.mamba_mixer(p, "", x, **kw), "full")
    o1, (c1, s1) = orc.mamba_mixer(p, "", x[:, :split], return_state=True, **kw)
    chk(o1, "out1")
    chk(c1, "conv_state1")
    chk(s1, "ssm_state1")
    o2, (c2, s2) = orc.mamba_mixer(p, "", x[:, split:], state=(c1, s1), return_state=True, **kw)
    chk(o2, "out2")
    chk(c2, "conv_state2")
    chk(s2, "ssm_state2")
    ssm = torch.zeros(x.shape[0], p["A_log"].shape[0], meta["d_state"], dtype=dt)
    chk(orc.mamba_mixer(p, "", x, ssm_state=ssm, **kw), "out_inplace")
    chk(ssm, "ssm_inplace")
    # streaming contract (scripts/check_streaming_state.py:55): chunked == full
    if dt == torch.float32:
        torch.testing.assert_close(torch.cat([o1, o2], 1), orc.mamba_mixer(p, "", x, **kw),
                                   rtol=1e-4, atol=1e-4)


MOD, MOD_META = load_golden("model_cases.npz")


def model_cfg(meta):
    m = dict(img_size=8, patch_size=4, depth=2, embed_dim=16, kernel_size=1, num_frames=4,
             fused_add_norm=False, rms_norm=False, residual_in_fp32=False,
             pool_type="cls+avg", norm_epsilon=1e-5, d_state=16, d_conv=4)
    m.update(meta["model"])
    return m


@pytest.mark.parametrize("name", sorted(MOD_META))
def test_oracle_encoder_matches_reference(name):
    meta = MOD_META[name]
    dt = torch.bfloat16 if meta["dtype"] == "bfloat16" else torch.float32
    p = {k: v.to(dt) for k, v in orc.params_from_npz(MOD, name + "/").items()}
    cfg = model_cfg(meta)
    x = _t(MOD, f"{name}/x", dt)
    rtol, atol = _tol(meta["dtype"])
    if dt == torch.bfloat16:
        rtol, atol = 5e-2, 5e-2
    chk = lambda a, k: torch.testing.assert_close(  # noqa: E731
        a.float(), _t(MOD, f"{name}/{k}"), rtol=rtol, atol=atol)
    for pool in ("cls+avg", "cls", "cls_cat_avg", "avg"):
        cfg["pool_type"] = pool
        xv, xp, _ = orc.encoder_forward(p, cfg, x)
        chk(xv, "x_vis")
        chk(xp, f"pool[{pool}]")
        if pool != "cls":
            _, xpt, _ = orc.encoder_forward(p, cfg, x, keep_temporal=True)
            chk(xpt, f"pool_kt[{pool}]")
    cfg["pool_type"] = "cls+avg"
    mask = torch.from_numpy(MOD[f"{name}/mask"].copy())
    xv, xp, _ = orc.encoder_forward(p, cfg, x, mask=mask)
    chk(xv, "x_vis_masked")
    chk(xp, "pool_masked")
    full, _, _ = orc.encoder_forward(p, cfg, x, add_pool_norm=False)
    chk(full, "full_noPool")
    half = meta["half"]
    k = cfg["kernel_size"]
    depth = cfg["depth"]
    d_inner = 2 * cfg["embed_dim"]
    st0 = [(torch.zeros(x.shape[0], d_inner, 4, dtype=dt),
            torch.zeros(x.shape[0], d_inner, 16, dtype=dt)) for _ in range(depth)]
    c1, _, st1 = orc.encoder_forward(p, cfg, x[:, :, :half], state=st0, add_pool_norm=False)
    chk(c1, "chunk1")
    for i, (cs, ss) in enumerate(st1):
        chk(cs, f"state1.{i}.conv")
        chk(ss, f"state1.{i}.ssm")
    c2, _, st2 = orc.encoder_forward(p, cfg, x[:, :, half:], state=st1,
                                     temporal_pos_offset=half // k, add_pool_norm=False)
    chk(c2, "chunk2")
    for i, (cs, ss) in enumerate(st2):
        chk(cs, f"state2.{i}.conv")
        chk(ss, f"state2.{i}.ssm")
    cfg["pool_type"] = "avg"
    xv2, xp2, _ = orc.encoder_forward(p, cfg, x[:, :, half:], state=st1,
                                      temporal_pos_offset=half // k)
    chk(xv2, "x_vis_chunk2_avg")
    chk(xp2, "pool_chunk2_avg")
    if dt == torch.float32:  # test_videomamba_regressions.py:562-588 (tighter)
        torch.testing.assert_close(torch.cat([c1, c2], 1), full, rtol=1e-4, atol=1e-4)


REF_, REF_META = load_golden("refiner_cases.npz")


@pytest.mark.parametrize("name", sorted(REF_META))
def test_oracle_refiner_matches_reference(name):
    """BiMambaRefinerBlock (models/refiner_backbone.py:98-135): 3-D / 4-D input, carried
    forward state, fused RMSNorm and LayerNorm blocks."""
    meta = REF_META[name]
    dt = torch.bfloat16 if meta["dtype"] == "bfloat16" else torch.float32
    p = {k: v.to(dt) for k, v in orc.params_from_npz(REF_, name + "/").items()}
    g = lambda k: _t(REF_, f"{name}/{k}", dt)  # noqa: E731
    blk = meta["block"]
    st = (g("state_fwd_conv"), g("state_fwd_ssm")) if meta["carried"] else None
    out, (nc, ns) = orc.refiner_forward(
        p, g("x"), state_fwd=st, fused=blk.get("fused_add_norm", True),
        residual_in_fp32=blk.get("residual_in_fp32", True), is_rms=blk.get("rms_norm", True))
    rtol, atol = _tol(meta["dtype"])
    chk = lambda a, k: torch.testing.assert_close(  # noqa: E731
        a.float(), _t(REF_, f"{name}/{k}"), rtol=rtol, atol=atol)
    chk(out, "out")
    chk(nc, "new_conv")
    chk(ns, "new_ssm")
