"""ORACLE — CPU restatement of the reference VideoMamba encoder forward.

TEST INFRASTRUCTURE, NOT PRODUCT.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import this module, and only as the checker
(or as the timed CPU baseline).  The product path (``videomamba_amd``) never imports
it and has no CPU fallback.

Pinning: every function below is checked in ``tests/test_oracle_golden.py`` against
the fixtures in ``tests/golden/*.npz``, which ``tests/golden/gen_golden.py`` produced by
running the reference model code itself (``/root/reference/models/videomamba``) in the
dev container.  The third-party kernels the reference calls (mamba-ssm 2.3.2.post1,
causal-conv1d 1.6.2.post1) are absent there; their published algorithms are restated
here and in ``tests/golden/_standins.py``; the scan values in the fixtures come from the
reference's own ``_selective_scan_ref``.

Everything is computed in fp32 on CPU.  When the model dtype ``dt`` is bf16 the
restatement rounds to bf16 at exactly the points where the reference materialises a
tensor in the model dtype ("→e").

Params are a flat ``{name: tensor}`` dict with the reference's state_dict keys.
"""

from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn.functional as F

Tensor = torch.Tensor


# ----------------------------------------------------------------------------- kernels
def selective_scan(u, delta, A, B, C, D=None, z=None, delta_bias=None,
                   delta_softplus=False, initial_state=None, return_last_state=False):
    """Selective scan; follows ``mamba_simple.py:30-106`` (``_selective_scan_ref``).

    u, delta, z: (b, d, l); A: (d, n); B, C: (b, n, l); D, delta_bias: (d,).
    fp32 internally, output rounded to u.dtype, last state fp32.
    """
    dtype_in = u.dtype
    u = u.float()
    delta = delta.float()
    if delta_bias is not None:
        delta = delta + delta_bias[..., None].float()
    if delta_softplus:
        delta = F.softplus(delta)  # threshold 20, as torch / mamba CUDA
    b, d, l = u.shape
    n = A.shape[1]
    A = A.float()
    Bf = B.float()
    Cf = C.float()
    h = torch.zeros(b, d, n) if initial_state is None else initial_state.float().clone()
    dA = torch.exp(delta[..., None] * A[None, :, None, :])  # (b, d, l, n)
    dBu = (delta * u)[..., None] * Bf.permute(0, 2, 1)[:, None, :, :]  # (b, d, l, n)
    ys = []
    for t in range(l):
        h = dA[:, :, t] * h + dBu[:, :, t]
        ys.append((h * Cf[:, None, :, t]).sum(-1))
    y = torch.stack(ys, dim=2) if l > 0 else torch.zeros(b, d, 0)
    if D is not None:
        y = y + u * D.float()[:, None]
    if z is not None:
        y = y * F.silu(z.float())
    y = y.to(dtype_in)
    return (y, h) if return_last_state else y


def selective_state_update(state, x, dt, A, B, C, D=None, z=None, dt_bias=None,
                           dt_softplus=False):
    """One-token scan step (mamba-ssm ``selective_state_update`` as called at
    ``mamba_simple.py:483-494``); updates ``state`` in place in its dtype."""
    dtf = dt.float()
    if dt_bias is not None:
        dtf = dtf + dt_bias.float()
    if dt_softplus:
        dtf = F.softplus(dtf)
    new = state.float() * torch.exp(dtf[..., None] * A.float()) \
        + (dtf * x.float())[..., None] * B.float()[:, None, :]
    state.copy_(new)
    out = (new * C.float()[:, None, :]).sum(-1)
    if D is not None:
        out = out + x.float() * D.float()
    if z is not None:
        out = out * F.silu(z.float())
    return out.to(x.dtype)


def causal_conv1d(x, weight, bias, silu=True, conv_state=None):
    """Depthwise causal conv (width W, left zero pad W-1) + SiLU; follows the slow path
    at ``mamba_simple.py:369-404``.  x: (b, d, l); weight: (d, W).

    With ``conv_state`` (b, d, W) the conv runs over ``cat([conv_state, x])`` and keeps
    the last l outputs (``:382-390``).  Returns (out, new_conv_state) where
    new_conv_state is the last W raw inputs (``:391-392`` / ``:401-404``).
    """
    b, d, l = x.shape
    w = weight.shape[-1]
    xin = x if conv_state is None else torch.cat([conv_state.to(x.dtype), x], dim=-1)
    out = F.conv1d(xin.float(), weight.float().reshape(d, 1, w),
                   None if bias is None else bias.float(), padding=w - 1, groups=d)
    out = out[..., : xin.shape[-1]][..., -l:] if l > 0 else out[..., :0]
    if silu:
        out = F.silu(out)
    new_state = F.pad(xin, (w - xin.shape[-1], 0)) if xin.shape[-1] < w else xin[..., -w:]
    return out.to(x.dtype), new_state


def causal_conv1d_update(x, conv_state, weight, bias, silu=True):
    """One-token conv step; rolls ``conv_state`` in place (``mamba_simple.py:468-474``)."""
    conv_state.copy_(torch.roll(conv_state, shifts=-1, dims=-1))
    conv_state[:, :, -1] = x
    o = (conv_state.float() * weight.float()).sum(-1)
    if bias is not None:
        o = o + bias.float()
    if silu:
        o = F.silu(o)
    return o.to(x.dtype)


def add_norm(x, residual, weight, bias, eps, prenorm, residual_in_fp32, is_rms):
    """Fused residual-add + RMSNorm/LayerNorm (mamba-ssm ``rms_norm_fn`` /
    ``layer_norm_fn`` as called at ``videomamba.py:152-166`` and ``:904-918``)."""
    xf = x.float()
    if residual is not None:
        xf = xf + residual.float()
        res_dtype = residual.dtype
    else:
        res_dtype = torch.float32 if residual_in_fp32 else x.dtype
    if is_rms:
        xhat = xf * torch.rsqrt((xf * xf).mean(-1, keepdim=True) + eps)
    else:
        mu = xf.mean(-1, keepdim=True)
        xhat = (xf - mu) * torch.rsqrt(((xf - mu) ** 2).mean(-1, keepdim=True) + eps)
    y = xhat * weight.float()
    if bias is not None:
        y = y + bias.float()
    y = y.to(x.dtype)
    return (y, xf.to(res_dtype)) if prenorm else y


# ----------------------------------------------------------------------------- mixer
def mamba_mixer(p: Dict[str, Tensor], prefix: str, hidden: Tensor, *, d_state: int,
                d_conv: int, state: Optional[Tuple[Tensor, Tensor]] = None,
                ssm_state: Optional[Tensor] = None, return_state: bool = False):
    """``Mamba.forward`` slow path (``mamba_simple.py:283-451``), stateless,
    ``state=(conv, ssm)`` and legacy in-place ``ssm_state`` variants."""
    dt_ = hidden.dtype
    W_in = p[prefix + "in_proj.weight"]
    d_inner = W_in.shape[0] // 2
    bsz, seqlen, _ = hidden.shape
    conv_state = None
    if state is not None:
        conv_state, ssm_state = state
    # in_proj, rounded to the model dtype (``:333-339``)
    xz = torch.einsum("dc,blc->bdl", W_in.float(), hidden.float()).to(dt_)
    if (prefix + "in_proj.bias") in p:
        xz = (xz.float() + p[prefix + "in_proj.bias"].float()[:, None]).to(dt_)
    A = -torch.exp(p[prefix + "A_log"].float())
    x, z = xz[:, :d_inner], xz[:, d_inner:]
    conv_w = p[prefix + "conv1d.weight"].reshape(d_inner, d_conv)
    conv_b = p.get(prefix + "conv1d.bias")
    xc, new_conv = causal_conv1d(x, conv_w, conv_b, silu=True, conv_state=conv_state)
    # x_proj / dt_proj (``:409-416``)
    Wx = p[prefix + "x_proj.weight"]
    dt_rank = Wx.shape[0] - 2 * d_state
    x_dbl = torch.einsum("bdl,jd->blj", xc.float(), Wx.float()).to(dt_)
    dtl, Bm, Cm = torch.split(x_dbl, [dt_rank, d_state, d_state], dim=-1)
    dlt = torch.einsum("dr,blr->bdl", p[prefix + "dt_proj.weight"].float(),
                       dtl.float()).to(dt_)
    Bm = Bm.permute(0, 2, 1)
    Cm = Cm.permute(0, 2, 1)
    use_inplace = ssm_state is not None and state is None and not return_state
    y, last = selective_scan(xc, dlt, A, Bm, Cm, p[prefix + "D"].float(), z=z,
                             delta_bias=p[prefix + "dt_proj.bias"].float(),
                             delta_softplus=True, initial_state=ssm_state,
                             return_last_state=True)
    out = torch.einsum("bdl,cd->blc", y.float(), p[prefix + "out_proj.weight"].float())
    if (prefix + "out_proj.bias") in p:
        out = out + p[prefix + "out_proj.bias"].float()
    out = out.to(dt_)
    if use_inplace:
        ssm_state.copy_(last)
    if return_state:
        return out, (new_conv, last)
    return out


# ----------------------------------------------------------------------------- block
def block_forward(p: Dict[str, Tensor], pre: str, h: Tensor, residual: Optional[Tensor], *,
                  fused: bool, residual_in_fp32: bool, is_rms: bool, eps: float, d_state: int,
                  d_conv: int, state: Optional[Tuple[Tensor, Tensor]] = None):
    """``Block.forward`` (``videomamba.py:120-246``): (fused) add + norm, then the mixer
    (stateful when ``state`` is given).  Returns ``(hidden, residual, new_state|None)``."""
    nw, nb = p[pre + "norm.weight"], p.get(pre + "norm.bias")
    C = h.shape[-1]
    if fused:  # ``:151-166``
        h, residual = add_norm(h, residual, nw, nb, eps, True, residual_in_fp32, is_rms)
    else:  # ``:141-150``
        residual = h if residual is None else residual + h
        r = residual.to(nw.dtype)
        if is_rms:
            h = add_norm(r, None, nw, None, eps, False, False, True)
        else:
            h = F.layer_norm(r.float(), (C,), nw.float(),
                             None if nb is None else nb.float(), eps).to(nw.dtype)
        if residual_in_fp32:
            residual = residual.float()
    if state is not None:
        h, st = mamba_mixer(p, pre + "mixer.", h, d_state=d_state, d_conv=d_conv, state=state,
                            return_state=True)
        return h, residual, st
    return mamba_mixer(p, pre + "mixer.", h, d_state=d_state, d_conv=d_conv), residual, None


def refiner_forward(p: Dict[str, Tensor], x: Tensor, *, state_fwd=None, state_bwd_init=None,
                    fused: bool = True, residual_in_fp32: bool = True, is_rms: bool = True,
                    eps: float = 1e-5, d_state: int = 16, d_conv: int = 4):
    """``BiMambaRefinerBlock.forward`` (``models/refiner_backbone.py:98-135``): forward
    block on the sequence, backward block on the time-flipped sequence (4-D input: frame
    order flipped, within-frame order kept, ``:61-68``), sigmoid gate, Linear.  States
    default to zeros (``:70-79``); only the forward block's new state is returned."""
    packed = None
    seq = x
    if x.ndim == 4:
        b, t, n, c = x.shape
        packed = (b, t, n)
        seq = x.reshape(b, t * n, c)
    elif x.ndim != 3:
        raise ValueError("Expected x to be [B, L, C] or [B, T, N, C].")

    def flip(v):
        if packed is None:
            return torch.flip(v, dims=[1])
        b_, t_, n_ = packed
        return torch.flip(v.reshape(b_, t_, n_, v.shape[-1]), dims=[1]).reshape(b_, t_ * n_, -1)

    dt_ = seq.dtype
    bsz = seq.shape[0]

    def zeros_state(pre):
        d_inner = p[pre + "mixer.in_proj.weight"].shape[0] // 2
        return (torch.zeros(bsz, d_inner, d_conv, dtype=dt_),
                torch.zeros(bsz, d_inner, d_state, dtype=dt_))

    kw = dict(fused=fused, residual_in_fp32=residual_in_fp32, is_rms=is_rms, eps=eps,
              d_state=d_state, d_conv=d_conv)
    st_f = state_fwd if state_fwd is not None else zeros_state("block_fwd.")
    out_f, _, new_f = block_forward(p, "block_fwd.", seq, None, state=st_f, **kw)
    st_b = state_bwd_init if state_bwd_init is not None else zeros_state("block_bwd.")
    out_b_rev, _, _ = block_forward(p, "block_bwd.", flip(seq), None, state=st_b, **kw)
    out_b = flip(out_b_rev)
    gin = torch.cat([out_f, out_b], dim=-1).float()
    lin = (gin @ p["fusion_gate.0.weight"].float().t() + p["fusion_gate.0.bias"].float()).to(dt_)
    gate = torch.sigmoid(lin.float()).to(dt_)  # nn.Linear then nn.Sigmoid, each in the dtype
    mix = (gate.float() * out_f.float()).to(dt_).float() + ((1.0 - gate.float()).to(dt_).float()
                                                             * out_b.float()).to(dt_).float()
    mix = mix.to(dt_)
    out = (mix.float() @ p["out_proj.weight"].float().t() + p["out_proj.bias"].float()).to(dt_)
    if packed is not None:
        out = out.reshape(*packed, out.shape[-1])
    return out, new_f


# ----------------------------------------------------------------------------- encoder
def _infer_spatial_grid(token_count: int, ref: Tuple[int, int]) -> Tuple[int, int]:
    """``videomamba.py:32-55``."""
    ref_ratio = ref[0] / ref[1]
    best, best_score = None, None
    for h in range(1, int(math.sqrt(token_count)) + 1):
        if token_count % h:
            continue
        w = token_count // h
        for hh, ww in ((h, w), (w, h)):
            s = (abs(hh / ww - ref_ratio), abs(hh - ref[0]) + abs(ww - ref[1]))
            if best_score is None or s < best_score:
                best_score, best = s, (hh, ww)
    return best


def encoder_forward(p: Dict[str, Tensor], cfg: dict, x: Tensor, *, mask=None,
                    keep_temporal: bool = False, state: Optional[Sequence] = None,
                    temporal_pos_offset: int = 0, add_pool_norm: bool = True):
    """``PretrainVideoMamba.forward`` (``videomamba.py:943-1067``) with
    ``forward_features`` (``:786-941``).  ``cfg`` keys: img_size, patch_size, depth,
    kernel_size, num_frames, fused_add_norm, rms_norm, residual_in_fp32, pool_type,
    norm_epsilon, d_state, d_conv.  ``state``: list of (conv, ssm) or None.

    Returns (x_vis, x_pool | None, new_state | None).
    """
    dt_ = p["patch_embed.proj.weight"].dtype
    k = cfg["kernel_size"]
    ps = cfg["patch_size"]
    ph, pw = (ps, ps) if isinstance(ps, int) else tuple(ps)  # tuple: ``:348-363``
    img = cfg["img_size"] if isinstance(cfg["img_size"], (tuple, list)) else (cfg["img_size"],) * 2
    eps = cfg.get("norm_epsilon", 1e-5)
    is_rms = cfg["rms_norm"]
    B_, _, T, H, W = x.shape
    assert T % k == 0
    x = x.to(dt_)
    # patch embed (``:359-368``)
    pe = F.conv3d(x.float(), p["patch_embed.proj.weight"].float(),
                  p["patch_embed.proj.bias"].float(), stride=(k, ph, pw)).to(dt_)
    _, C, Tt, Gh, Gw = pe.shape
    pos = p["pos_embed"]
    patch_pos = pos[:, 1:]
    bh, bw = img[0] // ph, img[1] // pw
    if bh * bw != patch_pos.shape[1]:
        bh, bw = _infer_spatial_grid(patch_pos.shape[1], (bh, bw))
    if (Gh, Gw) != (bh, bw):  # ``:621-644``
        pp = patch_pos.reshape(1, bh, bw, C).permute(0, 3, 1, 2)
        pp = F.interpolate(pp.float(), size=(Gh, Gw), mode="bicubic", align_corners=False)
        patch_pos = pp.permute(0, 2, 3, 1).reshape(1, Gh * Gw, C)
    patch_pos = patch_pos.to(dt_)
    tpe = p["temporal_pos_embedding"].to(dt_)  # ``:655-675``
    end = temporal_pos_offset + Tt
    if end > tpe.shape[1]:
        tp = F.interpolate(tpe.permute(0, 2, 1).float(), size=end, mode="linear",
                           align_corners=False).permute(0, 2, 1).to(dt_)
    else:
        tp = tpe
    tp = tp[:, temporal_pos_offset:end]
    tok = pe.permute(0, 2, 3, 4, 1).reshape(B_, Tt, Gh * Gw, C)
    tok = tok + patch_pos.unsqueeze(1)
    tok = tok + tp.unsqueeze(2)
    tok = tok.reshape(B_, Tt * Gh * Gw, C)
    has_cls = state is None or temporal_pos_offset <= 0
    if has_cls:
        cls = p["cls_token"].expand(B_, -1, -1) + pos[:, :1].to(dt_)
        h = torch.cat([cls, tok], dim=1)
    else:
        h = tok
    vis_pos = None
    if mask is not None:  # ``:753-784``
        vis = ~mask.bool()
        n_vis = int(vis.sum(1)[0])
        tp_ = torch.arange(h.shape[1]).unsqueeze(0).expand(B_, -1).masked_fill(~vis, h.shape[1])
        vis_pos = torch.sort(tp_, dim=1).values[:, :n_vis]
        h = h.gather(1, vis_pos.unsqueeze(-1).expand(-1, -1, C))
    residual = None
    new_state = [] if state is not None else None
    fused = cfg["fused_add_norm"]
    rif = cfg["residual_in_fp32"]
    for i in range(cfg["depth"]):
        h, residual, st = block_forward(
            p, f"layers.{i}.", h, residual, fused=fused, residual_in_fp32=rif, is_rms=is_rms,
            eps=eps, d_state=cfg["d_state"], d_conv=cfg["d_conv"],
            state=state[i] if state is not None else None)
        if state is not None:
            new_state.append(st)
    nw, nb = p["norm.weight"], p.get("norm.bias")
    if fused:  # ``:903-918``
        out = add_norm(h, residual, nw, nb, eps, False, rif, is_rms)
    else:  # ``:896-901``
        residual = h if residual is None else residual + h
        r = residual.to(nw.dtype)
        if is_rms:
            out = add_norm(r, None, nw, None, eps, False, False, True)
        else:
            out = F.layer_norm(r.float(), (C,), nw.float(),
                               None if nb is None else nb.float(), eps).to(nw.dtype)
    if not add_pool_norm:
        return out, None, new_state
    # pooling (``:983-1062``)
    cls_tok = out[:, :1] if has_cls else None
    patch = out[:, 1:] if has_cls else out
    pool = cfg["pool_type"]

    def pool_norm(v):
        return F.layer_norm(v.float(), (C,), p["pool_norm.weight"].float(),
                            p["pool_norm.bias"].float(), 1e-5).to(v.dtype)

    if pool == "cls":
        xp = pool_norm(cls_tok)
    else:
        if keep_temporal:
            hw = Gh * Gw
            if mask is None:
                avg = patch.reshape(B_, Tt, hw, C).mean(2)
            else:
                ppos = vis_pos[:, 1:] - 1 if has_cls else vis_pos
                fi = torch.div(ppos, hw, rounding_mode="floor")
                ssum = torch.zeros(B_, Tt, C, dtype=patch.dtype)
                ssum.scatter_add_(1, fi.unsqueeze(-1).expand(-1, -1, C), patch)
                cnt = torch.zeros(B_, Tt, 1, dtype=patch.dtype)
                cnt.scatter_add_(1, fi.unsqueeze(-1), torch.ones(B_, patch.shape[1], 1,
                                                                 dtype=patch.dtype))
                avg = ssum / cnt
        else:
            avg = patch.mean(1, keepdim=True)
        if pool == "cls+avg":
            xp = pool_norm(cls_tok + avg)
        elif pool == "cls_cat_avg":
            xp = pool_norm(torch.cat([cls_tok, avg], dim=1))
        else:
            xp = pool_norm(avg)
    return patch, xp, new_state


def params_from_npz(npz, prefix: str) -> Dict[str, Tensor]:
    """Collect ``{prefix}param.<key>`` arrays of a fixture into a state dict (fp32)."""
    out = {}
    tag = prefix + "param."
    for k in npz.files:
        if k.startswith(tag):
            out[k[len(tag):]] = torch.from_numpy(npz[k].copy())
    return out
