"""Pure-torch stand-ins for the third-party modules the reference imports.

TEST INFRASTRUCTURE ONLY — used by ``gen_golden.py`` to import and run the
reference model code (``/root/reference/models/videomamba/*.py``) in this
container, where the pinned third-party packages are absent:

* ``causal-conv1d==1.6.2.post1``  (``causal_conv1d_fn`` / ``causal_conv1d_update``)
* ``mamba-ssm==2.3.2.post1``      (``selective_scan_fn``, ``mamba_inner_fn``,
  ``selective_state_update``, ``RMSNorm`` / ``rms_norm_fn`` / ``layer_norm_fn``)
* ``timm>=1.0.22``                (``DropPath``, ``to_2tuple``, ``trunc_normal_``,
  ``_cfg``, ``_load_weights``)

Each stand-in restates the published algorithm of the pinned package, in fp32,
rounding to the input dtype exactly where the CUDA/Triton kernels store.  The
selective scan itself is NOT stood in: the generator rebinds the reference's own
``_selective_scan_ref`` (``models/videomamba/mamba_simple.py:30-106``) as
``selective_scan_fn`` so every scan value in the fixtures is reference arithmetic.
"""

from __future__ import annotations

import math
import sys
import types

import torch
import torch.nn as nn
import torch.nn.functional as F


# --------------------------------------------------------------------------- causal-conv1d
def causal_conv1d_fn(x, weight, bias=None, seq_idx=None, initial_states=None,
                     return_final_states=False, final_states_out=None, activation=None):
    """causal-conv1d 1.6.2 ``causal_conv1d_fn``: depthwise conv, left zero pad W-1,
    fp32 accumulate, optional SiLU, output in x.dtype.  Called by the reference at
    ``mamba_simple.py:383-399``."""
    assert seq_idx is None and initial_states is None and not return_final_states
    d, w = weight.shape
    out = F.conv1d(x.float(), weight.float().unsqueeze(1),
                   None if bias is None else bias.float(), padding=w - 1, groups=d)
    out = out[..., : x.shape[-1]]
    if activation in ("silu", "swish"):
        out = F.silu(out)
    return out.to(x.dtype)


def causal_conv1d_update(x, conv_state, weight, bias=None, activation=None,
                         cache_seqlens=None, conv_state_indices=None):
    """causal-conv1d ``causal_conv1d_update``: roll ``conv_state`` left by one, append
    x, dot with weight (fp32), optional SiLU.  ``conv_state`` is updated in place."""
    assert cache_seqlens is None and conv_state_indices is None
    unsqueeze = x.dim() == 2
    if unsqueeze:
        x = x.unsqueeze(-1)
    seqlen = x.shape[-1]
    outs = []
    for i in range(seqlen):
        conv_state.copy_(torch.roll(conv_state, shifts=-1, dims=-1))
        conv_state[:, :, -1] = x[:, :, i]
        o = (conv_state.float() * weight.float()).sum(-1)
        if bias is not None:
            o = o + bias.float()
        if activation in ("silu", "swish"):
            o = F.silu(o)
        outs.append(o.to(x.dtype))
    out = torch.stack(outs, dim=-1)
    return out.squeeze(-1) if unsqueeze else out


# --------------------------------------------------------------------------- mamba-ssm
def selective_state_update(state, x, dt, A, B, C, D=None, z=None, dt_bias=None,
                           dt_softplus=False):
    """mamba-ssm 2.3.2 Triton ``selective_state_update`` (one token): fp32 math, state
    stored back in its own dtype, output computed from the fp32 state."""
    dtf = dt.float()
    if dt_bias is not None:
        dtf = dtf + dt_bias.float()
    if dt_softplus:
        dtf = F.softplus(dtf)
    dA = torch.exp(dtf[..., None] * A.float())
    dBx = (dtf * x.float())[..., None] * B.float()[:, None, :]
    new_state = state.float() * dA + dBx
    state.copy_(new_state)
    out = (new_state * C.float()[:, None, :]).sum(-1)
    if D is not None:
        out = out + x.float() * D.float()
    if z is not None:
        out = out * F.silu(z.float())
    return out.to(x.dtype)


def mamba_inner_fn(*args, **kwargs):  # fast path is never used by the fixtures
    raise RuntimeError("mamba_inner_fn stand-in: fixtures use use_fast_path=False")


def _norm_fwd(x, weight, bias, residual, eps, prenorm, residual_in_fp32, is_rms):
    """mamba-ssm ``_layer_norm_fwd`` semantics: x (+ residual) summed in fp32, statistics
    on the fp32 sum, y = x_hat * w (+ b) stored in x.dtype; residual_out stored in
    residual.dtype, or fp32 when residual is None and residual_in_fp32."""
    xf = x.float()
    if residual is not None:
        xf = xf + residual.float()
        res_dtype = residual.dtype
    else:
        res_dtype = torch.float32 if residual_in_fp32 else x.dtype
    if is_rms:
        rstd = torch.rsqrt((xf * xf).mean(-1, keepdim=True) + eps)
        xhat = xf * rstd
    else:
        mean = xf.mean(-1, keepdim=True)
        var = ((xf - mean) ** 2).mean(-1, keepdim=True)
        xhat = (xf - mean) * torch.rsqrt(var + eps)
    y = xhat * weight.float()
    if bias is not None:
        y = y + bias.float()
    y = y.to(x.dtype)
    if prenorm:
        return y, xf.to(res_dtype)
    return y


def rms_norm_fn(x, weight, bias, residual=None, x1=None, weight1=None, bias1=None,
                eps=1e-6, dropout_p=0.0, rowscale=None, prenorm=False,
                residual_in_fp32=False, return_dropout_mask=False):
    return _norm_fwd(x, weight, bias, residual, eps, prenorm, residual_in_fp32, True)


def layer_norm_fn(x, weight, bias, residual=None, x1=None, weight1=None, bias1=None,
                  eps=1e-6, dropout_p=0.0, rowscale=None, prenorm=False,
                  residual_in_fp32=False, is_rms_norm=False, return_dropout_mask=False):
    return _norm_fwd(x, weight, bias, residual, eps, prenorm, residual_in_fp32,
                     is_rms_norm)


class RMSNorm(nn.Module):
    def __init__(self, hidden_size, eps=1e-5, dropout_p=0.0, device=None, dtype=None):
        super().__init__()
        self.eps = eps
        self.weight = nn.Parameter(torch.ones(hidden_size, device=device, dtype=dtype))
        self.register_parameter("bias", None)

    def forward(self, x, residual=None, prenorm=False, residual_in_fp32=False):
        return rms_norm_fn(x, self.weight, self.bias, residual=residual, eps=self.eps,
                           prenorm=prenorm, residual_in_fp32=residual_in_fp32)


# --------------------------------------------------------------------------- timm
class DropPath(nn.Module):
    def __init__(self, drop_prob=0.0, scale_by_keep=True):
        super().__init__()
        self.drop_prob = drop_prob

    def forward(self, x):
        if self.drop_prob == 0.0 or not self.training:
            return x
        keep = 1 - self.drop_prob
        mask = x.new_empty((x.shape[0],) + (1,) * (x.ndim - 1)).bernoulli_(keep)
        return x * mask / keep


def to_2tuple(x):
    if isinstance(x, (tuple, list)):
        return tuple(x)
    return (x, x)


def trunc_normal_(tensor, mean=0.0, std=1.0, a=-2.0, b=2.0):
    with torch.no_grad():
        def norm_cdf(v):
            return (1.0 + math.erf(v / math.sqrt(2.0))) / 2.0
        lo, hi = norm_cdf((a - mean) / std), norm_cdf((b - mean) / std)
        tensor.uniform_(2 * lo - 1, 2 * hi - 1)
        tensor.erfinv_()
        tensor.mul_(std * math.sqrt(2.0))
        tensor.add_(mean)
        tensor.clamp_(min=a, max=b)
        return tensor


def _cfg(url="", **kwargs):
    return {"url": url, **kwargs}


def _load_weights(model, checkpoint_path, prefix=""):
    raise RuntimeError("timm _load_weights stand-in is not available")


def install():
    """Register the stand-in modules in ``sys.modules`` (idempotent)."""
    def mod(name, **attrs):
        m = sys.modules.get(name) or types.ModuleType(name)
        for k, v in attrs.items():
            setattr(m, k, v)
        sys.modules[name] = m
        return m

    mod("causal_conv1d", causal_conv1d_fn=causal_conv1d_fn,
        causal_conv1d_update=causal_conv1d_update)
    mod("mamba_ssm")
    mod("mamba_ssm.ops")
    mod("mamba_ssm.ops.selective_scan_interface", mamba_inner_fn=mamba_inner_fn,
        # placeholder; gen_golden rebinds the reference's own _selective_scan_ref
        selective_scan_fn=lambda *a, **k: (_ for _ in ()).throw(RuntimeError("unbound")))
    mod("mamba_ssm.ops.triton")
    mod("mamba_ssm.ops.triton.selective_state_update",
        selective_state_update=selective_state_update)
    mod("mamba_ssm.ops.triton.layer_norm", RMSNorm=RMSNorm, layer_norm_fn=layer_norm_fn,
        rms_norm_fn=rms_norm_fn)
    mod("timm")
    mod("timm.layers")
    mod("timm.layers.drop", DropPath=DropPath)
    mod("timm.layers.helpers", to_2tuple=to_2tuple)
    mod("timm.layers.weight_init", trunc_normal_=trunc_normal_)
    mod("timm.models")
    mod("timm.models.vision_transformer", _cfg=_cfg, _load_weights=_load_weights)
