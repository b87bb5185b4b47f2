"""VideoMamba encoder on the HIP kernels (``models/videomamba/videomamba.py`` surface).

Public classes and functions keep the reference's names, signatures, state_dict keys,
initialisation, error types and messages: ``Block``, ``create_block``, ``PatchEmbed``,
``PretrainVideoMamba``, ``load_state_dict``, ``build_videomamba``.

``PretrainVideoMamba.forward_features`` runs its own layer loop on a padded token buffer
(B, Lp, C), Lp = round_up(L, 8), padded rows held at exactly zero:

    tubelet patch embed + pos adds (HIP, MFMA) -> [CLS row] -> optional mask gather
    per layer: fused residual-add + RMSNorm (HIP) -> Mamba mixer (HIP conv/scan + GEMMs)
    final add + norm fused with the pooling sums (HIP) -> pool tail + LayerNorm (HIP)
    -> (x_vis, x_pool[, state])

which is the same computation as calling ``Block.forward`` per layer on the unpadded
tokens (``Block.forward`` itself is kept for callers that use blocks directly).
"""

from __future__ import annotations

import logging
import math
import threading
from functools import partial
from typing import Any, Callable, Dict, List, Optional, Tuple, Union, cast

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch import Tensor

from . import kernels as K
from . import options
from . import phase_lock as _phase
from .layers import DropPath, RMSNorm, round_up, to_2tuple, trunc_normal_, warn_if_grad
from .mamba_simple import InferenceParamsLike, Mamba
from .streaming import (STREAMING_CONTRACT_VERSION, ForwardReturnSemantics, StateShape,
                        forward_return_semantics as _return_semantics)

logger = logging.getLogger(__name__)

LayerState = Union[Tensor, Tuple[Tensor, Tensor]]
StateCollection = Union[List[LayerState], Tuple[LayerState, ...], Dict[int, LayerState]]


def _infer_spatial_grid(token_count: int, reference_grid: Tuple[int, int]) -> Tuple[int, int]:
    """Factor ``token_count`` into (h, w) closest in aspect ratio, then size, to the
    reference grid (``videomamba.py:32-55``)."""
    if token_count <= 0:
        raise ValueError("Position embedding must contain at least one spatial token.")
    rh, rw = reference_grid
    target = float(rh) / float(rw)
    candidates = []
    for h in range(1, int(math.sqrt(token_count)) + 1):
        if token_count % h == 0:
            w = token_count // h
            candidates += [(h, w), (w, h)]
    if not candidates:
        raise ValueError(f"Unable to infer spatial grid from token count {token_count}.")
    return min(candidates, key=lambda hw: (abs(hw[0] / hw[1] - target),
                                           abs(hw[0] - rh) + abs(hw[1] - rw)))


def _norm_kind(norm: nn.Module) -> bool:
    """True for RMSNorm, False for LayerNorm (the two norms fused_add_norm supports)."""
    return isinstance(norm, RMSNorm)


# ----------------------------------------------------------------------------- Block
class NextNorm:
    """The next block's fused add + RMSNorm, offered to a mixer's out_proj
    (vm_linear_add_norm_fwd): the norm's fp32 weight and eps, the residual stream (updated in
    place), the buffer for the normalised rows, and whether the out_proj did it."""

    def __init__(self, w32: Tensor, eps: float):
        self.w32, self.eps = w32, eps
        self.residual: Optional[Tensor] = None
        self.hn: Optional[Tensor] = None
        self.done = False


# ----------------------------------------------------------------------------- Block
class Block(nn.Module):
    """Add -> norm -> mixer block returning (hidden_states, residual[, state])
    (``videomamba.py:87-253``)."""

    def __init__(self, dim: int, mixer_cls: Callable[[int], nn.Module],
                 norm_cls: Callable[[int], nn.Module] = nn.LayerNorm,
                 fused_add_norm: bool = False, residual_in_fp32: bool = False,
                 drop_path: float = 0.0):
        super().__init__()
        self.residual_in_fp32 = residual_in_fp32
        self.fused_add_norm = fused_add_norm
        self.mixer = mixer_cls(dim)
        self.norm = norm_cls(dim)
        self.drop_path = DropPath(drop_path) if drop_path > 0.0 else nn.Identity()
        if self.fused_add_norm:
            assert isinstance(self.norm, (nn.LayerNorm, RMSNorm)), \
                "Only LayerNorm and RMSNorm are supported for fused_add_norm"

    def _add_norm(self, hidden_states: Tensor, residual: Optional[Tensor], inplace: bool = False):
        nw, nb, eps = self.norm.weight, self.norm.bias, self.norm.eps
        is_rms = _norm_kind(self.norm)
        if self.fused_add_norm:
            h = hidden_states if residual is None else self.drop_path(hidden_states)
            # internal residual buffers are updated in place; a caller's tensor never is
            return K._norm(h, nw, nb, residual, True, self.residual_in_fp32, eps, is_rms,
                           residual_out=residual if inplace and residual is not None else None,
                           owner=self.norm)
        residual = hidden_states if residual is None else residual + self.drop_path(hidden_states)
        hidden = K._norm(residual.to(nw.dtype), nw, nb, None, False, False, eps, is_rms,
                         owner=self.norm)
        if self.residual_in_fp32:
            residual = residual.to(torch.float32)
        return hidden, residual

    def forward(self, hidden_states: Tensor, residual: Optional[Tensor] = None,
                inference_params: Optional[InferenceParamsLike] = None,
                use_checkpoint: bool = False, ssm_state: Optional[Tensor] = None,
                state: Optional[Tuple[Tensor, Tensor]] = None, return_state: bool = False):
        """hidden_states = Mixer(Norm(residual + hidden_states)).  ``use_checkpoint`` is
        accepted for API parity (the HIP path is inference-only, nothing to recompute)."""
        if state is not None and ssm_state is not None:
            raise ValueError("Pass either state or ssm_state, not both.")
        K.require_gpu(hidden_states, residual, what="VideoMamba")
        with torch.no_grad():
            hidden, residual = self._add_norm(hidden_states, residual)
        if state is not None:
            if return_state:
                hidden, new_state = self.mixer(hidden, inference_params=inference_params,
                                               state=state, return_state=True)
                return hidden, residual, new_state
            hidden = self.mixer(hidden, inference_params=inference_params, state=state,
                                return_state=False)
            return hidden, residual
        hidden = self.mixer(hidden, inference_params=inference_params, ssm_state=ssm_state)
        return hidden, residual

    def forward_padded(self, hidden: Tensor, residual: Optional[Tensor], seqlen: int,
                       state=None, ssm_state=None, return_state: bool = False, conv_out=None,
                       pre: Optional["NextNorm"] = None, next_norm: Optional["NextNorm"] = None):
        """Model-internal: same as ``forward`` on the padded (B, Lp, C) buffers.  ``pre``: the
        previous block's out_proj already ran this block's add + norm (``pre.done``): use its
        normalised rows and updated residual.  ``next_norm``: offer the NEXT block's norm to
        this block's out_proj (vm_linear_add_norm_fwd)."""
        idx = getattr(self, "layer_idx", None)
        _phase.pre_start(idx)  # sub-batch streams: after the previous part's pre phase
        if pre is not None and pre.done:
            hn, residual = pre.hn, pre.residual
        else:
            hn, residual = self._add_norm(hidden, residual, inplace=True)
        if next_norm is not None:
            next_norm.residual = residual
            next_norm.hn = torch.empty_like(hn)
        res = self.mixer.forward_padded(hn, seqlen, ssm_state=ssm_state, state=state,
                                        return_state=return_state, conv_out=conv_out,
                                        next_norm=next_norm)
        _phase.pre_done(idx)  # (the token-major mixer marked it after conv_proj already)
        if return_state:
            return res[0], residual, res[1]
        return res, residual, None

    def allocate_inference_cache(self, batch_size: int, max_seqlen: int, dtype=None, **kwargs):
        return self.mixer.allocate_inference_cache(batch_size, max_seqlen, dtype=dtype, **kwargs)


def create_block(d_model: int, ssm_cfg: Optional[Dict[str, object]] = None,
                 norm_epsilon: float = 1e-5, drop_path: float = 0.0, rms_norm: bool = True,
                 residual_in_fp32: bool = True, fused_add_norm: bool = True,
                 layer_idx: Optional[int] = None, bimamba: bool = True, device=None, dtype=None):
    """``videomamba.py:256-291``: blocks are always unidirectional (bimamba=False); the
    bidirectional composition lives in ``BiMambaRefinerBlock``."""
    fk = {k: v for k, v in (("device", device), ("dtype", dtype)) if v is not None}
    mixer_cls = partial(Mamba, layer_idx=layer_idx, bimamba=False, **(ssm_cfg or {}), **fk)
    norm_cls = partial(RMSNorm if rms_norm else nn.LayerNorm, eps=norm_epsilon)
    block = Block(d_model, mixer_cls, norm_cls=norm_cls, drop_path=drop_path,
                  fused_add_norm=fused_add_norm, residual_in_fp32=residual_in_fp32)
    object.__setattr__(block, "layer_idx", layer_idx)
    return block


def _init_weights(module, n_layer, initializer_range=0.02, rescale_prenorm_residual=True,
                  n_residuals_per_layer=1):
    """Mamba init (``videomamba.py:295-324``): zero Linear biases (except dt bias), and
    kaiming-uniform / sqrt(n_layer) for every mixer's out_proj."""
    if isinstance(module, nn.Linear):
        if module.bias is not None and not getattr(module.bias, "_no_reinit", False):
            nn.init.zeros_(module.bias)
    elif isinstance(module, nn.Embedding):
        nn.init.normal_(module.weight, std=initializer_range)
    if rescale_prenorm_residual:
        for name, p in module.named_parameters():
            if name in ("out_proj.weight", "fc2.weight"):
                nn.init.kaiming_uniform_(p, a=math.sqrt(5))
                with torch.no_grad():
                    p /= math.sqrt(n_residuals_per_layer * n_layer)


def segm_init_weights(m):
    if isinstance(m, nn.Linear):
        trunc_normal_(m.weight, std=0.02)
        if m.bias is not None:
            nn.init.constant_(m.bias, 0)
    elif isinstance(m, nn.LayerNorm):
        nn.init.constant_(m.bias, 0)
        nn.init.constant_(m.weight, 1.0)


# ----------------------------------------------------------------------------- patch embed
class PatchEmbed(nn.Module):
    """Tubelet embedding Conv3d(kernel = stride = (kernel_size, ph, pw)), square or
    rectangular patches as in ``videomamba.py:340-364``; the conv runs as the HIP
    implicit-GEMM kernel."""

    def __init__(self, img_size=224, patch_size=16, kernel_size=1, in_chans=3, embed_dim=768):
        super().__init__()
        img = to_2tuple(img_size)
        patch = to_2tuple(patch_size)
        self.img_size = img
        self.patch_size = patch
        self.num_patches = (img[1] // patch[1]) * (img[0] // patch[0])
        self.tubelet_size = kernel_size
        self.proj = nn.Conv3d(in_chans, embed_dim, kernel_size=(kernel_size, patch[0], patch[1]),
                              stride=(kernel_size, patch[0], patch[1]))

    def embed_tokens(self, x: Tensor, spos: Tensor, tpos: Tensor, out: Tensor, row0: int,
                     cls: Optional[Tensor] = None, cls_pos: Optional[Tensor] = None,
                     pad_rows: int = 0):
        K.patch_embed(x, self.proj.weight, self.proj.bias, spos, tpos, out, row0,
                      out.stride(0), cls=cls, cls_pos=cls_pos, pad_rows=pad_rows,
                      bias32=K.f32_cached(self, self.proj.bias, "b"))

    def forward(self, x: Tensor) -> Tensor:
        K.require_gpu(x, what="PatchEmbed")
        B, _, T, H, W = x.shape
        ph, pw = self.patch_size
        Tt, Gh, Gw = T // self.tubelet_size, H // ph, W // pw
        C = self.proj.out_channels
        dt = self.proj.weight.dtype
        out = torch.empty((B, Tt * Gh * Gw, C), dtype=dt, device=x.device)
        with torch.no_grad():
            zs = torch.zeros((Gh * Gw, C), dtype=dt, device=x.device)
            zt = torch.zeros((Tt, C), dtype=dt, device=x.device)
            self.embed_tokens(x, zs, zt, out, 0)
        return out.view(B, Tt, Gh, Gw, C).permute(0, 4, 1, 2, 3)


# ----------------------------------------------------------------------------- encoder
class _ThreadStreams(threading.local):
    by_device: Optional[Dict[Any, List[torch.cuda.Stream]]] = None


_SIDE_STREAMS = _ThreadStreams()


def _side_streams(device: torch.device, n: int) -> List[torch.cuda.Stream]:
    """n persistent HIP streams of ``device`` for sub-batch forwards, created once per
    calling host thread.  Per thread because two callers' split forwards on shared streams
    could deadlock the device: each part waits on its partner's phase events, and with both
    callers' parts interleaved on the same two streams a wait of one caller can sit behind
    the other caller's wait on work queued after it.  The first runs at high priority: its
    kernels dispatch first, so the halves drift apart and one's scan meets the other's
    memory-bound kernels more often (B = 896: 825-831 vs 838-843 ms per step,
    profiles/r05zn_stream_priority.jsonl)."""
    if _SIDE_STREAMS.by_device is None:
        _SIDE_STREAMS.by_device = {}
    key = (device.type, device.index)
    have = _SIDE_STREAMS.by_device.setdefault(key, [])
    while len(have) < n:
        have.append(torch.cuda.Stream(device, priority=-1 if not have else 0))
    return have[:n]


def _issue_phase_locked(issue: Callable[[int], None], lock: "_phase.PhaseLock", parts: int,
                        device: torch.device) -> None:
    """Issue sub-batch ``i`` by ``issue(i)`` under ``lock`` (phase_lock.py): part 0 from the
    calling thread, the others from one host thread each, with the caller's device, grad
    and inference modes (thread-local in torch).  A failing part releases its phase events
    so the others drain; the first error is raised after every part returned."""
    grad, infer = torch.is_grad_enabled(), torch.is_inference_mode_enabled()
    errors: List[Optional[BaseException]] = [None] * parts

    def work(i: int) -> None:
        _phase.bind(lock, i)
        try:
            with torch.cuda.device(device), torch.inference_mode(infer), \
                    torch.set_grad_enabled(grad):
                issue(i)
        except BaseException as e:  # noqa: BLE001 - re-raised below, on the caller's thread
            errors[i] = e
            lock.release(i)
        finally:
            _phase.bind(None, 0)

    threads = [threading.Thread(target=work, args=(i,), daemon=True) for i in range(1, parts)]
    for t in threads:
        t.start()
    work(0)
    for t in threads:
        t.join()
    for e in errors:
        if e is not None:
            raise e


class PretrainVideoMamba(nn.Module):
    streaming_contract_version: str = STREAMING_CONTRACT_VERSION

    def __init__(self, img_size: int = 224, patch_size: int = 16, depth: int = 24,
                 embed_dim: int = 192, channels: int = 3, drop_path_rate: float = 0.0,
                 ssm_cfg: Optional[Dict[str, object]] = None, norm_epsilon: float = 1e-5,
                 initializer_cfg: Optional[Dict[str, object]] = None,
                 fused_add_norm: bool = True, rms_norm: bool = True,
                 residual_in_fp32: bool = True, bimamba: bool = True,
                 pool_type: str = "cls+avg", kernel_size: int = 1, num_frames: int = 8,
                 device=None, dtype=None, use_checkpoint: bool = False,
                 checkpoint_num: int = 0, add_pool_norm: bool = True):
        fk = {k: v for k, v in (("device", device), ("dtype", dtype)) if v is not None}
        super().__init__()
        if not bimamba:
            raise NotImplementedError(
                "This minimal VideoMamba package only supports bimamba=True.")
        self.residual_in_fp32 = residual_in_fp32
        self.fused_add_norm = fused_add_norm
        self.use_checkpoint = use_checkpoint
        self.checkpoint_num = checkpoint_num
        self.depth = depth
        self.pool_type = pool_type
        logger.info("Use checkpoint: %s, checkpoint number: %s, pool type: %s",
                    use_checkpoint, checkpoint_num, pool_type)
        self.d_model = self.num_features = self.embed_dim = embed_dim

        self.patch_embed = PatchEmbed(img_size=img_size, patch_size=patch_size,
                                      kernel_size=kernel_size, in_chans=channels,
                                      embed_dim=embed_dim)
        num_patches = self.patch_embed.num_patches
        self.cls_token = nn.Parameter(torch.zeros(1, 1, embed_dim))
        self.pos_embed = nn.Parameter(torch.zeros(1, num_patches + 1, embed_dim))
        self.temporal_pos_embedding = nn.Parameter(
            torch.zeros(1, num_frames // kernel_size, embed_dim))
        dpr = [v.item() for v in torch.linspace(0, drop_path_rate, depth)]
        inter_dpr = [0.0] + dpr
        self.drop_path = DropPath(drop_path_rate) if drop_path_rate > 0.0 else nn.Identity()
        self.layers = nn.ModuleList([
            create_block(embed_dim, ssm_cfg=ssm_cfg, norm_epsilon=norm_epsilon,
                         rms_norm=rms_norm, residual_in_fp32=residual_in_fp32,
                         fused_add_norm=fused_add_norm, layer_idx=i, bimamba=bimamba,
                         drop_path=inter_dpr[i], **fk)
            for i in range(depth)])
        self.norm = (RMSNorm if rms_norm else nn.LayerNorm)(embed_dim, eps=norm_epsilon, **fk)
        self.add_pool_norm = add_pool_norm
        if add_pool_norm:
            self.pool_norm = nn.LayerNorm(embed_dim)

        self.apply(segm_init_weights)
        trunc_normal_(self.pos_embed, std=0.02)
        self.apply(partial(_init_weights, n_layer=depth, **(initializer_cfg or {})))

    # ------------------------------------------------------------------ state API
    def _mixers(self):
        return [layer.mixer for layer in self.layers]

    def allocate_inference_cache(self, batch_size: int, max_seqlen: int, dtype=None, **kwargs):
        return {i: layer.allocate_inference_cache(batch_size, max_seqlen, dtype=dtype, **kwargs)
                for i, layer in enumerate(self.layers)}

    def init_ssm_state(self, batch_size: int, dtype=None, device=None, as_dict: bool = False):
        states = []
        for layer in self.layers:
            _, s = layer.allocate_inference_cache(batch_size, max_seqlen=1, dtype=dtype)
            states.append(s if device is None else s.to(device=device))
        return dict(enumerate(states)) if as_dict else states

    def allocate_state(self, batch_size: int, dtype=None, device=None, as_dict: bool = False):
        """Per-layer zero (conv_state, ssm_state) for chunked execution (contract
        ``self.streaming_contract_version``)."""
        states = [m.allocate_state(batch_size, dtype=dtype, device=device) for m in self._mixers()]
        return dict(enumerate(states)) if as_dict else states

    def init_state(self, batch_size: int, dtype=None, device=None, as_dict: bool = False):
        """Backward-compatible alias for ``allocate_state``."""
        return self.allocate_state(batch_size=batch_size, dtype=dtype, device=device,
                                   as_dict=as_dict)

    def expected_state_shapes(self, batch_size: int) -> Dict[int, StateShape]:
        if batch_size <= 0:
            raise ValueError("batch_size must be a positive integer.")
        return {i: StateShape(conv_state=(batch_size, int(m.d_inner), int(m.d_conv)),
                              ssm_state=(batch_size, int(m.d_inner), int(m.d_state)))
                for i, m in enumerate(self._mixers())}

    def forward_return_semantics(self) -> ForwardReturnSemantics:
        return _return_semantics(self.add_pool_norm)

    @torch.jit.ignore()
    def no_weight_decay(self):
        return {"pos_embed", "cls_token", "temporal_pos_embedding"}

    def get_num_layers(self):
        return len(self.layers)

    @torch.jit.ignore()
    def load_pretrained(self, checkpoint_path, prefix=""):
        raise NotImplementedError("ViT .npz weight loading is not part of the VideoMamba "
                                  "encoder; use load_state_dict(...) with a plain state_dict.")

    # ------------------------------------------------------------------ helpers
    def _get_layer_state(self, state, layer_idx: int):
        if state is None:
            return None
        if isinstance(state, dict):
            return state.get(layer_idx)
        if isinstance(state, (list, tuple)):
            return state[layer_idx]
        raise TypeError("state must be a list, tuple, or dict indexed by layer id")

    def _validate_temporal_length(self, frame_count: int) -> int:
        k = self.patch_embed.tubelet_size
        if frame_count <= 0:
            raise ValueError("Input must contain at least one frame.")
        if frame_count % k:
            raise ValueError(
                f"Input frame count ({frame_count}) must be divisible by tubelet size ({k}).")
        return frame_count // k

    def _spatial_token_grid(self, height: int, width: int) -> Tuple[int, int]:
        ph, pw = self.patch_embed.patch_size
        if height < ph or width < pw:
            raise ValueError("Input spatial size must be at least one patch: "
                             f"got ({height}, {width}) with patch size ({ph}, {pw}).")
        return height // ph, width // pw

    def _get_spatial_pos_embedding(self, grid_h: int, grid_w: int, dtype=None, device=None):
        device = self.pos_embed.device if device is None else device
        dtype = self.pos_embed.dtype if dtype is None else dtype
        patch_pos = self.pos_embed[:, 1:]
        ph, pw = self.patch_embed.patch_size
        bh, bw = self.patch_embed.img_size[0] // ph, self.patch_embed.img_size[1] // pw
        if bh * bw != patch_pos.shape[1]:
            bh, bw = _infer_spatial_grid(patch_pos.shape[1], (bh, bw))
        if (grid_h, grid_w) == (bh, bw):
            return patch_pos.to(device=device, dtype=dtype)
        grid = patch_pos.reshape(1, bh, bw, self.embed_dim).permute(0, 3, 1, 2).float()
        grid = F.interpolate(grid, size=(grid_h, grid_w), mode="bicubic", align_corners=False)
        return grid.permute(0, 2, 3, 1).reshape(1, grid_h * grid_w, self.embed_dim).to(
            device=device, dtype=dtype)

    def _has_cls_token_for_forward(self, ssm_state, temporal_pos_offset: int) -> bool:
        if ssm_state is None or temporal_pos_offset <= 0:
            return True
        first = self._get_layer_state(ssm_state, 0)
        return not (isinstance(first, (list, tuple)) and len(first) == 2)

    def _get_temporal_pos_embedding(self, seqlen: int, offset: int = 0, dtype=None, device=None):
        """Temporal embedding slice [offset, offset+seqlen); linearly interpolated to
        ``offset+seqlen`` entries when that exceeds the table (``videomamba.py:655-675``)."""
        if offset < 0:
            raise ValueError("temporal_pos_offset must be non-negative.")
        device = self.temporal_pos_embedding.device if device is None else device
        dtype = self.temporal_pos_embedding.dtype if dtype is None else dtype
        table = self.temporal_pos_embedding.to(device=device, dtype=dtype)
        end = offset + seqlen
        if end > table.shape[1]:
            table = F.interpolate(table.permute(0, 2, 1).float(), size=end, mode="linear",
                                  align_corners=False).permute(0, 2, 1).to(dtype=dtype)
        return table[:, offset:end]

    def _normalize_mask(self, mask, batch_size, token_count, device, require_cls_visible):
        if mask is None:
            return None
        if mask.ndim != 2:
            raise ValueError("mask must be 2D with shape [B, N].")
        if mask.shape[0] != batch_size:
            raise ValueError(
                f"mask batch size mismatch: expected {batch_size}, got {mask.shape[0]}.")
        mask = mask.to(device=device, dtype=torch.bool)
        if mask.shape[1] != token_count:
            raise ValueError(
                f"mask token length mismatch: expected {token_count}, got {mask.shape[1]}.")
        if require_cls_visible and token_count > 0 and bool(mask[:, 0].any()):
            raise ValueError("mask must keep CLS token visible (mask[:, 0] must be False).")
        return mask

    def _visible_token_positions(self, mask, batch_size, token_count, device,
                                 require_cls_visible):
        """(normalized mask, ascending visible positions per sample) or (None, None)."""
        mask = self._normalize_mask(mask, batch_size, token_count, device, require_cls_visible)
        if mask is None:
            return None, None
        visible = ~mask
        counts = visible.sum(dim=1)
        if counts.numel() > 0 and not bool((counts == counts[0]).all()):
            raise ValueError("mask must keep the same number of visible tokens per sample; "
                             f"got per-sample counts: {counts.tolist()}.")
        n_vis = int(counts[0].item()) if counts.numel() > 0 else 0
        if counts.numel() > 0 and n_vis <= 0:
            raise ValueError("mask must keep at least one visible token per sample.")
        pos = torch.arange(token_count, device=device).unsqueeze(0).expand(batch_size, -1)
        pos = pos.masked_fill(mask, token_count)
        return mask, torch.sort(pos, dim=1).values[:, :n_vis]

    def _frame_bounds(self, visible_positions, temporal_tokens, tokens_per_frame,
                      has_cls_token):
        """Row bounds (B, T'+1) int32 of each frame's visible patch tokens in the gathered
        order, plus the largest frame; the masked keep_temporal groups of
        ``videomamba.py:702-751`` (positions are ascending, so a frame's tokens are
        contiguous).  Raises the reference's ValueError when a frame has none."""
        head = 1 if has_cls_token else 0
        starts = head + torch.arange(temporal_tokens + 1, device=visible_positions.device,
                                     dtype=visible_positions.dtype) * tokens_per_frame
        bounds = torch.searchsorted(visible_positions.contiguous(),
                                    starts.expand(visible_positions.shape[0], -1).contiguous())
        counts = bounds[:, 1:] - bounds[:, :-1]
        if counts.numel() and bool((counts == 0).any()):
            raise ValueError("keep_temporal with masking requires at least one visible patch "
                             "token for each temporal slice.")
        return bounds.to(torch.int32).contiguous(), int(counts.max().item())

    # ------------------------------------------------------------------ layer loop
    def _run_layers(self, h, residual, L, ssm_state, conv_out=None):
        """The depth loop over padded buffers: (h, residual, new_states|None, tuple_out).
        ``conv_out`` (depth, B, D, d_conv) receives the new conv states (graph runner)."""
        new_states = None
        tuple_out = False
        fuse = self._fuse_out_norm_ok(h)
        pending = None
        for idx, layer in enumerate(self.layers):
            nxt = None
            if fuse and idx + 1 < len(self.layers):
                nn_ = self.layers[idx + 1].norm
                nxt = NextNorm(K.f32_cached(nn_, nn_.weight, "w"), nn_.eps)
            layer_state = self._get_layer_state(ssm_state, idx)
            full = isinstance(layer_state, (list, tuple)) and len(layer_state) == 2
            if full and new_states is None:
                if isinstance(ssm_state, dict):
                    new_states = {}
                else:
                    new_states = [None] * len(self.layers)
                    tuple_out = isinstance(ssm_state, tuple)
            if full:
                h, residual, layer_state = layer.forward_padded(
                    h, residual, L, state=tuple(layer_state), return_state=True,
                    conv_out=None if conv_out is None else conv_out[idx], pre=pending,
                    next_norm=nxt)
            else:
                h, residual, _ = layer.forward_padded(h, residual, L, ssm_state=layer_state,
                                                      pre=pending, next_norm=nxt)
            if new_states is not None:
                new_states[idx] = layer_state
            pending = nxt
        return h, residual, new_states, tuple_out

    def _fuse_out_norm_ok(self, h: Tensor) -> bool:
        """Every block's add + norm after the first may run inside the previous block's
        out_proj (vm_linear_add_norm_fwd) when the blocks use the fused RMSNorm with an fp32
        residual on bf16 activations and no stochastic depth is active; each mixer then
        decides per call (its out_proj must take the row-invariant HIP GEMM)."""
        if not options.get().fuse_out_norm or h.dtype != torch.bfloat16:
            return False
        C = self.embed_dim
        if C % 8 or C > 1024:
            return False
        for layer in self.layers:
            if not (layer.fused_add_norm and layer.residual_in_fp32 and _norm_kind(layer.norm)
                    and (isinstance(layer.drop_path, nn.Identity) or not layer.training)):
                return False
        return True

    def _final_norm_pool(self, h, residual, L, has_cls, visible, pool, out=None):
        """Final add + norm of the padded buffer straight into contiguous (B, L, C)
        features, fused with the pooling sums (``vm_norm_pool_fwd``), then the pool tail
        (``vm_pool_finish_fwd``): (features, x_pool | None).  ``pool`` is None (no pooling)
        or (keep_temporal, temporal_tokens, tokens_per_frame)."""
        nw, nb, eps = self.norm.weight, self.norm.bias, self.norm.eps
        is_rms = _norm_kind(self.norm)
        C = self.embed_dim
        if C % 4 or C > 2048:
            raise NotImplementedError(f"embed_dim {C}: the HIP final norm takes C % 4 == 0, "
                                      "C <= 2048")
        if not self.fused_add_norm:  # ``:896-901``: add in the residual dtype, cast, norm
            residual = h if residual is None else residual + self.drop_path(h)
            h, residual = residual.to(nw.dtype).contiguous(), None
        elif residual is not None and residual.dtype != h.dtype and not self.residual_in_fp32:
            residual = residual.to(h.dtype)
        w32, b32 = K.f32_cached(self.norm, nw, "w"), K.f32_cached(self.norm, nb, "b")
        head = 1 if has_cls else 0
        npatch = L - head
        mode = self.pool_type
        sums = pool is not None and mode != "cls"
        groups, group_rows, bounds, max_rows = 1, npatch, None, npatch
        if sums:
            if npatch == 0:
                raise ValueError("mask must keep at least one patch token visible when using "
                                 f"pool_type='{mode}'.")
            keep_temporal, tt, per_frame = pool
            if keep_temporal:
                if visible is None:
                    groups, group_rows, max_rows = tt, per_frame, per_frame
                else:
                    bounds, max_rows = self._frame_bounds(visible, tt, per_frame, has_cls)
                    groups, group_rows = tt, 0
        feats, ws = K.norm_pool(h, residual, L, w32, b32, eps, is_rms, head=head,
                                groups=groups, group_rows=group_rows, bounds=bounds,
                                max_group_rows=max_rows, sums=sums, out=out)
        if pool is None:
            return feats, None
        pn = self.pool_norm
        if not isinstance(pn, nn.LayerNorm) or len(pn.normalized_shape) != 1:
            raise NotImplementedError("pool_norm must be an nn.LayerNorm over the channels")
        x_pool = K.pool_finish(ws, feats, mode=mode, keep_temporal=bool(pool[0]),
                               groups=groups, group_rows=group_rows, bounds=bounds,
                               max_group_rows=max_rows, has_cls=has_cls,
                               lnw32=K.f32_cached(pn, pn.weight, "w"),
                               lnb32=K.f32_cached(pn, pn.bias, "b"), ln_eps=pn.eps)
        return feats, x_pool

    # ------------------------------------------------------------------ forward
    def _embed(self, x: Tensor, has_cls: bool, temporal_pos_offset: int, tpos=None):
        """Patch embed + positional adds (+ CLS row) into a zero-padded (B, Lp, C) buffer.
        ``tpos`` (1, T', C) replaces the temporal-embedding slice (graph replay keeps it in a
        static buffer that is refilled per chunk)."""
        Bsz, _, T, H, W = x.shape
        k = self.patch_embed.tubelet_size
        ph, pw = self.patch_embed.patch_size
        Tt, Gh, Gw = T // k, H // ph, W // pw
        dt = self.patch_embed.proj.weight.dtype
        spos = self._get_spatial_pos_embedding(Gh, Gw, dtype=dt, device=x.device)
        if tpos is None:
            tpos = self._get_temporal_pos_embedding(Tt, offset=temporal_pos_offset, dtype=dt,
                                                    device=x.device)
        L = Tt * Gh * Gw + (1 if has_cls else 0)
        Lp = round_up(L)
        buf = torch.empty((Bsz, Lp, self.embed_dim), dtype=dt, device=x.device)
        # the CLS row (cls_token + pos_embed[:, :1] in the model dtype) and the zero padding
        # rows are written by the patch-embed launch itself
        cls = self.cls_token.detach().to(dt) if has_cls else None
        cls_pos = self.pos_embed.detach()[0, 0].to(dt) if has_cls else None
        self.patch_embed.embed_tokens(x, spos[0], tpos[0], buf, 1 if has_cls else 0,
                                      cls=cls, cls_pos=cls_pos, pad_rows=Lp - L)
        return buf, L, Tt, Gh * Gw

    def forward_features(self, x: Tensor, mask: Optional[Tensor] = None, use_image: bool = False,
                         ssm_state: Optional[StateCollection] = None,
                         temporal_pos_offset: int = 0):
        """Features (B, N_vis, C) [+ next state] (``videomamba.py:786-941``)."""
        if x.ndim != 5:
            raise ValueError("x must have shape [B, C, T, H, W].")
        self._validate_temporal_length(x.shape[2])
        K.require_gpu(x, what="VideoMamba")
        warn_if_grad(x, self.patch_embed.proj.weight)
        with torch.no_grad():
            return self._forward_features(x, mask, ssm_state, temporal_pos_offset)

    def _forward_features(self, x, mask, ssm_state, temporal_pos_offset, tpos=None):
        feats, _, st = self._encode(x, mask, ssm_state, temporal_pos_offset, tpos=tpos)
        return feats if ssm_state is None else (feats, st)

    def _encode(self, x, mask, ssm_state, temporal_pos_offset, tpos=None, pool=None,
                conv_out=None, feats_out=None, split=True):
        """(features (B, N_vis, C), x_pool | None, state result | None).  ``feats_out``: a
        (B, N_vis, C) buffer with contiguous rows the features are written into; ``split``
        False keeps this call on the current stream (a sub-batch never splits again)."""
        parts = (self._stream_parts(x, ssm_state, tpos, conv_out)
                 if split and mask is None and feats_out is None else 1)
        if parts > 1:
            return self._encode_streams(x, mask, ssm_state, temporal_pos_offset, pool, parts)
        has_cls = self._has_cls_token_for_forward(ssm_state, temporal_pos_offset)
        h, L, _, _ = self._embed(x, has_cls, temporal_pos_offset, tpos=tpos)
        Bsz = x.shape[0]
        _, visible = self._visible_token_positions(mask, Bsz, L, x.device,
                                                   require_cls_visible=has_cls)
        if visible is not None:
            gathered = h[:, :L].gather(1, visible.unsqueeze(-1).expand(-1, -1, self.embed_dim))
            L = gathered.shape[1]
            h = torch.zeros((Bsz, round_up(L), self.embed_dim), dtype=h.dtype, device=h.device)
            h[:, :L] = gathered

        h, residual, new_states, tuple_out = self._run_layers(h, None, L, ssm_state, conv_out)
        feats, x_pool = self._final_norm_pool(h, residual, L, has_cls, visible, pool,
                                              out=feats_out)

        if new_states is not None and isinstance(new_states, list):
            if any(s is None for s in new_states):
                raise ValueError("Expected full state for all layers.")
            st = tuple(new_states) if tuple_out else new_states
        elif ssm_state is None:
            st = None
        elif new_states is not None:
            st = new_states
        else:
            st = ssm_state
        return feats, x_pool, st

    # ------------------------------------------------------------------ batch streams
    def _stream_parts(self, x, ssm_state, tpos, conv_out) -> int:
        """How many sub-batches (one HIP stream each) this forward runs as:
        ``options.batch_streams`` from ``batch_stream_min_clips`` clips and
        ``batch_stream_min_work`` clip-channels (B x d_inner) up, outside graph
        capture and the graph runner's buffers, when every layer's state (if any) is one kind
        (full (conv, ssm) pairs of one conv dtype, or legacy ssm-only tensors).

        It also stays on one stream under autocast (thread-local in torch: the
        issue threads would not inherit it), with the fused out_proj + add + RMSNorm
        (``options.fuse_out_norm``: its pollers assume every producer workgroup of the
        launch runs, which a concurrent launch on another stream can prevent), and when the
        patch embed, the mixers and the final norm do not share one dtype (the split
        forward's shared features buffer takes that dtype; the one-stream forward writes the
        final norm's output dtype).  And it splits only where every projection runs on the
        row-invariant HIP GEMM (``projection_gemm == "hip"``, bf16, in_proj / out_proj K in
        the HIP GEMM's set, the fused conv_proj for x_proj): a library GEMM picks its kernel
        by the row count, so a half-batch could round differently from the whole batch, and
        the split forward promises the one-stream forward's bits."""
        o = options.get()
        n = int(o.batch_streams)
        B = x.shape[0]
        d_inner = int(self.layers[0].mixer.d_inner) if len(self.layers) else 0
        if (n <= 1 or B < max(int(o.batch_stream_min_clips), 2)
                or B * d_inner < int(o.batch_stream_min_work) or tpos is not None
                or conv_out is not None
                or (x.is_cuda and torch.cuda.is_current_stream_capturing())
                or torch.is_autocast_enabled("cuda") or o.fuse_out_norm
                or not self._row_invariant_projections(x, -(-B // min(n, B)))):
            return 1
        if ssm_state is not None:
            kinds = set()
            for idx in range(len(self.layers)):
                st = self._get_layer_state(ssm_state, idx)
                if isinstance(st, (list, tuple)) and len(st) == 2:
                    kinds.add(("full", st[0].dtype))
                elif isinstance(st, Tensor):
                    kinds.add(("ssm", None))
                else:
                    return 1
            if len(kinds) != 1:
                return 1
        return min(n, B)

    def _features_dtype(self) -> Optional[torch.dtype]:
        """The dtype every forward's features take when the patch embed, every mixer and
        the final norm share one parameter dtype (then the one-stream forward's final norm
        writes it whether or not ``fused_add_norm``); None when they differ."""
        dt = self.patch_embed.proj.weight.dtype
        if self.norm.weight.dtype != dt:
            return None
        for layer in self.layers:
            mx = layer.mixer
            if mx.in_proj.weight.dtype != dt or mx.out_proj.weight.dtype != dt:
                return None
        return dt

    def _row_invariant_projections(self, x: Tensor, part: int) -> bool:
        """Every mixer projection of a bf16 forward of ``part``-clip sub-batches of ``x``
        runs on the HIP GEMM (whose rows do not depend on the row count):
        ``options.projection_gemm == "hip"``, one bf16 dtype over the model, the token-major
        mixer, in_proj / out_proj K in vm_linear_fwd's unrolled set, no projection bias, and
        the fused conv_proj for x_proj (dt_proj runs in it or in the scan) at the sub-batch's
        extents (the longest chunk kind: with the CLS row)."""
        from .mamba_simple import _SMALL_GEMM_K
        o = options.get()
        if (o.projection_gemm != "hip" or o.mixer_layout == "cm"
                or self._features_dtype() != torch.bfloat16):
            return False
        gh, gw = self._spatial_token_grid(x.shape[-2], x.shape[-1])
        L = self._validate_temporal_length(x.shape[2]) * gh * gw + 1
        hn = torch.empty((1, 1, self.embed_dim), dtype=torch.bfloat16,
                         device=x.device).expand(part, round_up(L), self.embed_dim)
        for layer in self.layers:
            mx = layer.mixer
            if (mx.in_proj.weight.shape[1] not in _SMALL_GEMM_K
                    or mx.out_proj.weight.shape[1] not in _SMALL_GEMM_K
                    or mx.in_proj.bias is not None or mx.out_proj.bias is not None
                    or not mx._fused_conv_proj_ok(hn, L)):
                return False
        return True

    def _prepare_param_caches(self) -> None:
        """Materialise every parameter-derived cache (fp32 copies, padded projection
        weights) on the current stream before a forward forks into sub-batch streams: a
        cache first built inside one sub-batch's stream would be read by the others
        unordered."""
        for layer in self.layers:
            layer.mixer._fp32_params()
            layer.mixer._padded_proj_weights()
            K.f32_cached(layer.norm, layer.norm.weight, "w")
            K.f32_cached(layer.norm, getattr(layer.norm, "bias", None), "b")
        K.f32_cached(self.norm, self.norm.weight, "w")
        K.f32_cached(self.norm, getattr(self.norm, "bias", None), "b")
        pn = getattr(self, "pool_norm", None)
        if isinstance(pn, nn.LayerNorm):
            K.f32_cached(pn, pn.weight, "w")
            K.f32_cached(pn, pn.bias, "b")
        K.f32_cached(self.patch_embed, self.patch_embed.proj.bias, "b")

    def _encode_streams(self, x, mask, ssm_state, temporal_pos_offset, pool, parts):
        """_encode as ``parts`` sub-batches on their own streams, joined before returning.
        Sub-batch states are views of the caller's tensors (ssm states advance in place as
        in the one-stream forward); new conv states land in slices of one fresh buffer."""
        dev = x.device
        B = x.shape[0]
        cut = [B * i // parts for i in range(parts + 1)]
        cur = torch.cuda.current_stream(dev)
        streams = _side_streams(dev, parts)
        self._prepare_param_caches()
        depth = len(self.layers)
        full = False
        conv_new = None
        if ssm_state is not None:
            st0 = self._get_layer_state(ssm_state, 0)
            full = isinstance(st0, (list, tuple))
            if full:
                m0 = self.layers[0].mixer
                conv_new = torch.empty((depth, B, m0.d_inner, m0.d_conv), dtype=st0[0].dtype,
                                       device=dev)

        def part_state(a, b):
            if ssm_state is None:
                return None
            def sl(st):
                if isinstance(st, Tensor):
                    return st[a:b]
                return type(st)(t[a:b] for t in st) if isinstance(st, tuple) else [t[a:b] for t in st]
            if isinstance(ssm_state, dict):
                return {k: sl(v) for k, v in ssm_state.items()}
            items = [sl(v) for v in ssm_state]
            return tuple(items) if isinstance(ssm_state, tuple) else items

        # every part writes its rows of one features buffer (no concatenation pass)
        has_cls = self._has_cls_token_for_forward(ssm_state, temporal_pos_offset)
        gh, gw = self._spatial_token_grid(x.shape[-2], x.shape[-1])
        L = self._validate_temporal_length(x.shape[2]) * gh * gw + (1 if has_cls else 0)
        feats = torch.empty((B, L, self.embed_dim), dtype=self._features_dtype(), device=dev)
        outs: List[Any] = [None] * parts

        def issue(i: int) -> None:
            a, b = cut[i], cut[i + 1]
            with torch.cuda.stream(streams[i]):
                outs[i] = self._encode(
                    x[a:b], None, part_state(a, b), temporal_pos_offset, pool=pool,
                    conv_out=None if conv_new is None else conv_new[:, a:b],
                    feats_out=feats[a:b], split=False)

        for s in streams[:parts]:
            s.wait_stream(cur)
        if parts > 1 and options.get().batch_stream_lock:
            _issue_phase_locked(issue, _phase.PhaseLock(parts, depth), parts, dev)
        else:
            for i in range(parts):
                issue(i)
        for s in streams[:parts]:
            cur.wait_stream(s)
        x_pool = None if outs[0][1] is None else torch.cat([o[1] for o in outs], 0)
        if ssm_state is None:
            st = None
        elif full:
            def layer(idx):
                old = self._get_layer_state(ssm_state, idx)
                return (conv_new[idx], old[1])  # the ssm state advanced in place
            if isinstance(ssm_state, dict):  # as the one-stream path: one entry per layer
                st = {idx: layer(idx) for idx in range(depth)}
            else:
                items = [layer(idx) for idx in range(depth)]
                st = tuple(items) if isinstance(ssm_state, tuple) else items
        else:
            st = ssm_state  # legacy ssm-only tensors, advanced in place
        return feats, x_pool, st

    def forward(self, x: Tensor, mask: Optional[Tensor] = None, use_image: bool = False,
                keep_temporal: bool = False, ssm_state: Optional[StateCollection] = None,
                temporal_pos_offset: int = 0):
        """(x_vis, x_pool[, next_state]) with ``add_pool_norm``, else x_vis[, next_state]
        (``videomamba.py:943-1067``)."""
        if x.ndim != 5:
            raise ValueError("x must have shape [B, C, T, H, W].")
        gh, gw = self._spatial_token_grid(x.shape[-2], x.shape[-1])
        per_frame = gh * gw
        temporal_tokens = self._validate_temporal_length(x.shape[2])
        has_cls = self._has_cls_token_for_forward(ssm_state, temporal_pos_offset)
        if not self.add_pool_norm:
            return self.forward_features(x, mask, use_image, ssm_state=ssm_state,
                                         temporal_pos_offset=temporal_pos_offset)
        self._check_pool(has_cls)
        K.require_gpu(x, what="VideoMamba")
        warn_if_grad(x, self.patch_embed.proj.weight)
        with torch.no_grad():
            feats, x_pool, st = self._encode(x, mask, ssm_state, temporal_pos_offset,
                                             pool=(bool(keep_temporal), temporal_tokens,
                                                   per_frame))
        patch = feats[:, 1:] if has_cls else feats
        return (patch, x_pool) if ssm_state is None else (patch, x_pool, st)

    def _check_pool(self, has_cls: bool) -> None:
        pool = self.pool_type
        if pool not in K.POOL_MODES:
            raise ValueError(f"Unsupported pool_type: {pool}")
        if pool in {"cls", "cls+avg", "cls_cat_avg"} and not has_cls:
            raise ValueError(
                f"pool_type='{pool}' requires a CLS token, but continuation "
                "streaming chunks (temporal_pos_offset > 0 with full state) do not include CLS. "
                "Use pool_type='avg' for chunked streaming.")


# ----------------------------------------------------------------------------- loading
def load_state_dict(pretrained_path, model, ckpt_num_frame, num_frames):
    """Load a plain state_dict checkpoint with spatial (bicubic) and temporal (linear)
    positional-embedding interpolation (``videomamba.py:1070-1147``).  Only the
    ``weights_only=True`` loader is used."""
    logger.info("Loading pretrained weights from %s", pretrained_path)
    ckpt = torch.load(pretrained_path, map_location="cpu", weights_only=True)
    if not isinstance(ckpt, dict):
        raise TypeError("Expected a plain state_dict (dict) checkpoint.")
    if "model" in ckpt or "module" in ckpt:
        raise ValueError("Checkpoint wrapper keys ('model'/'module') are not supported. "
                         "Pass a plain state_dict checkpoint.")
    pe = model.patch_embed
    pos = ckpt["pos_embed"]
    C = pos.shape[-1]
    n_extra = model.pos_embed.shape[-2] - pe.num_patches
    gh, gw = pe.img_size[0] // pe.patch_size[0], pe.img_size[1] // pe.patch_size[1]
    if gh * gw != pe.num_patches:
        raise ValueError(f"Model patch grid size mismatch: {gh}x{gw} != num_patches({pe.num_patches}).")
    oh, ow = _infer_spatial_grid(pos.shape[-2] - n_extra, (gh, gw))
    if (oh, ow) != (gh, gw):
        logger.info("Position interpolate from %dx%d to %dx%d", oh, ow, gh, gw)
        grid = pos[:, n_extra:].reshape(-1, oh, ow, C).permute(0, 3, 1, 2)
        grid = F.interpolate(grid, size=(gh, gw), mode="bicubic", align_corners=False)
        grid = grid.permute(0, 2, 3, 1).reshape(-1, gh * gw, C)
        ckpt["pos_embed"] = torch.cat((pos[:, :n_extra], grid), dim=1)
    if ckpt_num_frame is None or ckpt_num_frame <= 0:
        raise ValueError("ckpt_num_frame must be a positive integer when loading pretrained weights.")
    t_old = ckpt_num_frame // pe.tubelet_size
    t_new = num_frames // pe.tubelet_size
    if t_old != t_new:
        logger.info("Temporal interpolate from %d to %d", t_old, t_new)
        tpe = ckpt["temporal_pos_embedding"].permute(0, 2, 1)
        tpe = F.interpolate(tpe, size=(t_new,), mode="linear", align_corners=False)
        ckpt["temporal_pos_embedding"] = tpe.permute(0, 2, 1)
    msg = model.load_state_dict(ckpt, strict=True)
    logger.info(msg)


_BUILD_FIELDS = ("channels", "img_size", "patch_size", "depth", "embed_dim", "drop_path_rate",
                 "ssm_cfg", "norm_epsilon", "fused_add_norm", "rms_norm", "residual_in_fp32",
                 "bimamba", "pool_type", "kernel_size", "num_frames", "use_checkpoint",
                 "checkpoint_num")


def build_videomamba(config, add_pool_norm=True):
    """Build from ``config.vision_encoder`` (``videomamba.py:1150-1200``); every field is
    required (``channels`` first: a config with ``in_chans`` raises AttributeError)."""
    vc = config.vision_encoder
    kw = {name: getattr(vc, name) for name in _BUILD_FIELDS}
    model = PretrainVideoMamba(add_pool_norm=add_pool_norm, **kw)
    object.__setattr__(model, "default_cfg", {"url": ""})
    pretrained = vc.pretrained
    if pretrained is not None:
        load_state_dict(pretrained_path=pretrained, model=model,
                        ckpt_num_frame=vc.ckpt_num_frame, num_frames=kw["num_frames"])
    else:
        logger.info("No pretrained weights!!!")
    return model
