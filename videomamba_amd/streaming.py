"""Streaming-state contract (public API surface).

Behaviour, names and error messages follow ``models/videomamba/streaming.py:7-133`` of
the reference so callers written against it work unchanged:
``STREAMING_CONTRACT_VERSION``, ``StateShape``, ``ForwardReturnSemantics``,
``forward_return_semantics``, ``model_forward_return_semantics``,
``expected_state_shapes``, ``allocate_state``, ``validate_state``.

Per layer the state is ``(conv_state, ssm_state)`` with shapes
``(B, d_inner, d_conv)`` and ``(B, d_inner, d_state)``.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Protocol, Sequence, Tuple, Union

import torch
from torch import Tensor

STREAMING_CONTRACT_VERSION = "1.0.0"

LayerState = Tuple[Tensor, Tensor]
StreamingState = Union[List[LayerState], Tuple[LayerState, ...], Dict[int, LayerState]]


@dataclass(frozen=True)
class StateShape:
    conv_state: Tuple[int, int, int]
    ssm_state: Tuple[int, int, int]


@dataclass(frozen=True)
class ForwardReturnSemantics:
    without_state: str
    with_state: str


def forward_return_semantics(add_pool_norm: bool) -> ForwardReturnSemantics:
    """Frozen return arity of ``PretrainVideoMamba.forward`` (README "Output API")."""
    if bool(add_pool_norm):
        return ForwardReturnSemantics("(x_vis, x_pool)", "(x_vis, x_pool, next_state)")
    return ForwardReturnSemantics("x_vis", "(x_vis, next_state)")


class _HasLayers(Protocol):
    layers: Sequence[object]
    add_pool_norm: bool


def model_forward_return_semantics(model: _HasLayers) -> ForwardReturnSemantics:
    return forward_return_semantics(bool(getattr(model, "add_pool_norm", True)))


def _mixer_dims(idx: int, layer: object) -> Tuple[int, int, int]:
    mixer = getattr(layer, "mixer", None)
    if mixer is None:
        raise TypeError(f"Layer {idx} does not expose a mixer attribute.")
    try:
        return (int(getattr(mixer, "d_inner")), int(getattr(mixer, "d_conv")),
                int(getattr(mixer, "d_state")))
    except (AttributeError, TypeError, ValueError) as exc:
        raise TypeError(
            f"Layer {idx} mixer does not expose integer d_inner/d_conv/d_state.") from exc


def expected_state_shapes(model: _HasLayers, batch_size: int) -> Dict[int, StateShape]:
    if batch_size <= 0:
        raise ValueError("batch_size must be a positive integer.")
    shapes: Dict[int, StateShape] = {}
    for idx, layer in enumerate(model.layers):
        d_inner, d_conv, d_state = _mixer_dims(idx, layer)
        shapes[idx] = StateShape(conv_state=(batch_size, d_inner, d_conv),
                                 ssm_state=(batch_size, d_inner, d_state))
    return shapes


def allocate_state(model: object, batch_size: int, dtype=None, device=None,
                   as_dict: bool = False) -> StreamingState:
    """Zero per-layer state via the model's ``allocate_state`` (or ``init_state``)."""
    for name in ("allocate_state", "init_state"):
        fn = getattr(model, name, None)
        if callable(fn):
            return fn(batch_size, dtype=dtype, device=device, as_dict=as_dict)
    raise TypeError("Model does not expose allocate_state(...) or init_state(...).")


def _layer_items(state: StreamingState, depth: int) -> List[object]:
    if isinstance(state, dict):
        want = set(range(depth))
        have = set(state.keys())
        if have != want:
            raise ValueError(
                f"State dict keys mismatch: expected {sorted(want)}, got {sorted(have)}.")
        return [state[i] for i in range(depth)]
    if isinstance(state, (list, tuple)):
        if len(state) != depth:
            raise ValueError(f"State length mismatch: expected {depth}, got {len(state)}.")
        return list(state)
    raise TypeError("State must be a list, tuple, or dict indexed by layer id.")


def validate_state(model: _HasLayers, state: StreamingState, batch_size: int) -> None:
    shapes = expected_state_shapes(model, batch_size)
    for idx, item in enumerate(_layer_items(state, len(shapes))):
        if not isinstance(item, (list, tuple)) or len(item) != 2:
            raise TypeError("Each layer state must be a 2-tuple: (conv_state, ssm_state).")
        conv_state, ssm_state = item
        if not (torch.is_tensor(conv_state) and torch.is_tensor(ssm_state)):
            raise TypeError("conv_state and ssm_state must both be tensors.")
        want = shapes[idx]
        got_conv, got_ssm = tuple(conv_state.shape), tuple(ssm_state.shape)
        if got_conv != want.conv_state:
            raise ValueError(f"Layer {idx} conv_state shape mismatch: expected "
                             f"{want.conv_state}, got {got_conv}.")
        if got_ssm != want.ssm_state:
            raise ValueError(f"Layer {idx} ssm_state shape mismatch: expected "
                             f"{want.ssm_state}, got {got_ssm}.")
