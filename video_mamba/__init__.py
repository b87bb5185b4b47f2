"""Stable public import surface (the reference's ``video_mamba`` package,
``video_mamba/__init__.py:1-42``), backed by the MI355X-native ``videomamba_amd``."""

from videomamba_amd.determinism import (DeterminismConfig, add_determinism_args,
                                        configure_determinism,
                                        configure_determinism_from_args)
from videomamba_amd.refiner_backbone import BiMambaRefinerBlock
from videomamba_amd.streaming import (STREAMING_CONTRACT_VERSION, ForwardReturnSemantics,
                                      LayerState, StateShape, StreamingState, allocate_state,
                                      expected_state_shapes, forward_return_semantics,
                                      model_forward_return_semantics, validate_state)
from videomamba_amd.videomamba import PretrainVideoMamba, build_videomamba

__all__ = [
    "DeterminismConfig",
    "ForwardReturnSemantics",
    "LayerState",
    "BiMambaRefinerBlock",
    "PretrainVideoMamba",
    "STREAMING_CONTRACT_VERSION",
    "StateShape",
    "StreamingState",
    "add_determinism_args",
    "allocate_state",
    "build_videomamba",
    "configure_determinism",
    "configure_determinism_from_args",
    "expected_state_shapes",
    "forward_return_semantics",
    "model_forward_return_semantics",
    "validate_state",
]
