"""``video_mamba.streaming`` alias (reference ``video_mamba/streaming.py``)."""
from videomamba_amd.streaming import (STREAMING_CONTRACT_VERSION, ForwardReturnSemantics,
                                      LayerState, StateShape, StreamingState, allocate_state,
                                      expected_state_shapes, forward_return_semantics,
                                      model_forward_return_semantics, validate_state)

__all__ = ["STREAMING_CONTRACT_VERSION", "ForwardReturnSemantics", "LayerState", "StateShape",
           "StreamingState", "allocate_state", "expected_state_shapes",
           "forward_return_semantics", "model_forward_return_semantics", "validate_state"]
