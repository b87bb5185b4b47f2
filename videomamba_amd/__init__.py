"""MI355X-native VideoMamba encoder (gfx950 HIP kernels behind the reference's API).

Import the public surface from ``video_mamba`` (the reference's stable import name);
this package holds the implementation:

* ``csrc/``          hand-written HIP kernels + the C ABI (``include/videomamba_hip.h``)
* ``_lib``           ctypes binding of ``libvideomamba_hip.so`` (fails loudly if missing)
* ``kernels``        operator shims with the reference's kernel call shapes
* ``mamba_simple``   Mamba mixer;  ``videomamba``  encoder / builder / loader
* ``streaming``      streaming-state contract;  ``determinism``  seeding knobs
* ``refiner_backbone``  BiMambaRefinerBlock;  ``sharding``  batch-sharded multi-GPU runner
"""

from .determinism import (DeterminismConfig, add_determinism_args, configure_determinism,
                          configure_determinism_from_args)
from .refiner_backbone import BiMambaRefinerBlock
from .streaming import (STREAMING_CONTRACT_VERSION, ForwardReturnSemantics, LayerState,
                        StateShape, StreamingState, allocate_state, expected_state_shapes,
                        forward_return_semantics, model_forward_return_semantics,
                        validate_state)
from .videomamba import PretrainVideoMamba, build_videomamba

__all__ = [
    "DeterminismConfig", "ForwardReturnSemantics", "LayerState", "BiMambaRefinerBlock",
    "PretrainVideoMamba", "STREAMING_CONTRACT_VERSION", "StateShape", "StreamingState",
    "add_determinism_args", "allocate_state", "build_videomamba", "configure_determinism",
    "configure_determinism_from_args", "expected_state_shapes", "forward_return_semantics",
    "model_forward_return_semantics", "validate_state",
]
