"""``video_mamba.determinism`` alias (reference ``video_mamba/determinism.py``)."""
from videomamba_amd.determinism import (DeterminismConfig, add_determinism_args,
                                        configure_determinism,
                                        configure_determinism_from_args)

__all__ = ["DeterminismConfig", "add_determinism_args", "configure_determinism",
           "configure_determinism_from_args"]
