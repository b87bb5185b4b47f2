"""``video_mamba.mamba_simple`` alias (reference ``video_mamba/mamba_simple.py``)."""
from videomamba_amd.mamba_simple import InferenceParamsLike, Mamba

__all__ = ["InferenceParamsLike", "Mamba"]
