"""``video_mamba.refiner_backbone`` alias (reference ``video_mamba/refiner_backbone.py``)."""
from videomamba_amd.refiner_backbone import BiMambaRefinerBlock

__all__ = ["BiMambaRefinerBlock"]
