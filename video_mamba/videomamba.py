"""``video_mamba.videomamba`` alias (reference ``video_mamba/videomamba.py``)."""
from videomamba_amd.videomamba import PretrainVideoMamba, build_videomamba, load_state_dict

__all__ = ["PretrainVideoMamba", "build_videomamba", "load_state_dict"]
