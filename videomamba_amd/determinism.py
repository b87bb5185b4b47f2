"""Determinism knobs (public API surface; ``video_mamba/determinism.py:10-96``).

``configure_determinism`` seeds python / numpy / torch (all devices) and sets the
torch algorithm switches; the CLI helpers expose the same flags.  On ROCm the
``cudnn`` switches address MIOpen and the ``allow_tf32`` switches are accepted and
recorded (gfx950 has no TF32 math mode).  The HIP kernels of this package are
deterministic regardless (no atomics on any path).
"""

from __future__ import annotations

import argparse
import random
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch


@dataclass(frozen=True)
class DeterminismConfig:
    seed: int = 0
    deterministic: bool = False
    warn_only: bool = True
    cudnn_benchmark: bool = True
    allow_tf32: bool = True


def configure_determinism(seed: int, deterministic: bool, warn_only: bool = True,
                          cudnn_benchmark: Optional[bool] = None,
                          allow_tf32: Optional[bool] = None) -> DeterminismConfig:
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)  # also seeds every visible GPU generator
    benchmark = (not deterministic) if cudnn_benchmark is None else bool(cudnn_benchmark)
    tf32 = (not deterministic) if allow_tf32 is None else bool(allow_tf32)
    torch.backends.cudnn.benchmark = benchmark
    torch.backends.cudnn.deterministic = bool(deterministic)
    torch.use_deterministic_algorithms(bool(deterministic), warn_only=warn_only)
    matmul = getattr(getattr(torch.backends, "cuda", None), "matmul", None)
    if matmul is not None:
        matmul.allow_tf32 = tf32
    torch.backends.cudnn.allow_tf32 = tf32
    return DeterminismConfig(seed=seed, deterministic=bool(deterministic),
                             warn_only=bool(warn_only), cudnn_benchmark=benchmark,
                             allow_tf32=tf32)


_TRI = {"on": True, "off": False, "auto": None}


def add_determinism_args(parser: argparse.ArgumentParser) -> argparse.ArgumentParser:
    parser.add_argument("--seed", type=int, default=0, help="Random seed.")
    parser.add_argument("--deterministic", action="store_true",
                        help="Enable deterministic PyTorch algorithms and cuDNN mode.")
    parser.add_argument("--deterministic-warn-only", action="store_true",
                        help="Use warn-only mode for deterministic algorithm enforcement.")
    parser.add_argument("--cudnn-benchmark", choices=list(_TRI), default="auto",
                        help="cuDNN benchmark mode. auto => inverse of --deterministic.")
    parser.add_argument("--allow-tf32", choices=list(_TRI), default="auto",
                        help="TF32 matmul/convolution mode. auto => inverse of --deterministic.")
    return parser


def configure_determinism_from_args(args: argparse.Namespace) -> DeterminismConfig:
    return configure_determinism(seed=int(args.seed), deterministic=bool(args.deterministic),
                                 warn_only=bool(args.deterministic_warn_only),
                                 cudnn_benchmark=_TRI[args.cudnn_benchmark],
                                 allow_tf32=_TRI[args.allow_tf32])
