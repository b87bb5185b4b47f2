"""Tuned library GEMMs for the projection layers (in_proj / x_proj / dt_proj / out_proj).

The projections are plain library GEMMs (hipBLASLt / rocBLAS through torch).  PyTorch's
TunableOp benchmarks every available solution for a GEMM shape and records the winner;
the results for this package's shapes on gfx950 ship in ``tuning/tunableop_gfx950.csv``
and are loaded read-only, so a fresh process uses the tuned kernels with no tuning cost.
Shapes missing from the file fall back to the library heuristic.

    VM_GEMM_TUNING=0    leave TunableOp alone
    VM_GEMM_TUNING=tune record new shapes into the results file (slow; run on the target)
"""

from __future__ import annotations

import os

import torch

RESULTS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuning",
                       "tunableop_gfx950.csv")
_done = False


def enable_tuned_gemms() -> bool:
    """Idempotent.  Returns True when TunableOp is active for this process."""
    global _done
    if _done:
        return torch.cuda.tunable.is_enabled()
    _done = True
    mode = os.getenv("VM_GEMM_TUNING", "1").lower()
    if mode in ("0", "off", "false", "no") or not torch.cuda.is_available():
        return False
    tune = mode == "tune"
    if not tune and not os.path.exists(RESULTS):
        return False
    tun = torch.cuda.tunable
    os.makedirs(os.path.dirname(RESULTS), exist_ok=True)
    tun.set_filename(RESULTS, insert_device_ordinal=False)
    tun.enable(True)
    tun.tuning_enable(tune)
    if tune:
        tun.set_max_tuning_duration(int(os.getenv("VM_GEMM_TUNING_MS", "60")))
        tun.set_max_tuning_iterations(int(os.getenv("VM_GEMM_TUNING_ITERS", "20")))
    else:
        tun.read_file(RESULTS)
    return True
