"""Tuned library GEMMs for the projection layers (in_proj / x_proj / dt_proj / out_proj).

The projections are plain library GEMMs (hipBLASLt / rocBLAS through torch).  PyTorch's
TunableOp benchmarks every available solution for a GEMM shape and records the winner;
the results for this package's shapes on gfx950 ship in ``tuning/tunableop_gfx950.csv``
and are loaded read-only, so a fresh process uses the tuned kernels with no tuning cost.
Shapes missing from the file fall back to the library heuristic.

Scope: TunableOp is a process-wide switch in PyTorch, so this module turns it on only
around the mixer's own GEMM calls (:func:`tuned`) and restores the caller's setting
afterwards — other GEMMs in the user's process are untouched.  It stays off when
``torch.are_deterministic_algorithms_enabled()`` (the determinism contract) or when
``options.gemm_tuning == "off"``; ``"tune"`` records new shapes into the results file.
"""

from __future__ import annotations

import contextlib
import os
import threading

import torch

from . import options

RESULTS = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuning",
                       "tunableop_gfx950.csv")
_loaded = {"mode": None}
# TunableOp's enable flags are process-wide: nested and concurrent users (the sub-batch
# forward's issue threads) share one switch, turned on by the first to enter and restored to
# the caller's setting by the last to leave (one thread's exit must not switch it
# off under another thread's GEMM)
_lock = threading.Lock()
_users = {"n": 0, "saved": None, "mode": None}


def _prepare(mode: str) -> bool:
    """Load the results file once per mode; False when TunableOp cannot be used."""
    if _loaded["mode"] == mode:
        return True
    if not torch.cuda.is_available():
        return False
    tun = torch.cuda.tunable
    tune = mode == "tune"
    if not tune and not os.path.exists(RESULTS):
        return False
    tun.set_filename(RESULTS, insert_device_ordinal=False)
    if tune:
        os.makedirs(os.path.dirname(RESULTS), exist_ok=True)
        tun.set_max_tuning_duration(60)
        tun.set_max_tuning_iterations(20)
    else:
        tun.read_file(RESULTS)
    _loaded["mode"] = mode
    return True


@contextlib.contextmanager
def tuned():
    """Run the enclosed GEMMs with the shipped TunableOp results (see module doc).
    Re-entrant and thread-safe: the switch stays on while any thread is inside."""
    mode = options.get().gemm_tuning
    if mode == "off" or torch.are_deterministic_algorithms_enabled():
        yield False
        return
    tun = torch.cuda.tunable
    with _lock:
        if _users["n"] == 0:
            if not _prepare(mode):
                ok = False
            else:
                _users["saved"] = (tun.is_enabled(), tun.tuning_is_enabled())
                _users["mode"] = mode
                tun.enable(True)
                tun.tuning_enable(mode == "tune")
                ok = True
        else:
            ok = _users["mode"] is not None
        if ok:
            _users["n"] += 1
    if not ok:
        yield False
        return
    try:
        yield True
    finally:
        with _lock:
            _users["n"] -= 1
            if _users["n"] == 0:
                was_on, was_tuning = _users["saved"]
                tun.tuning_enable(was_tuning)
                tun.enable(was_on)
                _users["saved"] = _users["mode"] = None
