"""Phase lock for sub-batch streams (``options.batch_stream_lock``).

The model's forward can split a large batch into parts, each on its own HIP stream
(``PretrainVideoMamba._encode_streams``).  Each layer has two phases:
  - the "pre" phase: add + norm, in_proj and conv_proj, bound by HBM and the matrix cores;
  - the scan and out_proj, with the scan bound by VALU issue.

Left to themselves, the parts' pre phases often run side by side.  Then HBM-bound or
GEMM kernels share the chip with kernels bound by the same unit.

The lock orders the pre phases in a ring:
  - part p > 0 starts layer l's pre phase after part p - 1 finished it;
  - part 0 starts layer l after the last part finished layer l - 1.
So one part's scan runs beside another part's pre phase, and no two pre phases overlap.
B = 896 as two parts, same bits every time:
  - in one process, alternating: 809.8–810.2 vs 817.8–818.7 ms per step, and 822.7–823.8 vs
    829.0–829.9 on another box (``profiles/r05zzd_phase_lock.jsonl``, ``r05zzc``);
  - in separate processes, alternating: 820.6–823.3 vs 823.4–830.7 ms
    (``r05zzf_lock_ab.jsonl``).
So the lock gains 0.3–1.1 %.

The ordering is GPU-side: a HIP event per (part, layer), recorded after the pre phase is
issued and waited on by the next part's stream.  The host threads only wait until that
event has been recorded, because a stream can only wait on an event that was recorded
before the wait was issued.  So each part issues its layers from its own host thread.  The
ring's order cannot deadlock.  A part that fails releases every one of its events (the
waits on an unrecorded event pass), so the other parts drain and the error is re-raised.

The reference has no counterpart: it runs one batch on one stream
(``models/videomamba/videomamba.py:943-1067``)."""
from __future__ import annotations

import threading
from typing import Callable, List, Optional

__all__ = ["PhaseLock", "current", "pre_start", "pre_done", "bind"]

_TLS = threading.local()


class PhaseLock:
    """Ring order over ``parts`` x ``depth`` layer pre phases.  ``record(part, idx)``
    marks the end of a pre phase on the caller's stream; ``wait(part, idx)`` makes the
    caller's stream wait for it (defaults: HIP events on the current stream)."""

    def __init__(self, parts: int, depth: int, record: Optional[Callable[[int, int], None]] = None,
                 wait: Optional[Callable[[int, int], None]] = None):
        if parts < 1 or depth < 0:
            raise ValueError("PhaseLock needs parts >= 1 and depth >= 0")
        self.parts, self.depth = parts, depth
        self._flags: List[List[threading.Event]] = [
            [threading.Event() for _ in range(depth)] for _ in range(parts)]
        if record is None or wait is None:
            import torch
            events = [[torch.cuda.Event() for _ in range(depth)] for _ in range(parts)]

            def record(part: int, idx: int) -> None:  # noqa: F811
                events[part][idx].record(torch.cuda.current_stream())

            def wait(part: int, idx: int) -> None:  # noqa: F811
                torch.cuda.current_stream().wait_event(events[part][idx])
        self._record, self._wait = record, wait

    def _after(self, part: int, idx: int) -> None:
        self._flags[part][idx].wait()
        self._wait(part, idx)

    def pre_start(self, part: int, idx: int) -> None:
        """Before part ``part`` issues layer ``idx``'s pre phase."""
        if not 0 <= idx < self.depth:
            return
        if part > 0:
            self._after(part - 1, idx)
        elif idx > 0 and self.parts > 1:
            self._after(self.parts - 1, idx - 1)

    def pre_done(self, part: int, idx: int) -> None:
        """After part ``part`` issued layer ``idx``'s pre phase (idempotent)."""
        if not 0 <= idx < self.depth or self._flags[part][idx].is_set():
            return
        self._record(part, idx)
        self._flags[part][idx].set()

    def release(self, part: int) -> None:
        """Unblock every waiter on ``part`` (after a failure: its events stay unrecorded)."""
        for f in self._flags[part]:
            f.set()


def bind(lock: Optional[PhaseLock], part: int) -> None:
    """Attach this host thread to ``part`` of ``lock`` (None detaches)."""
    _TLS.lock = lock
    _TLS.part = part


def current():
    """(lock, part) of this host thread, or (None, 0)."""
    return getattr(_TLS, "lock", None), getattr(_TLS, "part", 0)


def pre_start(idx: Optional[int]) -> None:
    lock, part = current()
    if lock is not None and idx is not None:
        lock.pre_start(part, idx)


def pre_done(idx: Optional[int]) -> None:
    lock, part = current()
    if lock is not None and idx is not None:
        lock.pre_done(part, idx)
