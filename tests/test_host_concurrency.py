"""Host-side concurrency of the sub-batch forward, on CPU:
the per-thread override slots, the re-entrant TunableOp switch and the split guards.  The
GPU side (two processes with their own issue threads, bitwise) is
tests/test_sharding_gloo.py::test_gpu_encoder_batch_sharded_world2_matches_single_process."""

import threading

import pytest
import torch

from videomamba_amd import gemm_tuning, options
from videomamba_amd import kernels as K
from videomamba_amd.videomamba import PretrainVideoMamba


def test_override_slots_are_per_thread():
    """A graph capture's scratch / sync / counter buffers, entered on one thread, never
    reach a launch issued by another thread (another sub-batch stream)."""
    seen = {}
    bufs = [torch.zeros(16, dtype=torch.uint8) for _ in range(3)]
    entered, done = threading.Event(), threading.Event()

    def other():
        entered.wait(5)
        seen["ws"] = K._WS_OVERRIDE.value
        seen["sync"] = K._SYNC_OVERRIDE.value
        seen["cnt"] = K._CNT_OVERRIDE.value
        seen["scratch"] = K.scratch(torch.device("cpu"), 7, 8)
        done.set()

    t = threading.Thread(target=other)
    t.start()
    with K.scratch_override(bufs[0]), K.sync_override(bufs[1]), K.counter_override(bufs[2]):
        assert K._WS_OVERRIDE.value is bufs[0] and K.scratch(torch.device("cpu"), 0, 8) is bufs[0]
        entered.set()
        done.wait(5)
    t.join(5)
    assert seen["ws"] is None and seen["sync"] is None and seen["cnt"] is None
    assert seen["scratch"] is not bufs[0] and seen["scratch"].numel() >= 8
    assert K._WS_OVERRIDE.value is None and K._CNT_OVERRIDE.value is None


class _FakeTunable:
    def __init__(self):
        self.on, self.tuning, self.log = False, False, []

    def is_enabled(self):
        return self.on

    def tuning_is_enabled(self):
        return self.tuning

    def enable(self, v=True):
        self.on = bool(v)
        self.log.append(("enable", self.on))

    def tuning_enable(self, v=True):
        self.tuning = bool(v)


def test_tuned_switch_is_refcounted_across_threads(monkeypatch):
    """TunableOp's switch is process-wide: with two issue threads inside tuned(), the first
    one's exit must leave it on for the other; the last exit restores the
    caller's setting."""
    fake = _FakeTunable()
    monkeypatch.setattr(torch.cuda, "tunable", fake)
    monkeypatch.setattr(gemm_tuning, "_prepare", lambda mode: True)
    monkeypatch.setattr(torch, "are_deterministic_algorithms_enabled", lambda: False)
    a_in, b_in, a_out = threading.Event(), threading.Event(), threading.Event()
    states = {}

    def a():
        with gemm_tuning.tuned() as ok:
            assert ok
            a_in.set()
            b_in.wait(5)
        a_out.set()

    def b():
        a_in.wait(5)
        with gemm_tuning.tuned() as ok:
            assert ok
            b_in.set()
            a_out.wait(5)
            states["after_a_exit"] = fake.is_enabled()
        states["after_b_exit"] = fake.is_enabled()

    with options.override(gemm_tuning="on"):
        ta, tb = threading.Thread(target=a), threading.Thread(target=b)
        ta.start()
        tb.start()
        ta.join(10)
        tb.join(10)
    assert states == {"after_a_exit": True, "after_b_exit": False}
    assert gemm_tuning._users["n"] == 0
    # nested on one thread: one enable, one restore
    fake.log.clear()
    with options.override(gemm_tuning="on"), gemm_tuning.tuned(), gemm_tuning.tuned():
        assert fake.is_enabled()
    assert fake.log == [("enable", True), ("enable", False)]


def _model(embed_dim=192, dtype=torch.bfloat16):
    torch.manual_seed(0)
    return PretrainVideoMamba(img_size=32, patch_size=16, depth=2, embed_dim=embed_dim,
                              num_frames=4).to(dtype)


def test_split_guards_on_the_host():
    """The split forward only where every projection is the row-invariant HIP GEMM on one
    bf16 dtype and the fused out_proj + norm is off (PretrainVideoMamba._stream_parts);
    autocast is covered on the GPU (torch disables it without a device)."""
    x = torch.zeros(6, 3, 4, 32, 32, dtype=torch.bfloat16)
    m = _model()
    with options.override(batch_streams=2, batch_stream_min_clips=2, batch_stream_min_work=0):
        assert m._stream_parts(x, None, None, None) == 2
        assert m._stream_parts(x[:1], None, None, None) == 1
        with options.override(fuse_out_norm=True):
            assert m._stream_parts(x, None, None, None) == 1
        with options.override(projection_gemm="library"):
            assert m._stream_parts(x, None, None, None) == 1
        with options.override(mixer_layout="cm"):
            assert m._stream_parts(x, None, None, None) == 1
        assert _model(embed_dim=64)._stream_parts(x, None, None, None) == 1  # K = 64: library
        assert _model(dtype=torch.float32)._stream_parts(x.float(), None, None, None) == 1
        m.norm.float()
        assert m._features_dtype() is None and m._stream_parts(x, None, None, None) == 1
