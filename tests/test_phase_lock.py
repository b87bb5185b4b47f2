"""The sub-batch phase lock's ring order (videomamba_amd/phase_lock.py), on the host: the
GPU-side record / wait are replaced by a log, so the order the lock enforces between host
threads is checked without a device.  The GPU forward with the lock is covered bitwise by
test_gpu_model.py::test_batch_streams_forward_is_bitwise_the_one_stream_forward."""
import threading
import time

import pytest

from videomamba_amd.phase_lock import PhaseLock, bind, current, pre_done, pre_start


def _run(parts, depth, fail=None, jitter=0.0):
    log, mu = [], threading.Lock()

    def note(*ev):
        with mu:
            log.append(ev)

    lock = PhaseLock(parts, depth, record=lambda p, i: note("rec", p, i),
                     wait=lambda p, i: note("wait", p, i))
    errors = [None] * parts

    def work(part):
        bind(lock, part)
        try:
            for idx in range(depth):
                pre_start(idx)
                note("start", part, idx)
                if jitter:
                    time.sleep(jitter * ((part + idx) % 3))
                if fail == (part, idx):
                    raise RuntimeError("boom")
                pre_done(idx)
                pre_done(idx)  # idempotent (the block's fallback after the mixer's mark)
        except RuntimeError as e:
            errors[part] = e
            lock.release(part)
        finally:
            bind(None, 0)

    th = [threading.Thread(target=work, args=(p,)) for p in range(parts)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=30)
        assert not t.is_alive(), "phase lock deadlocked"
    return log, errors


@pytest.mark.parametrize("parts,depth", [(2, 6), (3, 5), (1, 4)])
def test_ring_order(parts, depth):
    log, errors = _run(parts, depth, jitter=0.002)
    assert errors == [None] * parts
    pos = {e: i for i, e in enumerate(log)}
    assert sum(1 for e in log if e[0] == "rec") == parts * depth  # one record per phase
    for p in range(parts):
        for i in range(depth):
            if p > 0:  # part p's pre phase starts after part p - 1's was recorded
                assert pos[("rec", p - 1, i)] < pos[("wait", p - 1, i)] < pos[("start", p, i)]
            elif i > 0 and parts > 1:  # part 0's next layer after the last part's
                assert pos[("rec", parts - 1, i - 1)] < pos[("start", 0, i)]
    assert current() == (None, 0)


@pytest.mark.parametrize("fail", [(0, 2), (1, 0), (1, 3)])
def test_failing_part_releases_the_others(fail):
    log, errors = _run(2, 5, fail=fail)
    assert isinstance(errors[fail[0]], RuntimeError)
    other = 1 - fail[0]
    assert errors[other] is None
    assert ("start", other, 4) in log  # the other part ran every layer


def test_bad_shape():
    with pytest.raises(ValueError):
        PhaseLock(0, 3, record=lambda p, i: None, wait=lambda p, i: None)


@pytest.mark.parametrize("embed,batch,want", [(576, 1344, 2), (576, 224, 2), (576, 112, 1),
                                              (192, 512, 1), (192, 672, 2), (384, 336, 2)])
def test_split_rule_model_and_bench_agree(embed, batch, want, monkeypatch):
    """PretrainVideoMamba._stream_parts (the forward's split) and bench.py's
    _sub_batch_streams (what the bench line reports, and the per-launch batch its roofline
    leg times) apply the same rule: options.batch_streams from batch_stream_min_clips clips
    and batch_stream_min_work clip-channels (B x d_inner) up (for the bench's bf16 models,
    whose projections all run on the row-invariant HIP GEMM)."""
    import os
    import sys

    import torch

    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    from videomamba_amd.videomamba import PretrainVideoMamba

    model = PretrainVideoMamba(img_size=32, patch_size=16, depth=1, embed_dim=embed,
                               num_frames=2, pool_type="avg").to(torch.bfloat16)
    x = torch.empty(batch, 3, 2, 32, 32, device="meta", dtype=torch.bfloat16)
    monkeypatch.setattr(torch.cuda, "is_current_stream_capturing", lambda: False)  # no device
    assert model._stream_parts(x, None, None, None) == want
    assert bench._sub_batch_streams(batch, embed) == want
