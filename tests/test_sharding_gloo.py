"""Batch-sharded multi-process path on CPU (gloo, world_size 2): shard ranges, the
max-over-ranks clock and the pooled-feature all-gather.  The encoder
itself needs the GPU; what is tested here is everything around it that differs at N>1."""

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from videomamba_amd.sharding import gather_pooled, max_over_ranks, shard_batch, shard_range


def test_shard_range_covers_batch_exactly():
    for n in (0, 1, 7, 32, 33):
        for world in (1, 2, 3, 8):
            spans = [shard_range(n, world, r) for r in range(world)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
            sizes = [b - a for a, b in spans]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(4, 2, 2)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        x = torch.arange(5 * 3, dtype=torch.float32).view(5, 1, 3)
        local = shard_batch(x, world, rank)
        # a rank-dependent "elapsed time": the max must be the slowest rank's
        t = max_over_ranks(1.0 + rank, torch.device("cpu"))
        pooled = gather_pooled(local * 2)
        q.put((rank, local.shape[0], t, pooled.tolist()))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_shards_clock_and_gather():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    x = torch.arange(5 * 3, dtype=torch.float32).view(5, 1, 3)
    assert [o[1] for o in out] == [3, 2]          # 5 clips: ranks own 3 + 2
    assert all(o[2] == 2.0 for o in out)          # max over ranks
    for o in out:                                 # every rank sees the global pooled batch
        assert torch.equal(torch.tensor(o[3]), x * 2)


def _bench_stub(extra):
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(root, "bench.py"), "--stub-cpu", "--gpus", "2", "--steps", "4",
           "--warmup", "1"] + extra
    env = dict(os.environ, OMP_NUM_THREADS="1")
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=root)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout  # rank 0 prints exactly one JSON line
    return json.loads(lines[0])


def test_bench_control_flow_world2_weak_scaling():
    """bench.py's own N=2 path under torchrun (gloo, encoder stubbed): ranks from the env,
    a fixed batch per rank (C3, weak scaling), barrier-bracketed timing whose clock is the
    slowest rank's (rank 1 sleeps 4 ms per step), one JSON line from rank 0."""
    line = _bench_stub([])
    assert line["n_gpus"] == 2 and line["scaling"] == "weak"
    # C3 default: 1344 clips per rank (two 672-clip sub-batch streams on a GPU)
    assert line["config"]["per_gpu_batch"] == 1344 and line["config"]["global_batch"] == 2688
    assert line["ms_per_step"] >= 4.0  # the slower rank sets the step time
    want = 2688 * 16 * 196 * 4 / (line["ms_per_step"] * 4 / 1e3)
    assert abs(line["value"] - want) / want < 1e-3
    assert line["per_gpu_value"] * 2 == pytest.approx(line["value"], rel=1e-6)


def test_bench_control_flow_world2_m32_default_is_weak_1344_per_rank():
    """C4 (--config m32) without --global-batch keeps 1344 clips per rank (two 672-clip
    sub-batch streams, as C3; a launch of whole scan-grid rounds; 84 per GPU at N = 8 from a
    fixed 672 would have measured the batch choice, not the sharding): weak scaling, global
    batch = world x 1344, and the metric names the workload actually run."""
    line = _bench_stub(["--config", "m32"])
    assert line["scaling"] == "weak"
    assert line["config"]["per_gpu_batch"] == 1344 and line["config"]["global_batch"] == 2688
    assert line["metric"].endswith("VideoMamba-M 32f 224")
    assert _bench_stub(["--config", "ti8"])["metric"].endswith("VideoMamba-Ti 8f 224")


def test_bench_metric_name_is_the_baseline_metric_for_c3():
    import json
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    want = json.load(open(os.path.join(root, "BASELINE.json")))["metric"]
    assert bench.metric_name(bench.CONFIGS["m16"]) == want


def test_bench_cpu_baseline_threads_are_the_process_share(monkeypatch):
    """The CPU baseline runs on the CPUs the bench process may use: OMP_NUM_THREADS when set
    (16 on a one-GPU box), else the cgroup quota or the affinity mask — never the whole
    shared host that os.cpu_count() reports."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    monkeypatch.setenv("OMP_NUM_THREADS", "16")
    assert bench._cpu_share(256) == 16
    monkeypatch.delenv("OMP_NUM_THREADS")
    share = bench._cpu_share(3)
    assert 1 <= share <= max(3, os.cpu_count() or 1)


def test_bench_control_flow_world2_global_batch_split():
    """--global-batch (C4): one global batch split by shard_range — 5 clips on 2 ranks is
    3 + 2; scaling is strong and value counts the global batch once."""
    line = _bench_stub(["--config", "m32", "--global-batch", "5"])
    assert line["scaling"] == "strong" and line["config"]["global_batch"] == 5
    assert line["config"]["per_gpu_batch"] == 3  # rank 0's shard
    want = 5 * 32 * 196 * 4 / (line["ms_per_step"] * 4 / 1e3)
    assert abs(line["value"] - want) / want < 1e-3


def _encoder_shard_worker(rank, world, port, q, split=False):
    """One rank of the batch-sharded encoder: its contiguous clip range through the HIP
    encoder on cuda:0, then the pooled-feature all-gather (gloo, so CPU tensors).  ``split``:
    the rank's shard runs as the phase-locked two-stream sub-batch forward (its own host
    issue threads), as bench.py's ranks do at their 1344-clip batch."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from videomamba_amd import options
        torch.manual_seed(0)
        model = _shard_model(split)
        x = torch.randn(_SHARD_CLIPS, 3, 4, 64, 64, generator=torch.Generator().manual_seed(1))
        local = shard_batch(x, world, rank)
        kw = dict(batch_streams=2, batch_stream_lock=True, batch_stream_min_clips=2,
                  batch_stream_min_work=0) if split else dict(batch_streams=1)
        with torch.no_grad(), options.override(**kw):
            model = model.to("cuda:0")
            xl = local.to("cuda:0")
            parts = model._stream_parts(xl, None, None, None)
            xv, xp = model(xl)
        pooled = gather_pooled(xp.float().cpu())  # gloo: fp32 rows (bf16 converts exactly)
        q.put((rank, local.shape[0], xv.cpu(), pooled, parts))
    finally:
        dist.destroy_process_group()


_SHARD_CLIPS = 6


def _shard_model(split):
    """The sharded-encoder test model: embed_dim 192 (in_proj / out_proj on the row-invariant
    HIP GEMM, which the sub-batch split requires), bf16 when ``split``."""
    from videomamba_amd.videomamba import PretrainVideoMamba
    model = PretrainVideoMamba(img_size=64, patch_size=16, depth=3, embed_dim=192,
                               num_frames=4).eval()
    return model.to(torch.bfloat16) if split else model


@pytest.mark.gpu
@pytest.mark.parametrize("split", [False, True])
def test_gpu_encoder_batch_sharded_world2_matches_single_process(split):
    """SURVEY §8e on hardware we have: 2 fresh processes (gloo, both on cuda:0) each run
    their shard of a 6-clip batch through the HIP encoder and all-gather x_pool.  Every
    rank's features equal the single-process forward of the same shard bit for bit, and the
    gathered x_pool equals the single-process forward of the whole batch.  ``split``
    (VERDICT r5 #4): each rank's 3 clips run as the phase-locked two-stream sub-batch
    forward, so two processes, each with its own host issue threads, run concurrently on one
    GPU; their features and pooled rows are bit-equal to one process on one stream (bf16:
    every projection on the row-invariant HIP GEMM).  fp32 (library GEMMs, whose kernel
    choice depends on the row count) compares x_pool at 1e-5."""
    from videomamba_amd import options
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_encoder_shard_worker, args=(r, world, port, q, split))
             for r in range(world)]
    for p in procs:
        p.start()
    out = sorted((q.get(timeout=300) for _ in range(world)), key=lambda o: o[0])
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    torch.manual_seed(0)
    model = _shard_model(split).to("cuda:0")
    x = torch.randn(_SHARD_CLIPS, 3, 4, 64, 64, generator=torch.Generator().manual_seed(1))
    with torch.no_grad(), options.override(batch_streams=1):
        xv_all, xp_all = model(x.to("cuda:0").to(model.patch_embed.proj.weight.dtype))
        for rank, n, xv, pooled, parts in out:
            a, b = shard_range(_SHARD_CLIPS, world, rank)
            assert n == b - a
            assert parts == (2 if split else 1)
            xv_ref, _ = model(x[a:b].to("cuda:0").to(xv_all.dtype))
            assert torch.equal(xv, xv_ref.cpu())
            assert pooled.shape == xp_all.shape
            if split:
                assert torch.equal(pooled, xp_all.float().cpu())
            else:
                torch.testing.assert_close(pooled, xp_all.float().cpu(), rtol=1e-5, atol=1e-5)
    assert torch.equal(out[0][3], out[1][3])  # every rank holds the same gathered batch


def test_in_step_scan_fraction_reproduces_from_committed_trace():
    """the scan's in-step HBM fraction (the kernel's own begin-end times in a
    committed rocprofv3 trace of a bench command) is what bench.py reports as
    roofline.in_step.trace, and scripts/traffic_summary.py in-step reproduces it from the
    same file; the isolated figure (roofline.frac) is larger."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    algo = 672 * 1152 * 3137 * 4 * 2 + 2 * 672 * 16 * 3137 * 2 + 4 * 1152 * 16 + 8 * 1152 \
        + 2 * 672 * 1152 * 16 * 2
    tr = bench._trace_in_step(algo, 672)
    assert tr is not None and tr["source"] == bench.IN_STEP_TRACES[0][0]
    assert bench._trace_in_step(algo, 112) is None  # no committed trace of 112-clip launches
    out = subprocess.run([sys.executable, os.path.join(root, "scripts", "traffic_summary.py"),
                          "in-step", os.path.join(root, tr["source"]), "672"],
                         capture_output=True, text=True, check=True).stdout
    rec = json.loads(out)
    assert rec["bytes_per_launch"] == algo
    assert abs(rec["trace_frac"] - tr["frac"]) < 1e-4 and abs(rec["trace_avg_us"] - tr["avg_us"]) < 0.01
    line = json.load(open(os.path.join(root, "profiles", "r06v_bench.json")))
    assert line["roofline"]["frac"] > tr["frac"]
