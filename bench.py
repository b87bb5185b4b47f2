"""VideoMamba encoder benchmark on MI355X (BASELINE.json metric).

    python bench.py [--gpus N --steps K --warmup W --batch B]
    torchrun --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

Workload (config C3 of BASELINE.json; the metric is quoted on VideoMamba-M 16f 224):
VideoMamba-M (d576, depth 32), 16x224x224 clips, bf16, one stateful streaming chunk per
step (chunk_size 32 > 16 temporal tokens, so the clip is one chunk carrying
(conv_state, ssm_state) through every layer), random-init weights (seed 0), synthetic
clips.  A step = one forward of B clips per GPU; clips shard by batch across ranks with
no collective on the data path (weak scaling).  value = video tokens (B*T*196, CLS
excluded) per second summed over all ranks, timed as the max over ranks.

Other configs: --config m32 (VideoMamba-M 32x224^2, C4: 1344 clips per rank by default, two
672-clip sub-batch streams as in C3, so the 1/2/4/8-GPU curve keeps every GPU at the batch
where the scan holds its occupancy —
weak scaling; --global-batch G instead splits G clips across ranks with
sharding.shard_range — strong scaling; run under torchrun for the 8-GPU case), --config ti8
--full-sequence (C2).  The metric name follows the config ("<model> <T>f 224").  The
roofline block is always the scan at the M-16f shape.

--stub-cpu replaces the encoder by a trivial CPU op and runs the same rank / barrier /
max-over-ranks / JSON-line control flow on the gloo backend (tests/test_sharding_gloo.py
launches it under torchrun with 2 ranks).

Extra fields: chunk_p50_ms (B=1 chunk latency, HIP-graph replay; chunk_p50_eager_ms the
eager launch path), b1_kernels (per-stage roofline fractions of one M layer at the B=1
chunk shape), roofline of the selective-scan kernel
(HIP-event timed at the bench shape; algorithmic bytes per launch), cpu_baseline (the
CPU oracle on one M-16f clip, rank 0 at N=1 only).
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# Measured gfx950 issue costs (tools/probes/valu_rate.hip, >=2 waves/SIMD): cycles per
# wave64 instruction per SIMD.  The scan's irreducible work per (element, state) is one
# v_exp_f32 plus four fp32 mul/fma (delta*A, (delta*u)*B, h update, y += h*C).
CYC_EXP, CYC_FMA, SIMDS, CLOCK_HZ = 8.2, 2.8, 1024, 2.4e9
# The same scan instruction stream with its global loads and stores removed
# (tools/probes/scan_lab.hip "voff no vmem", profiles/r01c_scan_lab.txt): us per clip-layer
# at M-16f.  What the kernel's own VALU/SALU work costs with no memory at all.
LAB_NO_MEMORY_US_PER_CLIP_LAYER = 9.67

CONFIGS = {
    # C3 (default): 1344 clips per GPU = two 672-clip sub-batch streams with their layer
    # phases locked (options.batch_streams / batch_stream_lock; each launch's scan grid runs
    # ~3 whole rounds): 909.6-910.0 vs 920.1-923.3 us per clip at 896 (2 x 448), 908.3-908.8
    # at 1792, same box alternating (profiles/r05zzn_batch_lock_sweep.jsonl); before the lock
    # 896 and 1344 ran alike (921-934 / 925 us, r05zd_batch_sweep.jsonl, r05ze_*)
    "m16": dict(depth=32, embed_dim=576, frames=16, name="VideoMamba-M", batch=1344),
    # C4: the same 1344 clips per GPU (two locked 672-clip streams): 3.516-3.535 M vs
    # 3.488-3.508 M at 896, alternating on one box (profiles/r05zzq_m32_batch_ab.jsonl;
    # before the lock r05zg_*: 3.373 M at 896 with two streams, 3.316 M at 448 on one)
    "m32": dict(depth=32, embed_dim=576, frames=32, name="VideoMamba-M", batch=1344),
    "ti8": dict(depth=24, embed_dim=192, frames=8, name="VideoMamba-Ti",  # C1 / C2 shape
                batch=512),
}


def _args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=None, help="clips per GPU (C3, weak scaling)")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="clips split across all ranks (C4, strong scaling)")
    ap.add_argument("--stub-cpu", action="store_true",
                    help="CPU/gloo control-flow check with the encoder stubbed out")
    ap.add_argument("--config", default="m16", choices=sorted(CONFIGS))
    ap.add_argument("--p50-chunks", type=int, default=100)
    ap.add_argument("--scan-reps", type=int, default=50)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-b1", action="store_true",
                    help="skip the B=1 chunk latency and per-stage B=1 rooflines (batch sweeps)")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="oracle threads (0: every CPU this process may use, see _cpu_share)")
    ap.add_argument("--scan-dt-proj", default="auto", choices=("auto", "on", "off"),
                    help="options.scan_dt_proj: dt_proj inside the scan at chip-filling batches")
    ap.add_argument("--batch-streams", type=int, default=0,
                    help="options.batch_streams (sub-batch HIP streams per forward; 0: default)")
    ap.add_argument("--dist-backend", default="nccl", choices=("nccl", "gloo"),
                    help="process group backend for N > 1 (nccl = RCCL over xGMI; gloo only to "
                         "rehearse the multi-rank path with several ranks on one GPU)")
    ap.add_argument("--full-sequence", action="store_true",
                    help="stateless full-sequence forward (C2) instead of a stateful chunk")
    a = ap.parse_args()
    a.batch_default = a.batch is None
    if a.batch is None:
        # 448 clips per launch: the single-pass scan grid (9 workgroups per clip, 8 resident
        # per CU) runs ~2 full rounds; at 336 (1.5 rounds) the dt_proj-in-scan kernel loses
        # 15 % in the partial second round (profiles/r03c_batch_sweep.txt).  M-16f runs two
        # such launches side by side (CONFIGS)
        a.batch = CONFIGS[a.config].get("batch", 448)
    return a


def _progress(msg):
    """One progress line on stderr per bench stage (the JSON line stays alone on stdout)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def _sync_barrier(world):
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()


def _pmc_traffic(shape, kernel):
    """(HBM bytes per scan launch, source file) from the committed rocprofv3
    FETCH_SIZE/WRITE_SIZE passes (profiles/scan_traffic_*.json, calibrated gfx950 read /
    write ratios applied) when they were taken at this shape and kernel form; (None, None)
    otherwise.  PMC collection needs its own profiler run, so it is not repeated inside the
    timed bench: the JSON line says where the number comes from."""
    import glob
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "scan_traffic_*.json")))[::-1]:
        with open(path) as f:
            rec = json.load(f)
        if rec.get("shape") == shape and rec.get("kernel", "").startswith(kernel):
            return int(rec["hbm_bytes_per_launch"]), os.path.relpath(path, ROOT)
    return None, None


def scan_roofline(batch, reps, device, layout="tm", dtp=False):
    """Time the scan kernel at the bench shape (layer-0 geometry, padded layout) with HIP
    events on the launch stream; algorithmic bytes per launch per SURVEY.md 8(d).  The
    scan activates delta itself (the model's call: delta_bias, delta_softplus=True).
    layout "tm": the model's token-major buffers (u, dt: (B*Lp, D); z inside xz (B*Lp, 2D);
    B/C inside x_dbl (B*Lp, R+2N)); "cm": channel-major (D, B*Lp) buffers.
    dtp: the kernel the bf16 mixer runs at this batch with dt_proj folded in
    (vm_selective_scan_dtproj_fwd: dt from the x_dbl rows, no dt rows).  ``frac`` stays on
    the SURVEY 8(d) byte formula (which counts a delta stream); ``own_bytes_per_launch`` /
    ``frac_own_bytes`` price what the fused kernel itself must move (u, z, y, B|C rows,
    dt_low rows, states)."""
    from videomamba_amd import kernels as K
    from videomamba_amd.layers import round_up

    D, N, L, R = 1152, 16, 3137, 36
    Lp = round_up(L)
    n = batch * Lp
    g = torch.Generator(device=device).manual_seed(1)
    bf = torch.bfloat16
    A = -torch.arange(1, N + 1, device=device, dtype=torch.float32).repeat(D, 1).contiguous()
    Dv = torch.ones(D, device=device)
    bias = torch.full((D,), -4.0, device=device)
    h = torch.zeros(batch, D, N, device=device, dtype=bf)
    if layout == "tm":
        u = torch.randn(n, D, device=device, generator=g).to(bf)
        dt = (0.5 * torch.randn(n, D, device=device, generator=g) - 4.0).to(bf)
        xz = torch.randn(n, 2 * D, device=device, generator=g).to(bf)
        xdbl = torch.randn(n, R + 2 * N, device=device, generator=g).to(bf)
        z, Bm, Cm = xz[:, D:], xdbl[:, R:], xdbl[:, R + N:]
        y = torch.empty_like(u)
        s_u, s_z, s_bc = (Lp * D, 1, D), (Lp * 2 * D, 1, 2 * D), (Lp * (R + 2 * N), 1, R + 2 * N)
    else:
        u = torch.randn(D, n, device=device, generator=g).to(bf)
        dt = (0.5 * torch.randn(D, n, device=device, generator=g) - 4.0).to(bf)
        z = torch.randn(D, n, device=device, generator=g).to(bf)
        bc = torch.randn(2 * N, n, device=device, generator=g).to(bf)
        Bm, Cm = bc[:N], bc[N:]
        y = torch.empty_like(u)
        s_u = s_z = s_bc = (Lp, n, 1)
    stream = torch.cuda.current_stream(device).cuda_stream

    def launch():
        K.scan_raw(u, s_u, dt, s_u, A, Bm, s_bc, Cm, s_bc, Dv, z, s_z, bias, True,
                   h, (h.stride(0), h.stride(1)), h, (h.stride(0), h.stride(1)), y, s_u, Lp,
                   batch, D, L, N, 1, stream)

    if dtp:
        xdbl[:, :R] = (0.5 * torch.randn(n, R, device=device, generator=g)).to(bf)
        wdt = torch.zeros(D, 64, device=device, dtype=bf)
        wdt[:, :R] = (torch.randn(D, R, device=device, generator=g) / R ** 0.5).to(bf)
        E = R + 2 * N

        def launch():  # noqa: F811
            K.scan_dtproj_raw(u, s_u, xdbl, (Lp * E, E), R, wdt, A, Bm, s_bc, Cm, s_bc, Dv, z,
                              s_z, bias, h, (h.stride(0), h.stride(1)), h,
                              (h.stride(0), h.stride(1)), y, s_u, Lp, batch, D, L, N, stream)

    for _ in range(5):
        launch()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        launch()
    e1.record()
    torch.cuda.synchronize()
    avg_s = e0.elapsed_time(e1) / 1e3 / reps
    e = 2
    algo = batch * D * L * 4 * e + 2 * batch * N * L * e + 4 * D * N + 8 * D + 2 * batch * D * N * e
    achieved = algo / avg_s / 1e9
    floor_s = batch * D * L * N / 64 * (CYC_EXP + 4 * CYC_FMA) / SIMDS / CLOCK_HZ
    own = (batch * D * L * 3 * e + 2 * batch * N * L * e + batch * L * R * e + 4 * D * N
           + 8 * D + 2 * batch * D * N * e + D * R * e) if dtp else algo
    shape = f"B={batch} D={D} L={L} N={N} bf16, stateful"
    kname = ("vm::scan_seq_dtp_kernel" if dtp else "vm::scan_seq_kernel") if layout == "tm" \
        else "vm::scan_v5_kernel"
    traffic, tsrc = _pmc_traffic(shape, kname)
    return {"bound": "hbm", "kernel": kname, "layout": layout, "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_source": (f"committed rocprofv3 PMC passes at this shape ({tsrc}), not "
                               "measured in this run" if tsrc else None),
            "avg_us": round(avg_s * 1e6, 2),
            "bytes_per_launch": algo, "shape": shape,
            "own_bytes_per_launch": own,
            "frac_own_bytes": round(own / avg_s / 1e9 / HBM_PEAK_GBS, 4),
            "valu_model": {"floor_us": round(floor_s * 1e6, 2),
                           "frac_of_valu_floor": round(floor_s / avg_s, 4),
                           "no_memory_us": round(LAB_NO_MEMORY_US_PER_CLIP_LAYER * batch, 1),
                           "frac_of_no_memory": round(
                               LAB_NO_MEMORY_US_PER_CLIP_LAYER * batch * 1e-6 / avg_s, 4),
                           "note": "1 exp + 4 fma-class per (element, state) at measured gfx950 "
                                   "issue costs, 2.4 GHz; the HBM floor is below it"}}


# the committed rocprofv3 --kernel-trace --stats summary of a default bench command, whose
# scan launches all ran inside the two-stream step (scripts/round_evidence.sh PART=1)
# (each a default C3 bench at 1344 clips: 672-clip scan launches)
IN_STEP_TRACES = (("profiles/r06v_bench_kernel_stats.csv", 672),
                  ("profiles/r06j_bench_kernel_stats.csv", 672),
                  ("profiles/r05zzp_bench_kernel_stats.csv", 672))


def _trace_in_step(algo, batch, kname="scan_seq_dtp_kernel"):
    """The scan's average launch in the newest committed bench trace (its own begin-end
    times) and the HBM fraction on the same bytes; None when no trace of launches of this
    many clips is committed (another --batch prices nothing against it)."""
    import csv
    for rel, tb in IN_STEP_TRACES:
        if tb != batch:
            continue
        path = os.path.join(ROOT, rel)
        if not os.path.exists(path):
            continue
        rows = [r for r in csv.DictReader(open(path)) if kname in r["Name"]]
        calls = sum(int(r["Calls"]) for r in rows)
        if not calls:
            continue
        avg_us = sum(float(r["TotalDurationNs"]) for r in rows) / calls / 1e3
        return {"avg_us": round(avg_us, 2), "launches": calls,
                "frac": round(algo / (avg_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4), "source": rel}
    return None


def scan_in_step(step, L=3137, D=1152, N=16):
    """The scan as the timed step sees it: one more, untimed step with a
    HIP-event pair recorded around every token-major scan launch on its own launch stream
    (mamba_simple.scan_event_log), so the duration includes the other sub-batch stream's
    kernels sharing the CUs.  Priced with the same SURVEY 8(d) bytes as ``roofline``; the
    median launch is the headline (the first layer of each stream starts beside the patch
    embed, the last beside the final norm)."""
    from videomamba_amd.mamba_simple import scan_event_log
    torch.cuda.synchronize()
    with torch.no_grad(), scan_event_log() as log:
        step()
    torch.cuda.synchronize()
    if not log:
        return None
    us = sorted(a.elapsed_time(b) * 1e3 for a, b, _ in log)
    batch = log[0][2]
    e = 2
    algo = batch * D * L * 4 * e + 2 * batch * N * L * e + 4 * D * N + 8 * D + 2 * batch * D * N * e
    med = statistics.median(us)
    mean = sum(us) / len(us)
    return {"batch_per_launch": batch,
            "trace": _trace_in_step(algo, batch),
            "events": {"launches": len(us), "median_us": round(med, 2), "mean_us": round(mean, 2),
                       "min_us": round(us[0], 2), "max_us": round(us[-1], 2),
                       "frac": round(algo / (med * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)},
            "note": "trace: the kernel's own begin-end in the committed rocprofv3 trace of a "
                    "bench command (scripts/traffic_summary.py in-step reproduces it); events: "
                    "HIP events around each scan launch of one more, untimed step of this run "
                    "(mamba_simple.scan_event_log), from the stream reaching the launch to its "
                    "end — it includes waiting for CU slots the other sub-batch stream's "
                    "kernels hold, so it reads lower"}


MFMA_BF16_PEAK_TFLOPS = 2500.0  # dense bf16 MFMA (MI355X_MICROARCH.md; no sparsity)


def _graph_us(fn, reps, calls=20):
    """Average device time of fn() as replayed from a captured HIP graph of ``calls``
    back-to-back calls (HIP events around ``reps`` replays): what the B = 1 chunk's own graph
    sees per kernel, including the dependent-kernel boundary — eager launches from Python at
    these sizes measure the host's issue rate instead (~20 us per call).  Kernel scratch
    comes from one buffer owned here (scratch_override), as the chunk graph's does."""
    from videomamba_amd import kernels as K
    ws = torch.empty(1 << 27, dtype=torch.uint8, device="cuda")
    with K.scratch_override(ws):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(3):
                fn()
        torch.cuda.current_stream().wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(calls):
                fn()
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / (reps * calls)


def _event_us(fn, reps):
    """Average HIP-event time of fn() on the current stream, after warm-up."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def b1_kernel_rooflines(device, reps=50):
    """Per-kernel roofline fractions of one VideoMamba-M layer at the B=1 streaming-chunk
    shape (L=3137, padded 3144 rows): each stage launched alone, HIP-event timed on the
    launch stream, against its algorithmic bytes (HBM-bound kernels) or flops (GEMMs).
    Stages: add+RMSNorm (x bf16 + residual fp32 in, residual fp32 + normed bf16 out),
    in_proj GEMM, fused conv+x_proj (+ conv state out; + dt_proj only when the mixer keeps it
    there), the scan (scan_roofline at B=1: the segmented chunk form, computing dt_proj per
    segment when the mixer does), out_proj GEMM — each the kernel the mixer runs for a
    one-clip chunk (the projections on the row-invariant HIP GEMM, clips=1).  Since round 6
    the mixer runs in_proj with the conv + x_proj partials in its epilogue at this batch
    (``in_proj_conv``: vm_in_proj_conv_proj_fwd, its two launches), and ``layer_us_sum``
    adds the stages the mixer runs; in_proj / conv_proj stay listed for comparison.  Every
    stage but the scan is timed from a captured HIP graph (_graph_us: the chunk graph's own
    per-kernel cost; the eager host-issued timing of rounds 1-5 is ``us_eager``)."""
    from videomamba_amd import kernels as K
    from videomamba_amd.layers import round_up
    from videomamba_amd.mamba_simple import Mamba, _linear

    torch.manual_seed(0)
    C, L = 576, 3137
    Lp = round_up(L)
    bf = torch.bfloat16
    mx = Mamba(d_model=C, layer_idx=0).to(device, bf).eval()
    Dm, N, R, W = mx.d_inner, mx.d_state, mx.dt_rank, mx.d_conv
    E = R + 2 * N
    stream = torch.cuda.current_stream(device).cuda_stream
    x = torch.randn(Lp, C, device=device, dtype=bf)
    res = torch.randn(Lp, C, device=device)
    w32 = torch.ones(C, device=device)
    hn = torch.empty(Lp, C, device=device, dtype=bf)
    xz = torch.randn(Lp, 2 * Dm, device=device, dtype=bf)
    y = torch.randn(Lp, Dm, device=device, dtype=bf)
    u = torch.empty(Lp, Dm, device=device, dtype=bf)
    dt = torch.empty(Lp, Dm, device=device, dtype=bf)
    xdbl = torch.empty(Lp, E, device=device, dtype=bf)
    cs_in = torch.randn(1, Dm, W, device=device, dtype=bf)
    cs_out = torch.empty(1, Dm, W, device=device, dtype=bf)
    _, _, _, cw, cb = mx._fp32_params()
    wx_pad, wdt_pad = mx._padded_proj_weights()
    out = {}

    def hbm(name, us, nbytes):
        gbs = nbytes / us / 1e3
        out[name] = {"us": round(us, 2), "bound": "hbm", "achieved": round(gbs, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4)}

    def mfma(name, us, flops):
        tf = flops / us / 1e6
        out[name] = {"us": round(us, 2), "bound": "mfma", "achieved": round(tf, 1),
                     "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s",
                     "frac": round(tf / MFMA_BF16_PEAK_TFLOPS, 4)}

    def stage(name, fn, kind, amount):
        (hbm if kind == "hbm" else mfma)(name, _graph_us(fn, reps), amount)
        out[name]["us_eager"] = round(_event_us(fn, reps), 2)

    with torch.no_grad():
        stage("add_norm", lambda: K.add_norm_raw(x, res, w32, None, hn, res, Lp, C, 1e-5, True,
                                                 torch.cuda.current_stream().cuda_stream),
              "hbm", 12 * Lp * C)
        hn.normal_()
        stage("in_proj", lambda: _linear(hn, mx.in_proj.weight, clips=1), "mfma",
              2 * Lp * C * 2 * Dm)
        # the mixer's choice at this shape: dt_proj inside the segmented scan (no dt rows)
        dtp = mx._dtp_ok(hn.view(1, Lp, C), L)
        wd, dto = (None, None) if dtp else (wdt_pad, dt)
        stage("conv_proj", lambda: K.conv_proj_raw(
            xz, (Lp * 2 * Dm, 2 * Dm), cw, cb, cs_in, (cs_in.stride(0), cs_in.stride(1)),
            cs_out, (cs_out.stride(0), cs_out.stride(1)), wx_pad, E, wd, R, u,
            (Lp * Dm, Dm), xdbl, (Lp * E, E), dto, (Lp * Dm, Dm), Lp, 1, Dm, L, W,
            torch.cuda.current_stream().cuda_stream), "hbm",
            2 * Lp * ((2 if dtp else 3) * Dm + E) + 2 * wx_pad.numel()
            + (0 if dtp else 2 * wdt_pad.numel()))
        fused = mx._in_proj_conv_ok(hn.view(1, Lp, C), L, not dtp)
        if fused:  # what the mixer runs at this batch instead of the two stages above
            stage("in_proj_conv", lambda: K.in_proj_conv_proj_raw(
                hn, mx.in_proj.weight, xz[:, Dm:], cw, cb, cs_in,
                (cs_in.stride(0), cs_in.stride(1)), cs_out, (cs_out.stride(0), cs_out.stride(1)),
                wx_pad, E, wdt_pad, R, u, xdbl, dto, Lp, 1, Dm, L, W,
                torch.cuda.current_stream().cuda_stream), "mfma",
                2 * Lp * C * 2 * Dm + 2 * Lp * Dm * E)
        sc = scan_roofline(1, reps, device, "tm", dtp=dtp)
        out["scan"] = {k: sc[k] for k in ("avg_us", "bound", "achieved", "peak", "unit", "frac")}
        out["scan"]["us"] = out["scan"].pop("avg_us")
        out["scan"]["dt_proj_inside"] = bool(dtp)
        stage("out_proj", lambda: _linear(y, mx.out_proj.weight, clips=1), "mfma",
              2 * Lp * Dm * C)
    run = ["add_norm"] + (["in_proj_conv"] if fused else ["in_proj", "conv_proj"]) + ["scan",
                                                                                      "out_proj"]
    out["layer_us_sum"] = round(sum(out[k]["us"] for k in run), 2)
    out["layer_stages"] = run
    out["shape"] = f"VideoMamba-M layer, B=1, L={L} (padded {Lp}), bf16, stages launched alone"
    return out


def _oracle_clip_seconds(cfg, runs=3):
    """Median wall time of the oracle's fp32 B=1 forward of one clip, after one warm-up."""
    from oracle import videomamba_oracle as orc
    from videomamba_amd.videomamba import PretrainVideoMamba

    torch.manual_seed(0)
    m = PretrainVideoMamba(depth=cfg["depth"], embed_dim=cfg["embed_dim"],
                           num_frames=cfg["frames"])
    p = {k: v.detach() for k, v in m.state_dict().items()}
    ocfg = dict(img_size=224, patch_size=16, depth=cfg["depth"], kernel_size=1,
                num_frames=cfg["frames"], fused_add_norm=True, rms_norm=True,
                residual_in_fp32=True, pool_type="cls+avg", norm_epsilon=1e-5, d_state=16,
                d_conv=4)
    x = torch.randn(1, 3, cfg["frames"], 224, 224)
    times = []
    with torch.no_grad():
        for i in range(runs + 1):
            t0 = time.perf_counter()
            orc.encoder_forward(p, ocfg, x)
            if i:
                times.append(time.perf_counter() - t0)
    return statistics.median(times)


# The timed oracle against the reference's own CPU path, both timed warm in one session on
# the same 8 threads of the build container (scripts/cpu_calibration.py): the port's time
# over the reference's, per config.  Read from the committed record at run time.
CPU_CALIBRATION_FILE = os.path.join(ROOT, "profiles", "r03_cpu_calibration.json")


def _cpu_calibration():
    try:
        with open(CPU_CALIBRATION_FILE) as f:
            rec = json.load(f)
    except (OSError, ValueError):
        return None
    return {"threads": rec.get("threads"), "cpu_model": rec.get("cpu_model"),
            "oracle_over_reference_s_per_clip": {
                k: v["oracle_over_reference"] for k, v in rec.get("configs", {}).items()},
            "reference_s_per_clip": {
                k: v["reference_s_per_clip"] for k, v in rec.get("configs", {}).items()},
            "source": os.path.relpath(CPU_CALIBRATION_FILE, ROOT)}


def _cpu_info():
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = os.cpu_count()
    return model, affinity


def _cpu_share(affinity):
    """The host CPUs this process may actually run on: OMP_NUM_THREADS when the launcher set
    it (16 on a one-GPU box), else the cgroup CPU quota, else the affinity mask.
    os.cpu_count() counts the whole shared host (256 on the GPU boxes): the round-4 bench at
    256 oracle threads on a 16-CPU share ran past the box's 180 s no-output limit."""
    env = os.environ.get("OMP_NUM_THREADS", "").strip()
    if env.isdigit() and int(env) > 0:
        return int(env)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            return max(1, int(int(quota) / int(period)))
    except (OSError, ValueError):
        pass
    return max(1, affinity or os.cpu_count() or 1)


def cpu_baseline(cfg, threads):
    """the CPU path on the host cores, fp32 B=1, one clip of the bench
    config and of C1 (Ti 8x224^2).  The code timed is the oracle (the CPU restatement
    pinned to the reference), and ``value`` is its measured rate on these cores.  Beside it,
    ``reference_estimate`` scales that rate by the oracle-vs-reference time ratio of one
    calibration session (profiles/r03_cpu_calibration.json: 8 threads of the build
    container's Xeon, not these cores) — an estimate of the reference's own CPU rate, never
    the headline.  ``threads`` 0 = every CPU this process may use
    (``_cpu_share``: the box's share of the host; SURVEY 8(d)'s os.cpu_count() counts the
    whole shared host and oversubscribes the share 16x there).  Median of 2 after 1
    warm-up: a bounded sample (~10-30 s of CPU work) so the bench stays within minutes."""
    model, affinity = _cpu_info()
    share = _cpu_share(affinity)
    if threads <= 0:
        threads = share
    ti = CONFIGS["ti8"]
    torch.set_num_threads(threads)
    dt = _oracle_clip_seconds(cfg, runs=2)
    dt_c1 = _oracle_clip_seconds(ti, runs=2)
    cal = _cpu_calibration()
    key = {16: "m16", 8: "ti8"}.get(cfg["frames"]) if cfg["embed_dim"] in (576, 192) else None
    ratios = (cal or {}).get("oracle_over_reference_s_per_clip", {})
    ratio, ratio_c1 = ratios.get(key), ratios.get("ti8")
    port = cfg["frames"] * 196 / dt
    port_c1 = ti["frames"] * 196 / dt_c1
    est = None
    if ratio:
        est = {"value": round(port * ratio, 2), "unit": "video-tokens/s",
               "basis": f"the measured oracle rate x its time ratio to the reference's own CPU "
                        f"forward ({ratio}), taken once at {cal.get('threads')} threads on "
                        f"{cal.get('cpu_model')}; not re-measured on these cores",
               "calibration": cal}
    return {"value": round(port, 2),
            "unit": "video-tokens/s", "cores": threads, "kind": "port",
            "value_basis": "the oracle (oracle/videomamba_oracle.py) timed on these cores",
            "reference_estimate": est,
            "cpu_model": model, "host_cpu_count": os.cpu_count(), "affinity_cpus": affinity,
            "cpu_share": share,
            "threads_policy": "the CPUs this process may use (OMP_NUM_THREADS / cgroup quota / "
                              "affinity); os.cpu_count() counts the whole shared host",
            "sample": f"1 clip {cfg['name']} {cfg['frames']}x224^2 fp32 B=1, full forward, "
                      f"median of 2 after 1 warm-up ({dt:.2f} s at {threads} threads), "
                      "oracle/videomamba_oracle.py",
            "c1": {"value": round(port_c1, 2), "unit": "video-tokens/s",
                   "reference_estimate": round(port_c1 * ratio_c1, 2) if ratio_c1 else None,
                   "sample": f"C1: 1 clip {ti['name']} {ti['frames']}x224^2 fp32 B=1, median "
                             f"of 2 after 1 warm-up ({dt_c1:.2f} s)"}}


def _timed_steps(step, steps, warmup, world, device, sync):
    """W untimed steps, then K steps bracketed by barrier + device sync on both sides;
    returns the slowest rank's elapsed seconds (max over ranks)."""
    from videomamba_amd.sharding import max_over_ranks

    def barrier():
        sync()
        if world > 1:
            dist.barrier()
        sync()

    out = None
    with torch.no_grad():
        for _ in range(warmup):
            out = step()
        barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            out = step()
        barrier()
        elapsed = time.perf_counter() - t0
    return max_over_ranks(elapsed, device), out


def metric_name(cfg):
    """BASELINE.json's metric, named for the workload actually run (the headline string
    exactly for the C3 default, VideoMamba-M 16f)."""
    return (f"video-tokens/sec per GPU + streaming-chunk p50 latency, "
            f"{cfg['name']} {cfg['frames']}f 224")


def _base_line(args, cfg, world, global_batch, per_rank, elapsed, strong):
    T = cfg["frames"]
    ms_per_step = elapsed / args.steps * 1e3
    value = global_batch * T * 196 * args.steps / elapsed
    return {
        "metric": metric_name(cfg),
        "value": round(value, 1), "unit": "video-tokens/s", "n_gpus": world,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": True, "scaling": "strong" if strong else "weak",
        "vs_baseline": None, "dtype": "bf16",
        "data": "synthetic clips (randn), random-init weights (seed 0)",
        "config": {"workload": f"{cfg['name']} {T}x224^2 bf16, " + (
                       "full-sequence forward per step" if args.full_sequence else
                       "one stateful streaming chunk (chunk_size 32) per step"),
                   "model": cfg["name"], "global_batch": global_batch,
                   "per_gpu_batch": per_rank, "frames": T, "seq_len": 1 + T * 196,
                   "parallelism": f"batch-sharded x{world}, no data-path collectives",
                   "sub_batch_streams": _sub_batch_streams(per_rank, cfg["embed_dim"])},
        "per_gpu_value": round(value / world, 1),
    }


def _sub_batch_streams(batch, embed_dim=576):
    """How many HIP streams the model's forward splits this per-GPU batch over
    (options.batch_streams from batch_stream_min_clips clips and batch_stream_min_work
    clip-channels, d_inner = 2 x embed_dim; bit-identical to one stream) —
    the rule of PretrainVideoMamba._stream_parts."""
    try:
        from videomamba_amd import options
    except Exception:  # the CPU stub run
        return 1
    o = options.get()
    split = (batch >= max(int(o.batch_stream_min_clips), 2)
             and batch * 2 * embed_dim >= int(o.batch_stream_min_work))
    return int(o.batch_streams) if split else 1


def main_stub_cpu(args):
    """The bench's multi-rank control flow on CPU/gloo with the encoder replaced by a small
    matmul: rank/world from torchrun, per-rank batch, timed region, max over ranks, one
    JSON line from rank 0."""
    from videomamba_amd.sharding import dist_env, shard_range

    rank, _, world = dist_env()
    if world > 1:
        dist.init_process_group("gloo")
    cfg = CONFIGS[args.config]
    if args.global_batch:
        a, b = shard_range(args.global_batch, world, rank)
        per_rank, global_batch, strong = b - a, args.global_batch, True
    else:
        per_rank, global_batch, strong = args.batch, args.batch * world, False
    w = torch.randn(64, 64)
    x = torch.randn(max(per_rank, 1), 64)

    def step():
        time.sleep(0.002 * (1 + rank))  # ranks differ: the max must be the slowest
        return x @ w

    elapsed, _ = _timed_steps(step, args.steps, args.warmup, world, torch.device("cpu"),
                              lambda: None)
    if rank == 0:
        line = _base_line(args, cfg, world, global_batch, per_rank, elapsed, strong)
        line["stub"] = "cpu"
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main():
    args = _args()
    if args.stub_cpu:
        return main_stub_cpu(args)
    from videomamba_amd.sharding import dist_env, shard_range

    rank, local, world = dist_env()
    # one rank per GPU (local rank = device); a gloo rehearsal on a box with fewer GPUs than
    # ranks shares them round-robin
    dev_index = local if args.dist_backend == "nccl" else local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(dev_index)
    device = torch.device("cuda", dev_index)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group("gloo")

    from videomamba_amd import options
    from videomamba_amd.videomamba import PretrainVideoMamba

    options.get().scan_dt_proj = args.scan_dt_proj
    if args.batch_streams > 0:
        options.get().batch_streams = args.batch_streams
    cfg = CONFIGS[args.config]
    torch.manual_seed(0)
    model = PretrainVideoMamba(depth=cfg["depth"], embed_dim=cfg["embed_dim"],
                               num_frames=cfg["frames"], pool_type="cls+avg")
    model = model.to(device=device, dtype=torch.bfloat16).eval()
    T = cfg["frames"]
    global_batch = args.global_batch
    if global_batch:  # --global-batch: one global batch split across ranks (strong scaling)
        a, b = shard_range(global_batch, world, rank)
        B, strong = b - a, True
    else:  # C3: a fixed batch per rank (weak scaling)
        B, strong, global_batch = args.batch, False, args.batch * world
    g = torch.Generator(device=device).manual_seed(1000 + rank)
    x = torch.randn(B, 3, T, 224, 224, device=device, generator=g).to(torch.bfloat16)
    state = model.allocate_state(B, dtype=torch.bfloat16, device=device)

    def step():
        if args.full_sequence:
            return model(x)
        return model(x, ssm_state=state, temporal_pos_offset=0)

    _progress(f"model built, B={B}: {args.warmup} warm-up + {args.steps} timed steps")
    elapsed, out = _timed_steps(step, args.steps, args.warmup, world, device,
                                torch.cuda.synchronize)
    assert torch.isfinite(out[1].float()).all()
    _progress(f"timed: {elapsed / args.steps * 1e3:.1f} ms per step")
    from videomamba_amd import kernels as K
    K.check_scan_sync()  # no one-launch scan hand-off timed out (outside the timed region)
    line = _base_line(args, cfg, world, global_batch, B, elapsed, strong)

    # streaming-chunk p50 latency at B=1 (one stateful chunk of the same clip shape):
    # replayed from a captured HIP graph (videomamba_amd/graphs.py), and eager for reference
    from videomamba_amd.graphs import StreamingChunkGraph
    with torch.no_grad():
        x1 = x[:1].contiguous()
        st1 = model.allocate_state(1, dtype=torch.bfloat16, device=device)
        runner = StreamingChunkGraph(model, batch=1, frames=T)

        def chunk_lat(fn):
            lat = []
            for i in range(args.p50_chunks + 3):
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                if i >= 3:
                    lat.append((time.perf_counter() - t1) * 1e3)
            return statistics.median(lat)

        p50_eager = p50_graph = None
        if not args.no_b1:
            _progress("B=1 chunk latency (eager, then graph replay)")
            outs = []
            p50_eager = chunk_lat(lambda: outs.append(
                model(x1, ssm_state=st1, temporal_pos_offset=0)[1]))
            p50_graph = chunk_lat(lambda: outs.append(runner.run(x1, temporal_pos_offset=0)[1]))
            # the B=1 legs run the one-launch chunked scan: a timed-out block hand-off there
            # poisons its outputs with NaN, so no latency is reported unless none happened
            runner.check()
            K.check_scan_sync()
            assert all(bool(torch.isfinite(o.float()).all()) for o in outs[-3:] + outs[:3]), \
                "non-finite B=1 chunk output"
        from videomamba_amd.mamba_simple import mixer_layout
        mx0 = model.layers[0].mixer
        # the scan as the step launches it: one sub-batch stream's clips per launch
        rb = max(B // _sub_batch_streams(B, cfg["embed_dim"]), 1)
        hn0 = torch.empty((1, 1, cfg["embed_dim"]), device=device,
                          dtype=torch.bfloat16).expand(rb, 3144, cfg["embed_dim"])
        _progress("scan roofline leg")
        roof = scan_roofline(rb, args.scan_reps, device,
                             mixer_layout(rb, cfg["embed_dim"] * 2, device),
                             dtp=cfg["embed_dim"] == 576 and mx0._dtp_ok(hn0, 3137))
        if cfg["embed_dim"] == 576 and T == 16 and not args.full_sequence:  # the C3 step
            _progress("scan in-step leg")
            roof["in_step"] = scan_in_step(step)
        b1 = b1_kernel_rooflines(device) if cfg["embed_dim"] == 576 and not args.no_b1 else None

    if rank == 0:
        line.update({
            "chunk_p50_ms": round(p50_graph, 3) if p50_graph is not None else None,
            "chunk_p50_eager_ms": round(p50_eager, 3) if p50_eager is not None else None,
            "chunk_p50_batch": 1, "chunk_p50_mode": "hipGraph replay (StreamingChunkGraph)",
            "roofline": roof,
        })
        if b1 is not None:
            line["b1_kernels"] = b1
        if world == 1 and not args.no_cpu_baseline:
            _progress("CPU baseline (oracle)")
            line["cpu_baseline"] = cpu_baseline(cfg, args.cpu_threads)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
