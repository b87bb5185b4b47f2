"""Long-video streaming benchmark (BASELINE.json config C5): VideoMamba-M, 1024 frames per
clip fed as 16 stateful chunks of 64 frames (temporal_pos_offset advancing, conv/ssm state
carried through all 32 layers), bf16, synthetic clips, random-init weights (seed 0).

    python scripts/bench_long_video.py [--batch 1] [--frames 1024] [--chunk 64] [--reps 2]

Prints one JSON line: video tokens per second over the whole clip(s), per-chunk latency
(p50 over every chunk of the timed passes) and the first/continuation chunk sequence
lengths (12545 / 12544 at chunk 64).
"""

from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--frames", type=int, default=1024)
    ap.add_argument("--chunk", type=int, default=64)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--eager", action="store_true", help="eager launches instead of hipGraph replay")
    ap.add_argument("--check-chunks", type=int, default=4,
                    help="chunks compared against one full-sequence forward (fp32 state)")
    a = ap.parse_args()
    from videomamba_amd.videomamba import PretrainVideoMamba

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    # num_frames = the whole clip so temporal positions slice exactly (no interpolation)
    model = PretrainVideoMamba(depth=32, embed_dim=576, num_frames=a.frames,
                               pool_type="cls+avg", add_pool_norm=False)
    model = model.to(device=dev, dtype=torch.bfloat16).eval()
    g = torch.Generator(device=dev).manual_seed(5)
    x = torch.randn(a.batch, 3, a.frames, 224, 224, device=dev, generator=g).to(torch.bfloat16)
    nchunks = a.frames // a.chunk

    runner = None
    if not a.eager:
        from videomamba_amd.graphs import StreamingChunkGraph
        runner = StreamingChunkGraph(model, batch=a.batch, frames=a.chunk)

    def clip_pass(lat):
        state = model.allocate_state(a.batch, dtype=torch.bfloat16, device=dev)
        if runner is not None:
            runner.reset_state()
        out = None
        for c in range(nchunks):
            t1 = time.perf_counter()
            xc = x[:, :, c * a.chunk:(c + 1) * a.chunk]
            if runner is not None:
                out = runner.run(xc, temporal_pos_offset=c * a.chunk)
            else:
                out, state = model(xc, ssm_state=state, temporal_pos_offset=c * a.chunk)
            torch.cuda.synchronize()
            if lat is not None:
                lat.append((time.perf_counter() - t1) * 1e3)
        return out

    with torch.no_grad():
        for _ in range(a.warmup):
            clip_pass(None)
        torch.cuda.synchronize()
        lat = []
        t0 = time.perf_counter()
        for _ in range(a.reps):
            out = clip_pass(lat)
        elapsed = time.perf_counter() - t0
    assert torch.isfinite(out.float()).all()
    tokens = a.reps * a.batch * a.frames * 196

    # chunked == full: the first check-chunks chunks streamed with an fp32
    # state against one full-sequence forward over the same frames; relative error of the
    # patch tokens of the last chunk (the stitched prefix is the same comparison earlier)
    rel = None
    if a.check_chunks > 0:
        with torch.no_grad():
            nc = min(a.check_chunks, nchunks)
            st = model.allocate_state(a.batch, dtype=torch.float32, device=dev)
            for c in range(nc):
                # add_pool_norm=False: (x_vis, next_state); x_vis is the whole chunk
                xv, st = model(x[:, :, c * a.chunk:(c + 1) * a.chunk], ssm_state=st,
                               temporal_pos_offset=c * a.chunk)
            full = model(x[:, :, :nc * a.chunk])
            ref = full[:, -xv.shape[1]:].float()
            rel = ((xv.float() - ref).norm() / ref.norm()).item()
    print(json.dumps({
        "workload": f"VideoMamba-M {a.frames} frames as {nchunks} x chunk{a.chunk}, carried "
                    f"state, bf16, B={a.batch}",
        "mode": "eager" if a.eager else "hipGraph replay (StreamingChunkGraph)",
        "video_tokens_per_s": round(tokens / elapsed, 1),
        "clip_s": round(elapsed / a.reps, 4),
        "chunk_p50_ms": round(statistics.median(lat), 3),
        "chunk_first_ms": round(lat[0], 3),
        "seq_len_first_chunk": 1 + a.chunk * 196, "seq_len_next_chunks": a.chunk * 196,
        "peak_mem_gb": round(torch.cuda.max_memory_allocated(dev) / 1e9, 2),
        "chunked_vs_full_rel": rel,
        "chunked_vs_full_frames": min(a.check_chunks, nchunks) * a.chunk,
        "data": "synthetic clips (randn), random-init weights (seed 0)",
    }), flush=True)


if __name__ == "__main__":
    main()
