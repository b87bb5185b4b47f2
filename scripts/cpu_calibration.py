"""Cross-calibrate the CPU baseline (BASELINE.md "CPU-baseline plan"): in ONE session, on
the same threads, time

* the oracle's fp32 B=1 forward (oracle/videomamba_oracle.py — the timed leg of bench.py's
  cpu_baseline, the thing that travels to the GPU box), and
* the reference's own CPU forward (/root/reference models/videomamba/videomamba.py imported
  as-is through tests/golden/gen_golden.py's route: pure-torch stand-ins for the absent
  mamba-ssm / causal-conv1d / timm, the scan = the reference's _selective_scan_ref),

each as the median of 3 runs after 1 warm-up, on identical weights (the reference model's
seeded init, loaded into the oracle) and an identical clip.  Dev container only (needs
/root/reference); the committed result is profiles/r03_cpu_calibration.json.

    python scripts/cpu_calibration.py --threads 8 > profiles/r03_cpu_calibration.json
"""
import argparse
import json
import os
import platform
import statistics
import subprocess
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))

CONFIGS = {"ti8": dict(depth=24, embed_dim=192, frames=8),
           "m16": dict(depth=32, embed_dim=576, frames=16)}


def _cpu_model():
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, check=True).stdout
        for line in out.splitlines():
            if line.startswith("Model name:"):
                return line.split(":", 1)[1].strip()
    except Exception:  # noqa: BLE001
        pass
    return platform.processor() or platform.machine()


def _median_s(fn, runs=3):
    times = []
    for i in range(runs + 1):
        t0 = time.perf_counter()
        fn()
        if i:
            times.append(time.perf_counter() - t0)
    return statistics.median(times), times


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--configs", nargs="+", default=["ti8", "m16"])
    a = ap.parse_args()
    torch.set_num_threads(a.threads)

    import gen_golden
    from oracle import videomamba_oracle as orc
    _, vm, _ = gen_golden._import_reference()

    out = {"threads": a.threads, "cpu_count": os.cpu_count(), "cpu_model": _cpu_model(),
           "torch": torch.__version__, "method": "median of 3 after 1 warm-up, fp32, B=1, "
           "same weights and clip for both sides, one process", "configs": {}}
    for name in a.configs:
        c = CONFIGS[name]
        torch.manual_seed(0)
        ref = vm.PretrainVideoMamba(depth=c["depth"], embed_dim=c["embed_dim"],
                                    num_frames=c["frames"], fused_add_norm=True, rms_norm=True,
                                    residual_in_fp32=True, pool_type="cls+avg",
                                    ssm_cfg={"use_fast_path": False}).eval()
        p = {k: v.detach().clone() for k, v in ref.state_dict().items()}
        ocfg = dict(img_size=224, patch_size=16, depth=c["depth"], kernel_size=1,
                    num_frames=c["frames"], fused_add_norm=True, rms_norm=True,
                    residual_in_fp32=True, pool_type="cls+avg", norm_epsilon=1e-5, d_state=16,
                    d_conv=4)
        x = torch.randn(1, 3, c["frames"], 224, 224)
        with torch.no_grad():
            t_orc, all_orc = _median_s(lambda: orc.encoder_forward(p, ocfg, x))
            with gen_golden._pretend_cuda():
                t_ref, all_ref = _median_s(lambda: ref(x))
                xv_r, xp_r = ref(x)
            xv_o, xp_o, _ = orc.encoder_forward(p, ocfg, x)
        rel = ((xv_o - xv_r).norm() / xv_r.norm()).item()
        out["configs"][name] = {
            "oracle_s_per_clip": round(t_orc, 3), "reference_s_per_clip": round(t_ref, 3),
            "oracle_over_reference": round(t_orc / t_ref, 3),
            "oracle_runs_s": [round(t, 3) for t in all_orc],
            "reference_runs_s": [round(t, 3) for t in all_ref],
            "video_tokens": c["frames"] * 196,
            "oracle_vs_reference_x_vis_rel": rel}
        print(json.dumps({name: out["configs"][name]}), file=sys.stderr, flush=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
