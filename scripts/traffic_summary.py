"""Summarise the round-evidence PMC passes for one kernel into profiles/scan_traffic_<round>.json
and print the SQ counter averages.

    python scripts/traffic_summary.py r01c 336 scan_seq_kernel

HBM bytes per launch come from rocprofv3 FETCH_SIZE and WRITE_SIZE (separate passes,
dispatches averaged).  MI355X_MICROARCH.md: on gfx950 FETCH_SIZE tallies 128-B read requests
at 64 B for 16-B-per-lane streaming reads, WRITE_SIZE is exact for 16-B stores, and other
access widths are uncalibrated — "calibrate on a known byte count in your own access
pattern".  The scan reads and writes 2-byte lanes (one 128-B row segment per wave and
operand per step), so the round also runs the same FETCH/WRITE passes on
tools/probes/scan_lab's calibration kernel: that access pattern, no scan math, a known byte
count.  The scan's counters are divided by the measured counter-to-bytes ratios.
"""
import collections
import csv
import glob
import json
import sys


def in_step(stats_csv, bench_json=None, batch=672, kname="scan_seq_dtp_kernel"):
    """The scan's HBM fraction as the bench step sees it, from committed
    files only: the rocprofv3 --stats kernel summary of a bench command (every launch of
    the scan there ran inside the step, beside the other sub-batch stream's kernels) and,
    when given, that command's bench line (its isolated ``roofline.frac`` and live
    ``roofline.in_step``).  Bytes: SURVEY 8(d) per stateful bf16 launch of ``batch`` clips.

        python scripts/traffic_summary.py in-step profiles/r05zzp_bench_kernel_stats.csv \
            [profiles/r05zzp_bench.json] [batch]
    """
    D_, L_, N_, e_ = 1152, 3137, 16, 2
    algo_ = (batch * D_ * L_ * 4 * e_ + 2 * batch * N_ * L_ * e_ + 4 * D_ * N_ + 8 * D_
             + 2 * batch * D_ * N_ * e_)
    rows = [r for r in csv.DictReader(open(stats_csv)) if kname in r["Name"]]
    calls = sum(int(r["Calls"]) for r in rows)
    avg_ns = sum(float(r["TotalDurationNs"]) for r in rows) / calls
    out = {"kernel": kname, "batch_per_launch": batch, "bytes_per_launch": algo_,
           "trace": stats_csv, "trace_launches": calls, "trace_avg_us": round(avg_ns / 1e3, 2),
           "trace_frac": round(algo_ / (avg_ns * 1e-9) / 8e12, 4)}
    if bench_json:
        line = json.load(open(bench_json))
        line = line.get("parsed", line)
        roof = line["roofline"]
        out["isolated_avg_us"], out["isolated_frac"] = roof["avg_us"], roof["frac"]
        ins = roof.get("in_step") or {}
        ev = ins.get("events", ins)  # round 6: {"trace": .., "events": ..}
        if "median_us" in ev:
            out["events_median_us"] = ev["median_us"]
            out["events_frac"] = ev["frac"]
        if ins.get("trace"):
            out["line_trace_frac"], out["line_trace_source"] = ins["trace"]["frac"], ins["trace"]["source"]
    print(json.dumps(out, indent=1))
    return out


if len(sys.argv) > 1 and sys.argv[1] == "in-step":
    a = sys.argv[2:]
    in_step(a[0], a[1] if len(a) > 1 and a[1].endswith(".json") else None,
            int(a[-1]) if len(a) > 1 and a[-1].isdigit() else 672)
    sys.exit(0)

rnd, batch, kname = sys.argv[1], int(sys.argv[2]), sys.argv[3]
base = f"gpurun_out/{rnd}"
D, L, N, e = 1152, 3137, 16, 2
Lp = (L + 7) // 8 * 8


def per_dispatch(pattern, kernel):
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(f"{base}/{pattern}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if kernel in r["Kernel_Name"]:
                vals[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {c: sum(d.values()) / len(d) for c, d in vals.items() if d}


fetch = per_dispatch("pmc_FETCH_SIZE", kname)["FETCH_SIZE"] * 1024
write = per_dispatch("pmc_WRITE_SIZE", kname)["WRITE_SIZE"] * 1024
algo = batch * D * L * 4 * e + 2 * batch * N * L * e + 4 * D * N + 8 * D + 2 * batch * D * N * e

# calibration kernel: reads u, delta, z rows and writes y rows of (batch * Lp, D) bf16
calib_read = 3.0 * batch * Lp * D * e
calib_write = 1.0 * batch * Lp * D * e
cf = per_dispatch("calib_FETCH_SIZE", "stream_kernel").get("FETCH_SIZE")
cw = per_dispatch("calib_WRITE_SIZE", "stream_kernel").get("WRITE_SIZE")
out = {"kernel": f"vm::{kname}" + ("" if "dtp" in kname else "<bf16>") + " (token-major, B/C as scalar loads)",
       "shape": f"B={batch} D={D} L={L} N={N} bf16, stateful",
       "fetch_size_bytes_raw": fetch, "write_size_bytes_raw": write,
       "algorithmic_bytes_per_launch": algo, "round": rnd}
if cf and cw:
    r_read = cf * 1024 / calib_read      # counter bytes per true byte, this access pattern
    r_write = cw * 1024 / calib_write
    out.update({
        "calibration": {"kernel": "tools/probes/scan_lab stream_kernel<1> (calib mode)",
                        "true_read_bytes": calib_read, "fetch_size_bytes": cf * 1024,
                        "true_write_bytes": calib_write, "write_size_bytes": cw * 1024,
                        "read_ratio": round(r_read, 4), "write_ratio": round(r_write, 4)},
        "hbm_bytes_per_launch": fetch / r_read + write / r_write,
        "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes on "
                  "scripts/bench_scan.py at the bench shape, each divided by the counter/true-"
                  "byte ratio measured the same way on a calibration kernel with the scan's "
                  "2-byte-lane access pattern and a known byte count (MI355X_MICROARCH.md "
                  "HBM section: uncalibrated widths must be calibrated)"})
else:
    out.update({"hbm_bytes_per_launch": 2 * fetch + write,
                "method": "FETCH_SIZE doubled (gfx950 16-B-lane correction) + WRITE_SIZE; "
                          "no calibration run found"})
json.dump(out, open(f"profiles/scan_traffic_{rnd}.json", "w"), indent=1)
print(json.dumps(out, indent=1))
for tag in ("pmc_SQ_WAVES", "pmc_SQ_ACTIVE_INST_VALU"):
    for c, v in sorted(per_dispatch(tag, kname).items()):
        print(f"{c:28s} {v:.4g}")
