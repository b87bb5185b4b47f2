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
