"""Summarise the round-evidence PMC passes for one kernel into profiles/scan_traffic_<round>.json
(HBM bytes per launch: FETCH_SIZE x2 per the gfx950 correction + WRITE_SIZE) and print the
SQ counter averages.   python scripts/traffic_summary.py r01b 336 scan_seq_kernel"""
import collections
import csv
import glob
import json
import sys

rnd, batch, kname = sys.argv[1], int(sys.argv[2]), sys.argv[3]
base = f"gpurun_out/{rnd}"


def per_dispatch(tag):
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(f"{base}/pmc_{tag}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if kname in r["Kernel_Name"]:
                vals[r["Counter_Name"]][r["Dispatch_Id"]] += float(r["Counter_Value"])
    return {c: sum(d.values()) / len(d) for c, d in vals.items() if d}


fetch = per_dispatch("FETCH_SIZE")["FETCH_SIZE"] * 1024
write = per_dispatch("WRITE_SIZE")["WRITE_SIZE"] * 1024
D, L, N, e = 1152, 3137, 16, 2
algo = batch * D * L * 4 * e + 2 * batch * N * L * e + 4 * D * N + 8 * D + 2 * batch * D * N * e
out = {"kernel": f"vm::{kname}<bf16> (token-major, B/C as scalar loads)",
       "shape": f"B={batch} D={D} L={L} N={N} bf16, stateful",
       "fetch_size_bytes_raw": fetch, "write_size_bytes": write,
       "hbm_bytes_per_launch": 2 * fetch + write, "algorithmic_bytes_per_launch": algo,
       "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes on "
                 "scripts/bench_scan.py at the bench shape (dispatches averaged); FETCH_SIZE "
                 "doubled per MI355X_MICROARCH.md (gfx950 tallies 128-B read requests at "
                 "64 B); u/delta/z are 2-byte-per-lane loads, for which that correction is "
                 "uncalibrated", "round": rnd}
json.dump(out, open(f"profiles/scan_traffic_{rnd}.json", "w"), indent=1)
print(json.dumps(out, indent=1))
for tag in ("SQ_WAVES", "SQ_ACTIVE_INST_VALU"):
    for c, v in sorted(per_dispatch(tag).items()):
        print(f"{c:28s} {v:.4g}")
