"""Summarise rocprofv3 counter CSVs: per-dispatch mean of each counter for kernels whose
name matches --kernel, grouped by the run directory prefix (variant)."""
import argparse, collections, csv, glob, os
ap = argparse.ArgumentParser()
ap.add_argument("root")
ap.add_argument("--kernel", default="scan")
a = ap.parse_args()
groups = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(a.root, "*", "*counter_collection.csv"))):
    tag = os.path.basename(os.path.dirname(f)).split("_p")[0]
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if a.kernel not in r["Kernel_Name"]:
            continue
        per[(r["Counter_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
    for (name, _), v in per.items():
        groups[tag][name].append(v)
for tag in sorted(groups):
    print(tag)
    for name in sorted(groups[tag]):
        vals = groups[tag][name]
        print(f"  {name:28s} {sum(vals)/len(vals):.5g}  (n={len(vals)})")
