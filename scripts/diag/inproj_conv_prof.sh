#!/bin/bash
# kernel-trace split of vm_in_proj_conv_proj_fwd's two launches per pricing variant
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r06e}
mkdir -p $O
for v in product ${VARIANTS:-ic_noepi ic_noconv ic_nopart ic_nou ic_nops ic_noz}; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v -o k -- python scripts/diag/inproj_conv_bench.py $v 1 > $O/$v.log 2>&1 || { echo $v failed; tail $O/$v.log; exit 1; }
  python - "$O/$v" "$v" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/k_kernel_stats.csv", recursive=True)[0]
rows = [r for r in csv.DictReader(open(f)) if "inproj_conv" in r["Name"] or "xdbl" in r["Name"] or "linear_dma" in r["Name"] or "conv_proj_fused" in r["Name"]]
print(sys.argv[2], {r["Name"].split("(")[0].split("::")[-1][:40]: round(float(r["AverageNs"]) / 1e3, 2) for r in rows})
PY
done
