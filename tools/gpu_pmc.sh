#!/bin/bash
# PMC passes over the bench (one counter group per rocprofv3 run, --kernel-trace only)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-pmc}
mkdir -p gpurun_out/prof
rocprofv3 -L > gpurun_out/prof/counters_list.txt 2>&1 || true
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp -d gpurun_out/prof/${TAG}_$i -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof/${TAG}_$i.log 2>&1 || echo "group $i ($grp) failed: $(tail -2 gpurun_out/prof/${TAG}_$i.log)"
done < "${PMC_FILE:-tools/pmc_groups.txt}"
python3 - <<PY
import csv, collections, glob, os
for d in sorted(glob.glob("gpurun_out/prof/${TAG}_*/")):
    f = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(f): continue
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "gi_dense" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        print(f"{k:32s} {sum(v)/len(v):.4g}")
PY
