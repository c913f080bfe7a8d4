#!/bin/bash
# PMC passes over the bench at the metric's batch (one counter group per
# rocprofv3 run, --kernel-trace only), summarised per kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-pmc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 5 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $OUT/g$i -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --ref-batch 0 ${BENCH_ARGS:-} > $OUT/g$i.log 2>&1 || { echo "group $i ($grp) failed rc=$?"; tail -3 $OUT/g$i.log; exit 1; }
done < "${PMC_FILE:-tools/pmc_r02.txt}"
python3 - "$OUT" <<'PY'
import csv, collections, glob, os, sys, json
out = {}
for d in sorted(glob.glob(os.path.join(sys.argv[1], "g*/"))):
    f = os.path.join(d, "run_counter_collection.csv")
    if not os.path.exists(f): continue
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "gi_dense" in r["Kernel_Name"] or "gi_wave" in r["Kernel_Name"] or "gi_block" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        out[k] = sum(v) / len(v)
print(json.dumps(out, indent=1))
json.dump(out, open(os.path.join(sys.argv[1], "pmc_summary.json"), "w"), indent=1)
PY
