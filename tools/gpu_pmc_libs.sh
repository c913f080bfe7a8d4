#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --kernel-trace only) of
# tools/solve_once.py on each listed library, summarised per library and
# counter for the n <= 16 kernel.
# usage: LIBS="head v8" [N=16 M=32 B=1048576 FAM=box] [PMC_FILE=tools/pmc_r02.txt] bash tools/gpu_pmc_libs.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
export N=${N:-16} M=${M:-32} B=${B:-1048576} FAM=${FAM:-box} REPS=${REPS:-2}
OUT=gpurun_out/${TAG:-pmc_libs}
mkdir -p $OUT
KPAT=${KPAT:-gi_dense}
for v in $LIBS; do
  lib=embedded-qp-solver_amd/lib/libqpb_$v.so; [ "$v" = head ] && lib=embedded-qp-solver_amd/lib/libqpb.so
  i=0
  while read -r grp; do
    [ -z "$grp" ] && continue
    i=$((i+1))
    QPB_LIB=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $OUT/$v/g$i -o run --output-format csv -- python3 tools/solve_once.py > $OUT/$v.g$i.log 2>&1 || { echo "$v group $i failed rc=$?"; tail -3 $OUT/$v.g$i.log; exit 1; }
  done < "${PMC_FILE:-tools/pmc_r02.txt}"
done
python3 - "$OUT" "$KPAT" $LIBS <<'PY'
import csv, collections, glob, os, sys, json
out = {}
for v in sys.argv[3:]:
    agg = collections.defaultdict(list)
    for f in glob.glob(os.path.join(sys.argv[1], v, "g*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if sys.argv[2] in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    out[v] = {k: sum(x) / len(x) for k, x in agg.items()}
    w = out[v].get("SQ_WAVES")
    if w:
        out[v]["per_wave"] = {k: round(x / w, 1) for k, x in out[v].items() if k.startswith("SQ_") and k != "SQ_WAVES"}
print(json.dumps(out, indent=1))
json.dump(out, open(os.path.join(sys.argv[1], "pmc_summary.json"), "w"), indent=1)
PY
