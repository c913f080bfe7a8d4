#!/bin/bash
# PMC A/B of libqpb variants on one (n, m, B, family) batch: for each variant
# (head = lib/libqpb.so, NAME = lib/libqpb_NAME.so) and each counter group of
# $PMC_FILE, one rocprofv3 --kernel-trace --pmc pass over tools/solve_once.py;
# per-kernel means of every counter (over its dispatches) -> gpurun_out/pmcab/summary.json
# usage: VARS="head orig" N=16 M=32 B=1048576 FAM=box PMC_FILE=tools/pmc_ab.txt tools/gpu_pmc_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
OUT=${PMC_OUT:-gpurun_out/pmcab}
export PMC_OUT=$OUT
mkdir -p $OUT
export N=${N:-16} M=${M:-32} B=${B:-1048576} FAM=${FAM:-box} REPS=${REPS:-2}
for v in ${VARS:-head}; do
  lib=embedded-qp-solver_amd/lib/libqpb.so
  [ "$v" != head ] && lib=embedded-qp-solver_amd/lib/libqpb_$v.so
  i=0
  while read -r grp; do
    [ -z "$grp" ] && continue
    i=$((i+1))
    QPB_LIB=$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $OUT/${v}_$i -o run --output-format csv -- python3 tools/solve_once.py > $OUT/${v}_$i.log 2>&1 || { echo "pmc $v group $i failed: $(tail -3 $OUT/${v}_$i.log)"; exit 1; }
  done < "${PMC_FILE:-tools/pmc_ab.txt}"
done
python3 - <<'PY'
import csv, collections, glob, json, os, re
OUT = os.environ["PMC_OUT"]
out = {}
for d in sorted(glob.glob(OUT + "/*_*/")):
    v = re.match(r".*/(.+)_\d+/$", d).group(1)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            if "generate" in r["Kernel_Name"] or "philox" in r["Kernel_Name"].lower():
                continue
            agg[(r["Kernel_Name"].split("(")[0][-40:], r["Counter_Name"])].append(float(r["Counter_Value"]))
        for (k, c), vals in agg.items():
            out.setdefault(v, {}).setdefault(k, {})[c] = sum(vals) / len(vals)
json.dump(out, open(OUT + "/summary.json", "w"), indent=1)
for v, ks in out.items():
    for k, cs in ks.items():
        w = cs.get("SQ_WAVES", 1) or 1
        print(v, k, json.dumps({c: round(x / w, 1) if c.startswith("SQ_") and c != "SQ_WAVES" else x for c, x in sorted(cs.items())}))
PY
