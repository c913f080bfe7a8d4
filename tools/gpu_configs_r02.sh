#!/bin/bash
# Round-2 measurement of the non-headline configs: kernel times (HIP events,
# config_sweep.py), a rocprofv3 kernel trace of the n=128 run, and its MFMA /
# VALU PMC counters in separate passes (--kernel-trace only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/cfg
mkdir -p $OUT
timeout -k 10 300 python3 tools/config_sweep.py > $OUT/configs.json 2> $OUT/configs.err || { echo "sweep failed"; tail $OUT/configs.err; exit 1; }
cat $OUT/configs.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/config_sweep.py c3_n128_m256 > $OUT/trace.log 2>&1 || { echo "trace failed"; tail $OUT/trace.log; exit 1; }
i=0
for grp in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_MFMA_MOPS_F64 GRBM_GUI_ACTIVE" "SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d $OUT/pmc$i -o run --output-format csv -- python3 tools/config_sweep.py c3_n128_m256 > $OUT/pmc$i.log 2>&1 || { echo "pmc $i failed"; tail -3 $OUT/pmc$i.log; exit 1; }
done
python3 - $OUT <<'PY'
import csv, collections, glob, os, sys, json
out = {}
for d in sorted(glob.glob(os.path.join(sys.argv[1], "pmc*/"))):
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        agg = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            if "gi_gram" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, v in agg.items():
            out[k] = sum(v) / len(v)
print(json.dumps(out, indent=1))
json.dump(out, open(os.path.join(sys.argv[1], "pmc_gram.json"), "w"), indent=1)
PY
find $OUT/trace -name "*kernel_stats.csv" -exec cp {} $OUT/kernel_stats.csv \;
head -5 $OUT/kernel_stats.csv
