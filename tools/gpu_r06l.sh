#!/bin/bash
# round 6: LDS counters of the n <= 16 kernel (one PMC pass, kernel trace only)
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r6l}; mkdir -p $O
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_UNALIGNED_STALL -d $O/pmc_lds -o run --output-format csv -- python3 bench.py --no-cpu-baseline --ref-batch 0 --box-reps 0 --dense-reps 0 --pipeline-streams 0 --sustain-seconds 0 --settle-seconds 0 --steps 5 --warmup 1 > $O/pmc_lds.log 2>&1 || { echo "pmc failed"; tail -5 $O/pmc_lds.log; exit 1; }
python3 - $O <<'PY'
import csv, sys, collections
o = sys.argv[1]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f"{o}/pmc_lds/run_counter_collection.csv")):
    if "gi_dense_kernel" in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
w = sum(acc["SQ_WAVES"]) / len(acc["SQ_WAVES"])
print({k: round(sum(v) / len(v) / w, 2) for k, v in acc.items() if k != "SQ_WAVES"}, "per wave; waves", w)
PY
