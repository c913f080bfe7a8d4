#!/bin/bash
# round 6: the n <= 16 kernel's x solves capturing each component at a
# distinct address per lane (lib/libqpb_xdiag.so; the shipped kernel stores
# it from all 16 lanes of a QP to one address): parity, interleaved timing,
# and the LDS bank-conflict counter of the variant
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
export TMPDIR=/tmp
O=gpurun_out/${OUT:-r6d2}; mkdir -p $O
V=${V:-xdiag}
QPB_LIB=embedded-qp-solver_amd/lib/libqpb_$V.so timeout -k 10 400 python -u -m pytest tests/test_gpu_active_set.py tests/test_gpu_metric_batch.py tests/test_gpu_size_sweep.py -x -q --timeout 200 --timeout-method thread > $O/pytest_$V.log 2>&1; rc=$?
tail -2 $O/pytest_$V.log; [ $rc -ne 0 ] && exit $rc
for cfg in "1048576 box" "1048576 dense" "65536 box"; do set -- $cfg
  echo "== ab B=$1 $2" && B=$1 FAM=$2 ROUNDS=6 REPS=6 timeout -k 10 400 python tools/ab.py ${ORDER:-head $V} > $O/ab_$1_$2.json 2> $O/ab_$1_$2.err || { tail -5 $O/ab_$1_$2.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_$1_$2.json'));[print(k, v['median_us'], v['min_us'], v['same_as_first']) for k,v in d['variants'].items()]"
done
QPB_LIB=embedded-qp-solver_amd/lib/libqpb_$V.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS -d $O/pmc_lds -o run --output-format csv -- python3 bench.py --no-cpu-baseline --ref-batch 0 --box-reps 0 --dense-reps 0 --pipeline-streams 0 --sustain-seconds 0 --settle-seconds 0 --steps 5 --warmup 1 > $O/pmc_lds.log 2>&1 || { echo "pmc failed"; tail -5 $O/pmc_lds.log; exit 1; }
python3 - $O <<'PY'
import csv, sys, collections
o = sys.argv[1]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f"{o}/pmc_lds/run_counter_collection.csv")):
    if "gi_dense_kernel" in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
w = sum(acc["SQ_WAVES"]) / len(acc["SQ_WAVES"])
print({k: round(sum(v) / len(v) / w, 2) for k, v in acc.items() if k != "SQ_WAVES"}, "per wave")
PY
exit 0
