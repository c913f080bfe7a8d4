#!/bin/bash
# round 5: persistent launch v2 (ticket taken in the output phase, static
# first group, per-XCD queues with a load-scan steal; no spills): parity of
# the variant (p4) on the active-set + metric-batch tests, then interleaved
# A/B against the one-wave-per-group launch (head).  Each GPU step
# time-limited; the first failure ends it.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/${OUT:-r5t}; mkdir -p $O
echo "== tests (p4)" && QPB_LIB=$PWD/embedded-qp-solver_amd/lib/libqpb_p4.so timeout -k 10 600 python -u -m pytest tests/test_gpu_active_set.py tests/test_gpu_metric_batch.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_p4.log 2>&1; rc=$?; tail -2 $O/pytest_p4.log; [ $rc -ne 0 ] && exit $rc
for c in "1048576 box" "1048576 dense" "131072 box" "65536 box" "8192 box"; do
  set -- $c
  B=$1 FAM=$2 ROUNDS=5 REPS=5 timeout -k 10 300 python tools/ab.py head p4 > $O/ab_$1_$2.json || exit 1
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['B'], d['family'], {k:(v['median_us'],v['same_as_first']) for k,v in d['variants'].items()})" $O/ab_$1_$2.json
done
exit 0
