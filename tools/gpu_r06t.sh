#!/bin/bash
# round 6: the n <= 16 kernel's dynamic tail (claim_tail_group; variants
# lib/libqpb_t{4,8,16}.so: 1/4, 1/8, 1/16 of the groups in the tail) against
# the shipped kernel.  Parity first (the tail tests and the metric batch on
# t8), then interleaved timing at the metric's batch (box, dense) and at
# 262 144 QPs, the tail's threshold.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/${OUT:-r6t}; mkdir -p $O
QPB_LIB=embedded-qp-solver_amd/lib/libqpb_t8.so timeout -k 10 400 python -u -m pytest tests/test_gpu_tail.py tests/test_gpu_metric_batch.py -x -v --timeout 200 --timeout-method thread > $O/pytest_t8.log 2>&1; rc=$?
tail -3 $O/pytest_t8.log; [ $rc -ne 0 ] && exit $rc
for cfg in "1048576 box" "1048576 dense" "262144 box"; do set -- $cfg
  echo "== ab B=$1 $2" && B=$1 FAM=$2 ROUNDS=6 REPS=6 timeout -k 10 400 python tools/ab.py ${VARIANTS:-head t8 t16 t4} > $O/ab_$1_$2.json 2> $O/ab_$1_$2.err || { tail -5 $O/ab_$1_$2.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_$1_$2.json'));[print(k, v['median_us'], v['min_us'], v['same_as_first']) for k,v in d['variants'].items()]"
done
exit 0
