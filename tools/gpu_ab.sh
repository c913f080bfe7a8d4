#!/bin/bash
# A/B session: parity tests on each candidate library, then interleaved
# kernel timing (tools/ab.py) at the metric's batch and at 65,536.
# usage: VARIANTS="head v1" TESTV="v1" bash tools/gpu_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
for v in ${TESTV:-}; do
  lib=embedded-qp-solver_amd/lib/libqpb_$v.so; [ "$v" = head ] && lib=embedded-qp-solver_amd/lib/libqpb.so
  QPB_LIB=$lib timeout -k 10 300 python -u -m pytest tests/test_gpu_active_set.py tests/test_gpu_metric_batch.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/pytest_$v.log 2>&1; rc=$?
  echo "pytest $v rc=$rc"; tail -2 gpurun_out/ab/pytest_$v.log; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python tools/ab.py $VARIANTS > gpurun_out/ab/ab1m.json 2>gpurun_out/ab/ab.err || { tail gpurun_out/ab/ab.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/ab/ab1m.json'));print('B1M', json.dumps({k:(v['median_us'],v['same_as_first'],v['iters_mean']) for k,v in d['variants'].items()}))"
B=65536 ROUNDS=5 REPS=10 timeout -k 10 300 python tools/ab.py $VARIANTS > gpurun_out/ab/ab65k.json 2>>gpurun_out/ab/ab.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/ab/ab65k.json'));print('B65536', json.dumps({k:(v['median_us'],v['same_as_first']) for k,v in d['variants'].items()}))"
