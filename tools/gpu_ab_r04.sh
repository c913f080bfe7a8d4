#!/bin/bash
# round-4 A/B session: parity of the head library on the n<=16 tests, then
# interleaved kernel timing of head against named variants (tools/build_variant.sh)
# at the metric's 1M batch, box and dense families.   usage: VARS="orig nomfma" tools/gpu_ab_r04.sh
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out/ab4 || exit 1
TESTS=${TESTS-tests/test_gpu_active_set.py tests/test_gpu_metric_batch.py}
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > gpurun_out/ab4/pytest_head.log 2>&1 || { tail -30 gpurun_out/ab4/pytest_head.log; exit 1; }
  echo "pytest head: $(tail -1 gpurun_out/ab4/pytest_head.log)"
fi
summ() { python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], json.dumps({k:(v['median_us'],v['same_as_first'],round(v['iters_mean'],3)) for k,v in d['variants'].items()}))" "$1" "$2"; }
ROUNDS=${ROUNDS:-8} timeout -k 10 300 python tools/ab.py head $VARS > gpurun_out/ab4/ab1m_box.json || exit 1; summ gpurun_out/ab4/ab1m_box.json dense-kernel-1M-box
ROUNDS=${ROUNDS:-6} FAM=dense timeout -k 10 300 python tools/ab.py head $VARS > gpurun_out/ab4/ab1m_dense.json || exit 1; summ gpurun_out/ab4/ab1m_dense.json dense-kernel-1M-dense
