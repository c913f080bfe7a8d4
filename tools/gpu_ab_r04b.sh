#!/bin/bash
# round-4 A/B session over the three active-set kernels: parity of the head
# library on the n<=16 / box / n<=32 tests, then interleaved kernel timing of
# head against named variants (lib/libqpb_<name>.so): n=16 dense kernel at 1M
# (box and dense families), the box kernel at 1M, the n=32 kernel at 262,144.
#   usage: VARS="base" tools/gpu_ab_r04b.sh
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out/ab4b || exit 1
O=gpurun_out/ab4b
TESTS=${TESTS-tests/test_gpu_active_set.py tests/test_gpu_metric_batch.py tests/test_gpu_box.py tests/test_gpu_wave_kernel.py}
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > $O/pytest_head.log 2>&1 || { tail -30 $O/pytest_head.log; exit 1; }
  echo "pytest head: $(tail -1 $O/pytest_head.log)"
fi
summ() { python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], json.dumps({k:(v.get('median_us'),v.get('same_as_first'),round(v.get('iters_mean',0),3)) for k,v in d['variants'].items()}))" "$1" "$2"; }
ROUNDS=${ROUNDS:-8} timeout -k 10 300 python tools/ab.py head $VARS > $O/ab1m_box.json || exit 1; summ $O/ab1m_box.json n16-1M-box
ROUNDS=${ROUNDS:-6} FAM=dense timeout -k 10 300 python tools/ab.py head $VARS > $O/ab1m_dense.json || exit 1; summ $O/ab1m_dense.json n16-1M-dense
[ -n "$NOBOX" ] || { timeout -k 10 300 python tools/ab_box_variants.py head $VARS > $O/ab_boxkernel.json || exit 1; cat $O/ab_boxkernel.json | head -c 600; echo; }
[ -n "$NO32" ] || { timeout -k 10 300 python tools/ab_n32.py head $VARS > $O/ab_n32.json || exit 1; summ $O/ab_n32.json n32-262k-dense; }
