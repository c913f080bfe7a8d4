#!/bin/bash
# reference-replica session: the bitwise tests against the compiled reference
# (every n, grid reuse, compat drop-in), then REF Newton / ADMM / GD timing at
# configs[3]'s n = 128, B = 16 384 against named variants (VARS).
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out/ref4 || exit 1
O=gpurun_out/ref4
timeout -k 10 900 python -u -m pytest tests/test_gpu_reference_modes.py tests/test_gpu_compat.py -x -q --timeout 600 --timeout-method thread > $O/pytest_ref.log 2>&1; rc=$?; tail -3 $O/pytest_ref.log; [ $rc -ne 0 ] && exit $rc
for mode in newton admm gd; do
  ITERS=$([ $mode = admm ] && echo 1000 || echo 10) ROUNDS=3 MODE=$mode timeout -k 10 600 python tools/ab_ref.py head $VARS > $O/ab_ref_$mode.json || exit 1
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], {k:(round(v['median_ms'],2),v['bitwise_as_first']) for k,v in d['variants'].items()})" $O/ab_ref_$mode.json $mode
done
