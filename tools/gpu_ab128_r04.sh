#!/bin/bash
# n = 128 (configs[3]) A/B: parity of each variant on the n <= 128 tests, then
# interleaved kernel timing against head, box and dense families.
#   usage: VARS="gspec" tools/gpu_ab128_r04.sh
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out/ab128 || exit 1
O=gpurun_out/ab128
for v in $VARS; do
  QPB_LIB=embedded-qp-solver_amd/lib/libqpb_$v.so timeout -k 10 500 python -u -m pytest tests/test_gpu_block_kernel.py -x -q --timeout 400 --timeout-method thread > $O/pytest_$v.log 2>&1; rc=$?
  echo "pytest $v: $(tail -1 $O/pytest_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
summ() { python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], json.dumps({k:(v.get('median_us'),v.get('same_as_first')) for k,v in d['variants'].items()}))" "$1" "$2"; }
N=128 M=256 B=16384 FAM=box ROUNDS=${ROUNDS:-4} REPS=2 timeout -k 10 400 python tools/ab_n32.py head $VARS > $O/ab_box.json || exit 1; summ $O/ab_box.json box
N=128 M=256 B=16384 FAM=dense ROUNDS=${ROUNDS:-3} REPS=2 timeout -k 10 400 python tools/ab_n32.py head $VARS > $O/ab_dense.json || exit 1; summ $O/ab_dense.json dense
