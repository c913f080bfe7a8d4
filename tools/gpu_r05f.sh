#!/bin/bash
# round 5: gi_gram with y = L^{-1} f computed inside the factorisation
# (head) against y after it (lib/libqpb_gy0.so): n <= 128 parity, then
# interleaved kernel times at configs[3], box and dense
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/r5f; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_block_kernel.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
N=128 M=256 B=16384 FAM=box ROUNDS=3 REPS=2 timeout -k 10 300 python tools/ab_n32.py head gy0 > $O/ab_box.json || exit 1
N=128 M=256 B=16384 FAM=dense ROUNDS=3 REPS=2 timeout -k 10 300 python tools/ab_n32.py head gy0 > $O/ab_dense.json || exit 1
python3 -c "
import json
for f in ('box','dense'):
    d=json.load(open('$O/ab_'+f+'.json')); print(f, {k:(v['median_us'],v['iters_mean'],v['x_maxdiff_vs_first']) for k,v in d['variants'].items()})"
exit 0
