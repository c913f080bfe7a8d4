#!/bin/bash
# round 6: gi_gram v4.6 (D and y formed inside the blocked Cholesky) against
# v4.5 (lib/libqpb_g45.so): the n <= 128 parity tests, interleaved kernel
# times at configs[3] (box and dense families), and the section stamps.
# Each GPU step time-limited; the first failure ends it.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/${OUT:-r6b}; mkdir -p $O
echo "== tests" && timeout -k 10 600 python -u -m pytest tests/test_gpu_block_kernel.py tests/test_gpu_size_sweep.py -x -v --timeout 300 --timeout-method thread > $O/pytest_gram.log 2>&1; rc=$?; tail -3 $O/pytest_gram.log; [ $rc -ne 0 ] && exit $rc
echo "== ab box" && N=128 M=256 B=16384 FAM=box ROUNDS=3 REPS=3 timeout -k 10 300 python tools/ab_n32.py head g45 > $O/ab_box.json 2> $O/ab_box.err || { tail -5 $O/ab_box.err; exit 1; }
cat $O/ab_box.json
echo "== ab dense" && N=128 M=256 B=16384 FAM=dense ROUNDS=3 REPS=3 timeout -k 10 300 python tools/ab_n32.py head g45 > $O/ab_dense.json 2> $O/ab_dense.err || { tail -5 $O/ab_dense.err; exit 1; }
cat $O/ab_dense.json
echo "== stamps" && timeout -k 10 300 python tools/gram_time.py > $O/gram_time.txt 2>&1 || { tail -5 $O/gram_time.txt; exit 1; }
cat $O/gram_time.txt
exit 0
