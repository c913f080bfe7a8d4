#!/bin/bash
# round 5: the rotated-basis n <= 128 kernel (gi_gram v5, lib/libqpb.so) --
# parity tests, interleaved A/B against round 4's v4.5 (lib/libqpb_v45.so),
# box and dense at configs[3] (n = 128, m = 256, B = 16 384), section stamps
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/r5c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_block_kernel.py tests/test_gpu_size_sweep.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -4 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
N=128 M=256 B=16384 FAM=box ROUNDS=3 REPS=2 timeout -k 10 300 python tools/ab_n32.py head v45 > $O/ab_box.json || exit 1; cat $O/ab_box.json
N=128 M=256 B=16384 FAM=dense ROUNDS=3 REPS=2 timeout -k 10 300 python tools/ab_n32.py head v45 > $O/ab_dense.json || exit 1; cat $O/ab_dense.json
timeout -k 10 200 python tools/gram_time.py > $O/gram_time.txt 2>&1; cat $O/gram_time.txt
exit 0
