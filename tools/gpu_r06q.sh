#!/bin/bash
# round 6: the n <= 128 kernel with its triangular solves capturing the
# broadcast components and the A loads' addresses clamped (SGPR spills
# 685 -> 54; lib/libqpb_gcap.so) against the shipped kernel: parity on the
# variant, then interleaved timing at configs[3] (box and dense families).
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/${OUT:-r6q}; mkdir -p $O
V=${V:-gcap}; VS=${VS:-$V}
QPB_LIB=embedded-qp-solver_amd/lib/libqpb_$V.so timeout -k 10 500 python -u -m pytest tests/test_gpu_block_kernel.py tests/test_gpu_box.py tests/test_gpu_size_sweep.py -x -q --timeout 300 --timeout-method thread > $O/pytest_$V.log 2>&1; rc=$?
tail -2 $O/pytest_$V.log; [ $rc -ne 0 ] && exit $rc
for fam in box dense; do
  echo "== ab $fam" && N=128 M=256 B=16384 FAM=$fam ROUNDS=4 REPS=3 timeout -k 10 400 python tools/ab_n32.py ${ORDER:-head $VS} > $O/ab_$fam.json 2> $O/ab_$fam.err || { tail -5 $O/ab_$fam.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_$fam.json'));[print(k, v['median_us'], v['iters_mean'], v['x_maxdiff_vs_first'], v['ok_frac']) for k,v in d['variants'].items()]"
done
exit 0
