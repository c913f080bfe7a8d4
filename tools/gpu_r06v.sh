#!/bin/bash
# round 6: the n <= 32 wave kernel's output solves with captured components
# (no lane masks, no SGPR spills; lib/libqpb_wcap.so) against the shipped
# kernel: parity on the variant, then interleaved timing at configs[4]'s
# shape (dense and box families) and through qpb_solve_box.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/${OUT:-r6v}; mkdir -p $O
V=${V:-wcap}
QPB_LIB=embedded-qp-solver_amd/lib/libqpb_$V.so timeout -k 10 400 python -u -m pytest tests/test_gpu_wave_kernel.py tests/test_gpu_box.py tests/test_gpu_active_set.py -x -q --timeout 250 --timeout-method thread > $O/pytest_$V.log 2>&1; rc=$?
tail -2 $O/pytest_$V.log; [ $rc -ne 0 ] && exit $rc
for fam in dense box; do
  echo "== ab $fam" && FAM=$fam ROUNDS=5 REPS=4 timeout -k 10 400 python tools/ab_n32.py ${ORDER:-head $V} > $O/ab_$fam.json 2> $O/ab_$fam.err || { tail -5 $O/ab_$fam.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_$fam.json'));[print(k, v['median_us'], v.get('iters_mean'), v.get('x_maxdiff_vs_first'), v.get('ok_frac')) for k,v in d['variants'].items()]"
done
exit 0
