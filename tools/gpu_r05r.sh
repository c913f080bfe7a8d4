#!/bin/bash
# round 5: the column-scaled R (back substitution without a product per
# step): the GPU suite, then interleaved A/B against v11.5.  Each GPU step
# time-limited; the first failure ends it.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/r5r; mkdir -p $O
echo "== tests" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for c in "1048576 box" "1048576 dense" "131072 box" "65536 box"; do
  set -- $c
  B=$1 FAM=$2 ROUNDS=5 REPS=5 timeout -k 10 300 python tools/ab.py head v115 > $O/ab_$1_$2.json || exit 1
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['B'], d['family'], {k:(v['median_us'],v['same_as_first'],round(v['iters_mean'],4)) for k,v in d['variants'].items()})" $O/ab_$1_$2.json
done
exit 0
