#!/bin/bash
# round 5: gi_wave at 12 waves per CU (R stride 33, exchange row in R's
# column 0: 12,688 B per wave): the GPU suite, then interleaved A/B against
# the round-4 layout (oldwave) at configs[4]'s shape.  Each GPU step
# time-limited; the first failure ends it.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/r5k; mkdir -p $O
echo "== tests" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for fam in dense box; do
  FAM=$fam ROUNDS=4 REPS=4 timeout -k 10 300 python tools/ab_n32.py head oldwave > $O/ab_n32_$fam.json || exit 1
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('$fam', {k:(v['median_us'],v.get('same_as_first')) for k,v in d['variants'].items()})" $O/ab_n32_$fam.json
done
exit 0
