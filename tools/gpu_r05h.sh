#!/bin/bash
# round 5: 12 waves per CU (LDS slot 426 -> 410 doubles in gi_dense and
# gi_box): the GPU suite, interleaved A/B against the round-4 slot (old16,
# oldbox), and the wave timeline of the new build.  Each GPU step
# time-limited; the first failure ends it.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/${OUT:-r5h}; mkdir -p $O
echo "== tests" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for c in "1048576 box" "1048576 dense" "131072 box" "65536 box"; do
  set -- $c
  B=$1 FAM=$2 ROUNDS=4 REPS=5 timeout -k 10 300 python tools/ab.py head old16 > $O/ab_$1_$2.json || exit 1
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['B'], d['family'], {k:(v['median_us'],v['same_as_first']) for k,v in d['variants'].items()})" $O/ab_$1_$2.json
done
BOXAPI=1 B=1048576 ROUNDS=4 REPS=5 timeout -k 10 300 python tools/ab.py head oldbox > $O/ab_boxapi.json || exit 1
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('boxapi', d['B'], {k:(v['median_us'],v['same_as_first']) for k,v in d['variants'].items()})" $O/ab_boxapi.json
export QPB_LIB=$PWD/embedded-qp-solver_amd/lib/libqpb_wtrace.so
timeout -k 10 300 python -u tools/wave_timeline.py 1048576 box > $O/wtrace_1M.txt 2>&1 || exit 1
grep -A16 '"slot_fill"' $O/wtrace_1M.txt; grep -A3 cu_max $O/wtrace_1M.txt
exit 0
