#!/bin/bash
# round 5: bank-disjoint LDS slot pairs (400-double stride) in gi_dense and
# gi_box: the GPU suite, interleaved A/B against v11.5 / gi_box v2.2, and the
# LDS counters of both n <= 16 builds.  Each GPU step time-limited; the first
# failure ends it.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/r5s; mkdir -p $O
echo "== tests" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for c in "1048576 box" "1048576 dense" "131072 box" "65536 box"; do
  set -- $c
  B=$1 FAM=$2 ROUNDS=5 REPS=5 timeout -k 10 300 python tools/ab.py head v115 > $O/ab_$1_$2.json || exit 1
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['B'], d['family'], {k:(v['median_us'],v['same_as_first']) for k,v in d['variants'].items()})" $O/ab_$1_$2.json
done
BOXAPI=1 B=1048576 ROUNDS=5 REPS=5 timeout -k 10 300 python tools/ab.py head box22 > $O/ab_boxapi.json || exit 1
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('boxapi', {k:(v['median_us'],v['same_as_first']) for k,v in d['variants'].items()})" $O/ab_boxapi.json
echo "== lds pmc" && LIBS="head v115" PMC_FILE=tools/pmc_lds.txt TAG=pmc_lds_r05s timeout -k 10 400 bash tools/gpu_pmc_libs.sh > $O/pmc_lds.log 2>&1; rc=$?; tail -30 $O/pmc_lds.log; [ $rc -ne 0 ] && exit $rc
exit 0
