#!/bin/bash
# A/B session: VALU probe, parity tests on each candidate library, interleaved
# kernel timing (tools/ab.py).  usage: VARIANTS="v0 v1" TESTV="v1" bash tools/gpu_ab.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
timeout -k 10 60 ./tools/probe/valu_probe > gpurun_out/ab/probe.txt 2>&1 && tail -1 gpurun_out/ab/probe.txt
for v in ${TESTV:-}; do
  QPB_LIB=embedded-qp-solver_amd/lib/libqpb_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_active_set.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/pytest_$v.log 2>&1; rc=$?
  echo "pytest $v rc=$rc"; tail -2 gpurun_out/ab/pytest_$v.log; [ $rc -gt 1 ] && exit $rc
done
timeout -k 10 300 python tools/ab.py $VARIANTS > gpurun_out/ab/ab65k.json 2>gpurun_out/ab/ab.err || { tail gpurun_out/ab/ab.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/ab/ab65k.json'));print('B65536', {k:(v['median_us'],v['same_as_first']) for k,v in d['variants'].items()})"
B=262144 ROUNDS=4 REPS=5 timeout -k 10 300 python tools/ab.py $VARIANTS > gpurun_out/ab/ab262k.json 2>>gpurun_out/ab/ab.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/ab/ab262k.json'));print('B262144', {k:(v['median_us'],v['same_as_first']) for k,v in d['variants'].items()})"
