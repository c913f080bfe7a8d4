#!/bin/bash
# round 6 measurement of the shipped tree: every GPU test, smoke, the bench
# line + rocprofv3 kernel trace + PMC passes (tools/gpu_measure.sh, TAG r06),
# the batch scan and the config sweep.  Each GPU step time-limited; the first
# failure ends it.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/${OUT:-r6m}; mkdir -p $O
echo "== tests" && timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -2 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
echo "== measure" && TAG=${MTAG:-r06} timeout -k 10 1200 bash tools/gpu_measure.sh > $O/measure.log 2>&1; rc=$?; grep -E '"value"|kernel_ms|avg_ns|hbm_bytes_per_launch|effective_clock' $O/measure.log | head -12; [ $rc -ne 0 ] && exit $rc
echo "== batch scan" && timeout -k 10 300 python tools/batch_scan.py > $O/batch_scan.json 2> $O/batch_scan.err || { tail -5 $O/batch_scan.err; exit 1; }
cat $O/batch_scan.json
echo "== configs" && timeout -k 10 900 python tools/config_sweep.py > $O/configs.json 2> $O/configs.err || { tail -5 $O/configs.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/configs.json'));[print(k, v.get('kernel_ms'), v.get('qps_per_s'), v.get('ok_frac')) for k,v in d.items() if isinstance(v, dict)]"
exit 0
