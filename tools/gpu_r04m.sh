#!/bin/bash
# round-4 measurement on the shipped tree: every GPU test, the bench line +
# rocprofv3 stats + PMC passes (tools/gpu_measure.sh), the config sweep.
# Each GPU step time-limited; the first failure ends it.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/${OUTDIR:-m4}; mkdir -p $O
echo "== tests" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -2 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
echo "== measure" && TAG=r04 timeout -k 10 1200 bash tools/gpu_measure.sh > $O/measure.log 2>&1; rc=$?; tail -40 $O/measure.log; [ $rc -ne 0 ] && exit $rc
echo "== sweep" && timeout -k 10 600 python tools/config_sweep.py > $O/configs.json 2> $O/configs.err && cat $O/configs.json
