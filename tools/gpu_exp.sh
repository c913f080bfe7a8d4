#!/bin/bash
# Quick kernel experiment: GPU parity tests of the n<=16 kernel, the ablation
# sweep and the batch scan.  Each GPU step has its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof
TAG=${TAG:-exp}
timeout -k 10 300 python -u -m pytest tests/test_gpu_active_set.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_$TAG.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/batch_scan.py > gpurun_out/prof/scan_$TAG.json 2> gpurun_out/prof/scan_$TAG.err || { echo "scan failed"; tail -3 gpurun_out/prof/scan_$TAG.err; exit 1; }
cat gpurun_out/prof/scan_$TAG.json
timeout -k 10 300 python tools/prof_sweep.py > gpurun_out/prof/sweep_$TAG.json 2> gpurun_out/prof/sweep_$TAG.err || { echo "sweep failed"; exit 1; }
grep -E "iters_mean|maxit|wave_trips|m0" gpurun_out/prof/sweep_$TAG.json
