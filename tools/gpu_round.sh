#!/bin/bash
# One GPU session: parity tests, then a short bench.  Each GPU step has its own
# time limit; a crash/timeout (anything but pytest's 0/1) stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 420 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -25 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after GPU step failure"; exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 3 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
rc=$?
echo "bench rc=$rc"; tail -5 gpurun_out/bench.log
exit $rc
