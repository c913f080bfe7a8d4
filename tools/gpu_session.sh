#!/bin/bash
# One GPU session: GPU parity tests, then the round's measurement
# (tools/gpu_measure.sh: bench line with CPU baseline, rocprofv3 kernel trace
# + stats, FETCH_SIZE / WRITE_SIZE PMC passes).  Every GPU step has its own
# time limit; anything but pytest's 0/1 stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -5
  if [ $rc -ne 0 ]; then tail -40 gpurun_out/pytest_gpu.log; exit $rc; fi
fi
bash tools/gpu_measure.sh
