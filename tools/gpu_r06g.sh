#!/bin/bash
# round 6: the reference replicas' huge layout (128 < n <= 1024) bitwise
# against the compiled reference, the reference-mode suite around it, and the
# compat layer on the GPU.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/${OUT:-r6g}; mkdir -p $O
echo "== tests" && timeout -k 10 900 python -u -m pytest tests/test_gpu_reference_modes.py tests/test_gpu_compat.py -x -v --timeout 600 --timeout-method thread > $O/pytest_ref.log 2>&1; rc=$?; tail -3 $O/pytest_ref.log; [ $rc -ne 0 ] && exit $rc
exit 0
