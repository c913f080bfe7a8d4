#!/bin/bash
# round 6: the box entry point up to n = 128 (the BOX form of qpb_gi_gram.hip)
# and the wider oracle samples, then the gi_gram setup variants (tools/gpu_r06e.sh).
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/${OUT:-r6f}; mkdir -p $O
echo "== tests" && timeout -k 10 900 python -u -m pytest tests/test_gpu_box.py tests/test_gpu_mixed.py tests/test_gpu_active_set.py -x -v --timeout 600 --timeout-method thread > $O/pytest_box.log 2>&1; rc=$?; tail -3 $O/pytest_box.log; [ $rc -ne 0 ] && exit $rc
OUT=${OUT:-r6f} bash tools/gpu_r06e.sh
