#!/bin/bash
# round 5: wave timeline of the shipped n = 16 kernel (tools/wave_timeline.py,
# QPB_WAVE_TRACE build lib/libqpb_wtrace.so): slot fill, per-CU residency,
# hand-over gaps, tail, unprofiled shader clock.  Each GPU step time-limited;
# the first failure ends it.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/wtrace${TAG:-}; mkdir -p $O
export QPB_LIB=$PWD/embedded-qp-solver_amd/lib/libqpb_${LIBNAME:-wtrace}.so
for a in "1048576 box" "131072 box"; do
  echo "== $a"
  timeout -k 10 300 python -u tools/wave_timeline.py $a > $O/log_${a// /_}.txt 2>&1; rc=$?
  grep -v amdgpu.ids $O/log_${a// /_}.txt
  [ $rc -ne 0 ] && exit $rc
done
exit 0
