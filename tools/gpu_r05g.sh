#!/bin/bash
# round 5: wave timeline of the shipped n = 16 kernel (tools/wave_timeline.py,
# QPB_WAVE_TRACE build lib/libqpb_wtrace.so): slot fill, hand-over gaps, tail,
# unprofiled shader clock.  Each GPU step time-limited; the first failure ends it.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/wtrace; mkdir -p $O
export QPB_LIB=$PWD/embedded-qp-solver_amd/lib/libqpb_wtrace.so
for a in "1048576 box" "1048576 dense" "131072 box" "65536 box"; do
  echo "== $a"
  timeout -k 10 300 python -u tools/wave_timeline.py $a > $O/log_${a// /_}.txt 2>&1; rc=$?
  cat $O/log_${a// /_}.txt | grep -v amdgpu.ids
  [ $rc -ne 0 ] && exit $rc
done
exit 0
