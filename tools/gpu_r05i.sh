#!/bin/bash
# round 5: wave timeline with the input-arrival stamp, ends taken before and
# after the output stores drain (wtrace / wtrace2).  Each GPU step
# time-limited; the first failure ends it.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/r5i; mkdir -p $O
for v in wtrace wtrace2; do
  QPB_LIB=$PWD/embedded-qp-solver_amd/lib/libqpb_$v.so timeout -k 10 300 python -u tools/wave_timeline.py 1048576 box > $O/$v.txt 2>&1 || exit 1
  echo "== $v"; grep -B2 -A40 '"input_wait_us"' $O/$v.txt | grep -v "^ *[0-9.]*,*$" | head -60
done
exit 0
