#!/bin/bash
# round 5: the batch scan with back-to-back launch times (-> profiles/
# batch_scan.json) and the wave timeline's clock by start time at 131 072 and
# 1 M (a single launch after an idle gap).  Each GPU step time-limited; the
# first failure ends it.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/r5w; mkdir -p $O
timeout -k 10 400 python tools/batch_scan.py > $O/batch_scan.json 2> $O/batch_scan.err || { tail -5 $O/batch_scan.err; exit 1; }
grep -E '"B(65536|131072|262144|1048576)(_b2b)?_us"|T1M' $O/batch_scan.json
export QPB_LIB=$PWD/embedded-qp-solver_amd/lib/libqpb_wtrace.so
for a in "131072 box" "1048576 box"; do
  timeout -k 10 300 python -u tools/wave_timeline.py $a > $O/log_${a// /_}.txt 2>&1 || exit 1
  python3 -c "
import json,sys
d=json.load(open('gpurun_out/wtrace/wave_timeline_'+sys.argv[2]+'_'+sys.argv[1]+'.json'))
print(sys.argv[1], 'clock by start (100us bins)', d['shader_clock_GHz_by_start_100us'][:20])
" $a
done
exit 0
