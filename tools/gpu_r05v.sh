#!/bin/bash
# round 5: wave timelines of the final n <= 16 build (v11.5, QPB_WAVE_TRACE):
# the metric's batch (box, dense) and the N = 8 shard size.  Each GPU step
# time-limited; the first failure ends it.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/r5v; mkdir -p $O
export QPB_LIB=$PWD/embedded-qp-solver_amd/lib/libqpb_wtrace.so
for a in "1048576 box" "1048576 dense" "131072 box" "65536 box"; do
  timeout -k 10 300 python -u tools/wave_timeline.py $a > $O/log_${a// /_}.txt 2>&1 || exit 1
  python3 -c "
import json,sys
d=json.load(open('gpurun_out/wtrace/wave_timeline_'+sys.argv[2]+'_'+sys.argv[1]+'.json'))
print(sys.argv[1], sys.argv[2], 'span', d['span_us'], 'fill', round(d['slot_fill'],3), 'cu_max', d['cu_max_resident_waves'], 'gap', round(d['slot_handover_gap_us']['mean'],2), 'clock', round(d['shader_clock_GHz']['p50'],3), 'xcd spread', round(max(d['last_end_us_by_xcd'])-min(d['last_end_us_by_xcd']),1))
" $a
done
exit 0
