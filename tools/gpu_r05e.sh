#!/bin/bash
# round 5: the launch tail -- waves past trip T raise
# their issue priority (QPB_TAIL_PRIO = 6, 9, 12) against head: interleaved
# kernel times at the per-GPU shard sizes of N = 8 / 2 / 1 and configs[1]
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/r5e; mkdir -p $O
for B in 65536 131072 1048576; do
  B=$B ROUNDS=4 REPS=5 timeout -k 10 300 python tools/ab.py head prio6 prio9 prio12 > $O/ab_prio_$B.json || exit 1
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['B'], {k:(v['median_us'],v['same_as_first']) for k,v in d['variants'].items()})" $O/ab_prio_$B.json
done
exit 0
