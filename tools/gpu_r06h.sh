#!/bin/bash
# round 6: gi_gram with the two triangular solves blocked by the diagonal
# tiles' inverses (-DGRAM_BLK, lib/libqpb_gblk.so) against the shipped kernel,
# interleaved at configs[3] (box and dense), and the reference-mode tests.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/${OUT:-r6h}; mkdir -p $O
for fam in box dense; do
  echo "== ab $fam" && N=128 M=256 B=16384 FAM=$fam ROUNDS=4 REPS=3 timeout -k 10 400 python tools/ab_n32.py head gblk > $O/ab_$fam.json 2> $O/ab_$fam.err || { tail -5 $O/ab_$fam.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_$fam.json'));[print(k, v['median_us'], v['iters_mean'], v['x_maxdiff_vs_first'], v['ok_frac']) for k,v in d['variants'].items()]"
done
for nm in 48:96 100:200; do n=${nm%%:*}; m=${nm##*:}
  echo "== ab n=$n" && N=$n M=$m B=8192 FAM=dense ROUNDS=3 REPS=3 timeout -k 10 300 python tools/ab_n32.py head gblk > $O/ab_n$n.json 2> $O/ab_n$n.err || { tail -5 $O/ab_n$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_n$n.json'));[print(k, v['median_us'], v['iters_mean'], v['x_maxdiff_vs_first'], v['ok_frac']) for k,v in d['variants'].items()]"
done
[ -n "$WITH_TESTS" ] && OUT=${OUT:-r6h} bash tools/gpu_r06g.sh
exit 0
