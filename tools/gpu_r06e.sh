#!/bin/bash
# round 6: gi_gram v4.5 setup variants, interleaved at configs[3] (box and
# dense): gl = built without machine LICM; g2h = the diagonal-tile sweep on two
# DPP rows per tile row; gy = y = L^{-1} f formed block by block inside the
# Cholesky on wave 4; g2hy = both, without machine LICM.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/${OUT:-r6e}; mkdir -p $O
for fam in box dense; do
  echo "== ab $fam" && N=128 M=256 B=16384 FAM=$fam ROUNDS=3 REPS=3 timeout -k 10 400 python tools/ab_n32.py head gl g2h gy g2hy > $O/ab_$fam.json 2> $O/ab_$fam.err || { tail -5 $O/ab_$fam.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_$fam.json'));[print(k, v['median_us'], v['iters_mean'], v['x_maxdiff_vs_first'], v['ok_frac']) for k,v in d['variants'].items()]"
done
exit 0
