#!/bin/bash
# round 6: the n <= 16 kernel built with other LLVM machine-scheduler
# strategies (lib/libqpb_{ilp,itilp,memcl}.so: max-ilp, iterative-ilp,
# max-memory-clause; same source, same instruction counts) against the
# shipped build, interleaved; parity on the first variant.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/${OUT:-r6s}; mkdir -p $O
V=${VARIANTS:-head ilp itilp memcl}
for cfg in "1048576 box" "1048576 dense" "65536 box"; do set -- $cfg
  echo "== ab B=$1 $2" && B=$1 FAM=$2 ROUNDS=6 REPS=6 timeout -k 10 400 python tools/ab.py $V > $O/ab_$1_$2.json 2> $O/ab_$1_$2.err || { tail -5 $O/ab_$1_$2.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/ab_$1_$2.json'));[print(k, v['median_us'], v['min_us'], v['same_as_first']) for k,v in d['variants'].items()]"
done
exit 0
