#!/bin/bash
# round 5: -mllvm -disable-machine-licm on the n <= 16 kernel (confirmation,
# more rounds), the box kernel and the n <= 32 wave kernel.  Each GPU step
# time-limited; the first failure ends it.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/r5p; mkdir -p $O
for c in "131072 box" "65536 box" "1048576 box" "1048576 dense" "262144 box"; do
  set -- $c
  B=$1 FAM=$2 ROUNDS=6 REPS=5 timeout -k 10 300 python tools/ab.py head nolicm > $O/ab_$1_$2.json || exit 1
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(d['B'], d['family'], {k:(v['median_us'],v['same_as_first']) for k,v in d['variants'].items()})" $O/ab_$1_$2.json
done
BOXAPI=1 B=1048576 ROUNDS=6 REPS=5 timeout -k 10 300 python tools/ab.py head boxnolicm > $O/ab_boxapi.json || exit 1
python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('boxapi', {k:(v['median_us'],v['same_as_first']) for k,v in d['variants'].items()})" $O/ab_boxapi.json
for fam in dense box; do
  FAM=$fam ROUNDS=5 REPS=4 timeout -k 10 300 python tools/ab_n32.py head wavenolicm > $O/ab_n32_$fam.json || exit 1
  python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print('n32 $fam', {k:v['median_us'] for k,v in d['variants'].items()})" $O/ab_n32_$fam.json
done
exit 0
