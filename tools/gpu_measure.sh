#!/bin/bash
# Round measurement session: bench line (with CPU baseline), rocprofv3 kernel
# trace + stats of the same command, FETCH_SIZE / WRITE_SIZE in separate PMC
# passes; summaries land in gpurun_out/measure_$TAG and are copied to profiles/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r02}
OUT=gpurun_out/measure_$TAG
mkdir -p $OUT
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed $?"; tail -5 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -5 $OUT/trace.log; exit 1; }
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c -d $OUT/pmc_$c -o run --output-format csv -- python3 bench.py --no-cpu-baseline --ref-batch 0 --steps 5 --warmup 1 > $OUT/pmc_$c.log 2>&1 || { echo "pmc $c failed"; tail -5 $OUT/pmc_$c.log; exit 1; }
done
python3 tools/summarize_profile.py $OUT > $OUT/summary.json && cat $OUT/summary.json
