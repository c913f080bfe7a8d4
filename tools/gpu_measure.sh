#!/bin/bash
# Round measurement session: bench line (with CPU baseline), rocprofv3 kernel
# trace + stats of the same command, FETCH_SIZE / WRITE_SIZE and two SQ
# counter groups in separate PMC passes (--kernel-trace only); summaries land
# in gpurun_out/measure_$TAG (tools/summarize_profile.py writes summary.json
# and the pmc_traffic.json candidate that bench.py reads from profiles/).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r03}
OUT=gpurun_out/measure_$TAG
mkdir -p $OUT
timeout -k 10 400 python bench.py > $OUT/bench.json 2> $OUT/bench.err || { echo "bench failed $?"; tail -5 $OUT/bench.err; exit 1; }
cat $OUT/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline --dense-reps 0 --pipeline-streams 0 --sustain-seconds 0 > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -5 $OUT/trace.log; exit 1; }
i=0
for c in FETCH_SIZE WRITE_SIZE \
         "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU" \
         "SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT SQ_WAIT_INST_LDS" \
         "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1)); name=$(echo $c | cut -d' ' -f1); [ $i -gt 2 ] && name=sq$((i-2)); [ $i -eq 5 ] && name=clk
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c -d $OUT/pmc_$name -o run --output-format csv -- python3 bench.py --no-cpu-baseline --ref-batch 0 --box-reps 0 --dense-reps 0 --pipeline-streams 0 --sustain-seconds 0 --steps 5 --warmup 1 > $OUT/pmc_$name.log 2>&1 || { echo "pmc $name failed"; tail -5 $OUT/pmc_$name.log; exit 1; }
done
python3 tools/summarize_profile.py $OUT > $OUT/summary.json && cat $OUT/summary.json
