#!/bin/bash
# Profiling session: ablation sweep, rocprofv3 kernel trace/stats of the bench,
# and PMC passes (counters in their own runs, --kernel-trace only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
TAG=${TAG:-r01}
timeout -k 10 300 python tools/prof_sweep.py > gpurun_out/prof/sweep_$TAG.json 2> gpurun_out/prof/sweep_$TAG.err || { echo "sweep failed $?"; tail gpurun_out/prof/sweep_$TAG.err; exit 1; }
cat gpurun_out/prof/sweep_$TAG.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/trace_$TAG -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof/trace_$TAG.log 2>&1 || { echo "trace failed $?"; tail gpurun_out/prof/trace_$TAG.log; exit 1; }
tail -2 gpurun_out/prof/trace_$TAG.log
for pmc in "${PMCS[@]:-}"; do :; done
i=0
for pmc in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "FETCH_SIZE" "WRITE_SIZE" "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_ANY SQ_INSTS_VALU_FMA_F64 SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $pmc -d gpurun_out/prof/pmc${i}_$TAG -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/prof/pmc${i}_$TAG.log 2>&1 || { echo "pmc $i failed $?"; tail -5 gpurun_out/prof/pmc${i}_$TAG.log; }
done
ls -R gpurun_out/prof | head -50
