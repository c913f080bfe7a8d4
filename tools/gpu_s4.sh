#!/bin/bash
# round-4 diagnostics session (one box): fp64 4x4x4 MFMA pipe sharing, the
# n=16 MFMA-setup variant against head (sections, max_iter splits, PMC), the
# n=128 rcp-pivot variant (parity + interleaved timing), the config sweep
# (the REF n=128 row with the restructured replicas).  Each GPU step is
# time-limited; the first failure ends the script.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/s4; mkdir -p $O
step() { echo "== $1"; }
step probe && timeout -k 10 60 ./tools/probe/mfma44_probe > $O/mfma44.txt 2>&1 && grep -v "^lane" $O/mfma44.txt || exit 1
step exp && QPB_LIB=embedded-qp-solver_amd/lib/libqpb_mfma.so timeout -k 10 200 python tools/exp_n16.py > $O/exp_mfma.json && timeout -k 10 200 python tools/exp_n16.py > $O/exp_head.json || exit 1
python3 - <<'PY'
import json
for v in ("head", "mfma"):
    d = json.load(open(f"gpurun_out/s4/exp_{v}.json"))
    print(v, {k: d[k] for k in d if k.startswith("kernel_ms")}, d["sections_us_per_wave"])
PY
step pmc && VARS="head mfma" PMC_OUT=$O/pmc16 tools/gpu_pmc_ab.sh || exit 1
step n128 && QPB_LIB=embedded-qp-solver_amd/lib/libqpb_gramboth.so timeout -k 10 300 python -u -m pytest tests/test_gpu_block_kernel.py -x -q --timeout 250 --timeout-method thread > $O/pytest_gramboth.log 2>&1; rc=$?; tail -1 $O/pytest_gramboth.log; [ $rc -ne 0 ] && exit $rc
N=128 M=256 B=16384 FAM=box ROUNDS=3 REPS=2 timeout -k 10 400 python tools/ab_n32.py head gramrcp grampipe gramboth > $O/ab128.json && python3 -c "import json;d=json.load(open('gpurun_out/s4/ab128.json'));print('n128', {k:v['median_us'] for k,v in d['variants'].items()})" || exit 1
step sweep && timeout -k 10 500 python tools/config_sweep.py c3_ref_newton > $O/configs_ref.json 2> $O/configs_ref.err && cat $O/configs_ref.json || { tail -5 $O/configs_ref.err; exit 1; }
step pmc128 && VARS="head" N=128 M=256 B=16384 FAM=box REPS=1 PMC_FILE=tools/pmc_gram4.txt PMC_OUT=$O/pmc128 tools/gpu_pmc_ab.sh || exit 1
step tests && timeout -k 10 600 python -u -m pytest tests/test_gpu_wave_kernel.py tests/test_gpu_dist.py tests/test_gpu_integration.py -x -q --timeout 400 --timeout-method thread > $O/pytest_s4.log 2>&1; rc=$?; tail -3 $O/pytest_s4.log; exit $rc
