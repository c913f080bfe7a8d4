#!/bin/bash
# round 5, after the 12-waves-per-CU layouts (qpb 0.12): every GPU test,
# smoke, the measurement (bench line + rocprofv3 stats + PMC passes, TAG
# r05b), the batch scan (-> profiles/batch_scan.json), the config sweep and
# the n = 32 VALU-class PMC.  Each GPU step time-limited; the first failure
# ends it.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/${OUT:-r5l}; mkdir -p $O
echo "== tests" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -2 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
echo "== measure" && TAG=${MTAG:-r05b} timeout -k 10 1200 bash tools/gpu_measure.sh > $O/measure.log 2>&1; rc=$?; grep -E '"value"|kernel_ms|avg_ns|hbm_bytes_per_launch|effective_clock' $O/measure.log | head -12; [ $rc -ne 0 ] && exit $rc
echo "== batch scan" && timeout -k 10 300 python tools/batch_scan.py > $O/batch_scan.json 2> $O/batch_scan.err || { tail -5 $O/batch_scan.err; exit 1; }
cat $O/batch_scan.json
echo "== configs" && timeout -k 10 600 python tools/config_sweep.py c1_n16_m32 c4_n32_m64 c4_n32_m64_mixed c4_n32_box_dense_path c4_n32_box_fast_path c3_n128_m256 > $O/configs.json 2> $O/configs.err || { tail -5 $O/configs.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/configs.json'));[print(k, v.get('kernel_ms'), v.get('qps_per_s')) for k,v in d.items() if isinstance(v, dict)]"
echo "== n32 pmc" && LIBS=head N=32 M=64 B=262144 FAM=dense KPAT=gi_wave_kernel PMC_FILE=tools/pmc_n32.txt TAG=pmc_n32_${MTAG:-r05b} timeout -k 10 400 bash tools/gpu_pmc_libs.sh > $O/pmc_n32.log 2>&1; rc=$?; tail -12 $O/pmc_n32.log; [ $rc -ne 0 ] && exit $rc
exit 0
