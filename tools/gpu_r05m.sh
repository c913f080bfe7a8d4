#!/bin/bash
# round-5 measurement on the shipped tree: every GPU test, smoke, the bench
# line + rocprofv3 stats + PMC passes (FETCH/WRITE, two SQ groups, the GRBM
# clock pass: tools/gpu_measure.sh), the n = 32 wave kernel's VALU classes and
# clock (the mixed-precision bound).  Each GPU step
# time-limited; the first failure ends it.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/${OUTDIR:-m5}; mkdir -p $O
echo "== tests" && timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 600 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
echo "== smoke" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -2 $O/smoke.log; [ $rc -ne 0 ] && exit $rc
echo "== measure" && TAG=r05 timeout -k 10 1200 bash tools/gpu_measure.sh > $O/measure.log 2>&1; rc=$?; tail -60 $O/measure.log; [ $rc -ne 0 ] && exit $rc
echo "== n32 pmc" && LIBS=head N=32 M=64 B=262144 FAM=dense KPAT=gi_wave_kernel PMC_FILE=tools/pmc_n32.txt TAG=pmc_n32_r05 timeout -k 10 400 bash tools/gpu_pmc_libs.sh > $O/pmc_n32.log 2>&1; rc=$?; tail -20 $O/pmc_n32.log; [ $rc -ne 0 ] && exit $rc
exit 0
