# n=32 (configs[4] shape) variant A/B: parity tests on TESTV, then interleaved timing of VARIANTS
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ab || exit 1
for v in $TESTV; do
  QPB_LIB=embedded-qp-solver_amd/lib/libqpb_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_wave_kernel.py tests/test_gpu_mixed.py -x -q --timeout 250 --timeout-method thread > gpurun_out/ab/pytest_$v.log 2>&1; rc=$?
  echo "pytest $v rc=$rc"; tail -1 gpurun_out/ab/pytest_$v.log; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 400 python tools/ab_n32.py $VARIANTS > gpurun_out/ab/ab32.json && python3 -c "import json;d=json.load(open('gpurun_out/ab/ab32.json'));print('n32', {k:v['median_us'] for k,v in d['variants'].items()})"
