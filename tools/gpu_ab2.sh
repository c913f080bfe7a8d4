# n=16 and n=32 variant A/B in one call (parity tests on the candidates first)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ab &&
QPB_LIB=embedded-qp-solver_amd/lib/libqpb_wdrop.so timeout -k 10 300 python -u -m pytest tests/test_gpu_wave_kernel.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/pytest_wdrop.log 2>&1 && tail -1 gpurun_out/ab/pytest_wdrop.log &&
QPB_LIB=embedded-qp-solver_amd/lib/libqpb_ddi.so timeout -k 10 300 python -u -m pytest tests/test_gpu_active_set.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab/pytest_ddi.log 2>&1 && tail -1 gpurun_out/ab/pytest_ddi.log &&
timeout -k 10 300 python tools/ab.py head d2l ddi > gpurun_out/ab/ab16.json && python3 -c "import json;d=json.load(open('gpurun_out/ab/ab16.json'));print('n16', {k:(v['median_us'],v['same_as_first']) for k,v in d['variants'].items()})" &&
timeout -k 10 300 python tools/ab_n32.py whead wdrop > gpurun_out/ab/ab32.json && python3 -c "import json;d=json.load(open('gpurun_out/ab/ab32.json'));print('n32', {k:v['median_us'] for k,v in d['variants'].items()})"
