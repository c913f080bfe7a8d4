cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ab || exit 1
QPB_LIB=embedded-qp-solver_amd/lib/libqpb_mxnew.so timeout -k 10 300 python -u -m pytest tests/test_gpu_mixed.py -x -q --timeout 250 --timeout-method thread > gpurun_out/ab/pytest_mxnew.log 2>&1; rc=$?; tail -1 gpurun_out/ab/pytest_mxnew.log; [ $rc -ne 0 ] && exit $rc
ROUNDS=3 REPS=2 timeout -k 10 400 python tools/ab_n32.py mxbase@32 mxnew@32 mxnew > gpurun_out/ab/ab_mixed.json && python3 -c "import json;d=json.load(open('gpurun_out/ab/ab_mixed.json'));print('n32', {k:(v['median_us'],v['redo_frac']) for k,v in d['variants'].items()})"
