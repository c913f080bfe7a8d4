# n=128 (configs[3]) variant A/B: parity on the first candidate, then interleaved timing
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ab &&
QPB_LIB=embedded-qp-solver_amd/lib/libqpb_${TESTV}.so timeout -k 10 300 python -u -m pytest tests/test_gpu_block_kernel.py -x -q --timeout 250 --timeout-method thread > gpurun_out/ab/pytest_${TESTV}.log 2>&1; rc=$?; tail -1 gpurun_out/ab/pytest_${TESTV}.log; [ $rc -ne 0 ] && exit $rc
N=128 M=256 B=16384 FAM=box ROUNDS=${ROUNDS:-3} REPS=${REPS:-2} timeout -k 10 400 python tools/ab_n32.py $VARIANTS > gpurun_out/ab/ab128.json && python3 -c "import json;d=json.load(open('gpurun_out/ab/ab128.json'));print('n128', {k:v['median_us'] for k,v in d['variants'].items()})"
