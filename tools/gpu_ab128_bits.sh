# n=128 (configs[3]) variant A/B with a bitwise check: BASEV and TESTV solve
# the same 2048 QPs (tools/dump_solution.py), outputs compared bit for bit,
# then the parity tests on TESTV and interleaved timing of VARIANTS
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/ab || exit 1
for v in $BASEV $TESTV; do
  N=128 M=256 B=2048 FAM=box QPB_LIB=embedded-qp-solver_amd/lib/libqpb_$v.so OUT=gpurun_out/ab/sol128_$v.npz timeout -k 10 120 python tools/dump_solution.py || exit 1
done
python tools/bitwise_cmp.py gpurun_out/ab/sol128_$BASEV.npz gpurun_out/ab/sol128_$TESTV.npz; echo "bitwise rc=$?"
QPB_LIB=embedded-qp-solver_amd/lib/libqpb_${TESTV}.so timeout -k 10 300 python -u -m pytest tests/test_gpu_block_kernel.py -x -q --timeout 250 --timeout-method thread > gpurun_out/ab/pytest_${TESTV}.log 2>&1; rc=$?; tail -1 gpurun_out/ab/pytest_${TESTV}.log; [ $rc -ne 0 ] && exit $rc
N=128 M=256 B=16384 FAM=box ROUNDS=${ROUNDS:-3} REPS=${REPS:-2} timeout -k 10 400 python tools/ab_n32.py $VARIANTS > gpurun_out/ab/ab128.json && python3 -c "import json;d=json.load(open('gpurun_out/ab/ab128.json'));print('n128', {k:v['median_us'] for k,v in d['variants'].items()})"
