cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
timeout -k 10 300 python -u -m pytest tests/test_gpu_active_set.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/ab/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/ab.py v0 v1 v0i v3 v4 > gpurun_out/ab/ab65k.json 2>gpurun_out/ab/ab.err || { tail gpurun_out/ab/ab.err; exit 1; }
cat gpurun_out/ab/ab65k.json
B=262144 ROUNDS=4 REPS=5 timeout -k 10 300 python tools/ab.py v0 v1 v0i v3 v4 > gpurun_out/ab/ab262k.json 2>>gpurun_out/ab/ab.err || exit 1
cat gpurun_out/ab/ab262k.json
