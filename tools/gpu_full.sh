# Full GPU test suite, then the config sweep (kernel times of every BASELINE config)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/full || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/full/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/full/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 tools/config_sweep.py > gpurun_out/full/configs.json 2> gpurun_out/full/configs.err || { tail -3 gpurun_out/full/configs.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/full/configs.json'));print({k:(round(v['kernel_ms'],3),round(v['frac_of_8TBs'],3)) for k,v in d.items() if 'kernel_ms' in v})"
