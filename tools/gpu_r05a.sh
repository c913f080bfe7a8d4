cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5a
timeout -k 10 300 python -u tools/group_probe.py > gpurun_out/r5a/group_probe.json 2> gpurun_out/r5a/group_probe.err || { tail -20 gpurun_out/r5a/group_probe.err; exit 1; }
cat gpurun_out/r5a/group_probe.json
timeout -k 10 400 python bench.py > gpurun_out/r5a/bench.json 2> gpurun_out/r5a/bench.err || { tail -5 gpurun_out/r5a/bench.err; exit 1; }
cat gpurun_out/r5a/bench.json
