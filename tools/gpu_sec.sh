cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/sec &&
timeout -k 10 200 python tools/sections.py > gpurun_out/sec/n16.json 2>gpurun_out/sec/err.log &&
timeout -k 10 200 python tools/sections.py n32 > gpurun_out/sec/n32.json 2>>gpurun_out/sec/err.log && cat gpurun_out/sec/n16.json gpurun_out/sec/n32.json
