#!/bin/bash
# quick iteration: GPU parity tests, the ablation sweep, the section profile
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prof
TAG=${TAG:-iter}
timeout -k 10 420 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after GPU step failure"; exit $rc; fi
timeout -k 10 300 python tools/prof_sweep.py > gpurun_out/prof/sweep_$TAG.json 2> gpurun_out/prof/sweep_$TAG.err
rc2=$?
cat gpurun_out/prof/sweep_$TAG.json; tail -3 gpurun_out/prof/sweep_$TAG.err
[ $rc2 -ne 0 ] && exit $rc2
timeout -k 10 200 python tools/sections.py > gpurun_out/prof/sections_$TAG.json 2> gpurun_out/prof/sections_$TAG.err
rc3=$?
cat gpurun_out/prof/sections_$TAG.json; tail -3 gpurun_out/prof/sections_$TAG.err
exit $rc3
