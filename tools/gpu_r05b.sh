#!/bin/bash
# round 5: the batch scan of the shipped tree (-> profiles/batch_scan.json, which
# bench.py's per-rank prediction reads), then the multi-GPU tests (per-rank
# block, digests) and the reference-replica tests (queried LDS sizing)
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/r5b; mkdir -p $O
timeout -k 10 300 python tools/batch_scan.py > $O/batch_scan.json 2> $O/batch_scan.err || { tail -5 $O/batch_scan.err; exit 1; }
cat $O/batch_scan.json; cp $O/batch_scan.json profiles/batch_scan.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_reference_modes.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -5 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
exit 0
