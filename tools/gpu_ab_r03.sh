#!/bin/bash
# round-3 A/B session: parity of each candidate, then interleaved kernel timing
# (n=16 dense kernel at 1M box + dense, box fast path, n=32 wave kernel)
cd "${GRAFT_REPO_ROOT:-.}" && mkdir -p gpurun_out/ab || exit 1
DV=${DV-vB}; BV=${BV-bB}; WV=${WV-wB}
for v in $DV; do
  QPB_LIB=embedded-qp-solver_amd/lib/libqpb_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_active_set.py tests/test_gpu_metric_batch.py -x -q --timeout 250 --timeout-method thread > gpurun_out/ab/pytest_$v.log 2>&1 || { tail -20 gpurun_out/ab/pytest_$v.log; exit 1; }
  echo "pytest $v: $(tail -1 gpurun_out/ab/pytest_$v.log)"
done
for v in $BV; do
  QPB_LIB=embedded-qp-solver_amd/lib/libqpb_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_box.py -x -q --timeout 250 --timeout-method thread > gpurun_out/ab/pytest_$v.log 2>&1 || { tail -20 gpurun_out/ab/pytest_$v.log; exit 1; }
  echo "pytest $v: $(tail -1 gpurun_out/ab/pytest_$v.log)"
done
for v in $WV; do
  QPB_LIB=embedded-qp-solver_amd/lib/libqpb_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_wave_kernel.py tests/test_gpu_mixed.py -x -q --timeout 250 --timeout-method thread > gpurun_out/ab/pytest_$v.log 2>&1 || { tail -20 gpurun_out/ab/pytest_$v.log; exit 1; }
  echo "pytest $v: $(tail -1 gpurun_out/ab/pytest_$v.log)"
done
summ() { python3 -c "import json,sys;d=json.load(open(sys.argv[1]));print(sys.argv[2], json.dumps({k:v['median_us'] for k,v in d['variants'].items()}))" "$1" "$2"; }
if [ -n "$DV" ]; then
  ROUNDS=8 timeout -k 10 300 python tools/ab.py head $DV > gpurun_out/ab/ab1m_box.json || exit 1; summ gpurun_out/ab/ab1m_box.json dense-kernel-1M-box
  ROUNDS=6 FAM=dense timeout -k 10 300 python tools/ab.py head $DV > gpurun_out/ab/ab1m_dense.json || exit 1; summ gpurun_out/ab/ab1m_dense.json dense-kernel-1M-dense
fi
if [ -n "$BV" ]; then
  ROUNDS=8 timeout -k 10 300 python tools/ab_box_variants.py head $BV > gpurun_out/ab/ab_box.json || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/ab/ab_box.json'));print('box-1M', {k:v['median_us'] for k,v in d.items()})"
fi
if [ -n "$WV" ]; then
  timeout -k 10 400 python tools/ab_n32.py head $WV > gpurun_out/ab/ab32.json || exit 1; summ gpurun_out/ab/ab32.json wave-n32-262k
fi
