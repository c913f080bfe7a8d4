#!/bin/bash
# round 6, first GPU session: the GPU tests touched this round (full active
# sets against the oracle's new rules, the DIAG_WAVE flag at small and odd
# sizes, the box path with absent bounds), then the config sweep with the
# success fraction read from the full solve.  Each GPU step time-limited; the
# first failure ends it.
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/${OUT:-r6a}; mkdir -p $O
echo "== tests" && timeout -k 10 600 python -u -m pytest tests/test_gpu_active_set.py tests/test_gpu_wave_kernel.py tests/test_gpu_box.py -x -v --timeout 300 --timeout-method thread > $O/pytest_sel.log 2>&1; rc=$?; tail -3 $O/pytest_sel.log; [ $rc -ne 0 ] && exit $rc
echo "== configs" && timeout -k 10 600 python tools/config_sweep.py c1_n16_m32 c4_n32_m64 c4_n32_m64_mixed c4_n32_box_dense_path c4_n32_box_fast_path c3_n128_m256 > $O/configs.json 2> $O/configs.err || { tail -5 $O/configs.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/configs.json'));[print(k, v.get('kernel_ms'), v.get('ok_frac')) for k,v in d.items() if isinstance(v, dict)]"
exit 0
