#!/bin/bash
# round 5: the n <= 32 box fast path (BOX form of gi_wave) -- box, wave and
# mixed tests; the config sweep with the mixed and box rows; section stamps
# of the fp64 wave kernel at configs[4] (the mixed-precision bound)
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/r5d; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_box.py tests/test_gpu_wave_kernel.py tests/test_gpu_mixed.py -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -4 $O/pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python tools/config_sweep.py c1_n16_m32 c4_n32_m64 c4_n32_m64_mixed c4_n32_box_dense_path c4_n32_box_fast_path c3_n128_m256 > $O/configs.json 2> $O/configs.err || { tail -5 $O/configs.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/configs.json'));print({k:(round(v['kernel_ms'],3),round(v['frac_of_8TBs'],3)) for k,v in d.items() if 'kernel_ms' in v})"
timeout -k 10 200 python tools/sections.py n32 > $O/sections_n32.json 2>&1; cat $O/sections_n32.json
exit 0
