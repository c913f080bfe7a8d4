#!/bin/bash
# round 6: the batch scan and the config sweep re-taken with their timers
# settling the GPU's clocks first
cd "${GRAFT_REPO_ROOT:-.}" || exit 1
O=gpurun_out/${OUT:-r6c}; mkdir -p $O
timeout -k 10 300 python tools/batch_scan.py > $O/batch_scan.json 2> $O/batch_scan.err || { tail -5 $O/batch_scan.err; exit 1; }
timeout -k 10 900 python tools/config_sweep.py > $O/configs.json 2> $O/configs.err || { tail -5 $O/configs.err; exit 1; }
python3 - $O <<'PY'
import json, sys
o = sys.argv[1]
d = json.load(open(f"{o}/batch_scan.json"))
print({k: v for k, v in d.items() if k.split("_")[0] in ("B65536", "B131072", "B1048576", "T1M", "fit")})
c = json.load(open(f"{o}/configs.json"))
for k, v in c.items():
    print(k, v.get("kernel_ms"), v.get("gpu_kernel_ms"), v.get("ok_frac"))
PY
