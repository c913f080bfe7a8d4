# n=32 (configs[4] shape) kernel: rocprofv3 kernel trace + one SQ counter pass (--kernel-trace only)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && OUT=gpurun_out/pmc32 && mkdir -p $OUT || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/solve_once.py > $OUT/trace.log 2>&1 || { tail -3 $OUT/trace.log; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $OUT/pmc -o run --output-format csv -- python3 tools/solve_once.py > $OUT/pmc.log 2>&1 || { tail -3 $OUT/pmc.log; exit 1; }
python3 - $OUT <<'PY'
import csv, collections, glob, json, os, sys
out = {}
for f in glob.glob(os.path.join(sys.argv[1], "pmc", "**", "*counter_collection.csv"), recursive=True):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "gi_wave_kernel" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {k: sum(v) / len(v) for k, v in agg.items()}
out["valu_insts_per_qp"] = out["SQ_INSTS_VALU"] / out["SQ_WAVES"]
for f in glob.glob(os.path.join(sys.argv[1], "trace", "**", "*kernel_stats.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "gi_wave_kernel" in r["Name"]:
            out["avg_ns"] = float(r["AverageNs"]); out["calls"] = int(r["Calls"])
print(json.dumps(out, indent=1))
json.dump(out, open(os.path.join(sys.argv[1], "pmc_n32.json"), "w"), indent=1)
PY
