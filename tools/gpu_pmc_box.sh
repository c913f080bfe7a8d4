# box fast path: PMC instruction counts of gi_box_kernel vs gi_dense_kernel on the same QPs (tools/ab_box.py)
cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && OUT=gpurun_out/pmcbox && mkdir -p $OUT || exit 1
ROUNDS=1 REPS=1 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE -d $OUT/pmc -o run --output-format csv -- python3 tools/ab_box.py > $OUT/pmc.log 2>&1 || { tail -3 $OUT/pmc.log; exit 1; }
python3 - $OUT <<'PY'
import csv, collections, glob, json, os, sys
res = {}
for f in glob.glob(os.path.join(sys.argv[1], "pmc", "**", "*counter_collection.csv"), recursive=True):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f)):
        for k in ("gi_box_kernel", "gi_dense_kernel"):
            if k in r["Kernel_Name"]:
                agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in agg.items():
        res[k] = {c: sum(v) / len(v) for c, v in d.items()}
        res[k]["valu_per_wave"] = res[k]["SQ_INSTS_VALU"] / res[k]["SQ_WAVES"]
        res[k]["lds_per_wave"] = res[k]["SQ_INSTS_LDS"] / res[k]["SQ_WAVES"]
print(json.dumps(res, indent=1))
json.dump(res, open(os.path.join(sys.argv[1], "pmc_box.json"), "w"), indent=1)
PY
