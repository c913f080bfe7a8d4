#!/usr/bin/env python3
"""Summarise a gpu_measure.sh session: kernel stats of the solver kernel, and
HBM traffic per launch from the PMC passes with the gfx950 corrections of
MI355X_MICROARCH.md §HBM (FETCH_SIZE and WRITE_SIZE are KiB; FETCH_SIZE reads
half the bytes of a wide coalesced stream -> x2; WRITE_SIZE exact for 16-B
streaming stores)."""
import csv
import json
import os
import sys

out_dir = sys.argv[1]
KERNEL = "gi_dense_kernel"


def rows(path):
    return list(csv.DictReader(open(path))) if os.path.exists(path) else []


res = {}
stats = rows(os.path.join(out_dir, "trace", "run_kernel_stats.csv"))
for r in stats:
    if KERNEL in r["Name"]:
        res["kernel"] = r["Name"].split("(")[0]
        res["calls"] = int(r["Calls"])
        res["avg_ns"] = float(r["AverageNs"])
        res["min_ns"] = float(r["MinNs"])
        res["max_ns"] = float(r["MaxNs"])
        res["pct_of_gpu_time"] = float(r["Percentage"])
# the timed steps alone: the trace command launches nothing of this kernel
# after them, so they are its last `steps` dispatches (the average above also
# holds the first launches after idle, slow while the clocks ramp, and the
# settle and warmup launches)
kt = rows(os.path.join(out_dir, "trace", "run_kernel_trace.csv"))
kd = [(float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) for r in kt if KERNEL in r.get("Kernel_Name", "")]
steps = int(os.environ.get("STEPS", 50))
if len(kd) >= steps:
    res["timed_steps"] = steps
    res["timed_avg_ns"] = sum(kd[-steps:]) / steps
    res["first_launch_ns"] = kd[0]
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    vals = [float(r["Counter_Value"]) for r in rows(os.path.join(out_dir, f"pmc_{c}", "run_counter_collection.csv"))
            if KERNEL in r["Kernel_Name"]]
    if vals:
        res[c + "_KiB_per_launch"] = sum(vals) / len(vals)
if "FETCH_SIZE_KiB_per_launch" in res and "WRITE_SIZE_KiB_per_launch" in res:
    fetch = 2.0 * res["FETCH_SIZE_KiB_per_launch"] * 1024  # gfx950: FETCH_SIZE counts half of a wide stream
    write = res["WRITE_SIZE_KiB_per_launch"] * 1024
    res["hbm_bytes_per_launch"] = fetch + write
    res["correction"] = "bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (MI355X_MICROARCH.md HBM section)"
# SQ counter groups: per-wave averages over the solver kernel's launches
sq = {}
for d in sorted(os.listdir(out_dir)) if os.path.isdir(out_dir) else []:
    if not d.startswith("pmc_sq"):
        continue
    per = {}
    for r in rows(os.path.join(out_dir, d, "run_counter_collection.csv")):
        if KERNEL in r["Kernel_Name"]:
            per.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    for k, v in per.items():
        sq[k] = sum(v) / len(v)
if sq.get("SQ_WAVES"):
    res["sq_per_wave"] = {k: v / sq["SQ_WAVES"] for k, v in sq.items() if k != "SQ_WAVES"}
    res["sq_waves_per_launch"] = sq["SQ_WAVES"]
# effective shader clock over the solver kernel: GRBM_GUI_ACTIVE sums the
# busy cycles of the 8 XCDs (MI355X_MICROARCH.md, DVFS give-back), so
# cycles / 8 / the kernel's duration in the same pass
clk = {}
for r in rows(os.path.join(out_dir, "pmc_clk", "run_counter_collection.csv")):
    if KERNEL in r["Kernel_Name"]:
        clk.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
kt = rows(os.path.join(out_dir, "pmc_clk", "run_kernel_trace.csv"))
durs = [float(r["End_Timestamp"]) - float(r["Start_Timestamp"]) for r in kt if KERNEL in r.get("Kernel_Name", "")]
if clk.get("GRBM_GUI_ACTIVE") and durs:
    ga = sum(clk["GRBM_GUI_ACTIVE"]) / len(clk["GRBM_GUI_ACTIVE"])
    dn = sum(durs) / len(durs)
    res["grbm_gui_active_per_launch"] = ga
    res["pmc_pass_kernel_ns"] = dn
    res["effective_clock_GHz"] = ga / 8.0 / dn
try:
    res["bench"] = json.loads(open(os.path.join(out_dir, "bench.json")).read().strip().splitlines()[-1])
    res["library"] = res["bench"].get("library")
except Exception:  # noqa: BLE001
    pass
# the candidate profiles/pmc_traffic.json (bench.py's roofline.traffic and
# valu_ceiling), keyed to the hot kernel's revision token of the library string
if "hbm_bytes_per_launch" in res and "sq_per_wave" in res and res.get("library"):
    lib = res["library"]
    inner = lib.split("(", 1)[1].rsplit(")", 1)[0]
    rev = next(t.split(":", 1)[0].strip() for t in inner.split(";") if t.strip().startswith("gi_dense"))
    spw = res["sq_per_wave"]
    cfg = res["bench"]["config"]
    pmc = {"config": {"n": cfg["n"], "m": cfg["m"], "batch_per_gpu": cfg["batch_per_gpu"], "family": cfg["family"]},
           "library": lib, "kernel_rev": rev, "hbm_bytes_per_launch": res["hbm_bytes_per_launch"],
           "source": f"{out_dir} (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, 2*FETCH+WRITE)",
           "valu_classes": {"VALU": spw.get("SQ_INSTS_VALU"), "FMA_F64": spw.get("SQ_INSTS_VALU_FMA_F64"),
                            "MUL_F64": spw.get("SQ_INSTS_VALU_MUL_F64"), "ADD_F64": spw.get("SQ_INSTS_VALU_ADD_F64"),
                            "TRANS_F64": spw.get("SQ_INSTS_VALU_TRANS_F64")},
           "valu_source": f"{out_dir} (rocprofv3 --pmc SQ_INSTS_VALU[_FMA_F64|_MUL_F64|_ADD_F64|_TRANS_F64] "
                          f"SQ_WAVES, {rev})"}
    json.dump(pmc, open(os.path.join(out_dir, "pmc_traffic.json"), "w"), indent=1)
print(json.dumps(res, indent=1))
