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
try:
    res["bench"] = json.loads(open(os.path.join(out_dir, "bench.json")).read().strip().splitlines()[-1])
    res["library"] = res["bench"].get("library")
except Exception:  # noqa: BLE001
    pass
print(json.dumps(res, indent=1))
