#!/usr/bin/env python3
"""does packed fp32 (v_pk_fma_f32 / v_pk_mul_f32, two fp32
FMAs per lane per instruction) reopen configs[4]'s mixed-precision path?

DESIGN.md §2.7 bounds a fused mixed kernel by T_mixed >= (0.871 r + 0.49) T_64,
with r the issue-cost ratio of the fp32 pass to the fp64 kernel over the
setup-and-loop instruction mix: the path can only win if r < 0.585.  Here r is
recomputed from the n = 32 kernel's PMC class mix per wave (the committed
profiles/r05/measure_c/pmc_n32.log) and the measured issue costs per wave
instruction (tools/probe/valu_probe.hip, profiles/r03/valu_probe_r03.jsonl):
fp64 FMA 5.24, MUL / ADD 5.47, fp64 transcendental 17.23, 32-bit 3.07,
v_pk_fma_f32 5.37 cycles (two FMAs: 2.69 per FMA).

Favourable to the packed design throughout: every fp64 FMA, MUL and ADD is
assumed to pair with another into one packed instruction (most of the
kernel's FMAs are v_fmac_f64_dpp with a row_newbcast operand, and VOP3P has no
DPP form, so each would really need its own broadcast move), the fp32
transcendentals are charged as the 32-bit class, and the 32-bit class (the
selection, reductions, selects, integer work) is unchanged.
usage: tools/mixed_packed_bound.py > profiles/r06/mixed_packed_bound.json"""
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
COST = {"FMA_F64": 5.24, "MUL_F64": 5.47, "ADD_F64": 5.47, "TRANS_F64": 17.23, "B32": 3.07, "PK_F32": 5.37}
THRESHOLD = 0.585  # r below which T_mixed's bound falls under T_64


def main():
    pw = json.load(open(os.path.join(ROOT, "profiles", "r05", "measure_c", "pmc_n32.log")))["head"]["per_wave"]
    fma, mul, add, trans = (pw["SQ_INSTS_VALU_" + k] for k in ("FMA_F64", "MUL_F64", "ADD_F64", "TRANS_F64"))
    b32 = pw["SQ_INSTS_VALU"] - fma - mul - add - trans
    c64 = fma * COST["FMA_F64"] + (mul + add) * COST["MUL_F64"] + trans * COST["TRANS_F64"] + b32 * COST["B32"]
    scalar32 = (fma + mul + add + trans) * COST["B32"] + b32 * COST["B32"]
    packed32 = (fma + mul + add) / 2.0 * COST["PK_F32"] + trans * COST["B32"] + b32 * COST["B32"]
    floor = b32 * COST["B32"]  # float arithmetic free: the 32-bit class alone
    out = {"source": "profiles/r05/measure_c/pmc_n32.log (gi_wave, n = 32, m = 64, B = 262 144, per wave)",
           "class_mix_per_wave": {"FMA_F64": fma, "MUL_F64": mul, "ADD_F64": add, "TRANS_F64": trans, "B32": b32},
           "issue_cycles_per_wave": {"fp64_kernel": c64, "fp32_scalar": scalar32, "fp32_packed": packed32,
                                     "float_work_free": floor},
           "r": {"fp32_scalar": scalar32 / c64, "fp32_packed": packed32 / c64, "float_work_free": floor / c64},
           "threshold": THRESHOLD,
           "bound_T_mixed_over_T64": {k: 0.871 * v + 0.49 for k, v in
                                      {"fp32_scalar": scalar32 / c64, "fp32_packed": packed32 / c64}.items()},
           "build": packed32 / c64 < THRESHOLD}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
