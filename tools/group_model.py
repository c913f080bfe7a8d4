#!/usr/bin/env python3
"""Issue-cycle model of the n = 16, m = 32 active-set kernel for three lane
mappings (VERDICT r04 item 1, step a):

  G = 4  the shipped gi_dense: 16 lanes per QP, two D rows per lane (MR = 2)
  G = 2  32 lanes per QP, one D row per lane, two QPs per wavefront: the
         owner writes its only row (no 35-v_cndmask row select, as gi_box),
         E halves (one 16-double row per lane)
  G = 1  64 lanes per QP (gi_wave, measured directly: tools/group_probe.py)

Two inputs:
 (1) trips.  The numpy Goldfarb-Idnani model (tools/gi_select_sim.py, dual
     steepest-edge rule, the kernel's formulation) gives every QP's iteration
     sequence (q before the iteration, ADD or DROP); the kernel runs one more
     trip per QP (the selection that finds no violated row).  A wavefront of G
     QPs runs max-over-the-group trips; the back substitution runs qmax = the
     group's largest q steps, the ADD column select one branch per distinct q,
     and a trip runs the DROP path when any QP of the group drops.
 (2) VALU per section, split into a part fixed per wavefront and a part per D
     row held by a lane, read off the gfx950 listing of gi_dense v11.3 (MR = 2
     instantiation; tools/asm_blocks.py block table):

       section          listing blocks           VALU  fixed  per row
       load + norms     LBB3_4                    100     30      35
       setup sweep      LBB3_8                    754    418     168   (D: 120 DPP FMAs + 3 per step)
       selection        LBB3_17..bb.19             26     10       8   (+2 per wave at G = 2: cross-half max)
       exchange write   bb.22                      36      1   35(MR-1) (owner's row select)
       slack product    LBB3_23                    61     25      18
       ratio + step     LBB3_41, LBB3_44, bb.45    48     48       0
       slack update     LBB3_13                    12      6       3
       ADD              LBB3_12 + column tree      76     28      24   (+6 per distinct q)
       DROP             LBB3_65..LBB3_106         ~190     60      65   (+19 per Givens step)
       back subst.      LBB3_39..64          2 per step (qmax steps)
       outputs          LBB3_164..               257    240       8

     Cycles per VALU class (tools/probe/valu_probe.hip): the per-row parts are
     DPP-fused fp64 FMAs (5.24 cycles), the fixed parts are charged the
     kernel's measured average (13 839 issue cycles / 2 962 VALU per wave =
     4.67 cycles, PMC of v11.3).

Output: trips per QP, VALU and issue cycles per QP for G = 4, 2, 1, and the
predicted kernel-time ratio against G = 4 at the same issue efficiency (the
G = 4 kernel's VALU issues ~89 % of its cycles at 3 waves per SIMD, so a 4th
wave per SIMD can recover at most the remaining ~11 %).
usage: tools/group_model.py [B] [family] > json"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import oracle  # noqa: E402
from gi_select_sim import gi  # noqa: E402

FMA_CYC, AVG_CYC = 5.24, 13839.0 / 2962.0
# (fixed per wave, per row per lane) VALU, from the listing (docstring table)
SEC = {
    "load": (30, 35), "sweep": (418, 168), "select": (10, 8), "slackprod": (25, 18),
    "ratio": (48, 0), "slackupd": (6, 3), "add": (28, 24), "drop": (60, 65), "out": (240, 8),
}
XCHG_SELECT = 35   # v_cndmask per extra row held by the owner lane
COLQ = 6           # ADD column-q branch tree, per distinct q in the wave
GIVENS = 19        # per Givens step of a DROP (R and D rotations, per wave)
BACKSUB = 2        # per back-substitution step


def traces(B, fam):
    H, f, A, b = oracle.family_generate(16, B, 20261015, family=fam, shift=1.0, box=10.0)
    out = []
    for i in range(B):
        tr = []
        gi(H[i], f[i], A[i], b[i], "proj", trace=tr)
        tr.append((None, "final"))  # the selection trip that finds nothing
        out.append(tr)
    return out


def cost_cycles(fixed, rows, extra_fixed=0.0):
    return (fixed + extra_fixed) * AVG_CYC + rows * FMA_CYC


def model(trs, G, MR):
    """VALU and issue cycles per QP for groups of G consecutive QPs, MR D rows per lane."""
    B = len(trs) // G * G
    valu = cyc = trips = 0.0
    for g0 in range(0, B, G):
        grp = trs[g0:g0 + G]
        T = max(len(t) for t in grp)
        trips += T
        v = c = 0.0

        def sec(name, extra=0.0):
            nonlocal v, c
            fx, pr = SEC[name]
            v += fx + extra + pr * MR
            c += cost_cycles(fx + extra, pr * MR)

        sec("load"); sec("sweep"); sec("out")
        for k in range(T):
            steps = [t[k] if k < len(t) else None for t in grp]
            live = [s for s in steps if s is not None and s[1] != "final"]
            sec("select", 2.0 if G == 2 else 0.0)
            if not live:
                continue
            # exchange: the owner's row select (MR - 1 extra rows), then the slack product
            v += 1 + XCHG_SELECT * (MR - 1)
            c += (1 + XCHG_SELECT * (MR - 1)) * AVG_CYC
            sec("slackprod")
            qmax = max(s[0] for s in live)
            v += BACKSUB * qmax
            c += BACKSUB * qmax * FMA_CYC
            if qmax > 0:
                sec("ratio")
            sec("slackupd")
            adds = [s for s in live if s[1] == "add"]
            drops = [s for s in live if s[1] == "drop"]
            if adds:
                nq = len({s[0] for s in adds})
                sec("add", COLQ * nq)
            if drops:
                gsteps = max(s[0] for s in drops)
                sec("drop", GIVENS * gsteps)
        valu += v
        cyc += c
    n = B
    return {"trips_per_wave": trips / (B / G), "valu_per_qp": valu / n, "issue_cycles_per_qp": cyc / n}


def main(B, fam):
    trs = traces(B, fam)
    its = np.array([len(t) for t in trs])
    res = {"family": fam, "B": B, "kernel_trips_per_qp": float(its.mean()), "max": int(its.max())}
    g4 = model(trs, 4, 2)
    g2 = model(trs, 2, 1)
    res["G4_gi_dense"] = g4
    res["G2_32lanes"] = g2
    res["G2_vs_G4_issue_cycles"] = g2["issue_cycles_per_qp"] / g4["issue_cycles_per_qp"]
    # a 4th wave per SIMD recovers at most the idle ~11 % of the G = 4 kernel's VALU cycles
    res["G2_best_case_time_ratio_with_4_waves"] = res["G2_vs_G4_issue_cycles"] * 0.89
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 2000, sys.argv[2] if len(sys.argv) > 2 else "box")
