#!/usr/bin/env python3
"""Can the n <= 16 kernel stop paying for finished QPs?  An issue-cycle model of
the schemes VERDICT r05 item 1 names, on the calibrated section costs of
tools/group_model.py (the v11.3 listing's VALU per section, split into a part
per wavefront and a part per D row; 7.42 vs 7.38 GPU trips per wave, 728 vs
740 PMC VALU per QP) and the per-QP iteration traces of the numpy
Goldfarb-Idnani model (tools/gi_select_sim.py, dual steepest edge).

A wavefront of G = 4 QPs (16 lanes each) issues every instruction for all four
rows; a row whose QP is finished or not yet started still costs its share.
Schemes, each keeping G = 4:

  base      the shipped launch: one wave per 4 consecutive QPs, max-of-4 trips.
  refill k  (i) a resident wave that, once k of its 4 rows are done, stores
            their outputs, loads k new QPs and runs the setup sweep for them
            while the running rows sit masked; the event costs the full output +
            load + sweep sections (SIMD: masked rows cost the same issue
            slots), charged once per event.  Free in the model (favourable to
            the scheme): the persistent loop's bookkeeping, its input-load
            latency (the wave would stall or must prefetch), its spills.
  spill C   (iii) the launch stops each wave after C trips; an unfinished QP
            writes its state (D 32x16, R, L, s, lambda, the key norms: ~7.7 KB)
            to HBM and a tail launch resumes the unfinished QPs four per wave
            (charged: the load section as the restore, the remaining trips
            lockstepped among the tail's QPs, the outputs).  The VALU of the
            spill itself is not charged (favourable); its bytes are reported.
  morph     (iv) when at most 2 of the 4 QPs are unfinished, they spread over the
            idle rows' lanes (32 lanes per QP, one D row per lane) for the rest
            of the wave: the per-row half of every trip section is saved.
  sort W    (ii) QPs regrouped inside windows of W by a predictor before the
            solve: the violated count at x0 (the only predictor available
            before the setup without another pass over the inputs; 0.39
            correlated with the iterations), and the true count (unreachable
            bound).  A predictor computed after the setup (e.g. the steepest-edge
            violation mass) would need every QP's ~7.7 KB state moved between
            waves: reported with that traffic.

Besides the model, one measured fact bounds every scheme: the launch with
max_iter = 1 (load, setup, one trip, outputs) takes 1.377 ms of the full
launch's 1.795 ms (profiles/r05/group_probe.json, box family, 1 M QPs), so the
whole rest of the active-set loop costs 0.42 ms; the lockstep waste is
1.76 / 6.38 of those trips, at most ~0.12 ms even if removed for free.

usage: tools/refill_model.py [B] [family] > profiles/r06/refill_model_<family>.json"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from group_model import AVG_CYC, BACKSUB, COLQ, FMA_CYC, GIVENS, SEC, XCHG_SELECT, traces  # noqa: E402

MR = 2
STATE_BYTES = 8 * (32 * 16 + 16 * 16 + 136 + 32 + 16) + 4 * 32 + 4 * 16  # D, R, L, s, lambda | fn2, act/idx
INPUT_BYTES = 6920  # algorithmic bytes per QP


def sec_cost(name, extra=0.0, mr=MR):
    fx, pr = SEC[name]
    return fx + extra + pr * mr, (fx + extra) * AVG_CYC + pr * mr * FMA_CYC


def trip_cost(steps, mr=MR):
    """VALU and issue cycles of one loop trip of a wave whose rows are at
    `steps` (a (q, 'add'|'drop') tuple, (None, 'final') or None = idle row);
    mr = 1: the 32-lanes-per-QP form (one D row per lane, +2 VALU for the
    cross-half key max, no owner row select)."""
    def sc(name, extra=0.0):
        return sec_cost(name, extra, mr)
    v, c = sc("select", 2.0 if mr == 1 else 0.0)
    live = [s for s in steps if s is not None and s[1] != "final"]
    if not live:
        return v, c
    v += 1 + XCHG_SELECT * (mr - 1)
    c += (1 + XCHG_SELECT * (mr - 1)) * AVG_CYC
    dv, dc = sc("slackprod")
    v, c = v + dv, c + dc
    qmax = max(s[0] for s in live)
    v += BACKSUB * qmax
    c += BACKSUB * qmax * FMA_CYC
    if qmax > 0:
        dv, dc = sc("ratio")
        v, c = v + dv, c + dc
    dv, dc = sc("slackupd")
    v, c = v + dv, c + dc
    adds = [s for s in live if s[1] == "add"]
    drops = [s for s in live if s[1] == "drop"]
    if adds:
        dv, dc = sc("add", COLQ * len({s[0] for s in adds}))
        v, c = v + dv, c + dc
    if drops:
        dv, dc = sc("drop", GIVENS * max(s[0] for s in drops))
        v, c = v + dv, c + dc
    return v, c


EV_SETUP = tuple(a + b for a, b in zip(sec_cost("load"), sec_cost("sweep")))
EV_OUT = sec_cost("out")


def run_groups(groups):
    """Lockstep waves over fixed groups (lists of traces): VALU, cycles, trips."""
    v = c = trips = 0.0
    for grp in groups:
        T = max(len(t) for t in grp)
        trips += T
        v += EV_SETUP[0] + EV_OUT[0]
        c += EV_SETUP[1] + EV_OUT[1]
        for k in range(T):
            dv, dc = trip_cost([t[k] if k < len(t) else None for t in grp])
            v, c = v + dv, c + dc
    return v, c, trips


def base(trs):
    B = len(trs) // 4 * 4
    v, c, trips = run_groups([trs[i:i + 4] for i in range(0, B, 4)])
    return {"valu_per_qp": v / B, "issue_cycles_per_qp": c / B, "trips_per_wave": trips / (B / 4)}


def refill(trs, k, waves=64):
    """(i): `waves` resident waves share the QP stream (dealt round-robin to
    the refill events in order of occurrence; the drain at the end included)."""
    B = len(trs)
    nxt = 0
    v = c = 0.0
    events = 0
    # each wave: rows = [trace, position] or None
    state = []
    for _ in range(waves):
        rows = []
        for _ in range(4):
            rows.append([trs[nxt], 0] if nxt < B else None)
            nxt += 1
        state.append(rows)
        v += EV_SETUP[0]
        c += EV_SETUP[1]
        events += 1
    active = True
    while active:
        active = False
        for rows in state:
            if all(r is None for r in rows):
                continue
            active = True
            steps = [r[0][r[1]] if r is not None and r[1] < len(r[0]) else None for r in rows]
            dv, dc = trip_cost(steps)
            v, c = v + dv, c + dc
            for r in rows:
                if r is not None:
                    r[1] += 1
            done = [i for i, r in enumerate(rows) if r is not None and r[1] >= len(r[0])]
            running = sum(1 for r in rows if r is not None and r[1] < len(r[0]))
            if done and (len(done) >= k or running == 0):
                # outputs of the finished rows, then (if the stream has QPs) load + setup of new ones
                v += EV_OUT[0]
                c += EV_OUT[1]
                refilled = False
                for i in done:
                    if nxt < B:
                        rows[i] = [trs[nxt], 0]
                        nxt += 1
                        refilled = True
                    else:
                        rows[i] = None
                if refilled:
                    v += EV_SETUP[0]
                    c += EV_SETUP[1]
                    events += 1
    return {"valu_per_qp": v / B, "issue_cycles_per_qp": c / B, "qps_per_setup_event": B / events}


def spill(trs, C):
    """(iii): first launch capped at C trips, the unfinished QPs resumed by a
    tail launch from their spilled state."""
    B = len(trs) // 4 * 4
    v = c = 0.0
    tail = []
    for i in range(0, B, 4):
        grp = trs[i:i + 4]
        T = min(max(len(t) for t in grp), C)
        v += EV_SETUP[0] + EV_OUT[0]
        c += EV_SETUP[1] + EV_OUT[1]
        for k in range(T):
            dv, dc = trip_cost([t[k] if k < len(t) else None for t in grp])
            v, c = v + dv, c + dc
        tail += [t[C:] for t in grp if len(t) > C]
    nt = len(tail)
    for i in range(0, nt, 4):
        grp = tail[i:i + 4]
        T = max(len(t) for t in grp)
        lv, lc = sec_cost("load")
        v += lv + EV_OUT[0]
        c += lc + EV_OUT[1]
        for k in range(T):
            dv, dc = trip_cost([t[k] if k < len(t) else None for t in grp])
            v, c = v + dv, c + dc
    extra = 2.0 * STATE_BYTES * nt / B
    return {"valu_per_qp": v / B, "issue_cycles_per_qp": c / B, "unfinished_frac": nt / B,
            "extra_hbm_bytes_per_qp": extra, "extra_bytes_frac": extra / INPUT_BYTES}


MORPH_VALU = 2 * 16 * 2 + 8  # permlane moves of a lane's second D row (16 doubles) and its row scalars


def morph(trs):
    """(iv) once at most 2 of a wave's 4 QPs are unfinished, their D rows are
    spread over the idle rows' lanes (v_permlane16/32_swap: a lane's second
    row moves to a lane of an idle row) and the rest of their trips run in
    the 32-lanes-per-QP form (one D row per lane).  Charged: the moves once
    per wave, the one-row form's trip costs afterwards.  Free (favourable):
    the second loop body's registers and code, the R / L slots (per QP in LDS,
    unchanged)."""
    B = len(trs) // 4 * 4
    v = c = 0.0
    for i in range(0, B, 4):
        grp = trs[i:i + 4]
        T = max(len(t) for t in grp)
        v += EV_SETUP[0] + EV_OUT[0]
        c += EV_SETUP[1] + EV_OUT[1]
        morphed = False
        for k in range(T):
            steps = [t[k] if k < len(t) else None for t in grp]
            if not morphed and sum(1 for t in grp if len(t) > k) <= 2:
                morphed = True
                v += MORPH_VALU
                c += MORPH_VALU * AVG_CYC
            dv, dc = trip_cost(steps, 1 if morphed else MR)
            v, c = v + dv, c + dc
    return {"valu_per_qp": v / B, "issue_cycles_per_qp": c / B}


def sorted_windows(trs, key, W):
    B = len(trs) // W * W
    order = np.concatenate([w0 + np.argsort(key[w0:w0 + W], kind="stable") for w0 in range(0, B, W)])
    v, c, trips = run_groups([[trs[j] for j in order[i:i + 4]] for i in range(0, B, 4)])
    return {"valu_per_qp": v / B, "issue_cycles_per_qp": c / B, "trips_per_wave": trips / (B / 4)}


def violated_at_x0(B, fam):
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
    import oracle
    H, f, A, b = oracle.family_generate(16, B, 20261015, family=fam, shift=1.0, box=10.0)
    nv = np.zeros(B)
    for i in range(B):
        L = np.linalg.cholesky(H[i])
        s = b[i] + np.linalg.solve(L, A[i].T).T @ np.linalg.solve(L, f[i])
        an = np.linalg.norm(A[i], axis=1)
        nv[i] = (s / an < -1e-10 * (1 + np.abs(b[i]) / an)).sum()
    return nv


def main(B, fam):
    trs = traces(B, fam)
    its = np.array([len(t) for t in trs], float)
    b0 = base(trs)
    ref = b0["issue_cycles_per_qp"]
    out = {"family": fam, "B": B, "kernel_trips_per_qp": float(its.mean()), "base_G4": b0,
           "ideal_no_lockstep_issue_cycles_ratio": None, "schemes": {}}
    # the unreachable bound: every trip charged as if all 4 rows were busy (no idle rows)
    lone = sum(trip_cost([t[k]] * 4)[1] / 4 for t in trs[: len(trs) // 4 * 4] for k in range(len(t)))
    setup_out = (EV_SETUP[1] + EV_OUT[1]) / 4
    out["ideal_no_lockstep_issue_cycles_ratio"] = (lone / (len(trs) // 4 * 4) + setup_out) / ref
    S = out["schemes"]
    for k in (1, 2, 3, 4):
        r = refill(trs, k)
        r["vs_base"] = r["issue_cycles_per_qp"] / ref
        S[f"refill_k{k}"] = r
    for C in (5, 6, 7, 8, 9):
        r = spill(trs, C)
        r["vs_base"] = r["issue_cycles_per_qp"] / ref
        S[f"spill_after_{C}_trips"] = r
    r = morph(trs)
    r["vs_base"] = r["issue_cycles_per_qp"] / ref
    S["morph_to_32_lanes_at_2_live"] = r
    nv = violated_at_x0(B, fam)
    for W in (16, 64):
        for name, key in (("violated_at_x0", nv), ("true_count", its)):
            r = sorted_windows(trs, key, W)
            r["vs_base"] = r["issue_cycles_per_qp"] / ref
            if name == "true_count":
                r["note"] = "unreachable: the count is known only after the solve"
            S[f"sort_w{W}_{name}"] = r
    S["sort_after_setup_any_predictor"] = {
        "extra_hbm_bytes_per_qp": 2.0 * STATE_BYTES, "extra_bytes_frac": 2.0 * STATE_BYTES / INPUT_BYTES,
        "note": "regrouping after the setup moves every QP's state between waves; bounded below by the "
                "true-count sort's cycles and above 2x the inputs' bytes"}
    best = min((v["vs_base"], k) for k, v in S.items() if "vs_base" in v and "true_count" not in k)
    out["best_buildable"] = {"scheme": best[1], "issue_cycles_vs_base": best[0],
                             "predicted_gain": 1.0 - best[0], "build_threshold": 0.08,
                             "build": 1.0 - best[0] >= 0.08}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 4000, sys.argv[2] if len(sys.argv) > 2 else "box")
