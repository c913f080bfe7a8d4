#!/usr/bin/env python3
"""Lockstep cost of four QPs per wavefront (n <= 16 kernel), in the numpy model
of tools/gi_select_sim.py (dual steepest-edge rule): the trips a wave runs are
the maximum of its four QPs' iteration counts.  Prints the mean trips per wave
for (a) the batch order, (b) QPs sorted inside windows of W by their initially
violated count (a predictor available after the setup) and by the true count
(the unreachable bound), and (c) a first launch capped at k trips whose
unfinished QPs are re-solved from scratch in lockstep groups of four (setup
charged as SETUP trips), and (d) the trips per wave for lockstep groups of
1, 2, 4 and 8 QPs (tools/group_model.py turns them into issue cycles).  usage: tools/lockstep_sim.py [B] [family]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle"))
import oracle  # noqa: E402
from gi_select_sim import gi  # noqa: E402

SETUP = 2.2  # setup sweep VALU in units of one loop trip (~600 / 275)


def main(B, fam):
    H, f, A, b = oracle.family_generate(16, B, 20261015, family=fam, shift=1.0, box=10.0)
    its = np.zeros(B, int)
    nv = np.zeros(B, int)
    for i in range(B):
        L = np.linalg.cholesky(H[i])
        D0 = np.linalg.solve(L, A[i].T).T
        s = b[i] + D0 @ np.linalg.solve(L, f[i])
        an = np.linalg.norm(A[i], axis=1)
        nv[i] = (s / an < -1e-10 * (1 + np.abs(b[i]) / an)).sum()
        its[i] = gi(H[i], f[i], A[i], b[i], "proj")[0]
    B4 = B // 4 * 4
    its, nv = its[:B4], nv[:B4]
    lock = lambda o: its[o].reshape(-1, 4).max(1).mean()  # noqa: E731
    print(f"{fam}: iterations {its.mean():.3f}, corr(iterations, violated at x0) {np.corrcoef(its, nv)[0, 1]:.2f}")
    print(f"  batch order: {lock(np.arange(B4)):.3f} trips per wave")
    # group sizes: trips a wavefront of G QPs runs (max over its group), per QP
    for G in (1, 2, 4, 8):
        BG = B // G * G
        print(f"  group size {G}: {its[:BG].reshape(-1, G).max(1).mean() if BG <= B4 else float('nan'):.3f} trips per wave")
    for W in (16, 64):
        for name, key in (("violated count", nv.astype(float)), ("true count", its.astype(float))):
            o = np.concatenate([w0 + np.argsort(key[w0:w0 + W], kind="stable") for w0 in range(0, B4, W)])
            print(f"  sorted in windows of {W} by {name}: {lock(o):.3f}")
    base = lock(np.arange(B4))
    for k in range(5, 11):
        p1 = np.minimum(its.reshape(-1, 4).max(1), k).mean()
        un = np.random.default_rng(0).permutation(its[its > k])
        un = un[: len(un) // 4 * 4]
        p2 = (un.reshape(-1, 4).max(1).mean() + SETUP) * len(un) / B4 if len(un) else 0.0
        print(f"  cap {k}: {(its > k).mean():.3f} unfinished, {p1 + p2:.3f} trip-equivalents per wave (uncapped {base:.3f})")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 4000, sys.argv[2] if len(sys.argv) > 2 else "box")
