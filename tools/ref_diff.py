#!/usr/bin/env python3
"""Diagnostic (GPU box): where do the REF-mode replicas (qpb_ref_solve,
qpb_matrix_invert) differ bitwise from the compiled reference C?  For each n,
draws QPs with the reference generator (refC), runs refC and the GPU replica
on the same inputs and reports, per mode, the bitwise-equal fraction and for
each differing QP: the GPU iteration count, whether its inverse was bitwise
equal, and the relative / ulp error.  usage: ref_diff.py [count]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embedded-qp-solver_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import qpb  # noqa: E402
from refc import RefC, available  # noqa: E402


def ulps(a, b):
    ia = a.view(np.int64)
    ib = b.view(np.int64)
    return np.abs(ia - ib)


def main(count=256):
    out = {}
    dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    for n in (4, 16, 32):
        for box in ("1e12", "1e2"):
            if not available(n, box):
                continue
            rc = RefC(n, box)
            P, q, x0 = rc.generate(seed=1234 + n, count=count)
            inv_ref = np.stack([rc.invert(P[i].copy()) for i in range(count)])
            inv_gpu = qpb.matrix_invert(dev(P)).cpu().numpy()
            inv_eq = np.all(inv_gpu == inv_ref, axis=(1, 2))
            res = {"inverse_bitwise": float(inv_eq.mean())}
            bx = float(box)
            modes = [("newton", qpb.REF_NEWTON, 10, rc.newton), ("admm", qpb.REF_ADMM, 10000, rc.admm)]
            for name, mode, iters, fn in modes:
                if name == "newton" and box != "1e12":
                    continue
                xr = fn(P, q, x0, iters)
                xg, it = qpb.ref_solve(mode, dev(P), dev(q), dev(x0), iterations=iters, box=(-bx, bx))
                xg = xg.cpu().numpy()
                it = it.cpu().numpy()
                eq = np.all(xg == xr, axis=1)
                rel = np.abs(xg - xr).max(axis=1) / np.abs(xr).max(axis=1)
                bad = np.nonzero(~eq)[0]
                res[name] = {
                    "bitwise": float(eq.mean()),
                    "max_rel": float(rel.max()),
                    "differ": [{"qp": int(i), "gpu_iters": int(it[i]), "inverse_bitwise": bool(inv_eq[i]),
                                "rel": float(rel[i]), "max_ulp": int(ulps(xg[i], xr[i]).max())}
                               for i in bad[:12]],
                    "differ_inverse_equal": int(np.sum(inv_eq[bad])),
                    "differ_count": int(bad.size),
                }
            out[f"n{n}_box{box}"] = res
            print(f"n={n} box={box}: inverse bitwise {res['inverse_bitwise']:.3f}; "
                  + "; ".join(f"{k} bitwise {v['bitwise']:.3f} (max rel {v['max_rel']:.1e})"
                              for k, v in res.items() if isinstance(v, dict)), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "ref_diff.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 256)
