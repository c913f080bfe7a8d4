#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ (run HERE, where
/root/reference exists; the GPU box only reads the committed .npz files).

Inputs/outputs come from
  * the compiled reference C (oracle/_ref/libqpref_*.so built by oracle/Makefile
    from the unmodified /root/reference sources): its generator
    (matrix_ops.c:677-734 in main.c:37-39 order), newton_method_with_line_search
    (qp_solvers.c:103-144), admm (:255-319), gradient_descent_with_line_search
    (:65-101), matrix_invert (matrix_ops.c:551-630);
  * the numpy oracle (oracle/oracle.py): qp_ref.py's unconstrained solve and the
    KKT-certified primal active-set solver for the constrained families.

Usage:  make -C oracle ref && python tests/golden/make_golden.py
"""
from __future__ import annotations

import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import oracle as O  # noqa: E402
from refc import RefC  # noqa: E402


def certify(H, f, A, b, res_list):
    x = np.stack([r.x for r in res_list])
    lam = np.stack([r.lam for r in res_list])
    act = np.stack([r.active for r in res_list])
    st = np.array([r.status for r in res_list])
    kk = O.kkt_residuals(H, f, A, b, x, lam)
    worst = max(float(v.max()) for v in kk.values())
    assert (st == 0).all(), st
    assert worst < 1e-9, kk
    return x, lam, act, worst


def box_as_dense(n, count, ub, lb):
    A = np.concatenate([np.broadcast_to(np.eye(n), (count, n, n)),
                        np.broadcast_to(-np.eye(n), (count, n, n))], axis=1).copy()
    b = np.concatenate([np.broadcast_to(ub, (count, n)), -np.broadcast_to(lb, (count, n))], axis=1).copy()
    return A, b


def ref_family(n, seed, count, gd_count):
    rc = RefC(n, "1e12")
    P, q, x0 = rc.generate(seed, count)
    P2, q2, x02 = O.ref_generate(seed, count, n)
    assert np.array_equal(P, P2) and np.array_equal(q, q2) and np.array_equal(x0, x02)
    out = dict(P=P, q=q, x0=x0)
    out["newton_x"] = rc.newton(P, q, x0, 10)            # HESS_ITERATIONS config.h:37
    out["admm_x_inactive"] = rc.admm(P, q, x0, 10000)    # ADMM_ITERATIONS config.h:38
    if gd_count:
        out["gd_x"] = rc.gd(P[:gd_count], q[:gd_count], x0[:gd_count], 10000)  # GRAD_ITERATIONS
    out["x_exact"] = np.stack([O.qp_ref_solve(P[i], q[i]) for i in range(count)])
    out["f_exact"] = np.array([O.eval_qp(P[i], q[i], out["x_exact"][i]) for i in range(count)])
    if n <= 16:
        out["inv"] = np.stack([rc.invert(P[i]) for i in range(count)])
    # active box +-1e2 (the survey's "active" reference box)
    ra = RefC(n, "1e2")
    out["admm_x_active"] = ra.admm(P, q, x0, 10000)
    A, b = box_as_dense(n, count, 1e2, -1e2)
    res = [O.active_set_solve(P[i], q[i], A[i], b[i]) for i in range(count)]
    x, lam, act, worst = certify(P, q, A, b, res)
    out.update(box_x=x, box_lam=lam, box_act=act, box_A=A, box_b=b)
    return out, dict(seed=seed, count=count, n=n, box_active=1e2, kkt_worst=worst)


def cond_family(n, seed, count, kind, box, m=None):
    H, f, A, b = O.family_conditioned(seed, count, n, m=m, box=box, kind=kind)
    res = [O.active_set_solve(H[i], f[i], A[i], b[i]) for i in range(count)]
    x, lam, act, worst = certify(H, f, A, b, res)
    out = dict(H=H, f=f, A=A, b=b, x=x, lam=lam, act=act, iters=np.array([r.iters for r in res]))
    meta = dict(seed=seed, count=count, n=n, m=int(A.shape[1]), kind=kind, box=box, kkt_worst=worst,
                mean_active=float(act.sum(1).mean()))
    if kind == "box" and n == 16 and box == 10:
        rc = RefC(16, "10")
        out["admm_x"] = rc.admm(H, f, np.zeros_like(f), 10000)
    return out, meta


def main():
    manifest = {"generator": "tests/golden/make_golden.py", "files": {}}
    jobs = [
        ("ref_n4", lambda: ref_family(4, 4001, 32, 32)),
        ("ref_n16", lambda: ref_family(16, 16001, 32, 8)),
        ("ref_n32", lambda: ref_family(32, 32001, 12, 0)),
        ("cond_box_n16", lambda: cond_family(16, 20261015, 64, "box", 10.0)),
        ("cond_dense_n16_m32", lambda: cond_family(16, 20261016, 64, "dense", 10.0, m=32)),
        ("cond_box_n4", lambda: cond_family(4, 20261017, 32, "box", 10.0)),
        ("cond_dense_n4_m8", lambda: cond_family(4, 20261018, 32, "dense", 10.0, m=8)),
        ("cond_dense_n10_m20", lambda: cond_family(10, 20261019, 32, "dense", 10.0, m=20)),
    ]
    for name, job in jobs:
        data, meta = job()
        path = os.path.join(HERE, name + ".npz")
        np.savez_compressed(path, **data)
        with open(path, "rb") as fp:
            meta["sha256"] = hashlib.sha256(fp.read()).hexdigest()
        meta["arrays"] = {k: list(v.shape) for k, v in data.items()}
        manifest["files"][name + ".npz"] = meta
        print(name, meta.get("kkt_worst"), os.path.getsize(path))
    with open(os.path.join(HERE, "manifest.json"), "w") as fp:
        json.dump(manifest, fp, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
