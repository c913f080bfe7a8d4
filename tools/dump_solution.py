#!/usr/bin/env python3
"""Solve one generated batch with the library QPB_LIB names and save x, lam,
active, status, iters to OUT (.npz), for bitwise comparisons of kernel
variants.  env: N (32), M (64), B (65536), FAM (dense), OUT, FLAGS (0)"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embedded-qp-solver_amd"))
import torch  # noqa: E402

import qpb  # noqa: E402

n, m, B = int(os.environ.get("N", 32)), int(os.environ.get("M", 64)), int(os.environ.get("B", 65536))
H, f, A, b = qpb.generate(n, B, 20261015, family=os.environ.get("FAM", "dense"), m=m)
sol = qpb.solve(H, f, A, b, flags=int(os.environ.get("FLAGS", 0)))
torch.cuda.synchronize()
np.savez(os.environ["OUT"], **{k: getattr(sol, k).cpu().numpy() for k in ("x", "lam", "active", "status", "iters")})
print("saved", os.environ["OUT"])
