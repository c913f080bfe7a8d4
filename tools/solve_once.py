#!/usr/bin/env python3
"""One generate + REPS solves of a (n, m, B, family) batch: a short program for
rocprofv3 passes.  env: N (32), M (64), B (262144), FAM (dense), REPS (2), FLAGS (0),
MAXIT (0 = the default cap; 1 = setup + one iteration)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embedded-qp-solver_amd"))
import torch  # noqa: E402

import qpb  # noqa: E402

n, m, B = int(os.environ.get("N", 32)), int(os.environ.get("M", 64)), int(os.environ.get("B", 262144))
fam = os.environ.get("FAM", "dense")
H, f, A, b = qpb.generate(n, B, 20261015, family=fam, m=m)
for _ in range(int(os.environ.get("REPS", 2))):
    sol = qpb.solve(H, f, A, b, flags=int(os.environ.get("FLAGS", 0)), max_iter=int(os.environ.get("MAXIT", 0)))
torch.cuda.synchronize()
print("ok", float(sol.iters.double().mean()), int((sol.status == qpb.OK).sum()))
