#!/usr/bin/env python3
"""Where the n = 128, m = 256 block kernel's time goes: kernel time against
max_iter (setup + k iterations), iteration / drop counts, B = 2048 (8 QPs per
CU) of the configs[3] box family."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embedded-qp-solver_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import qpb  # noqa: E402
from config_sweep import t_kernel  # noqa: E402


def main():
    B = int(os.environ.get("B", 2048))
    n = int(os.environ.get("N", 128))
    fam = os.environ.get("FAM", "box")
    H, f, A, b = qpb.generate(n, B, 20261015, family=fam)
    sol = qpb.solve(H, f, A, b)
    torch.cuda.synchronize()
    it = sol.iters.cpu().numpy().astype(np.int64)
    q = qpb.active_mask_to_bool(sol.active.cpu().numpy(), 2 * n).sum(1)
    drops = (it - 1 - q) // 2
    out = {"n": n, "B": B, "family": fam, "iters_mean": float(it.mean()), "iters_max": int(it.max()),
           "active_mean": float(q.mean()), "drops_mean": float(drops.mean()),
           "ok": float((sol.status.cpu().numpy() == 0).mean())}
    for mi in (1, 2, 5, 10, 20, 40, 0):
        out[f"maxit{mi or 'def'}_ms"] = t_kernel(lambda: qpb.solve(H, f, A, b, max_iter=mi, out=sol), 3)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
