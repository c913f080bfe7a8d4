#!/usr/bin/env python3
"""How much of the n = 16 kernel's lockstep waste (a wave of four QPs runs the
max of their trip counts) a regrouping could win: the bench's QPs solved once,
then the mean over groups of four of max(iters) for the launch order, for
groups formed after sorting windows of W QPs by a predictor, and by the
iteration count itself (the bound).  Predictors available after the setup:
the number of rows the unconstrained minimiser violates.
env: B (262144), SEED (20261015), OUT (gpurun_out/lockstep_probe.json)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embedded-qp-solver_amd"))
import torch  # noqa: E402

import qpb  # noqa: E402

B = int(os.environ.get("B", 262144))
n = 16
H, f, A, b = qpb.generate(n, B, int(os.environ.get("SEED", 20261015)), family="box", shift=1.0, box=10.0)
sol = qpb.solve(H, f, A, b)
torch.cuda.synchronize()
it = sol.iters.long()
x0 = -torch.linalg.solve(H, f.unsqueeze(-1)).squeeze(-1)
viol0 = ((A @ x0.unsqueeze(-1)).squeeze(-1) > b).sum(1)
nact = torch.zeros(B, dtype=torch.long, device=it.device)
for r in range(2 * n):
    nact += ((sol.active[:, 0].long() >> r) & 1)


def grouped(order):
    return float(it[order].view(-1, 4).max(1).values.double().mean())


res = {"B": B, "mean_iters": float(it.double().mean()), "max_iters": int(it.max()),
       "launch_order": grouped(torch.arange(B, device=it.device)),
       "corr_viol0_iters": float(torch.corrcoef(torch.stack([viol0.double(), it.double()]))[0, 1]),
       "corr_nact_iters": float(torch.corrcoef(torch.stack([nact.double(), it.double()]))[0, 1]),
       "hist_iters": torch.bincount(it).tolist(), "windows": {}}
for W in (8, 16, 32, 64, 256):
    row = {}
    for name, key in (("viol0", viol0), ("iters", it)):
        k = key.view(-1, W).double() + torch.rand(B // W, W, device=it.device) * 0.5  # random tie order
        order = (k.argsort(1) + torch.arange(0, B, W, device=it.device).unsqueeze(1)).reshape(-1)
        row[name] = grouped(order)
    res["windows"][str(W)] = row
print(json.dumps(res))
out = os.environ.get("OUT", os.path.join(ROOT, "gpurun_out", "lockstep_probe.json"))
os.makedirs(os.path.dirname(out), exist_ok=True)
json.dump(res, open(out, "w"), indent=1)
