import sys, os, json
sys.path.insert(0, "embedded-qp-solver_amd"); sys.path.insert(0, "oracle")
import numpy as np, torch, qpb, oracle as O
B = 16384
H, f, A, b = qpb.generate(128, B, 20261015, family="dense")
res = {}
for rep in range(2):
    sol = qpb.solve(H, f, A, b); torch.cuda.synchronize()
    x = sol.x.cpu().numpy(); lam = sol.lam.cpu().numpy()
    bad = []
    for k0 in range(0, B, 2048):
        sl = slice(k0, k0 + 2048)
        r = O.kkt_residuals(*(t[sl].cpu().numpy() for t in (H, f, A, b)), x[sl], lam[sl])
        worst = np.max(np.stack([np.abs(v).reshape(len(v), -1).max(1) if v.ndim > 1 else np.abs(v) for v in r.values()]), axis=0)
        bad += [int(k0 + i) for i in np.nonzero(worst > 1e-9)[0]]
    res[rep] = {"bad": bad[:20], "nbad": len(bad), "iters_bad": [int(sol.iters[i]) for i in bad[:20]], "x_hash": float(np.abs(x).sum())}
print(json.dumps(res))
