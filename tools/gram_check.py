#!/usr/bin/env python3
"""GPU check of the Gram-form n<=128 kernel (qpb_gi_gram.hip): oracle parity on
small counts per shape, KKT at a larger batch, and timing at BASELINE
configs[3] (n=128, m=256, B=16384) against the round-1 block kernel
(QPB_FLAG_DIAG_BLOCK).  Writes gpurun_out/gram_check.json."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "embedded-qp-solver_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402
import qpb  # noqa: E402

out = {}
dev = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
for n, m, kind, count in [(48, 96, "box", 6), (64, 128, "dense", 6), (33, 200, "dense", 4), (128, 256, "box", 4),
                          (128, 256, "dense", 3), (100, 40, "dense", 3)]:
    H, f, A, b = O.family_conditioned(2000 + n + m, count, n, m=m, box=10.0, kind=kind)
    sol = qpb.solve(dev(H), dev(f), dev(A), dev(b))
    torch.cuda.synchronize()
    x, lam, act, st, it = (t.cpu().numpy() for t in sol)
    r = O.kkt_residuals(H, f, A, b, x, lam)
    mask = qpb.active_mask_to_bool(act, m)
    errs, masks = [], []
    for i in range(count):
        ref = O.active_set_solve(H[i], f[i], A[i], b[i])
        errs.append(float(np.abs(x[i] - ref.x).max() / max(1.0, np.abs(ref.x).max())))
        masks.append(bool(np.array_equal(mask[i], ref.active)))
    key = f"{kind}_n{n}_m{m}"
    out[key] = {"status": st.tolist(), "iters": it.tolist(), "kkt": {k: float(v.max()) for k, v in r.items()},
                "xerr": errs, "mask_ok": masks}
    print(key, out[key], flush=True)

B = 16384
H, f, A, b = qpb.generate(128, B, 20261015, family="box")
for name, flags in [("gram", 0), ("block", 128)]:
    sol = qpb.solve(H, f, A, b, flags=flags)
    torch.cuda.synchronize()
    reps = 3 if flags == 0 else 1
    t0 = time.perf_counter()
    for _ in range(reps):
        sol = qpb.solve(H, f, A, b, flags=flags)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / reps * 1e3
    st = sol.status.cpu().numpy()
    it = sol.iters.cpu().numpy()
    rec = {"ms": ms, "qps": B / ms * 1e3, "ok_frac": float((st == 0).mean()), "iters_mean": float(it.mean()),
           "iters_max": int(it.max())}
    if name == "gram":
        Hn, fn, An, bn = (t.cpu().numpy() for t in (H, f, A, b))
        k = 2048
        r = O.kkt_residuals(Hn[:k], fn[:k], An[:k], bn[:k], sol.x.cpu().numpy()[:k], sol.lam.cpu().numpy()[:k])
        rec["kkt_first2048"] = {kk: float(v.max()) for kk, v in r.items()}
        xg = sol.x.clone()
    else:
        rec["x_vs_gram"] = float((sol.x - xg).abs().max().item())
    out[f"config3_{name}"] = rec
    print(name, rec, flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(out, open(os.path.join(ROOT, "gpurun_out", "gram_check.json"), "w"), indent=1)
