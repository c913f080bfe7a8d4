#!/usr/bin/env python3
"""Compare two dump_solution.py outputs: bitwise equality per array, and the
largest difference where they differ.  usage: bitwise_cmp.py a.npz b.npz"""
import json
import sys

import numpy as np

a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
res = {}
for k in a.files:
    x, y = a[k], b[k]
    same = x.shape == y.shape and np.array_equal(x.view(np.uint8), y.view(np.uint8))
    res[k] = {"bitwise": bool(same)}
    if not same and x.shape == y.shape and x.dtype.kind == "f":
        d = np.abs(x - y)
        res[k].update(max_abs=float(d.max()), rows_differing=int((d.reshape(len(d), -1) > 0).any(1).sum()))
print(json.dumps(res))
sys.exit(0 if all(v["bitwise"] for v in res.values()) else 3)
