import sys, os, time, torch
sys.path.insert(0, "embedded-qp-solver_amd")
import qpb
B = 16384
H, f, A, b = qpb.generate(128, B, 20261015, family="box")
for mi in (1, 2, 11, 21, 0):
    sol = qpb.solve(H, f, A, b, max_iter=mi); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3): sol = qpb.solve(H, f, A, b, max_iter=mi)
    torch.cuda.synchronize()
    print(mi, (time.perf_counter() - t0) / 3 * 1e3, "ms", float(sol.iters.float().mean()))
# unconstrained: setup only (no loop)
sol = qpb.solve(H, f); torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(3): sol = qpb.solve(H, f)
torch.cuda.synchronize(); print("m=0", (time.perf_counter() - t0) / 3 * 1e3, "ms")
names = ["chol", "D", "y+s", "select", "d", "w+r", "step+update", "outputs", "L restore", "x", "queue", "H load", "diag", "panel", "trailing", "step:t", "step:gemv", "step:upd", "step:keys"]
sec = torch.zeros(20, dtype=torch.int64, device="cuda")
sol = qpb.solve(H, f, A, b)
qpb.solve_sections(H, f, A, b, sec, out=sol); torch.cuda.synchronize()
v = sec.cpu().tolist()
import json
cus = torch.cuda.get_device_properties(0).multi_processor_count
print(json.dumps({nm: round(x / 100.0 / B, 3) for nm, x in zip(names, v)}), "us per QP (wall of its workgroup)")
