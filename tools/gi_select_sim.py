# Goldfarb-Idnani dual active-set in numpy (the kernel's formulation) with
# selectable constraint-selection rules; counts iterations (ADD + DROP).
# usage: N=32 python tools/gi_select_sim.py [B] [family] [rules...]
import os, sys, numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'oracle'))
import oracle

def gi(H, f, A, b, rule, tol=1e-10, trace=None):
    # trace: a list that receives (q, 'add' | 'drop') per iteration when given
    n = len(f); m = len(b)
    L = np.linalg.cholesky(H)
    D0 = np.linalg.solve(L, A.T).T          # A L^{-T}
    y = np.linalg.solve(L, f)
    s = b + D0 @ y
    an = np.linalg.norm(A, axis=1); dn = np.linalg.norm(D0, axis=1)
    W = []; R = np.zeros((0, 0)); lam = np.zeros(0)
    Dc = D0.copy()
    it = adds = drops = 0
    thr = -tol * (1 + np.abs(b) / an)        # on s/|a|
    while it < 300:
        q = len(W)
        act = np.zeros(m, bool); act[W] = True
        viol = (~act) & (s / an < thr)
        if not viol.any(): break
        if rule == 'anorm': key = s / an
        elif rule == 'dnorm': key = s / dn
        elif rule == 'raw': key = s
        elif rule == 'proj':
            fn = np.linalg.norm(Dc[:, q:], axis=1); fn[fn == 0] = np.inf; key = s / fn
        p = np.argmin(np.where(viol, key, np.inf))
        up = 0.0
        while True:
            it += 1
            q = len(W)
            d = Dc[p]; d1 = -d[:q]; d2 = d[q:]
            r = np.linalg.solve(R, d1) if q else np.zeros(0)
            t1 = np.inf; k = -1
            for j in range(q):
                if r[j] > 0 and lam[j] / r[j] < t1: t1 = lam[j] / r[j]; k = j
            nd2 = d2 @ d2
            t2 = -s[p] / nd2 if nd2 > 1e-24 * (d @ d) else np.inf
            t = min(t1, t2)
            if not np.isfinite(t): return it, adds, drops, None
            if np.isfinite(t2): s = s + t * (Dc[:, q:] @ d2)
            lam = lam - t * r; up += t
            if trace is not None:
                trace.append((q, 'add' if t2 <= t1 else 'drop'))
            if t2 <= t1:
                nrm = np.linalg.norm(d2)
                alpha = -nrm if d2[0] <= 0 else nrm      # kernel: Dpq <= 0 -> -|d2|
                v = d2.copy(); v[0] += alpha
                Dc[:, q:] -= np.outer(Dc[:, q:] @ v, v) * (2 / (v @ v))
                Rn = np.zeros((q + 1, q + 1)); Rn[:q, :q] = R; Rn[:q, q] = d1; Rn[q, q] = alpha
                R = Rn; W.append(p); lam = np.append(lam, up); adds += 1
                break
            drops += 1
            W.pop(k); lam = np.delete(lam, k); R = np.delete(R, k, axis=1)
            for j in range(k, q - 1):
                a_, bb = R[j, j], R[j + 1, j]
                h = np.hypot(a_, bb); c, sn = a_ / h, bb / h
                G = np.array([[c, sn], [-sn, c]])
                R[[j, j + 1], :] = G @ R[[j, j + 1], :]
                Dc[:, [j, j + 1]] = Dc[:, [j, j + 1]] @ G.T
            R = R[:q - 1, :]
    return it, adds, drops, sorted(W)

if __name__ == '__main__':
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    H, f, A, b = oracle.family_generate(int(os.environ.get('N', 16)), B, 20261015, family=sys.argv[2] if len(sys.argv) > 2 else 'box', shift=1.0, box=10.0)
    base = None
    for rule in sys.argv[3:] or ['anorm', 'dnorm', 'raw', 'proj']:
        its = []; dr = []; Ws = []
        for i in range(B):
            it, a, d, W = gi(H[i], f[i], A[i], b[i], rule)
            its.append(it); dr.append(d); Ws.append(W)
        its = np.array(its)
        ls = its[: (B // 4) * 4].reshape(-1, 4).max(1).mean()
        same = None
        if base is None: base = Ws
        else: same = np.mean([Ws[i] == base[i] for i in range(B)])
        print(rule, 'iters mean %.3f' % its.mean(), 'drops %.3f' % np.mean(dr), 'lockstep4 %.3f' % ls, 'same W', same, flush=True)
