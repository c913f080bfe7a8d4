import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "embedded-qp-solver_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


def kkt_max_residual_device(H, f, A, b, x, lam, chunk=65536):
    """oracle.kkt_residuals (the same four relative residuals, the same
    scales) evaluated with torch on the device, chunked over the batch, for
    certificates at full BASELINE batch sizes; returns the largest residual
    over all QPs and all four kinds."""
    import torch
    worst = 0.0
    for s in range(0, f.shape[0], chunk):
        e = slice(s, s + chunk)
        Hc, fc, Ac, bc, xc, lc = H[e], f[e], A[e], b[e], x[e], lam[e]
        r = torch.einsum("bij,bj->bi", Hc, xc) + fc + torch.einsum("bij,bi->bj", Ac, lc)
        xn = xc.abs().amax(1)
        stat = r.abs().amax(1) / (1.0 + fc.abs().amax(1) + Hc.abs().sum(2).amax(1) * xn)
        sc = 1.0 + bc.abs().amax(1) + Ac.abs().sum(2).amax(1) * xn
        slack = bc - torch.einsum("bij,bj->bi", Ac, xc)
        prim = torch.clamp(-slack.amin(1), min=0.0) / sc
        ln = 1.0 + lc.abs().amax(1)
        dual = torch.clamp(-lc.amin(1), min=0.0) / ln
        comp = (lc * slack).abs().amax(1) / (ln * sc)
        worst = max(worst, float(torch.stack([stat, prim, dual, comp]).max()))
    return worst
