"""Diagnostic: distance of the fused CG iterates (r.q read / conjugacy
identity) from the textbook recurrence and from each other, by iteration count."""
import os
import sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ["GG_KRON_FOLD_MIN"] = "8"
import torch
import oracle
import gp_grief_amd as gg


def rel(a, b):
    return float(np.linalg.norm(a - b) / np.linalg.norm(b))


for dims, s in (((30, 22, 14), 0.05), ((30, 22, 14), 2.0), ((24, 20, 16, 18), 0.05)):
    F = []
    for k, m in enumerate(dims):
        g = np.linspace(0.0, 1.0, m)
        F.append(oracle.cov_1d("RBF", g, g, 1.0, 0.15 * (1 + 0.05 * k)) + 1e-12 * np.eye(m))
    K = gg.tensors.KronMatrix(F, sym=True)
    n = int(np.prod(dims))
    b = torch.tensor(np.random.default_rng(11).standard_normal(n), device="cuda")
    for its in (5, 10, 15, 25):
        xs = {}
        for name, kw in (("tb", dict(recurrence="textbook")), ("rq0", dict(rq=0)),
                         ("rq1", dict(rq=1))):
            cg = gg.linalg.KronCG(K, s, **kw)
            cg.start(b, rtol=0.0)
            cg.iterate(its)
            xs[name] = cg.x.cpu().numpy()
        print(dims, s, its, "rq0-tb %.2e rq1-tb %.2e rq1-rq0 %.2e" % (
            rel(xs["rq0"], xs["tb"]), rel(xs["rq1"], xs["tb"]), rel(xs["rq1"], xs["rq0"])),
            flush=True)
