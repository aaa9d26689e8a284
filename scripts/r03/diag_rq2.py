"""Diagnostic: recursive vs true residual of the fused CG with each r.q source
(d = 3, 16 x 12 x 10, shift 1: test_cg_fused_state_is_textbook_after_iterate)."""
import os
import sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import oracle
import gp_grief_amd as gg

dims = (16, 12, 10)
F = []
for k, m in enumerate(dims):
    g = np.linspace(0.0, 1.0, m)
    F.append(oracle.cov_1d("RBF", g, g, 1.0, 0.15 * (1 + 0.05 * k)) + 1e-12 * np.eye(m))
K = gg.tensors.KronMatrix(F, sym=True)
n = int(np.prod(dims))
bh = np.random.default_rng(5).standard_normal(n)
b = torch.tensor(bh, device="cuda")
s = 1.0
print("fold mask", K._device().fold_mask())
for its in (2, 4, 8, 12, 16, 20, 25, 30):
    row = []
    for name, kw in (("tb", dict(recurrence="textbook")), ("rq0", dict(rq=0)), ("rq1", dict(rq=1))):
        cg = gg.linalg.KronCG(K, s, **kw)
        cg.start(b, rtol=0.0)
        cg.iterate(its)
        x = cg.x.cpu().numpy()
        rt = np.linalg.norm(bh - (oracle.kron_matvec(F, x) + s * x))
        row.append("%s rec %.6e true %.6e" % (name, cg.status()[2], rt))
    print(its, " | ".join(row), flush=True)
