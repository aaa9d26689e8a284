"""Debug helper: fused / textbook CG iteration counts on small folded grids."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import oracle  # noqa: E402


def main():
    import gp_grief_amd as gg
    ms = [int(v) for v in sys.argv[1].split(",")]
    F = [oracle.cov_1d("RBF", np.linspace(0, 1, m), np.linspace(0, 1, m), 1.0,
                       0.15 * (1 + 0.05 * k)) + 1e-12 * np.eye(m) for k, m in enumerate(ms)]
    K = gg.tensors.KronMatrix(F, sym=True)
    n = int(np.prod(ms))
    b = np.random.default_rng(3).standard_normal((n, 1))
    s = 0.05
    out = {"ms": ms, "fold_mask": K._device().fold_mask(),
           "xdefer_env": os.environ.get("GG_CG_XDEFER")}
    for rec in ("fused", "textbook"):
        for rep in range(2):
            x, info = gg.linalg.cg(K, b, shift=s, rtol=1e-10, recurrence=rec)
            out["%s_%d" % (rec, rep)] = (int(info), int(gg.linalg.cg.last.iters))
    xo, _, ito = oracle.cg_solve(lambda v: oracle.kron_matvec(F, v) + s * v, b[:, 0], rtol=1e-10)
    out["oracle"] = int(ito)
    print(out, flush=True)


if __name__ == "__main__":
    main()
