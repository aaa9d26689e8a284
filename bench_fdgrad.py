"""Finite-difference LML gradient of GP-GRIEF with kernel-parameter
optimisation (basemodel.py:328-361 + gp_grief_model.py:53-68)
on one MI355X: the C2 problem (3-D 128^3 grid, RBF per dim, p = 1000,
n = 100k), opt_kernel_params=True, reweight_eig_funs=False, so one gradient =
1 + 7 LMLs (noise, 3 variances, 3 lengthscales), each with its own eigen-basis,
Phi, Gram and Cholesky.  Times the gradient with the perturbed bases'
eigendecompositions batched into one launch (GriefKernel.prefetch_eigs) and
with them computed one by one, and prints one JSON line."""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def main():
    import torch
    import gp_grief_amd as gg
    import gp_grief_amd.grid  # noqa: F401
    import gp_grief_amd.kern  # noqa: F401
    import gp_grief_amd.models  # noqa: F401
    d, m, p, n, s = 3, 128, 1000, 100000, 0.01
    x = np.random.default_rng(0).random((n, d))
    y = (np.sin(6.0 * x).sum(axis=1) + 0.1 * np.random.default_rng(1).standard_normal(n))
    y = y.reshape(-1, 1)
    out = {"metric": "finite-difference LML gradient (opt_kernel_params), C2",
           "unit": "ms per gradient", "higher_is_better": False, "n_gpus": 1, "dtype": "f64",
           "data": "synthetic",
           "config": {"workload": "C2: 3-D 128^3 RBF, p = 1000, n = 100000, 8 LMLs per gradient"}}
    for label, batched in (("batched_eigs", True), ("sequential_eigs", False)):
        times = []
        for rep in range(3):
            kl = [gg.kern.RBF(1, variance=1.0, lengthscale=0.2 * (1 + 0.05 * i)) for i in range(d)]
            grid = gg.grid.InducingGrid(xg=[np.linspace(0, 1, m).reshape(-1, 1)] * d)
            kern = gg.kern.GriefKernel(kern_list=kl, grid=grid, n_eigs=p,
                                       reweight_eig_funs=False, opt_kernel_params=True)
            if not batched:
                kern.prefetch_eigs = lambda sets: 0
            model = gg.models.GPGriefModel(x, y, kern, noise_var=s)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ll, g = model.log_likelihood(return_gradient=True)
            torch.cuda.synchronize()
            times.append((time.perf_counter() - t0) * 1e3)
        out[label + "_ms"] = min(times)
        out[label + "_lml"] = float(np.squeeze(ll))
    out["value"] = out["batched_eigs_ms"]
    out["speedup_vs_sequential"] = out["sequential_eigs_ms"] / out["batched_eigs_ms"]
    print(json.dumps(out))


if __name__ == "__main__":
    main()
