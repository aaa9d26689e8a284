"""Time the pieces of GriefKernel._setup_inducing_cov at a GRIEF config (tuning
aid).  Usage: python tools/setup_profile.py [C2|C4|C5] [reps]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONF = {"C2": (3, 128, "RBF", 1000), "C4": (6, 64, "Matern52", 5000), "C5": (8, 32, "RBF", 10000)}


def main():
    import torch
    import gp_grief_amd as gg
    import gp_grief_amd.kern as kern_mod
    import gp_grief_amd.tensors as tens
    name = sys.argv[1] if len(sys.argv) > 1 else "C2"
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    d, m, kind, p = CONF[name]
    times = {}

    def wrap(mod, fname, key):
        f = getattr(mod, fname)

        def g(*a, **k):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = f(*a, **k)
            torch.cuda.synchronize()
            times.setdefault(key, []).append(1e3 * (time.perf_counter() - t0))
            return r
        import inspect
        if isinstance(inspect.getattr_static(mod, fname), staticmethod):
            g = staticmethod(g)
        setattr(mod, fname, g)

    wrap(kern_mod, "device_sym_eig_tridiag", "tridiag_values")
    wrap(kern_mod, "device_sym_eig_tridiag_vectors", "vectors")
    wrap(kern_mod, "device_sym_eig", "full_eig")
    for meth, key in (("cov_grid", "cov_grid"), ("_grid_factors_host", "factors"),
                      ("_select", "select"), ("_separated", "separated"),
                      ("_centro_vectors", "vectors_centro"),
                      ("_build_device_basis", "basis")):
        wrap(kern_mod.GriefKernel, meth, key)
    for r in range(reps):
        kl = [getattr(gg.kern, kind)(1, variance=1.0, lengthscale=0.2 * (1 + 0.05 * i))
              for i in range(d)]
        grid = gg.grid.InducingGrid(xg=[np.linspace(0, 1, m).reshape(-1, 1)] * d)
        k = gg.kern.GriefKernel(kern_list=kl, grid=grid, n_eigs=p)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        k._setup_inducing_cov()
        torch.cuda.synchronize()
        times.setdefault("setup_total", []).append(1e3 * (time.perf_counter() - t0))
    print(json.dumps({"config": name, **{k: round(min(v), 3) for k, v in times.items()}}))
    del tens


if __name__ == "__main__":
    main()
