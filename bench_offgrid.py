"""Off-grid posterior of the full-grid GP on one MI355X.

Workload: the C3 grid (4-D RBF 200^4, sigma^2 = 0.01, exact solve), M test
points off the grid.  One "step" = GPGridModel.predict(X*) = two device
Khatri-Rao contractions over the N = 1.6e9 grid (mean K(X*, grid) alpha and the
variance quadratic form), each 2 N M flop of FP64 MFMA GEMM plus a weighted
column sum that reads the GEMM output once (8 N M / m_{d-1} bytes).

Prints one JSON line: predictions/s, the GEMM roofline, and the CPU oracle
(oracle.kr_contract, NumPy) timed on a bounded sample of points.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=200)
    ap.add_argument("--dims", type=int, default=4)
    ap.add_argument("--points", type=int, default=1000)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--cpu-baseline", default="auto", choices=["auto", "off"])
    a = ap.parse_args()
    import torch
    import gp_grief_amd as gg
    import gp_grief_amd.kern  # noqa: F401
    import gp_grief_amd.models  # noqa: F401

    m, d, s, M = a.grid, a.dims, 0.01, a.points
    N = m ** d
    g = np.linspace(0.0, 1.0, m)
    ls = [0.1 * (1 + 0.05 * i) for i in range(d)]
    gk = gg.kern.GridKernel([gg.kern.RBF(1, variance=1.0, lengthscale=l) for l in ls])
    y = torch.randn(N, 1, dtype=torch.float64, device="cuda",
                    generator=torch.Generator(device="cuda").manual_seed(1))
    model = gg.models.GPGridModel([g.reshape(-1, 1)] * d, y, gk, noise_var=s, solver="exact")
    model.fit()
    xs = np.random.default_rng(2).uniform(0.0, 1.0, (M, d))
    for _ in range(a.warmup):
        model.predict(xs)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        mean, var = model.predict(xs)
    torch.cuda.synchronize()
    ms_step = (time.perf_counter() - t0) * 1e3 / a.steps

    # the mean contraction alone, timed with HIP events on torch's stream
    Kxz = gk.cov_kr(xs, model.xg)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    Kxz.contract(model._alpha)
    ev0.record()
    for _ in range(a.steps):
        Kxz.contract(model._alpha)
    ev1.record()
    torch.cuda.synchronize()
    ms_contract = ev0.elapsed_time(ev1) / a.steps
    flop = 2.0 * N * M
    out = {
        "metric": "off-grid GP posterior (mean + variance) on a %d-D %d^%d RBF grid" % (d, m, d),
        "value": M / (ms_step * 1e-3), "unit": "test points/s", "higher_is_better": True,
        "n_gpus": 1, "steps": a.steps, "warmup": a.warmup, "ms_per_step": ms_step,
        "dtype": "f64", "data": "synthetic",
        "config": {"workload": "C3 grid %d^%d, exact solve, M = %d off-grid points" % (m, d, M),
                   "grid": m, "dims": d, "points": M, "sigma2": s},
        "contract_ms": ms_contract,
        "roofline": {"bound": "mfma", "kernel": "gg_kr_contract (GEMM + weighted column sum)",
                     "achieved": flop / (ms_contract * 1e-3) / 1e12, "peak": 78.6,
                     "unit": "TFLOP/s", "frac": flop / (ms_contract * 1e-3) / 1e12 / 78.6,
                     "flop_per_contract": flop,
                     "gemm_output_bytes_per_contract": 8.0 * N * M / m * 2},
    }
    if a.cpu_baseline == "auto":
        import oracle
        alpha = model._alpha.cpu().numpy()
        blocks = [b for b in Kxz.A]
        k = 2
        t0 = time.perf_counter()
        oracle.kr_contract([b[:k] for b in blocks], alpha)
        dt = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": k / dt / 2.0, "unit": "test points/s",
                               "cores": int(os.environ.get("OMP_NUM_THREADS", os.cpu_count())),
                               "kind": "port",
                               "sample": "oracle.kr_contract (NumPy tensordot) on %d points, "
                                         "mean only, halved for mean + variance: %.1f s"
                                         % (k, dt)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
