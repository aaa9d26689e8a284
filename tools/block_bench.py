"""Block-basis operator and CG at 200^4: per-launch HIP-event
times of the matvec and of the fused CG iteration, one JSON line per leg.

  python tools/block_bench.py [--m 200] [--d 4] [--reps 5] [--iters 20] [--grid-cg]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--m", type=int, default=200)
    ap.add_argument("--d", type=int, default=4)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--grid-cg", action="store_true", help="also time the grid-basis CG")
    ap.add_argument("--no-matvec", action="store_true")
    ap.add_argument("--no-cg", action="store_true")
    ap.add_argument("--no-grid", action="store_true", help="skip the grid-basis matvec")
    a = ap.parse_args()
    import torch
    import gp_grief_amd as gg
    m, d = a.m, a.d
    g = np.linspace(0.0, 1.0, m)
    F = []
    for k in range(d):
        ell = 0.1 * (1 + 0.05 * k)
        F.append(np.exp(-0.5 * (g[:, None] - g[None, :]) ** 2 / ell ** 2) + 1e-12 * np.eye(m))
    K = gg.tensors.KronMatrix(F, sym=True)
    dk = K._device()
    ok, n, L = dk.block_info()
    out = {"m": m, "d": d, "block": ok, "launches": L, "block_n": n, "grid_n": m ** d,
           "padding": n / float(m ** d) if ok else None}
    if not a.no_matvec and ok:
        x = torch.randn(n, dtype=torch.float64, device="cuda")
        y = torch.empty_like(x)
        dk.block_matvec(x, out=y)
        torch.cuda.synchronize()
        lm, tot = dk.block_matvec_timed(x, y, a.reps)
        out["block_matvec_ms"] = tot / a.reps
        out["block_launch_ms"] = [v / a.reps for v in lm]
        if not a.no_grid:
            # plain grid-basis matvec for comparison
            xg = torch.randn(m ** d, dtype=torch.float64, device="cuda")   # grid layout
            y2 = torch.empty_like(xg)
            lm2, tot2 = dk.matvec_timed(xg, y2, a.reps)
            out["grid_matvec_ms"] = tot2 / a.reps
            out["grid_launch_ms"] = [v / a.reps for v in lm2]
            del y2, xg
        del x, y
        dk.release_work()
        torch.cuda.empty_cache()
    bases = [] if a.no_cg else (["block"] if ok else []) + (["grid"] if a.grid_cg or not ok else [])
    for basis in bases:
        b = torch.randn(m ** d, dtype=torch.float64, device="cuda")   # the grid's N
        s = gg.linalg.KronCG(K, 0.01, basis=basis)
        s.start(b, rtol=1e-14)
        s.iterate(3, close=False)
        torch.cuda.synchronize()
        s.profile(True)
        t0 = time.perf_counter()
        s.iterate(a.iters, close=False)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        nm, ms = s.profile_read()
        s.profile(False)
        t2 = time.perf_counter()
        s.close()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        out["cg_%s" % basis] = {"ms_per_iter": 1e3 * (t1 - t0) / a.iters,
                                "launch_ms": [v / max(nm, 1) for v in ms],
                                "close_ms": 1e3 * (t3 - t2), "iters": s.status()[0]}
        del s, b
        torch.cuda.empty_cache()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
