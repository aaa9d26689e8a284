"""P2 dense-kernel microbenchmarks on one MI355X (tuning aid, not a product path).

Times, with HIP events on torch's current stream, at the GRIEF config shapes:
  gram    A = Phi^T Phi, Phi n x p row-major: gp_grief_amd.dense.matmul
          (ta=True, lower triangle: n p^2 FLOP) and, for reference, the
          vendor library behind torch.matmul (full product: 2 n p^2 FLOP)
  potrf   gp_grief_amd.dense.Cholesky(P) vs torch.linalg.cholesky(P)
  potrs   Cholesky.solve (forward + backward) for one right-hand side
  eig     gp_grief_amd.tensors.device_sym_eig on d factors of size m
Usage: python tools/p2_kernels_bench.py [--shapes 100000x1000,100000x5000,...]
Prints one JSON line per measurement.
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timed(torch, fn, reps=3):
    fn()
    torch.cuda.synchronize()
    best = None
    for _ in range(reps):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        best = ms if best is None else min(best, ms)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="100000x1000,100000x5000,100000x10000")
    ap.add_argument("--what", default="gram,potrf,potrs,eig")
    ap.add_argument("--vendor", action="store_true", help="also time torch's library calls")
    a = ap.parse_args()
    import torch
    import gp_grief_amd as gg
    from gp_grief_amd import dense
    what = a.what.split(",")
    gen = torch.Generator(device="cuda")
    gen.manual_seed(0)
    for sh in a.shapes.split(","):
        n, p = [int(v) for v in sh.split("x")]
        Phi = torch.randn((n, p), dtype=torch.float64, device="cuda", generator=gen) / np.sqrt(n)
        if "gram" in what:
            A = torch.zeros((p, p), dtype=torch.float64, device="cuda")
            ms = timed(torch, lambda: dense.matmul(Phi, Phi, ta=True, C=A, uplo=1))
            rec = {"what": "gram", "n": n, "p": p, "ms": ms,
                   "tflops": n * p * p / ms / 1e9, "flop_rule": "n p^2 (lower triangle)"}
            if a.vendor:
                msv = timed(torch, lambda: torch.matmul(Phi.t(), Phi))
                rec.update(vendor_ms=msv, vendor_tflops=2.0 * n * p * p / msv / 1e9)
            print(json.dumps(rec), flush=True)
        if "potrf" in what or "potrs" in what:
            A = dense.matmul(Phi, Phi, ta=True)
            P = A + 0.01 * torch.eye(p, dtype=torch.float64, device="cuda")
            del A
            ch = [None]

            def f():
                ch[0] = dense.Cholesky(P)
            ms = timed(torch, f)
            rec = {"what": "potrf", "p": p, "ms": ms, "tflops": p ** 3 / 3.0 / ms / 1e9}
            if a.vendor:
                msv = timed(torch, lambda: torch.linalg.cholesky(P))
                rec.update(vendor_ms=msv, vendor_tflops=p ** 3 / 3.0 / msv / 1e9)
            L = torch.tril(ch[0].L)
            err = float((L @ L.t() - torch.tril(P) - torch.tril(P, -1).t()).abs().max()
                        / P.abs().max())
            rec["rel_err"] = err
            print(json.dumps(rec), flush=True)
            if "potrs" in what:
                b = torch.randn(p, dtype=torch.float64, device="cuda", generator=gen)
                ms = timed(torch, lambda: ch[0].solve(b, which=3))
                print(json.dumps({"what": "potrs", "p": p, "ms": ms}), flush=True)
                ms = timed(torch, lambda: ch[0].inverse_diag(), reps=1)
                print(json.dumps({"what": "inverse_diag", "p": p, "ms": ms}), flush=True)
            del P, ch
        del Phi
        torch.cuda.empty_cache()
    if "eig" in what:
        from gp_grief_amd.tensors import device_sym_eig
        for m, d in ((128, 3), (64, 6), (32, 8), (200, 4)):
            g = np.linspace(0, 1, m)
            F = [np.exp(-0.5 * (g[:, None] - g[None, :]) ** 2 / (0.2 * (1 + 0.05 * i)) ** 2)
                 + 1e-12 * np.eye(m) for i in range(d)]
            ms = timed(torch, lambda: device_sym_eig(F))
            print(json.dumps({"what": "eig", "m": m, "d": d, "ms": ms}), flush=True)


if __name__ == "__main__":
    main()
