"""Time the plain 200^4 Kronecker matvec (gg_kron_matvec, no CG fusions) on the
device, for kernel-trace / PMC runs of the mode products in isolation.

usage: python tools/matvec_bench.py [--reps 5] [--grid 200] [--dims 4]
Prints one JSON line: ms per matvec (HIP events) and the fold mask.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--grid", type=int, default=200)
    ap.add_argument("--dims", type=int, default=4)
    a = ap.parse_args()
    import torch
    import bench
    K, _ = bench.grid_factors(a.grid, a.dims)
    dk = K._device()
    n = a.grid ** a.dims
    x = bench.grid_rhs_device(a.grid, a.dims, torch, torch.device("cuda"))
    y = torch.empty_like(x)
    dk.matvec(x, out=y)
    torch.cuda.synchronize()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.reps):
        dk.matvec(x, out=y)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / a.reps
    print(json.dumps({"grid": a.grid, "dims": a.dims, "n": n, "ms_per_matvec": ms,
                      "fold_mask": dk.fold_mask(), "reps": a.reps}), flush=True)


if __name__ == "__main__":
    main()
