"""Interleaved A/B of the plain folded mode-product variants (GG_FOLD_VARIANT)
on the 200^4 Kronecker matvec, in one process: per round and variant, the
mean ms per matvec over --reps (HIP events) and the max relative difference of
its output against variant 0 (the variants reorder nothing in the sums: the
check is bitwise in practice).

usage: python tools/fold_variant_ab.py --variants 0,8,9,10 --rounds 3
Prints one JSON line per (round, variant).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="0,8,9,10")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--grid", type=int, default=200)
    ap.add_argument("--dims", type=int, default=4)
    a = ap.parse_args()
    import torch
    import bench
    K, _ = bench.grid_factors(a.grid, a.dims)
    dk = K._device()
    x = bench.grid_rhs_device(a.grid, a.dims, torch, torch.device("cuda"))
    y = torch.empty_like(x)
    ref = torch.empty_like(x)
    os.environ["GG_FOLD_VARIANT"] = "0"
    dk.matvec(x, out=ref)
    torch.cuda.synchronize()
    scale = float(ref.abs().max())
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    for rnd in range(a.rounds):
        for v in a.variants.split(","):
            os.environ["GG_FOLD_VARIANT"] = v
            dk.matvec(x, out=y)
            torch.cuda.synchronize()
            err = float((y - ref).abs().max()) / scale
            e0.record()
            for _ in range(a.reps):
                dk.matvec(x, out=y)
            e1.record()
            torch.cuda.synchronize()
            print(json.dumps({"round": rnd, "variant": v,
                              "ms_per_matvec": e0.elapsed_time(e1) / a.reps,
                              "rel_diff_vs_v0": err}), flush=True)
    os.environ["GG_FOLD_VARIANT"] = "0"


if __name__ == "__main__":
    main()
