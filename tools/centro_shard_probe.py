"""Per-rank compute of the parity-sharded CG (one rank's local operator), on
ONE GPU: for G = 2^K ranks, factors 0..K-1 of the 200^4 operator are split
into their even / odd (centrosymmetric) halves S_k, T_k (h x h), and rank g's
block of the operator is X_0 x ... x X_{K-1} x K_K x ... x K_{d-1} (X_k = S_k
or T_k by bit k of g).  Times the fused CG on that local operator (the
all-reduce of the dot products is not included).

usage: python tools/centro_shard_probe.py [--grid 200] [--dims 4] [--steps 10]
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def halves(F):
    m = F.shape[0]
    h = m // 2
    A = F[:h, :h]
    B = F[:h, m - 1:h - 1:-1]   # B[j, i] = F[j, m-1-i]
    return A + B, A - B


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=200)
    ap.add_argument("--dims", type=int, default=4)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--rotate", type=int, default=0,
                    help="1: the unsharded (folded) factors first in the local operator")
    a = ap.parse_args()
    import torch
    import bench
    import gp_grief_amd as gg
    from gp_grief_amd import linalg
    m, d = a.grid, a.dims
    _, F = bench.grid_factors(m, d)
    for G in [int(v) for v in a.worlds.split(",")]:
        K = int(round(np.log2(G)))
        for g in ([0, G - 1] if G > 1 else [0]):
            loc = []
            for k in range(d):
                if k < K:
                    S, T = halves(F[k])
                    loc.append(T if (g >> (K - 1 - k)) & 1 else S)
                else:
                    loc.append(F[k])
            if a.rotate:
                loc = loc[K:] + loc[:K]
            Kl = gg.tensors.KronMatrix([np.ascontiguousarray(f) for f in loc])
            n = int(np.prod([f.shape[0] for f in loc]))
            y = torch.ones(n, dtype=torch.float64, device="cuda")
            cg = linalg.KronCG(Kl, 0.01)
            cg.start(y, rtol=0.0, atol=0.0)
            cg.iterate(2)
            torch.cuda.synchronize()
            cg.profile(True)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            cg.iterate(a.steps)
            e1.record()
            torch.cuda.synchronize()
            nm, per = cg.profile_read()
            fm = Kl._device().fold_mask()
            print(json.dumps({"G": G, "rank": g, "rotate": a.rotate, "local_shape": [f.shape[0] for f in loc],
                              "fold_mask": fm, "ms_per_iteration": e0.elapsed_time(e1) / a.steps,
                              "launch_ms": [v / max(nm, 1) for v in per]}), flush=True)
            del cg, Kl, y
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
