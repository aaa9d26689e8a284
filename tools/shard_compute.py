"""Per-rank compute of the factor-0-sharded CG iteration, measured on ONE GPU.

For G = 1, 2, 4, 8 this builds rank 0's gg_kron_dist handle of the 200^4
operator (HipEngine(F, G, 0)) and times, with HIP events on the compute
stream, everything rank 0's GPU does in one DistKronCG iteration except the
exchanges: phase 1 (mode products 1..d-1 on N/G elements, the CG direction
update fused into the first), phase 2 (factor 0 on N/G), the shift / p.q
pass and the x / r update pass.  The exchanges (2 all-to-alls of N/G
elements, 2 scalar all-reduces) need the other GPUs and are reported only as
the bytes each rank moves.  The compute-only ceiling of the strong-scaling
speedup is T_1(fused single-GPU iteration) / T_G(rank compute).

usage: python tools/shard_compute.py [--grid 200] [--dims 4] [--reps 5]
Prints one JSON line per G.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", type=int, default=200)
    ap.add_argument("--dims", type=int, default=4)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--worlds", default="1,2,4,8")
    a = ap.parse_args()
    import torch
    import bench
    from gp_grief_amd.distributed import HipEngine
    m, d = a.grid, a.dims
    _, F = bench.grid_factors(m, d)
    n = m ** d
    dev = torch.device("cuda")
    for G in [int(v) for v in a.worlds.split(",")]:
        eng = HipEngine(F, G, 0)
        nl = eng.n_local
        x = bench.local_rhs(m, d, G, 0, torch, dev)
        r = x.clone()
        p = eng.zeros()
        send, recv, q = eng.empty(), eng.empty(), eng.empty()
        xs = eng.zeros()
        eng.local_dot(r, r)
        eng.cg_init(0.0, 0.0)
        recv.copy_(x)                      # a stand-in for exchange #1's result
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
        tot = [0.0] * 4
        for rep in range(a.reps + 1):
            ev[0].record()
            eng.phase1(p, send, r=r)       # p = r + beta p fused; local factors 1..d-1
            ev[1].record()
            eng.phase2(recv, q)            # factor 0 on N/G
            ev[2].record()
            eng.shift_dot(q, p, 0.01)      # q += s p ; local p.q
            ev[3].record()
            eng.cg_alpha()
            eng.cg_update(xs, r, p, q)     # x += a p, r -= a q ; local r.r
            ev[4].record()
            torch.cuda.synchronize()
            if rep > 0:
                for k in range(4):
                    tot[k] += ev[k].elapsed_time(ev[k + 1])
        per = [t / a.reps for t in tot]
        print(json.dumps({"G": G, "n_local": nl, "fold_mask": eng.fold_mask,
                          "phase1_ms": per[0], "phase2_ms": per[1], "shift_dot_ms": per[2],
                          "update_ms": per[3], "rank_compute_ms": sum(per),
                          "exchange_bytes_per_rank": 2 * 8.0 * nl * (G - 1) / G,
                          "allreduce_per_iteration": 2 if G > 1 else 0}), flush=True)
        del eng, x, r, p, send, recv, q, xs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
