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

--recurrence fused (DistKronCG's default at d >= 4): phase 1 carries the CG
prologue (r -= alpha q_old, p = r + beta p, r.r and p.q_old partials) and
the deferred x update; after phase 2 one pass forms q += shift p with p.q and
q.q, and the scalars kernel runs on the (here: local) 5-double reduction.
--recurrence textbook: the separate shift / p.q and x / r passes.  The
exchange's stand-in (recv = the right-hand side) makes the iterates
meaningless, so the run reports whether the CG state stayed finite (a
stopped CG skips its kernels and its times would be void).

usage: python tools/shard_compute.py [--grid 200] [--dims 4] [--reps 5]
                                     [--recurrence fused|textbook|both]
Prints one JSON line per G and recurrence.
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
    ap.add_argument("--recurrence", default="both", choices=["fused", "textbook", "both"])
    a = ap.parse_args()
    recs = ["fused", "textbook"] if a.recurrence == "both" else [a.recurrence]
    import torch
    import bench
    from gp_grief_amd.distributed import HipEngine
    m, d = a.grid, a.dims
    _, F = bench.grid_factors(m, d)
    n = m ** d
    dev = torch.device("cuda")
    for G in [int(v) for v in a.worlds.split(",")]:
        for rec in recs:
            eng = HipEngine(F, G, 0)
            if rec == "fused" and not eng.supports_fused:
                print(json.dumps({"G": G, "recurrence": rec, "skipped": "engine cannot fuse"}))
                del eng
                continue
            print(json.dumps(run_one(a, eng, G, rec, m, d, torch, bench, dev)), flush=True)
            del eng
            torch.cuda.empty_cache()


def run_one(a, eng, G, rec, m, d, torch, bench, dev):
    nl = eng.n_local
    x = bench.local_rhs(m, d, G, 0, torch, dev)
    r = x.clone()
    send, recv, q = eng.empty(), eng.empty(), eng.zeros()
    xs = eng.zeros()
    eng.local_dot(r, r)
    eng.cg_init(0.0, 0.0)
    recv.copy_(x)                      # a stand-in for exchange #1's result
    if rec == "fused":
        names = ["phase1_ms", "phase2_ms", "post_ms", "scalars_ms"]
        pb = [eng.zeros() for _ in range(4)]
    else:
        names = ["phase1_ms", "phase2_ms", "shift_dot_ms", "update_ms"]
        p = eng.zeros()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(5)]
    tot = [0.0] * 4
    for rep in range(a.reps + 1):
        ev[0].record()
        if rec == "fused":
            p_old, p_new = pb[0], pb[1]
            eng.phase1_fused(p_old, p_new, send, r, q, xs, 0.01, False)   # prologue + x side
            ev[1].record()
            eng.phase2(recv, q)                                     # factor 0 on N/G
            ev[2].record()
            eng.fused_post(q, p_new, 0.01)                          # p.q', q'.q' (reads)
            ev[3].record()
            eng.fused_scalars(p_new)                                # (after the all-reduce)
            ev[4].record()
            pb[0], pb[1], pb[2], pb[3] = p_new, pb[3], p_old, pb[2]
        else:
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
    it, done, rho, _ = eng.cg_status()
    per = [t / a.reps for t in tot]
    out = {"G": G, "recurrence": rec, "n_local": nl, "fold_mask": eng.fold_mask}
    out.update(zip(names, per))
    out.update({"rank_compute_ms": sum(per),
                "exchange_bytes_per_rank": 2 * 8.0 * nl * (G - 1) / G,
                "allreduce_per_iteration": (1 if rec == "fused" else 2) if G > 1 else 0,
                "cg_state_valid": bool(not done and rho == rho)})
    return out

if __name__ == "__main__":
    main()
