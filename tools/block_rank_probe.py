"""Per-rank compute of the block-sharded CG, measured
alone on ONE MI355X: for G = 2^K ranks, rank g owns the operator's parity
blocks [g 2^d / G, (g + 1) 2^d / G) (distributed.BlockHipEngine ->
gg_cg_create_blocks) and runs the fused CG on them through the same
gg_cg_iterate_partial / _finish pair the sharded solve uses; the all-reduce
between them is replaced by nothing (the rank's local sums drive its scalars:
the CG of its own block system, the same kernels and the same bytes).  Rank 0
and rank G - 1 (whose blocks differ in parity: S / T factors) are timed per
launch with the library's HIP events, plus the once-per-solve fold of the
grid right-hand side into the rank's blocks and the unfold of its solution.

usage: python tools/block_rank_probe.py [--grid 200] [--dims 4] [--steps 20]
                                        [--worlds 1,2,4,8] > out.jsonl
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
    ap.add_argument("--sigma2", type=float, default=0.01)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--worlds", default="1,2,4,8")
    a = ap.parse_args()
    import torch
    import bench
    from gp_grief_amd.distributed import BlockHipEngine
    m, d, s = a.grid, a.dims, a.sigma2
    n = m ** d
    K, F = bench.grid_factors(m, d)
    dev = torch.device("cuda", 0)
    for G in [int(v) for v in a.worlds.split(",")]:
        for g in ([0, G - 1] if G > 1 else [0]):
            eng = BlockHipEngine(K, G, g, s)
            yg = bench.grid_rhs_device(m, d, torch, dev)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(6)]
            ev[0].record()
            y = eng.fold(yg)
            ev[1].record()
            del yg
            x = eng.zeros()
            eng.start_partial(y, x)
            eng.start_finish(0.0, 0.0)
            for _ in range(a.warmup):
                eng.iterate_partial()
                eng.iterate_finish()
            torch.cuda.synchronize()
            eng.profile(True)
            ev[2].record()
            for _ in range(a.steps):
                eng.iterate_partial()
                eng.iterate_finish()
            ev[3].record()
            torch.cuda.synchronize()
            nm, per = eng.profile_read()
            eng.profile(False)
            eng.close_partial()
            eng.close_finish()
            ev[4].record()
            xg = eng.unfold(x)
            ev[5].record()
            torch.cuda.synchronize()
            it = eng.status()[0]
            nl = eng.n_local
            launch = [v / max(nm, 1) for v in per]
            ms_it = ev[2].elapsed_time(ev[3]) / a.steps
            flops = bench.block_launch_flops(nl, m, d)
            passes = bench.block_launch_passes(d, eng.xwin, eng.rderive)
            dom = max(range(len(launch)), key=lambda i: launch[i])
            rec = {
                "G": G, "rank": g, "blocks": [eng.blk0, eng.nblk], "n_local": nl,
                "x_window": eng.xwin, "r_derived": eng.rderive, "iterations": it,
                "ms_per_iteration": ms_it, "launch_ms": launch,
                "launch_ms_source": "HIP events the library records around each launch "
                                    "(gg_cg_profile) over %d iterations" % a.steps,
                "iteration_algorithmic_bytes": 8.0 * nl * sum(passes),
                "iteration_hbm_gbs": 8.0 * nl * sum(passes) / (ms_it * 1e-3) / 1e9,
                "dominant_launch": {
                    "position": dom, "ms": launch[dom], "passes": passes[dom],
                    "frac_hbm": 8.0 * nl * passes[dom] / (launch[dom] * 1e-3) / 1e9
                                / bench.HBM_PEAK_GBS,
                    "frac_mfma": flops[dom] / (launch[dom] * 1e-3) / 1e12
                                 / bench.FP64_MFMA_PEAK_TFLOPS},
                "fold_ms": ev[0].elapsed_time(ev[1]),
                "unfold_ms": ev[4].elapsed_time(ev[5]),
                "allreduce": "not included (5 doubles per iteration on the real job)",
            }
            print(json.dumps(rec), flush=True)
            del eng, x, y, xg
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
