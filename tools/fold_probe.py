"""Parity-block fold / unfold timing at 200^4 on one MI355X (tuning aid):
gg_kron_block_fold forward / inverse over all 2^d blocks and
gg_kron_block_fold_range over 1/2, 1/4 and 1/8 of them, HIP events on the
library's stream, best of `reps` after one warm-up each.

usage: python tools/fold_probe.py [--grid 200] [--dims 4] [--reps 3] > out.jsonl
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
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch
    import bench
    m, d = a.grid, a.dims
    K, F = bench.grid_factors(m, d)
    dk = K._device()
    n = m ** d
    nblk_all = 1 << d
    dev = torch.device("cuda", 0)
    xg = bench.grid_rhs_device(m, d, torch, dev)

    def timed(fn):
        fn()
        torch.cuda.synchronize()
        best = None
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1)
            best = ms if best is None else min(best, ms)
        return best

    xb = dk.block_fold_range(xg, 0, nblk_all)
    yg = torch.empty_like(xg)
    for G in (1, 2, 4, 8):
        nb = nblk_all // G
        nl = n // G
        out_f = torch.empty(nl, dtype=torch.float64, device=dev)
        ms_f = timed(lambda: dk.block_fold_range(xg, 0, nb, out=out_f))
        ms_i = timed(lambda: dk.block_fold_range(xb[:nl], 0, nb, inverse=True, out=yg))
        rec = {"G": G, "blocks": nb, "fold_ms": ms_f, "unfold_ms": ms_i,
               "fold_bytes": 8.0 * (n + nl), "unfold_bytes": 8.0 * (nl + n),
               "fold_gbs": 8.0 * (n + nl) / ms_f / 1e6, "unfold_gbs": 8.0 * (nl + n) / ms_i / 1e6}
        print(json.dumps(rec), flush=True)
        del out_f
    err = float((dk.block_fold_range(xb, 0, nblk_all, inverse=True, out=yg) - xg).abs().max())
    print(json.dumps({"round_trip_max_abs_err": err}), flush=True)


if __name__ == "__main__":
    main()
