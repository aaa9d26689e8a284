"""Phase timing of gg_potrf's block chain (tuning aid, not a product path).

Runs dense.Cholesky(P) at each size with GG_POTRF_PROF set, reads the per-
workgroup stamps the block kernel writes (100 MHz clock: start, after the
in-panel update, after the 64 x 64 factor, after the TRSM stores) and prints
one JSON line per size: the factor time, the block-launch spans by position
in the panel, the mean phase times and the gap between consecutive block
launches (first start of launch b + 1 minus last end of launch b).
Usage: python tools/potrf_prof.py [p,...] [--lookahead 0|1]
"""
import argparse
import json
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def analyse(path):
    raw = np.fromfile(path, dtype=np.int64)
    nblk, G, K = (int(v) for v in raw[:3])
    st = raw[3:].reshape(nblk, G, K).astype(np.float64) / 100.0   # us
    out = {"nblk": nblk, "blocks": []}
    prev_end = None
    for b in range(nblk):
        s = st[b]
        live = s[:, 0] > 0
        s = s[live]
        if len(s) == 0:
            continue
        start = s[:, 0].min()
        ends = np.where(s[:, 3] > 0, s[:, 3], s[:, 2])
        end = ends.max()
        rec = {"b": b, "wgs": int(live.sum()), "span_us": end - start,
               "update_us": float(np.mean(s[:, 1] - s[:, 0])),
               "factor_us": float(np.mean(s[:, 2] - s[:, 1])),
               "trsm_us": float(np.mean((s[:, 3] - s[:, 2])[s[:, 3] > 0])) if (s[:, 3] > 0).any() else 0.0,
               "start_skew_us": float(s[:, 0].max() - start),
               "gap_us": None if prev_end is None else float(start - prev_end)}
        prev_end = end
        out["blocks"].append(rec)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("sizes", nargs="?", default="10000")
    ap.add_argument("--lookahead", default="1")
    ap.add_argument("--dump", action="store_true", help="print every block")
    a = ap.parse_args()
    os.environ["GG_POTRF_LOOKAHEAD"] = a.lookahead
    import torch
    from gp_grief_amd import dense, native
    gen = torch.Generator(device="cuda")
    gen.manual_seed(0)
    for p in [int(v) for v in a.sizes.split(",")]:
        n = max(2 * p, 4000)
        Phi = torch.randn((n, p), dtype=torch.float64, device="cuda", generator=gen) / np.sqrt(n)
        P = dense.matmul(Phi, Phi, ta=True)
        P = torch.tril(P) + torch.tril(P, -1).t() + 0.01 * torch.eye(p, dtype=torch.float64, device="cuda")
        del Phi
        dense.Cholesky(P.clone())   # warm
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        ch = dense.Cholesky(P.clone())
        e1.record()
        torch.cuda.synchronize()
        ms_plain = e0.elapsed_time(e1)
        fd, path = tempfile.mkstemp(suffix=".bin")
        os.close(fd)
        os.environ["GG_POTRF_PROF"] = path
        native.knobs_reload()
        ch = dense.Cholesky(P.clone())
        torch.cuda.synchronize()
        del os.environ["GG_POTRF_PROF"]
        native.knobs_reload()
        res = analyse(path)
        os.unlink(path)
        L = torch.tril(ch.L)
        err = float((L @ L.t() - P).abs().max() / P.abs().max())
        bl = res["blocks"]
        pos = {}
        for r in bl:
            pos.setdefault(r["b"] % 4, []).append(r)
        summ = {"p": p, "ms": ms_plain, "rel_err": err, "lookahead": int(a.lookahead),
                "chain_span_ms": sum(r["span_us"] for r in bl) / 1e3,
                "gaps_ms": sum(r["gap_us"] or 0.0 for r in bl) / 1e3}
        for k, rs in sorted(pos.items()):
            summ["pos%d" % k] = {f: round(float(np.mean([r[f] for r in rs])), 2)
                                 for f in ("span_us", "update_us", "factor_us", "trsm_us",
                                           "start_skew_us")}
            summ["pos%d" % k]["gap_us"] = round(float(np.mean([r["gap_us"] or 0.0 for r in rs])), 2)
        print(json.dumps(summ), flush=True)
        if a.dump:
            for r in bl:
                print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in r.items()}))
        del P, ch
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
