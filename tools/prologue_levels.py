"""Prologue-launch levels per CG workspace allocation.

In one process: build the 200^4 operator once, then for each trial allocate a
fresh CG workspace (linalg.KronCG; GG_CG_VEC_PAD = the trial's pad between
the CG vectors), run W warm-up + K profiled fused iterations and print the
per-position mode-product times with the workspace's virtual address.  A
level that follows the allocation but not the pad points at physical page
placement; one that follows the pad at the vectors' relative offsets.

usage: python tools/prologue_levels.py [--grid 200] [--pads 0,0,0,1024,...]
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
    ap.add_argument("--pads", default="0,0,0,0,256,256,4096,4096,262144,262144")
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--hold", type=int, default=0,
                    help="keep this many earlier workspaces alive (changes placement)")
    a = ap.parse_args()
    import torch
    import bench
    from gp_grief_amd import linalg
    m, d = a.grid, a.dims
    K, _ = bench.grid_factors(m, d)
    y = bench.local_rhs(m, d, 1, 0, torch, torch.device("cuda"))
    held = []
    for t, pad in enumerate(int(v) for v in a.pads.split(",")):
        os.environ["GG_CG_VEC_PAD"] = str(pad)
        cg = linalg.KronCG(K, 0.01)
        cg.start(y, rtol=0.0, atol=0.0)
        cg.iterate(a.warmup)
        cg.profile(True)
        cg.iterate(a.steps)
        nm, per = cg.profile_read()
        cg.profile(False)
        va = int(cg.work.data_ptr())
        print(json.dumps({"trial": t, "pad": pad, "va_hex": hex(va), "va_mod_2MiB": va % (2 << 20),
                          "va_mod_1GiB": va % (1 << 30),
                          "pos_ms": [v / max(nm, 1) for v in per]}), flush=True)
        if a.hold > 0:
            held.append(cg)
            held = held[-a.hold:]
        del cg
        torch.cuda.synchronize()
        if a.hold == 0:
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
