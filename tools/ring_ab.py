"""A/B of the folded plain mode product: the chunked kernel (GG_FOLD_RING=0)
against the ring variants (gg_kron_ring.hip) on the 200^4 operator, interleaved
in one process, outputs checked bitwise.  Prints one JSON line per run."""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    import bench
    m, d = int(os.environ.get("AB_M", 200)), int(os.environ.get("AB_D", 4))
    variants = os.environ.get("AB_VARIANTS", "0,1,2,3,4,5").split(",")
    rounds = int(os.environ.get("AB_ROUNDS", 2))
    K, F = bench.grid_factors(m, d)
    dev = torch.device("cuda", 0)
    x = bench.grid_rhs_device(m, d, torch, dev)
    dk = K._device()
    ref = None
    for r in range(rounds):
        for v in variants:
            os.environ["GG_FOLD_RING"] = v
            y = torch.empty_like(x)
            dk.matvec(x, out=y)
            per, tot = dk.matvec_timed(x, y, 5)
            if ref is None:
                ref = y.clone()
            same = bool(torch.equal(y, ref))
            print(json.dumps({"round": r, "variant": v, "ms": tot / 5,
                              "per_position": [round(t / 5, 3) for t in per],
                              "bitwise_equal": same}), flush=True)
            del y
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
