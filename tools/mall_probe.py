"""Copy bandwidth vs working-set size on one MI355X (tuning aid, not a product path).

A buffer pair of S bytes is copied back and forth (read S + write S per copy);
small pairs stay in the 256 MB memory-side cache, large ones stream from HBM.
The ratio tells whether keeping a mode-product intermediate cache-resident
(slabs of the 200^4 tensor) could beat the HBM pass cost.
Prints one JSON line per size.
"""
import json

import torch


def main():
    for mb in (16, 32, 64, 96, 128, 192, 256, 512, 2048, 8192):
        n = mb * (1 << 20) // 8
        a = torch.ones(n, dtype=torch.float64, device="cuda")
        b = torch.empty_like(a)
        reps = max(4, min(400, 40000 // mb))
        for _ in range(3):
            b.copy_(a)
        torch.cuda.synchronize()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for i in range(reps):
            if i & 1:
                a.copy_(b)
            else:
                b.copy_(a)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        print(json.dumps({"what": "copy", "mb": mb, "ms": ms,
                          "gbps_rw": 2.0 * n * 8 / ms / 1e6}), flush=True)
        del a, b
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
