"""A/B the mode-product launch variants (GG_MP_VARIANT) on the m^d matvec,
interleaved in ONE process (cdna guide rule 24), on two inputs: N(0,1) data and
the bench's smooth grid right-hand side (clock / DVFS depends on the data).
Tuning tool only.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch
    import gp_grief_amd as gg
    import oracle
    from bench import grid_rhs_device
    m = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    d = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    variants = sys.argv[3].split(",") if len(sys.argv) > 3 else ["0", "1", "2", "3", "4"]
    rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    g = np.linspace(0, 1, m)
    F = [oracle.cov_1d("RBF", g, g, 1.0, 0.1 * (1 + 0.05 * k)) + 1e-12 * np.eye(m)
         for k in range(d)]
    K = gg.tensors.KronMatrix(F, sym=True)
    dev = torch.device("cuda")
    inputs = {"randn": torch.randn(m ** d, dtype=torch.float64, device=dev),
              "grid_rhs": grid_rhs_device(m, d, torch, dev)}
    y = torch.empty(m ** d, dtype=torch.float64, device=dev)
    res = {}
    for r in range(rounds):
        for v in variants:
            os.environ["GG_MP_VARIANT"] = v
            for name, x in inputs.items():
                K.matvec_device(x, shift=0.0, out=y)
                torch.cuda.synchronize()
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(3):
                    K.matvec_device(x, shift=0.0, out=y)
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1) / 3
                res.setdefault((v, name), []).append(ms)
    # every variant must give the same product (bitwise up to summation order)
    ref = None
    for v in variants:
        os.environ["GG_MP_VARIANT"] = v
        K.matvec_device(inputs["randn"], shift=0.0, out=y)
        torch.cuda.synchronize()
        if ref is None:
            ref = y.clone()
        err = float((y - ref).abs().max() / ref.abs().max())
        print(json.dumps({"variant": v, "max_rel_diff_vs_first": err}), flush=True)
        assert err < 1e-12, (v, err)
    for (v, name), ts in sorted(res.items()):
        ms = min(ts)
        print(json.dumps({"variant": v, "input": name, "matvec_ms_min": ms,
                          "matvec_ms_all": ts,
                          "tflops": 2.0 * m ** d * m * d / (ms * 1e-3) / 1e12}), flush=True)


if __name__ == "__main__":
    main()
