"""Device Cholesky (gg_potrf) against the vendor factor at several sizes, with
the look-ahead stream on and off (GG_POTRF_LOOKAHEAD).  Debug / tuning aid.
Prints one JSON line per (p, lookahead)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    from gp_grief_amd import dense
    import gp_grief_amd as gg
    sizes = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else
                              "300,1000,2500,5000,7500,10000").split(",")]
    print(json.dumps({"stream_priority_range": list(torch.cuda.Stream.priority_range())}),
          flush=True)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(0)
    for p in sizes:
        n = max(2 * p, 4000)
        Phi = torch.randn((n, p), dtype=torch.float64, device="cuda", generator=gen) / np.sqrt(n)
        P = Phi.t() @ Phi + 0.01 * torch.eye(p, dtype=torch.float64, device="cuda")
        del Phi
        Lv = torch.linalg.cholesky(P)
        for la in ("0", "1"):
            os.environ["GG_POTRF_LOOKAHEAD"] = la
            gg.native.knobs_reload()
            rec = {"p": p, "lookahead": int(la)}
            try:
                ch = dense.Cholesky(P.clone())
                L = torch.tril(ch.L)
                rec["rel_err_vs_vendor"] = float((L - Lv).abs().max() / Lv.abs().max())
                rec["ok"] = True
            except Exception as e:  # noqa: BLE001
                rec["ok"] = False
                rec["error"] = str(e)[:200]
            print(json.dumps(rec), flush=True)
        del P, Lv
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
