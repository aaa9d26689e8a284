"""Fidelity of the CPU baseline restatement (build container only).

bench.py's cpu_baseline times oracle.kron_matvec_dsymm -- the reference's
per-mode dsymm sequence (kron_matrix.py:74-96) restated -- because the
reference itself cannot travel to the GPU box.  This script times that
restatement against the reference's own KronMatrix.kronvec_prod on the same
factors and vector, here, at 100^4 and 150^4 (SURVEY 8d asks for +-15 %), and
checks the two agree numerically.  Writes profiles/r02_cpu_fidelity.json.

Imports /root/reference (through tests/golden/make_golden.import_reference),
so it never runs on the GPU box (.gpurunignore).
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))


def factors(m, d):
    import oracle
    g = np.linspace(0.0, 1.0, m)
    return [oracle.cov_1d("RBF", g, g, 1.0, 0.1 * (1 + 0.05 * (d - 1 - k))) + 1e-12 * np.eye(m)
            for k in range(d)]


def best_of(fn, reps):
    ts = []
    out = None
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        ts.append(time.perf_counter() - t0)
    return min(ts), ts, out


def main():
    from make_golden import import_reference
    import oracle
    gp = import_reference("/root/reference")
    from gp_grief.tensors import KronMatrix
    rows = []
    for m in (100, 150):
        d = 4
        F = factors(m, d)
        K = KronMatrix([np.asfortranarray(f) for f in F], sym=True)
        x = np.random.default_rng(1).standard_normal((m ** d, 1))
        t_ref, ts_ref, y_ref = best_of(lambda: K * x, 2)
        t_res, ts_res, y_res = best_of(lambda: oracle.kron_matvec_dsymm(F, x), 2)
        err = float(np.linalg.norm(y_res - y_ref[:, 0]) / np.linalg.norm(y_ref))
        rows.append({"grid": m, "dims": d, "n": m ** d,
                     "reference_kronvec_prod_s": t_ref, "reference_runs_s": ts_ref,
                     "restatement_dsymm_s": t_res, "restatement_runs_s": ts_res,
                     "ratio_restatement_over_reference": t_res / t_ref,
                     "rel_diff": err})
        print(json.dumps(rows[-1]), flush=True)
        del y_ref, y_res, x, K
    info = {"host": os.uname().nodename, "cpu_count": os.cpu_count(),
            "blas_threads": os.environ.get("OMP_NUM_THREADS", "default"),
            "note": "reference = gp_grief.tensors.KronMatrix.kronvec_prod imported from "
                    "/root/reference; restatement = oracle.kron_matvec_dsymm; best of 2 "
                    "runs each, same factors (bench.py recipe) and vector",
            "within_15pct": all(abs(r["ratio_restatement_over_reference"] - 1) <= 0.15
                                for r in rows),
            "rows": rows}
    out = os.path.join(ROOT, "profiles", "r02_cpu_fidelity.json")
    with open(out, "w") as f:
        json.dump(info, f, indent=1)
    print("wrote", out)
    del gp


if __name__ == "__main__":
    main()
