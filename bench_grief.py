"""P2 (GRIEF) fit benchmark: SURVEY 8(d) configs C2 / C4 / C5 on 1..N MI355X.

Not the driver's bench line (that is bench.py, the P1 200^4 CG).  This
measures the second half of the north star's hot path, GPGriefModel's fit
(gp_grief_model.py:78-87, 137-153, 203-245) and its adjoint gradient /
prediction, stage by stage with HIP events on the stream the C ABI launches
on:

  setup   GriefKernel._setup_inducing_cov: grid covariances, device Jacobi
          eigensolve of the d factors, host top-p selection (grief_kernel.py:168-190);
          its parts beside it: setup_factors (host covariances), setup_eigvals
          (device tridiagonalisation + bisection), setup_select (host top-p),
          setup_vectors (selected eigenvectors), setup_basis (device tables)
  phi     gg_grief_tables + gg_grief_phi (expand_SKC, tensors.py:97-128)
  gram    A = Phi^T Phi on FP64 MFMA (gp_grief_model.py:148), local rows
  reduce  the all-reduce of A over the ranks (RCCL; absent at N = 1)
  chol    P = A + diag(s/w), blocked potrf (:149-153)
  alpha   Woodbury solve (:228-235) + LML (:203-214)
  grad    adjoint gradient (:156-200)
  predict M = 1000 test points, mean + full M x M covariance (:89-125)
  cg      (--cg) the p-system solved instead by Jacobi-PCG with one RCCL
          all-reduce of p doubles per iteration (the "RCCL
          all-reduce CG" of C5): iterations, ms per iteration, alpha vs Cholesky

Inputs: xg_i = linspace(0, 1, m), x ~ U[0,1]^d (default_rng(0)),
n = 100 000, y = sum_i sin(6 x_i) + 0.1 eps (default_rng(1)), s = 0.01,
test points from default_rng(2); lengthscales 0.2 (1 + 0.05 i).  With N
ranks, rank g holds rows [g n / N, (g+1) n / N) (data-row sharding);
times are the max over ranks (strong scaling: n fixed).

Roofline per stage: gram is MFMA-bound (FLOP = n p^2, lower triangle only),
phi is HBM-bound (bytes = 8 n p written + 16 n U table reads).

cpu_baseline (N = 1 only): the oracle (NumPy/OpenBLAS restatement of the same
fit, oracle/grief.py) on a bounded row sample of the workload; the GPU fit on
the SAME sample is checked against it (LML relative difference reported).

Usage: python bench_grief.py [--gpus N] [--configs C2,C4,C5] [--repeats 3]
                             [--cpu auto|off] [--cg]
--gpus N > 1 without a launcher starts torch.distributed.run as a child.
Prints one JSON line per config (rank 0).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP64_MFMA_PEAK_TFLOPS = 78.6
HBM_PEAK_GBS = 8000.0

CONFIGS = {
    # name: (dims, m, kind, p, n, cpu sample rows)
    "C2": (3, 128, "RBF", 1000, 100000, 100000),
    "C4": (6, 64, "Matern52", 5000, 100000, 20000),
    "C5": (8, 32, "RBF", 10000, 100000, 10000),
}


def make_data(d, n, M=1000):
    x = np.random.default_rng(0).random((n, d))
    eps = np.random.default_rng(1).standard_normal(n)
    y = np.sin(6.0 * x).sum(axis=1) + 0.1 * eps
    xt = np.random.default_rng(2).random((M, d))
    return x, y.reshape(-1, 1), xt


def lengthscales(d):
    return [0.2 * (1.0 + 0.05 * i) for i in range(d)]


def build_model(gg, d, m, kind, p, x, y, s, comm=None, p_solver='chol'):
    kl = [getattr(gg.kern, kind)(1, variance=1.0, lengthscale=l) for l in lengthscales(d)]
    grid = gg.grid.InducingGrid(xg=[np.linspace(0, 1, m).reshape(-1, 1) for _ in range(d)])
    kern = gg.kern.GriefKernel(kern_list=kl, grid=grid, n_eigs=p)
    return gg.models.GPGriefModel(x, y, kern, noise_var=s, comm=comm, p_solver=p_solver)


class Stages(object):
    """HIP events on torch's current stream (the one the C ABI launches on)."""

    def __init__(self, torch):
        self.torch = torch
        self.ev = []

    def mark(self, name):
        e = self.torch.cuda.Event(enable_timing=True)
        e.record()
        self.ev.append((name, e))

    def read(self):
        self.torch.cuda.synchronize()
        out = {}
        for (n0, e0), (n1, e1) in zip(self.ev[:-1], self.ev[1:]):
            out[n1] = e0.elapsed_time(e1)
        return out


class Ctx(object):
    def __init__(self, torch, dist, world, rank):
        self.torch, self.dist, self.world, self.rank = torch, dist, world, rank

    def barrier(self):
        self.torch.cuda.synchronize()
        if self.dist is not None:
            self.dist.barrier()
        self.torch.cuda.synchronize()

    def max(self, v):
        if self.dist is None:
            return float(v)
        # through the host under gloo (the gloo-gpu rehearsal of bench.py)
        gloo = str(self.dist.get_backend()) == "gloo"
        t = self.torch.tensor([float(v)], dtype=self.torch.float64,
                              device="cpu" if gloo else "cuda")
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def comm(self):
        if self.dist is None:
            return None
        from gp_grief_amd.distributed import TorchExchange
        return TorchExchange()


def rows_of(ctx, n):
    b = np.linspace(0, n, ctx.world + 1).astype(int)
    return b[ctx.rank], b[ctx.rank + 1]


def gpu_fit(gg, ctx, d, m, kind, p, x, y, xt, s):
    """One cold fit through the public API, stage-timed. Returns (times ms, model, ll)."""
    torch = ctx.torch
    ctx.barrier()
    w0 = time.perf_counter()
    st = Stages(torch)
    st.mark("start")
    mdl = build_model(gg, d, m, kind, p, x, y, s, comm=ctx.comm())
    mdl.parameters                      # noqa: B018  (resolves dependent attributes)
    mdl.kern._stage_mark = st.mark      # setup_factors / _eigvals / _select / _vectors
    mdl.kern._setup_inducing_cov()
    mdl.kern._stage_mark = None
    st.mark("setup_basis")              # the device basis tables (_build_device_basis)
    mdl._w = mdl.kern.w
    xd = mdl._x_dev()                   # the host -> device copy of X (the boundary)
    st.mark("h2d")
    mdl._Phi = mdl.kern.phi_device(xd)
    st.mark("phi")
    A = torch.zeros((p, p), dtype=torch.float64, device=mdl._Phi.device)
    gg.dense.matmul(mdl._Phi, mdl._Phi, ta=True, C=A, uplo=mdl._gram_uplo)
    st.mark("gram")
    mdl._A = mdl._sum(A)
    st.mark("reduce")
    mdl._cov_setup()                    # A kept: P = A + diag(s/w), potrf
    st.mark("chol")
    ll = mdl.log_likelihood()           # alpha (Woodbury) + LML
    st.mark("alpha")
    ctx.barrier()
    wall_fit = ctx.max(time.perf_counter() - w0)
    ll2, grad = mdl.log_likelihood(return_gradient=True)
    st.mark("grad")
    mean, var = mdl.predict(xt)
    st.mark("predict")
    times = st.read()
    times = {k: ctx.max(v) for k, v in times.items()}
    # setup = the sum of its parts (factors on the host, device tridiagonal +
    # bisection eigenvalues, host top-p selection, selected eigenvectors,
    # device basis tables)
    times["setup"] = sum(v for k, v in times.items() if k.startswith("setup_"))
    times["fit_wall"] = 1e3 * wall_fit
    return times, mdl, float(np.squeeze(ll)), grad, mean, var


def cg_leg(gg, ctx, mdl_chol, d, m, kind, p, x, y, s):
    """The p-system by PCG (one p-vector all-reduce per iteration) on the same
    rows and basis; alpha against the Cholesky one."""
    torch = ctx.torch
    mdl = build_model(gg, d, m, kind, p, x, y, s, comm=ctx.comm(), p_solver='cg')
    mdl.kern = mdl_chol.kern            # same basis (eigen-selection already done)
    mdl.parameters                      # noqa: B018
    mdl._w = mdl.kern.w
    mdl._Phi = mdl_chol._Phi
    b = mdl._sum(gg.dense.matvec(mdl._Phi, mdl._y_dev(), trans=True))
    mdl._jacobi_diag(gg.device.to_device(s / np.asarray(mdl._w, dtype=np.float64)))
    ctx.barrier()
    t0 = time.perf_counter()
    z = mdl.solve_p_cg(b)
    ctx.barrier()
    dt = ctx.max(time.perf_counter() - t0)
    it = mdl.cg_iters[-1]
    zc = mdl_chol._Pchol.solve(b, which=3)
    err = float((z - zc).norm() / zc.norm())
    return {"iterations": it, "ms": 1e3 * dt, "ms_per_iteration": 1e3 * dt / max(it, 1),
            "allreduce_per_iteration": 1 if ctx.world > 1 else 0,
            "allreduce_bytes": 8 * p, "rtol": mdl.cg_rtol,
            "z_rel_diff_vs_cholesky": err}


def cpu_fit(d, m, kind, p, x, y, s):
    import oracle
    from oracle.grief import grief_inducing, grief_phi, grief_fit, grief_lml
    from bench import cpu_share
    threads, share = cpu_share()
    try:
        from threadpoolctl import threadpool_limits
        ctx = threadpool_limits(limits=threads)
    except Exception:  # pragma: no cover
        ctx = None
    specs = [(kind, 1.0, l) for l in lengthscales(d)]
    xg = [np.linspace(0, 1, m) for _ in range(d)]
    t0 = time.perf_counter()
    ind = grief_inducing(specs, xg, p)
    t1 = time.perf_counter()
    Phi = grief_phi(x, specs, xg, ind)
    t2 = time.perf_counter()
    fit = grief_fit(Phi, np.ones(ind["p"]), y, s)
    ll = grief_lml(fit, y)
    t3 = time.perf_counter()
    if ctx is not None:
        ctx.__exit__(None, None, None)
    del oracle
    return {"setup_s": t1 - t0, "phi_s": t2 - t1, "gram_chol_alpha_s": t3 - t2,
            "fit_s": t3 - t0, "threads": threads, "cpu_share": share, "lml": ll}


def run_config(gg, ctx, name, repeats, cpu, with_cg, s=0.01):
    torch = ctx.torch
    d, m, kind, p, n, n_cpu = CONFIGS[name]
    x, y, xt = make_data(d, n)
    lo, hi = rows_of(ctx, n)
    xl, yl = x[lo:hi], y[lo:hi]
    runs = []
    cg = None
    for r in range(repeats):
        times, mdl, ll, grad, mean, var = gpu_fit(gg, ctx, d, m, kind, p, xl, yl, xt, s)
        runs.append(times)
        U = mdl.kern._dev_basis["U"]
        uplo = mdl._gram_uplo
        if with_cg and r == repeats - 1:
            cg = cg_leg(gg, ctx, mdl, d, m, kind, p, xl, yl, s)
        del mdl
        torch.cuda.empty_cache()
    best = {k: min(rr[k] for rr in runs) for k in runs[0]}
    fit_ms = sum(best[k] for k in ("setup", "h2d", "phi", "gram", "reduce", "chol", "alpha"))
    n_rank = int(hi - lo)
    gram_flop = (1.0 if uplo else 2.0) * n_rank * p * p
    gram_tf = gram_flop / (best["gram"] * 1e-3) / 1e12
    phi_bytes = 8.0 * n_rank * p + 16.0 * n_rank * U
    phi_gbs = phi_bytes / (best["phi"] * 1e-3) / 1e9
    res = {
        "metric": "GRIEF fit (setup + Phi + Gram + all-reduce + Cholesky + alpha + LML)",
        "value": 1e3 / fit_ms, "unit": "fits/s", "fit_ms": fit_ms,
        "higher_is_better": True, "n_gpus": ctx.world, "dtype": "f64", "data": "synthetic",
        "scaling": "strong",
        "config": {"workload": name, "dims": d, "grid": m, "kernel": kind, "p": p, "n": n,
                   "rows_per_rank": n_rank, "sigma2": s, "U_selected_rows": U,
                   "repeats": repeats,
                   "parallelism": "single-gpu" if ctx.world == 1 else
                   "data rows x%d, Gram all-reduce (%s), replicated potrf"
                   % (ctx.world, "RCCL" if str(ctx.dist.get_backend()) == "nccl" else "gloo")},
        "stage_ms": best,
        "gram": {"bound": "mfma", "flop": gram_flop,
                 "flop_rule": "n p^2 per rank (lower triangle only)" if uplo
                 else "2 n p^2 (full GEMM)",
                 "achieved": gram_tf, "peak": FP64_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s",
                 "frac": gram_tf / FP64_MFMA_PEAK_TFLOPS},
        "phi": {"bound": "hbm", "bytes": phi_bytes, "achieved": phi_gbs,
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": phi_gbs / HBM_PEAK_GBS},
        "lml": ll,
    }
    if cg is not None:
        res["p_system_cg"] = cg
    if cpu and ctx.world == 1:
        xs, ys = x[:n_cpu], y[:n_cpu]
        c = cpu_fit(d, m, kind, p, xs, ys, s)
        # the GPU fit on the same sample, checked against the oracle
        t, mdl, ll_s, _, _, _ = gpu_fit(gg, ctx, d, m, kind, p, xs, ys, xt[:10], s)
        gpu_sample_ms = sum(t[k] for k in ("setup", "h2d", "phi", "gram", "reduce", "chol", "alpha"))
        res["cpu_baseline"] = {
            "value": 1.0 / c["fit_s"], "unit": "fits/s", "cores": c["threads"], "kind": "port",
            "host_cpu_count": os.cpu_count(), "cpu_share": c["cpu_share"],
            "sample": "oracle/grief.py fit on the first %d of the %d rows (NumPy/OpenBLAS, "
                      "%d threads): setup %.2f s, Phi %.2f s, Gram+chol+alpha %.2f s"
                      % (n_cpu, n, c["threads"], c["setup_s"], c["phi_s"],
                         c["gram_chol_alpha_s"]),
            "gpu_fit_ms_same_sample": gpu_sample_ms,
            "speedup_same_sample": c["fit_s"] * 1e3 / gpu_sample_ms,
            "lml_rel_diff_same_sample": abs(ll_s - c["lml"]) / abs(c["lml"]),
        }
        del mdl
        torch.cuda.empty_cache()
    return res


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--configs", default="C2,C4,C5")
    ap.add_argument("--repeats", type=int, default=3)
    ap.add_argument("--cpu", default="auto", choices=["auto", "off"])
    ap.add_argument("--cg", action="store_true")
    a = ap.parse_args()
    if os.environ.get("WORLD_SIZE") is None and a.gpus > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node",
               str(a.gpus), "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
               os.path.abspath(__file__)] + sys.argv[1:]
        sys.exit(subprocess.call(cmd))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    import torch
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
        dist.init_process_group("nccl")
    import gp_grief_amd as gg
    import gp_grief_amd.grid  # noqa: F401
    import gp_grief_amd.kern  # noqa: F401
    import gp_grief_amd.models  # noqa: F401
    gg.native.load()
    ctx = Ctx(torch, dist, world, rank)
    for name in a.configs.split(","):
        res = run_config(gg, ctx, name.strip(), a.repeats, a.cpu == "auto", a.cg)
        if rank == 0:
            print(json.dumps(res), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
