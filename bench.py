"""Benchmark: CG iterations/s on the 4-D RBF grid 200^4 (BASELINE.json configs[2]).

One "step" = one CG iteration on (K + s I) x = y, K = K_0 (x) K_1 (x) K_2 (x) K_3
(200 x 200 RBF factors, lengthscales 0.1*(1+0.05 i), jitter 1e-12, s = 0.01),
all vectors (y, x, r, p, q, matvec scratch: 6 x 12.8 GB) resident in HBM.

Prints ONE JSON line (rank 0):
  metric/value/unit   CG iterations per second, whole job
  roofline            the dominant kernel (the FP64 MFMA mode product) timed
                      with HIP events on the stream it runs on, against the
                      FP64 matrix peak; plus HBM GB/s of the whole matvec
  cpu_baseline        the CPU oracle (oracle/, NumPy + OpenBLAS) timed on this
                      host on a bounded sample of the same workload

  python bench.py [--gpus N] [--steps K] [--warmup W] [--grid 200] [--dims 4]
N > 1 is launched by torch.distributed.run (one process per GPU, RCCL): strong
scaling of the same single CG, factor 0 sharded over the ranks (two all-to-alls
per matvec, two scalar all-reduces per iteration); see DESIGN.md section 6.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

FP64_MFMA_PEAK_TFLOPS = 78.6   # MI355X FP64 matrix, dense (AMD spec)
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--grid", type=int, default=200)
    ap.add_argument("--dims", type=int, default=4)
    ap.add_argument("--sigma2", type=float, default=0.01)
    ap.add_argument("--cpu-baseline", default="auto", choices=["auto", "off"])
    ap.add_argument("--recurrence", default="fused", choices=["fused", "textbook"])
    return ap.parse_args()


def factors(m, d):
    import oracle  # factor construction only (m x m); the CPU leg below times it
    g = np.linspace(0.0, 1.0, m)
    return [oracle.cov_1d("RBF", g, g, 1.0, 0.1 * (1 + 0.05 * (d - 1 - k))) + 1e-12 * np.eye(m)
            for k in range(d)]


def grid_rhs_device(m, d, torch, dev, seed=1):
    """y = sum_i sin(6 xg_i) + 0.1 eps on the grid, built on the device."""
    g = torch.linspace(0.0, 1.0, m, dtype=torch.float64, device=dev)
    f = torch.sin(6.0 * g)
    y = torch.zeros([m] * d, dtype=torch.float64, device=dev)
    for k in range(d):
        shape = [1] * d
        shape[k] = m
        y += f.reshape(shape)
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed)
    y = y.reshape(-1)
    chunk = 1 << 27
    for i in range(0, y.numel(), chunk):
        n = min(chunk, y.numel() - i)
        y[i:i + n] += 0.1 * torch.randn(n, dtype=torch.float64, device=dev, generator=gen)
    return y


def local_rhs_device(m, d, world, rank, torch, dev, seed=1):
    """This rank's shard of the same right-hand side, in the sharded layout
    (m_1, ..., m_{d-1}, a) with a = i_0 - rank * m/world fastest."""
    s0 = m // world
    g = torch.linspace(0.0, 1.0, m, dtype=torch.float64, device=dev)
    f = torch.sin(6.0 * g)
    y = torch.zeros([m] * (d - 1) + [s0], dtype=torch.float64, device=dev)
    for k in range(d - 1):
        shape = [1] * d
        shape[k] = m
        y += f.reshape(shape)
    shape = [1] * d
    shape[d - 1] = s0
    y += f[rank * s0:(rank + 1) * s0].reshape(shape)
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed + 1000 * rank)
    y = y.reshape(-1)
    chunk = 1 << 27
    for i in range(0, y.numel(), chunk):
        n = min(chunk, y.numel() - i)
        y[i:i + n] += 0.1 * torch.randn(n, dtype=torch.float64, device=dev, generator=gen)
    return y


def run_sharded(a, world, rank, torch, dev, dist):
    """Strong scaling: one CG on the full grid, factor 0 sharded over ranks."""
    import gp_grief_amd as gg  # noqa: F401
    from gp_grief_amd.distributed import DistKronCG, HipEngine, TorchExchange
    m, d, s = a.grid, a.dims, a.sigma2
    F = factors(m, d)
    eng = HipEngine(F, world, rank)
    y = local_rhs_device(m, d, world, rank, torch, dev)
    ex = TorchExchange()
    mode = os.environ.get("GG_DIST_MODE", "auto")
    # every rank must take the same exchange: a push setup that fails on any
    # rank (IPC mapping of a peer's buffer) sends all ranks to all-to-all
    try:
        cg = DistKronCG(eng, ex, s, mode=mode)
        ok = 1.0
    except Exception as exc:  # noqa: BLE001
        print("rank %d: %s exchange setup failed (%s); using a2a" % (rank, mode, exc),
              file=sys.stderr, flush=True)
        cg, ok = None, 0.0
    flag = torch.tensor([ok], dtype=torch.float64, device=dev)
    dist.all_reduce(flag, op=dist.ReduceOp.MIN)
    if float(flag.item()) < 1.0:
        cg = DistKronCG(eng, ex, s, mode="a2a")
    if cg.mode == "push":
        # one matvec through the peer-memory exchange against the all-to-all
        # path on the same input; any disagreement falls back to all-to-all
        ref = DistKronCG(eng, ex, s, mode="a2a")
        ya, yp = eng.empty(), eng.empty()
        ref.apply(y.clone(), ya)
        cg.apply(y.clone(), yp)
        err = torch.stack([(ya - yp).abs().max(), ya.abs().max()])
        dist.all_reduce(err, op=dist.ReduceOp.MAX)
        del ref, ya, yp
        if not float(err[0]) <= 1e-12 * float(err[1]):
            cg = DistKronCG(eng, ex, s, mode="a2a")
        torch.cuda.empty_cache()
    cg.start(y, rtol=0.0, atol=0.0)
    cg.iterate(a.warmup)
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    cg.iterate(a.steps)
    torch.cuda.synchronize()
    dist.barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    it, done, rho, tol = cg.status()
    assert it == a.warmup + a.steps and np.isfinite(rho), (it, rho)
    n = m ** d
    return {
        "metric": "CG iters/sec + Kron-matvec achieved HBM GB/s, 4D RBF grid 200^4",
        "value": a.steps / dt,
        "unit": "CG iters/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": 1e3 * dt / a.steps,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {"workload": "4D RBF grid %d^%d, CG on (K + %g I) x = y, N = %d, factor 0 "
                               "sharded over %d GPUs" % (m, d, s, n, world),
                   "grid": m, "dims": d, "sigma2": s, "n": n,
                   "exchange": cg.mode,
                   "parallelism": ("shard factor-0 x%d: matvec exchange by %s, 2 scalar "
                                   "all-reduce per iteration (RCCL)"
                                   % (world, "peer-memory stores in the mode-product "
                                             "epilogues + 2 RCCL barriers"
                                      if cg.mode == "push" else "2 RCCL all-to-all"))},
    }


KERNEL_NAME = "gg::mode_product_kernel<13, 4, 3, 0, 3, true, 1, 2, 0>"


def pmc_traffic(m, d):
    """HBM bytes per launch of the dominant kernel from the committed PMC
    passes (tools/pmc_traffic.py), if they were taken on this kernel and
    workload; else None."""
    path = os.path.join(ROOT, "profiles", "r01_pmc_mode_product.json")
    if (m, d) != (200, 4) or not os.path.exists(path):
        return None, None
    rec = json.load(open(path))
    if KERNEL_NAME.replace("gg::", "") not in str(rec.get("kernel")):
        return None, None
    return rec["traffic_bytes"], os.path.relpath(path, ROOT)


def cpu_baseline(m, d, sigma2):
    """One CG iteration of the CPU oracle at the full grid (bounded sample)."""
    import oracle
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    try:
        from threadpoolctl import threadpool_limits
        ctx = threadpool_limits(limits=threads)
    except Exception:  # pragma: no cover
        ctx = None
    F = factors(m, d)
    n = m ** d
    rng = np.random.default_rng(1)
    block = rng.standard_normal(m ** min(d, 3))
    b = np.tile(block, n // block.size)
    mv = lambda v: oracle.kron_matvec(F, v) + sigma2 * v
    t0 = time.perf_counter()
    x, info, it = oracle.cg_solve(mv, b, rtol=0.0, maxiter=1)
    dt = time.perf_counter() - t0
    del x, b
    if ctx is not None:
        ctx.__exit__(None, None, None)
    return {"value": 1.0 / dt, "unit": "CG iters/s", "cores": threads, "kind": "port",
            "sample": "1 CG iteration of oracle.cg_solve on the full %d^%d grid "
                      "(NumPy/OpenBLAS, %d threads), %.1f s" % (m, d, threads, dt)}


def main():
    a = parse()
    import torch
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")
    else:
        dist = None
    dev = torch.device("cuda", torch.cuda.current_device())
    import gp_grief_amd as gg
    if world > 1:
        res = run_sharded(a, world, rank, torch, dev, dist)
        if rank == 0:
            print(json.dumps(res), flush=True)
        dist.destroy_process_group()
        return

    m, d, s = a.grid, a.dims, a.sigma2
    F = factors(m, d)
    K = gg.tensors.KronMatrix(F, sym=True)
    n = m ** d
    y = grid_rhs_device(m, d, torch, dev)
    solver = gg.linalg.KronCG(K, s, recurrence=a.recurrence)
    solver.start(y, rtol=0.0, atol=0.0)   # never "converges": exactly the steps asked for
    torch.cuda.synchronize()

    # ---- CG: warmup, then exactly `steps` iterations bracketed by barrier+sync
    solver.iterate(a.warmup, check_every=0)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    # live kernel timing: HIP events around every mode product of the timed
    # iterations, recorded by the library on the stream the kernels run on
    solver.profile(True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    solver.iterate(a.steps, check_every=0)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    dt = time.perf_counter() - t0
    n_mv, mode_ms = solver.profile_read()
    solver.profile(False)
    assert n_mv == a.steps, (n_mv, a.steps)
    if dist is not None:
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    it, conv, res, tol = solver.status()
    assert it == a.warmup + a.steps, (it, a.warmup, a.steps)
    assert np.isfinite(res)

    # dominant kernel: the plain mode product.  Positions of a matvec: 0 is the
    # CG-fused first product (prologue), 1 carries the fused x-update side
    # job, d-1 the fused epilogue (shift, p.q / r.q / q.q); the plain ones are
    # 1..d-2 (textbook) or 2..d-2 (fused).
    per_pos = [t / n_mv for t in mode_ms]
    plain = list(range(2 if solver.recurrence == "fused" else 1, d - 1)) or [d - 1]
    launch_ms = sum(per_pos[k] for k in plain) / len(plain)
    mv_ms = sum(per_pos)
    flop_launch = 2.0 * n * m
    achieved_tf = flop_launch / (launch_ms * 1e-3) / 1e12
    traffic, traffic_src = pmc_traffic(m, d)
    # algorithmic HBM bytes of one iteration (8 B per element per pass):
    # d mode products read + write 2N each; CG vectors (textbook) p-update
    # r, p -> p 3N; +s p / p.q read p 1N; x/r update 6N.  Fused: the same
    # vector passes ride on the mode products (first: r, q, p -> r, p; second:
    # x, p -> x; last: p, r): 10N either way (+ one closing update per
    # iterate() call in the fused case).
    mv_bytes = 8.0 * n * (2 * d + 1)
    it_bytes = 8.0 * n * (2 * d + 10)
    result = {
        "metric": "CG iters/sec + Kron-matvec achieved HBM GB/s, 4D RBF grid 200^4",
        "value": a.steps / dt,
        "unit": "CG iters/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": 1e3 * dt / a.steps,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {"workload": "4D RBF grid %d^%d, CG on (K + %g I) x = y, N = %d"
                               % (m, d, s, n),
                   "grid": m, "dims": d, "sigma2": s, "n": n,
                   "cg_recurrence": solver.recurrence,
                   "parallelism": "single-gpu"},
        "roofline": {"bound": "mfma", "achieved": achieved_tf, "peak": FP64_MFMA_PEAK_TFLOPS,
                     "unit": "TFLOP/s", "frac": achieved_tf / FP64_MFMA_PEAK_TFLOPS,
                     "traffic": traffic, "traffic_unit": "bytes per launch",
                     "traffic_source": traffic_src,
                     "kernel": KERNEL_NAME, "launch_ms": launch_ms,
                     "launch_ms_source": "HIP events around each launch in the timed region",
                     "algorithmic_bytes_per_launch": 16.0 * n,
                     "flop_per_launch": flop_launch},
        "mode_product_ms_by_position": per_pos,
        "matvec_ms": mv_ms,
        "matvec_tflops": 2.0 * n * m * d / (mv_ms * 1e-3) / 1e12,
        "matvec_hbm_gbs": mv_bytes / (mv_ms * 1e-3) / 1e9,
        "matvec_hbm_frac": mv_bytes / (mv_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
        "iteration_algorithmic_bytes": it_bytes,
        "iteration_hbm_gbs": it_bytes / (dt / a.steps) / 1e9,
        "outside_mode_products_ms": 1e3 * dt / a.steps - mv_ms,
    }
    if rank == 0 and world == 1 and a.cpu_baseline == "auto":
        del solver, y
        torch.cuda.empty_cache()
        result["cpu_baseline"] = cpu_baseline(m, d, s)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
