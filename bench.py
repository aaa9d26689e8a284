"""Benchmark: CG iterations/s on the 4-D RBF grid 200^4 (BASELINE.json configs[2]).

One "step" = one CG iteration on (K + s I) x = y, K = K_0 (x) K_1 (x) K_2 (x) K_3
(200 x 200 RBF factors built by gp_grief_amd.kern.GridKernel.cov_grid -- the
drop-in path, grid_kernel.py:56-115 -- lengthscales 0.1*(1+0.05 i), jitter
1e-12, s = 0.01), all vectors (y, x, r, two p buffers, q, matvec scratch:
7 x 12.8 GB) resident in HBM.

Prints ONE JSON line (rank 0):
  metric/value/unit   CG iterations per second, whole job
  roofline            the dominant kernel -- the mode-product launch position
                      with the largest share of the timed region, from HIP
                      events recorded by the library on the stream the kernels
                      run on -- against its binding roof (FP64 MFMA or HBM,
                      whichever floor is higher for that launch's algorithmic
                      FLOP and bytes); plus whole-matvec and whole-iteration
                      fractions
  cpu_baseline        the reference's CPU arithmetic restated
                      (oracle.kron_matvec_dsymm: kron_matrix.py:74-96's dsymm
                      sequence; fidelity vs the reference in
                      profiles/r02_cpu_fidelity.json) in a textbook CG on the
                      full grid, 1 warm-up + 3 timed iterations, host threads
  matvec              (--matvec R, default 5) the isolated K*x on the same
                      operator: HIP events per mode product, HBM / MFMA
                      fractions of the 8-pass matvec; not part of `value`
  lanczos             (--lanczos K, default 30) K steps of device Lanczos on
                      the same operator after the CG leg, per-step HIP events
                      recorded by the library (SLQ log-det leg of C3); not
                      part of `value`

  python bench.py [--gpus N] [--steps K] [--warmup W] [--grid 200] [--dims 4]
--gpus N > 1 without a launcher: this process starts
`python -m torch.distributed.run --nproc-per-node N ... bench.py` as a child
(before any GPU call) and exits with its status; under the launcher each rank
is one GPU (RCCL): strong scaling of the same single CG, factor 0 sharded over
the ranks.
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

FP64_MFMA_PEAK_TFLOPS = 78.6   # MI355X FP64 matrix, dense (AMD spec)
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E (MI355X_MICROARCH.md)
METRIC = "CG iters/sec + Kron-matvec achieved HBM GB/s, 4D RBF grid 200^4"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    # default 8: the x window (K = 8) is full from the 8th iteration on, so
    # the timed steps are steady state (the driver's W = 5 leaves its first two
    # timed iterations 6 and 7 of the 8 directions: 0.17 % of the timed bytes)
    ap.add_argument("--warmup", type=int, default=8)
    ap.add_argument("--grid", type=int, default=200)
    ap.add_argument("--dims", type=int, default=4)
    ap.add_argument("--sigma2", type=float, default=0.01)
    ap.add_argument("--cpu-baseline", default="auto", choices=["auto", "off"])
    ap.add_argument("--cpu-iters", type=int, default=3)
    ap.add_argument("--recurrence", default="fused", choices=["fused", "textbook"])
    # multi-GPU decomposition: parity blocks (no exchange) where the factors
    # allow it, else factor 0 sharded with two exchanges per matvec
    # multi-GPU decomposition: "block" = the parity-block basis's 2^d blocks
    # over 2^K ranks (no exchange); "parity" = factors 0..K-1 in the even /
    # odd basis (no exchange); "transpose" = factor 0 sharded (two exchanges
    # per matvec); "auto" = the first that applies, in that order
    ap.add_argument("--shard", default="auto", choices=["auto", "block", "parity", "transpose"])
    ap.add_argument("--lanczos", type=int, default=30,
                    help="also time this many device Lanczos steps (one probe; 0 = off; "
                         "single GPU only)")
    ap.add_argument("--matvec", type=int, default=5,
                    help="also time this many isolated K*x matvecs (HIP events per mode "
                         "product; 0 = off; single GPU only)")
    ap.add_argument("--exchange", default="auto", choices=["auto", "push", "a2a"])
    ap.add_argument("--fusion", type=int, default=None, choices=[0, 1, 2],
                    help="fused-CG layout (gg_cg_set_fusion); default: the library's")
    ap.add_argument("--grief", default="C2,C4,C5",
                    help="P2 GRIEF fits timed after the CG leg (bench_grief configs, "
                         "comma-separated; 'off' = none); not part of `value`")
    return ap.parse_args()


# ---------------------------------------------------------------- launcher
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(a):
    """One process per GPU via torch.distributed.run, started as a CHILD of
    this process before anything touched the GPU (never exec)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node", str(a.gpus), "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


# ---------------------------------------------------------------- inputs
def grid_factors(m, d):
    """The 200^4 operator's factors through the drop-in API:
    GridKernel([RBF_i]).cov_grid(xg, dim_noise_var=1e-12) (device kernels),
    returned as host arrays (factor k = input dimension d-1-k)."""
    import gp_grief_amd.kern as kern
    kl = [kern.RBF(1, variance=1.0, lengthscale=0.1 * (1 + 0.05 * i)) for i in range(d)]
    xg = [np.linspace(0.0, 1.0, m).reshape(-1, 1) for _ in range(d)]
    K = kern.GridKernel(kl).cov_grid(xg, dim_noise_var=1e-12)
    return K, [np.asarray(f, dtype=np.float64) for f in K.K]


RHS_NOISE = 0.6180339887498949   # golden-ratio increment of the index-based noise


def rhs_at(g, m, d, torch):
    """y[g] = sum_k sin(6 xg[i_k]) + 0.1 eps(g), xg = linspace(0, 1, m), i_k the
    digits of the global flat index g (C order), eps(g) = 2 frac(g phi) - 1 --
    a function of the global index alone, so the sharded layouts of every N
    hold exactly the single-GPU right-hand side."""
    gd = g.to(torch.float64)
    eps = 2.0 * torch.frac(gd * RHS_NOISE) - 1.0
    y = 0.1 * eps
    rest = g.clone()
    for _ in range(d):
        i = torch.remainder(rest, m)
        y += torch.sin(6.0 * i.to(torch.float64) / (m - 1))
        rest = torch.div(rest, m, rounding_mode="floor")
    return y


def grid_rhs_device(m, d, torch, dev):
    """The 200^4 right-hand side on the device, built in chunks."""
    n = m ** d
    y = torch.empty(n, dtype=torch.float64, device=dev)
    chunk = 1 << 26
    for i in range(0, n, chunk):
        k = min(chunk, n - i)
        y[i:i + k] = rhs_at(torch.arange(i, i + k, dtype=torch.int64, device=dev), m, d, torch)
    return y


def local_rhs(m, d, world, rank, torch, dev):
    """This rank's shard of the same right-hand side, in the sharded layout
    (m_1, ..., m_{d-1}, a) with a = i_0 - rank * m/world fastest: local index
    l = r s0 + a holds the global element g = (rank s0 + a) R + r, R = N / m."""
    s0 = m // world
    R = m ** (d - 1)
    nl = R * s0
    y = torch.empty(nl, dtype=torch.float64, device=dev)
    chunk = 1 << 26
    for i in range(0, nl, chunk):
        k = min(chunk, nl - i)
        l = torch.arange(i, i + k, dtype=torch.int64, device=dev)
        r = torch.div(l, s0, rounding_mode="floor")
        a = l - r * s0
        y[i:i + k] = rhs_at((rank * s0 + a) * R + r, m, d, torch)
    return y


def parity_local_rhs(m, d, world, rank, torch, dev):
    """This rank's block of the same right-hand side in the even / odd basis
    of factors 0..K-1 (G = 2^K; distributed.parity_fold, on the device): local
    index = C order over the local axes (distributed.parity_local_axes: the
    unsharded axes K..d-1 of size m, then the sharded 0..K-1 of size h = m / 2),
    and b~ = 2^(-K/2)
    sum over the 2^K mirror choices s of sign(s) y[g(s)] -- axis k takes
    digit i (s_k = 0) or m - 1 - i (s_k = 1, sign -1 when bit k of the rank,
    counted from the most significant, is set)."""
    from gp_grief_amd.distributed import parity_local_axes
    K = world.bit_length() - 1
    h = m // 2
    axes = parity_local_axes(d, world)            # global axis of each local axis
    sizes = [h if a < K else m for a in axes]
    nl = int(np.prod(sizes))
    y = torch.empty(nl, dtype=torch.float64, device=dev)
    chunk = 1 << 24
    scale = 2.0 ** (-0.5 * K)
    for i in range(0, nl, chunk):
        k = min(chunk, nl - i)
        rest = torch.arange(i, i + k, dtype=torch.int64, device=dev)
        digits = [None] * d                       # by global axis
        for pos in range(d - 1, -1, -1):
            digits[axes[pos]] = torch.remainder(rest, sizes[pos])
            rest = torch.div(rest, sizes[pos], rounding_mode="floor")
        acc = torch.zeros(k, dtype=torch.float64, device=dev)
        for sgn_bits in range(1 << K):
            g = torch.zeros(k, dtype=torch.int64, device=dev)
            sign = 1.0
            for ax in range(d):
                if ax < K and (sgn_bits >> (K - 1 - ax)) & 1:
                    idx = (m - 1) - digits[ax]
                    if (rank >> (K - 1 - ax)) & 1:
                        sign = -sign
                else:
                    idx = digits[ax]
                g = g * m + idx
            acc += sign * rhs_at(g, m, d, torch)
        y[i:i + k] = acc * scale
    return y


# ---------------------------------------------------------------- sharded
def _engine_factory():
    """HipEngine, or (tests only) GG_BENCH_ENGINE=module:Class, whose module
    may also provide make_factors(m, d) -- the CPU/gloo rehearsal of the
    launcher and the sharded orchestration."""
    spec = os.environ.get("GG_BENCH_ENGINE")
    if not spec:
        from gp_grief_amd.distributed import HipEngine
        return HipEngine, None
    import importlib
    mod_name, cls_name = spec.split(":")
    mod = importlib.import_module(mod_name)
    return getattr(mod, cls_name), getattr(mod, "make_factors", None)


def _all_reduce(dist, t, op):
    """All-reduce of a small tensor; through the host when the process group
    is gloo and the tensor lives on a GPU (the gloo-gpu rehearsal)."""
    if t.is_cuda and str(dist.get_backend()) == "gloo":
        h = t.cpu()
        dist.all_reduce(h, op=op)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=op)


def backend_fields(backend, world, torch, on_gpu):
    """How the ranks ran: the collective backend, the GPUs the box has, and
    the scaling label -- "rehearsal" when every rank shares fewer physical
    GPUs than ranks over gloo (GG_BENCH_BACKEND=gloo-gpu: a correctness and
    plumbing run, not a scaling result)."""
    phys = torch.cuda.device_count() if on_gpu else 0
    rehearsal = backend != "nccl" or phys < world
    return {"backend": "nccl (RCCL)" if backend == "nccl" else backend,
            "physical_gpus": phys,
            "scaling": "rehearsal" if rehearsal else "strong",
            "collectives": "RCCL" if backend == "nccl" else "gloo"}


def run_sharded(a, world, rank, torch, dev, dist, on_gpu, backend="nccl"):
    """Strong scaling: one CG on the full grid, sharded over the ranks."""
    from gp_grief_amd.distributed import DistKronCG, TorchExchange
    m, d, s = a.grid, a.dims, a.sigma2
    Engine, make_factors = _engine_factory()
    K = None
    if make_factors is not None:
        F = make_factors(m, d)
    else:
        K, F = grid_factors(m, d)
    shard = os.environ.get("GG_DIST_SHARD", a.shard)
    from gp_grief_amd.distributed import block_shard_ok, parity_ok
    if shard in ("auto", "block"):
        blk_spec = os.environ.get("GG_BENCH_BLOCK_ENGINE")   # tests: module:Class
        if K is None:
            from gp_grief_amd.tensors import KronMatrix
            K = KronMatrix(F, sym=True)
        if blk_spec or (on_gpu and block_shard_ok(K, world)):
            return run_block(a, world, rank, torch, dev, dist, on_gpu, K, F, backend)
        if shard == "block":
            raise SystemExit("bench.py: block sharding needs 2^K <= 2^d GPUs and a parity-block "
                             "basis")
    if shard in ("auto", "parity") and parity_ok(F, world):
        return run_parity(a, world, rank, torch, dev, dist, on_gpu, F, backend)
    if shard == "parity":
        raise SystemExit("bench.py: parity sharding needs 2^K GPUs and centrosymmetric factors")
    eng = Engine(F, world, rank)
    y = local_rhs(m, d, world, rank, torch, dev)
    ex = TorchExchange()
    sync = torch.cuda.synchronize if on_gpu else (lambda: None)
    mode = os.environ.get("GG_DIST_MODE", a.exchange)
    # the fused recurrence wherever the engine runs it (d >= 4, folded
    # factors 1..d-1), else the textbook one
    rec = "auto" if a.recurrence == "fused" else "textbook"
    if mode == "auto":
        # the library's default (DistKronCG): RCCL all-to-all; push (peer
        # stores over xGMI) is opt-in until it has run across devices
        mode = "a2a"
    # every rank must take the same exchange: a push setup that fails on any
    # rank (IPC mapping of a peer's buffer) sends all ranks to all-to-all
    try:
        cg = DistKronCG(eng, ex, s, mode=mode, recurrence=rec)
        ok = 1.0
    except Exception as exc:  # noqa: BLE001
        print("rank %d: %s exchange setup failed (%s); using a2a" % (rank, mode, exc),
              file=sys.stderr, flush=True)
        cg, ok = None, 0.0
    flag = torch.tensor([ok], dtype=torch.float64, device=dev)
    _all_reduce(dist, flag, dist.ReduceOp.MIN)
    if float(flag.item()) < 1.0:
        cg = DistKronCG(eng, ex, s, mode="a2a", recurrence=rec)
    if cg.mode == "push":
        # one matvec through the peer-memory exchange against the all-to-all
        # path on the same input; any disagreement falls back to all-to-all
        ref = DistKronCG(eng, ex, s, mode="a2a")
        ya, yp = eng.empty(), eng.empty()
        ref.apply(y.clone(), ya)
        cg.apply(y.clone(), yp)
        err = torch.stack([(ya - yp).abs().max(), ya.abs().max()])
        _all_reduce(dist, err, dist.ReduceOp.MAX)
        del ref, ya, yp
        if not float(err[0]) <= 1e-12 * float(err[1]):
            cg = DistKronCG(eng, ex, s, mode="a2a", recurrence=rec)
        if on_gpu:
            torch.cuda.empty_cache()
    cg.start(y, rtol=0.0, atol=0.0)
    cg.iterate(a.warmup, close=False)
    sync()
    dist.barrier()
    sync()
    if on_gpu:
        cg.profile(True, a.steps)   # HIP events between the phases, on the compute stream
    t0 = time.perf_counter()
    cg.iterate(a.steps, close=False)
    sync()
    dist.barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    _all_reduce(dist, t, dist.ReduceOp.MAX)
    dt = float(t.item())
    phases = None
    if on_gpu:
        ph = cg.profile_read()
        cg.profile(False)
    cg.close()                       # the once-per-solve closing update
    it, done, rho, tol = cg.status()
    assert it == a.warmup + a.steps and np.isfinite(rho), (it, rho)
    n = m ** d
    if on_gpu:
        # max over ranks of each phase's mean per iteration
        keys = sorted(ph)
        v = torch.tensor([ph[k] / a.steps for k in keys], dtype=torch.float64, device=dev)
        _all_reduce(dist, v, dist.ReduceOp.MAX)
        phases = dict(zip(keys, [float(u) for u in v.tolist()]))
    bf = backend_fields(backend, world, torch, on_gpu)
    res = {
        "metric": METRIC,
        "value": a.steps / dt,
        "unit": "CG iters/s",
        "n_gpus": dist.get_world_size(),
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": 1e3 * dt / a.steps,
        "higher_is_better": True,
        "scaling": bf["scaling"],
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "backend": bf["backend"],
        "physical_gpus": bf["physical_gpus"],
        "config": {"workload": "4D RBF grid %d^%d, CG on (K + %g I) x = y, N = %d, factor 0 "
                               "sharded over %d ranks" % (m, d, s, n, world),
                   "grid": m, "dims": d, "sigma2": s, "n": n,
                   "exchange": cg.mode,
                   "cg_recurrence": cg.recurrence,
                   "parallelism": ("shard factor-0 x%d: matvec exchange by %s, %s per "
                                   "iteration (%s)"
                                   % (world, "peer-memory stores in the mode-product "
                                             "epilogues + 2 barriers"
                                      if cg.mode == "push" else "2 all-to-all",
                                      "one 5-double all-reduce" if cg.recurrence == "fused"
                                      else "2 scalar all-reduces", bf["collectives"]))},
    }
    if phases is not None:
        res["phase_ms_per_iteration"] = phases
        res["local_roofline"] = sharded_roofline(phases, n, m, d, world,
                                                 getattr(eng, "fold_mask", 0))
    return res


def run_parity(a, world, rank, torch, dev, dist, on_gpu, F, backend="nccl"):
    """Strong scaling by parity sharding (distributed.ParityShardCG): rank g
    owns one block of the operator in the even / odd basis of factors
    0..K-1 -- no exchange, one all-reduce of five doubles per iteration."""
    from gp_grief_amd.distributed import ParityShardCG, TorchExchange
    m, d, s = a.grid, a.dims, a.sigma2
    ex = TorchExchange()
    spec = os.environ.get("GG_BENCH_PARITY_ENGINE")   # tests: module:Class
    eng = None
    if spec:
        import importlib
        mod_name, cls_name = spec.split(":")
        eng = getattr(importlib.import_module(mod_name), cls_name)(F, world, rank, s)
    cg = ParityShardCG(F, world, rank, ex, s, engine=eng)
    sync = torch.cuda.synchronize if on_gpu else (lambda: None)
    if on_gpu:
        y = parity_local_rhs(m, d, world, rank, torch, dev)
    else:
        from gp_grief_amd.distributed import parity_fold
        yg = rhs_at(torch.arange(m ** d, dtype=torch.int64), m, d, torch).numpy()
        y = torch.from_numpy(parity_fold(yg, [m] * d, world)[rank].copy())
    cg.start(y, rtol=0.0, atol=0.0)
    cg.iterate(a.warmup, close=False)
    sync()
    dist.barrier()
    sync()
    if on_gpu:
        cg.profile(True, a.steps)
    t0 = time.perf_counter()
    cg.iterate(a.steps, close=False)
    sync()
    dist.barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    _all_reduce(dist, t, dist.ReduceOp.MAX)
    dt = float(t.item())
    if on_gpu:
        ph = cg.profile_read()
        nm, per = cg.e.profile_read()
        cg.profile(False)
    cg.close()                       # the once-per-solve closing update
    it, conv, res, tol = cg.status()
    assert it == a.warmup + a.steps and np.isfinite(res), (it, res)
    n = m ** d
    K = world.bit_length() - 1
    bf = backend_fields(backend, world, torch, on_gpu)
    res_ = {
        "metric": METRIC,
        "value": a.steps / dt,
        "unit": "CG iters/s",
        "n_gpus": dist.get_world_size(),
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": 1e3 * dt / a.steps,
        "higher_is_better": True,
        "scaling": bf["scaling"],
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "backend": bf["backend"],
        "physical_gpus": bf["physical_gpus"],
        "config": {"workload": "4D RBF grid %d^%d, CG on (K + %g I) x = y, N = %d, "
                               "parity-sharded over %d ranks" % (m, d, s, n, world),
                   "grid": m, "dims": d, "sigma2": s, "n": n,
                   "exchange": "none",
                   "cg_recurrence": "fused",
                   "local_factor_orders": [f.shape[0] for f in cg.e.local_factors]
                   if hasattr(cg.e, "local_factors") else None,
                   "parallelism": ("parity-shard factors 0..%d over %d ranks: the operator is "
                                   "block-diagonal in their even / odd basis, each rank owns "
                                   "one block; no exchange, one 5-double all-reduce per "
                                   "iteration (%s)" % (K - 1, world, bf["collectives"]))},
    }
    if on_gpu:
        keys = sorted(ph)
        v = torch.tensor([ph[k] / a.steps for k in keys] + [x / max(nm, 1) for x in per],
                         dtype=torch.float64, device=dev)
        _all_reduce(dist, v, dist.ReduceOp.MAX)
        vals = [float(u) for u in v.tolist()]
        res_["phase_ms_per_iteration"] = dict(zip(keys, vals[:len(keys)]))
        res_["local_launch_ms"] = vals[len(keys):]
        nl = n / world
        passes = float(sum(launch_passes(d, "fused", 0, True, True)))
        res_["local_passes_per_iteration"] = passes
        lm = res_["phase_ms_per_iteration"].get("launches", 0.0)
        if lm > 0:
            res_["local_gbs"] = passes * 8.0 * nl / (lm * 1e-3) / 1e9
            res_["local_frac_hbm"] = res_["local_gbs"] / HBM_PEAK_GBS
    return res_


def run_block(a, world, rank, torch, dev, dist, on_gpu, K, F, backend="nccl"):
    """Strong scaling by block sharding (distributed.BlockHipEngine): the
    operator in its parity-block basis is block diagonal over the 2^d parity
    patterns; rank g of G = 2^K owns blocks [g 2^d / G, (g + 1) 2^d / G) and
    runs the single-GPU block kernels on them (d - 1 launches per iteration).
    No exchange; one all-reduce of five doubles per iteration.  The right-hand
    side is folded on the device from the grid vector into the rank's blocks
    (gg_kron_block_fold_range) and the solution unfolded the same way; both are
    once per solve, timed beside the iterations."""
    from gp_grief_amd.distributed import BlockHipEngine, ParityShardCG, TorchExchange
    m, d, s = a.grid, a.dims, a.sigma2
    n = m ** d
    spec = os.environ.get("GG_BENCH_BLOCK_ENGINE")   # tests: module:Class (host arrays)
    if spec:
        import importlib
        mod_name, cls_name = spec.split(":")
        Engine = getattr(importlib.import_module(mod_name), cls_name)
    else:
        Engine = BlockHipEngine
    eng = Engine(K, world, rank, s)
    ex = TorchExchange()
    sync = torch.cuda.synchronize if on_gpu else (lambda: None)
    fold_ms = unfold_ms = xred_ms = xgat_ms = unfold_all_ms = None
    if on_gpu:
        yg = grid_rhs_device(m, d, torch, dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        y = eng.fold(yg)
        e1.record()
        sync()
        fold_ms = e0.elapsed_time(e1)
        del yg
        torch.cuda.empty_cache()
    else:
        y = eng.fold(rhs_at(torch.arange(n, dtype=torch.int64), m, d, torch).numpy())
    cg = ParityShardCG(F, world, rank, ex, s, engine=eng)
    cg.start(y, rtol=0.0, atol=0.0)
    cg.iterate(a.warmup, close=False)
    sync()
    dist.barrier()
    sync()
    # HIP events on the GPU (host timestamps in the CPU rehearsal)
    cg.profile(True, a.steps)
    t0 = time.perf_counter()
    cg.iterate(a.steps, close=False)
    sync()
    dist.barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], dtype=torch.float64, device=dev)
    _all_reduce(dist, t, dist.ReduceOp.MAX)
    dt = float(t.item())
    ph = cg.profile_read()
    nm, per = eng.profile_read()
    cg.profile(False)
    cg.close()                       # the once-per-solve closing update
    it, conv, res, tol = cg.status()
    assert it == a.warmup + a.steps and np.isfinite(res), (it, res)
    if on_gpu:
        # the solution's way back: this rank's contribution to P^T x (one
        # pass over N), summed over the ranks by one all-reduce of N doubles
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        xg = eng.unfold(cg.x)
        e1.record()
        sync()
        unfold_ms = e0.elapsed_time(e1)
        if backend == "nccl":
            e0.record()
            dist.all_reduce(xg)
            e1.record()
            sync()
            xred_ms = e0.elapsed_time(e1)
        del xg
        torch.cuda.empty_cache()
        # the default way back (distributed.block_solution): an all-gather of
        # the N / G shares, then the whole unfold on every rank.  Timed with
        # RCCL only: in the one-card rehearsal the ranks' two more grid-sized
        # buffers push the card's shared HBM past its size and the driver
        # evicts buffers to host memory (the unfold then ran 1.5 s against
        # 13.5 ms alone, tools/fold_probe.py)
        if backend == "nccl":
            e0.record()
            xa = ex.all_gather(cg.x)
            e1.record()
            sync()
            xgat_ms = e0.elapsed_time(e1)
            e0.record()
            xg = eng.unfold_all(xa)
            e1.record()
            sync()
            unfold_all_ms = e0.elapsed_time(e1)
            del xa, xg
            torch.cuda.empty_cache()
    nl = n // world
    bf = backend_fields(backend, world, torch, on_gpu)
    ms_per_step = 1e3 * dt / a.steps
    res_ = {
        "metric": METRIC,
        "value": a.steps / dt,
        "unit": "CG iters/s",
        "n_gpus": dist.get_world_size(),
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": bf["scaling"],
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "backend": bf["backend"],
        "physical_gpus": bf["physical_gpus"],
        "config": {"workload": "4D RBF grid %d^%d, CG on (K + %g I) x = y, N = %d, "
                               "block-sharded over %d ranks" % (m, d, s, n, world),
                   "grid": m, "dims": d, "sigma2": s, "n": n,
                   "exchange": "none",
                   "cg_recurrence": "fused",
                   "cg_basis": "block",
                   "blocks_per_rank": (1 << d) // world,
                   "cg_x_window": int(getattr(eng, "xwin", 0)),
                   "cg_r_derived": bool(getattr(eng, "rderive", False)),
                   "n_per_rank": nl,
                   "launches_per_iteration": d - 1,
                   "timed_region": "exactly `steps` fused CG iterations continuing the "
                                   "warm-up's open recurrence; fold, closing update and "
                                   "unfold (once per solve) outside it",
                   "parallelism": ("block-shard: the operator's 2^%d parity blocks, %d per "
                                   "rank (factors 0..%d's parity bits = the rank); no "
                                   "exchange, one 5-double all-reduce per iteration (%s)"
                                   % (d, (1 << d) // world, world.bit_length() - 2,
                                      bf["collectives"]))},
        "cpu_baseline": {"value": None, "unit": "CG iters/s",
                         "reference": "the n_gpus = 1 line's cpu_baseline (the bench contract "
                                      "times the CPU baseline on rank 0 at N = 1 only); the "
                                      "same single CG on the same grid"},
    }
    if ph:
        keys = sorted(ph)
        v = torch.tensor([ph[k] / a.steps for k in keys] + [x / max(nm, 1) for x in per] +
                         [fold_ms or 0.0, unfold_ms or 0.0, unfold_all_ms or 0.0],
                         dtype=torch.float64, device=dev)
        _all_reduce(dist, v, dist.ReduceOp.MAX)
        vals = [float(u) for u in v.tolist()]
        phases = dict(zip(keys, vals[:len(keys)]))
        per_pos = vals[len(keys):len(keys) + len(per)]
        res_["phase_ms_per_iteration"] = phases
        res_["local_launch_ms"] = per_pos
        # the dominant kernel of a rank (its blocks are whole blocks: the
        # single-GPU block roofline with n -> N / G)
        roof, extra = roofline_report(per_pos, nl, m, d, "fused", ms_per_step, block=True,
                                      xwin=int(getattr(eng, "xwin", 0)),
                                      rderive=bool(getattr(eng, "rderive", False)))
        roof["scope"] = "per rank: the rank's dominant launch on its N / G elements " \
                        "(max over ranks of the per-launch %s means)" \
                        % ("HIP-event" if on_gpu else "host-timer (CPU rehearsal engine)")
        roof["traffic_source"] = "no PMC passes for the sharded layout"
        res_["roofline"] = roof
        res_["local_matvec_ms"] = extra["matvec_ms"]
        res_["local_iteration_floor_ms"] = extra["iteration_floor_ms"]
        ar = phases.get("allreduce", 0.0)
        res_["allreduce"] = {"ms_per_iteration": ar, "share_of_iteration": ar / ms_per_step,
                             "doubles_per_iteration": 5, "collectives": bf["collectives"]}
        res_["fold_ms"] = vals[-3] if on_gpu else None
        res_["unfold_ms"] = vals[-2] if on_gpu else None
        res_["fold_unfold_bytes_per_rank"] = 8.0 * (n + nl)
        # the solution's two ways back, once per solve (rank 0's events; the
        # unfolds max over ranks): "reduce" = unfold_ms + solution_allreduce_ms,
        # "gather" (distributed.solve's default) = solution_allgather_ms +
        # unfold_all_ms
        res_["unfold_all_ms"] = vals[-1] if unfold_all_ms is not None else None
        if xred_ms is not None:
            res_["solution_allreduce_ms"] = xred_ms
        if xgat_ms is not None:
            res_["solution_allgather_ms"] = xgat_ms
    return res_


def sharded_roofline(phases, n, m, d, world, fold_mask):
    """Per-rank achieved rates of the two local MFMA phases (DESIGN.md section
    6): phase 1 = factors 1..d-1 on N/G elements, phase 2 = factor 0 on N/G;
    a folded factor (centrosymmetric split) does m instead of 2 m FLOP per
    element.  Bytes: X read + Y written per mode product."""
    nl = n / world

    def flop(k):
        return (1.0 if (fold_mask >> k) & 1 else 2.0) * nl * m

    out = {}
    for name, ks in (("phase1", range(1, d)), ("phase2", [0])):
        ms = phases.get(name)
        if not ms:
            continue
        f = sum(flop(k) for k in ks)
        b = 16.0 * nl * len(ks)
        out[name] = {"ms": ms, "flop": f, "bytes": b,
                     "tflops": f / (ms * 1e-3) / 1e12, "gbs": b / (ms * 1e-3) / 1e9,
                     "frac_mfma": f / (ms * 1e-3) / 1e12 / FP64_MFMA_PEAK_TFLOPS,
                     "frac_hbm": b / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS}
    ex = sum(phases.get(k, 0.0) for k in ("exchange1", "exchange2"))
    out["exchange_ms"] = ex
    out["exchange_bytes_per_rank"] = 2 * 8.0 * nl * (world - 1) / world
    if ex > 0:
        out["exchange_gbs_per_rank"] = out["exchange_bytes_per_rank"] / (ex * 1e-3) / 1e9
    return out


# ---------------------------------------------------------------- roofline
def launch_passes(d, recurrence, fusion=0, xdefer=False, rq=False):
    """Algorithmic 8-byte passes over N of each mode-product launch position of
    one CG iteration (reads + writes, gg_kron.hip kron_apply / MpFuse),
    averaged over iterations.  xdefer: the x update runs every other
    iteration as x += c0 p0 + c1 p1 (4 passes per two iterations, 2 per
    iteration on average instead of 3).  rq: r.q from the conjugacy identity
    (gg_cg_set_rq 1), so the epilogue reads p only."""
    if d == 1:
        return [4] if recurrence == "fused" else [5]
    passes = [2] * d
    if recurrence == "fused":
        # prologue: r, q_old read, r written (p_old is X); layout 0 also writes p_new
        passes[0] += 3 if fusion else 4
        # epilogue: p and r read (shift, p.q, r.q; p only with the conjugacy
        # r.q); layouts 1/2 also write p_new
        passes[d - 1] += 3 if fusion else (1 if rq else 2)
        xp = 2.0 if (xdefer and fusion != 2) else 3.0
        if fusion == 2:
            passes[d - 1] += 2  # x += alpha p_old in the epilogue (x read + written)
        elif d >= 4:
            passes[1] += xp / 2  # side job on the first half of x
            passes[2] += xp / 2  # ... second half (gg_kron.hip kron_apply split_side)
        else:
            passes[1] += xp      # side job: x update (x, p read; x written)
    else:
        passes[0] += 2          # prologue: r read, p written in place
        passes[d - 1] += 1      # epilogue: p read (shift, p.q)
    return passes


def block_launch_passes(d, xwin=0, rderive=False):
    """Passes over N of each launch of the fused CG iteration in the
    parity-block basis (gg_kronb.hip block_apply; d - 1 launches): the first
    (axis 0, in place) carries the prologue -- p_old (its MFMA operand), r and
    q_old read, r, p_new and the output written; the last (the pair of
    innermost axes, blk_pair_lds_kernel) reads its input and p_new, writes q,
    and carries the x side job: xwin = 0, mode 2's balanced pairs (half of x
    per iteration: x, p_{j-2}, p_{j-1} read, x written = 2 passes); xwin = K,
    mode 3's window (one of K regions of x read and written, its K pending
    directions read = (K + 2) / K passes); the ones between are plain.
    rderive (round 6): the prologue keeps no r -- it reads p_{j-2} in place of
    r and stores no r, one pass fewer."""
    passes = [2.0] * (d - 1)
    passes[0] += 3.0 if rderive else 4.0
    passes[-1] += 1.0 + ((xwin + 2.0) / xwin if xwin >= 2 else 2.0)
    return passes


def block_launch_kernels(d):
    kinds = ["plain"] * (d - 1)
    kinds[0] = "prologue"
    kinds[-1] = "pair-epilogue-side"
    return kinds


def block_launch_flops(n, m, d):
    """MFMA FLOP per launch: an h x h factor (h = m / 2) per element of its
    axis is 2 n h = n m; the pair launch applies two."""
    fl = [1.0 * n * m] * (d - 1)
    fl[-1] = 2.0 * n * m
    return fl


def launch_kernels(d, recurrence, fusion=0):
    """The kernel instantiation of each launch position (gg_kron.hip kron_apply
    selects it per position): positions that share one are one rocprof row."""
    if d == 1:
        return ["epilogue"]
    kinds = ["plain"] * d
    kinds[0] = "prologue"
    kinds[d - 1] = "epilogue"
    if recurrence == "fused" and fusion != 2:
        kinds[1] = "side"
        if d >= 4:
            kinds[2] = "side"
    return kinds


def dominant_group(per_pos, kinds):
    """Positions of the kernel with the largest total time per iteration (the
    rocprof-dominant kernel by total time)."""
    tot = {}
    for k, t in zip(kinds, per_pos):
        tot[k] = tot.get(k, 0.0) + t
    best = max(tot, key=tot.get)
    return [i for i, k in enumerate(kinds) if k == best], best


def roofline_report(per_pos, n, m, d, recurrence, ms_per_step, fusion=0, fold_mask=0,
                    xdefer=False, rq=False, block=False, xwin=0, rderive=False):
    """fold_mask bit k: mode product k runs on the centrosymmetric split
    (gg_kron_fold_mask), executing n m MFMA FLOP instead of the dense 2 n m;
    the roofline prices the work the kernel actually does.  block: the CG runs
    in the parity-block basis (d - 1 launches)."""
    if block:
        flops = block_launch_flops(n, m, d)
        passes = block_launch_passes(d, xwin, rderive)
        kinds = block_launch_kernels(d)
    else:
        flops = [(1.0 if (fold_mask >> k) & 1 else 2.0) * n * m for k in range(d)]
        passes = launch_passes(d, recurrence, fusion, xdefer, rq)
        kinds = launch_kernels(d, recurrence, fusion)
    L = len(kinds)
    group, kind = dominant_group(per_pos, kinds)
    dom = group[0]
    flop = flops[dom]
    t = float(np.mean([per_pos[i] for i in group])) * 1e-3   # per-launch average
    byts = 8.0 * n * float(np.mean([passes[i] for i in group]))
    f_mfma = flop / (FP64_MFMA_PEAK_TFLOPS * 1e12)
    f_hbm = byts / (HBM_PEAK_GBS * 1e9)
    bound = "mfma" if f_mfma >= f_hbm else "hbm"
    tf = flop / t / 1e12
    gbs = byts / t / 1e9
    mv_s = sum(per_pos) * 1e-3
    it_bytes = 8.0 * n * sum(passes)
    floor_it = max(sum(flops) / (FP64_MFMA_PEAK_TFLOPS * 1e12), it_bytes / (HBM_PEAK_GBS * 1e9))
    roof = {
        "bound": bound,
        "achieved": tf if bound == "mfma" else gbs,
        "peak": FP64_MFMA_PEAK_TFLOPS if bound == "mfma" else HBM_PEAK_GBS,
        "unit": "TFLOP/s" if bound == "mfma" else "GB/s",
        "frac": (f_mfma if bound == "mfma" else f_hbm) / t,
        "traffic": None, "traffic_unit": "bytes per launch",
        "kernel": "%s, %s kernel (launch position%s %s of %d; %s CG, layout %d)"
                  % ("parity-block launch" if block else "mode product", kind,
                     "s" if len(group) > 1 else "", ", ".join(str(i) for i in group), L,
                     recurrence, fusion),
        "selection": "the kernel with the largest total time per iteration (rocprof "
                     "groups launches by kernel); per-launch averages over its positions",
        "positions": group,
        "launch_ms": t * 1e3,
        "launch_ms_source": "HIP events the library records around each launch, on the "
                            "stream it launches on, over the timed iterations",
        "flop_per_launch": flop, "algorithmic_bytes_per_launch": byts,
        "flop_rule": ("parity-block basis: n m MFMA FLOP per h x h factor applied (h = m/2), "
                      "2 n m for the pair launch" if block else
                      "n m MFMA FLOP (centrosymmetric even/odd split: two h x h GEMMs, "
                      "h = m/2; the dense product is 2 n m)" if (fold_mask >> dom) & 1
                      else "2 n m (dense factor)"),
        "passes_per_launch": byts / (8.0 * n),
        "frac_mfma": f_mfma / t, "frac_hbm": f_hbm / t,
        "achieved_tflops": tf, "achieved_gbs": gbs,
    }
    big = int(np.argmax(per_pos))
    extra = {
        "largest_launch": {"position": big, "launch_ms": per_pos[big],
                           "passes": passes[big],
                           "frac_hbm": 8.0 * n * passes[big] / (HBM_PEAK_GBS * 1e9)
                           / (per_pos[big] * 1e-3),
                           "frac_mfma": f_mfma / (per_pos[big] * 1e-3)},
        "mode_product_ms_by_position": per_pos,
        "launch_kinds": kinds,
        "passes_by_position": passes,
        "matvec_ms": 1e3 * mv_s,
        "matvec_tflops": sum(flops) / mv_s / 1e12,
        "matvec_frac": sum(flops) / mv_s / 1e12 / FP64_MFMA_PEAK_TFLOPS,
        "matvec_dense_equivalent_tflops": d * 2.0 * n * m / mv_s / 1e12,
        "fold_mask": fold_mask,
        "matvec_hbm_gbs": 8.0 * n * (2 * L + 1) / mv_s / 1e9,
        "matvec_hbm_frac": 8.0 * n * (2 * L + 1) / mv_s / 1e9 / HBM_PEAK_GBS,
        "iteration_algorithmic_bytes": it_bytes,
        "iteration_hbm_gbs": it_bytes / (ms_per_step * 1e-3) / 1e9,
        "iteration_floor_ms": 1e3 * floor_it,
        "iteration_frac_vs_fused_floor": 1e3 * floor_it / ms_per_step,
        "outside_mode_products_ms": ms_per_step - 1e3 * mv_s,
    }
    return roof, extra


PMC_JSON = os.path.join("profiles", "r04", "pmc_mode_product.json")
PMC_JSON_BLOCK = os.path.join("profiles", "r06", "pmc_block.json")
# the sources that decide the CG launches' HBM traffic
KERNEL_SOURCES = ["gp_grief_amd/csrc/gg_kron.hip", "gp_grief_amd/csrc/gg_kron_fold.hip",
                  "gp_grief_amd/csrc/gg_mp.h", "gp_grief_amd/csrc/gg_internal.h",
                  "gp_grief_amd/csrc/gg_vec.hip", "gp_grief_amd/csrc/gg_kron_ring.hip",
                  "gp_grief_amd/csrc/gg_kronb.hip"]


def kernel_source_hash():
    import hashlib
    h = hashlib.sha256()
    for rel in KERNEL_SOURCES:
        with open(os.path.join(ROOT, rel), "rb") as f:
            h.update(rel.encode() + b"\0" + f.read())
    return h.hexdigest()


def pmc_traffic(m, d, positions, recurrence, fusion=0, fold_mask=0, xdefer=True, rq=False,
                block=False, xwin=0, rderive=False):
    """HBM bytes per launch of the dominant kernel (averaged over its launch
    positions) from the committed PMC passes (tools/pmc_traffic.py) -- only
    when they were taken on this workload, recurrence, fusion layout and fold
    state, by kernels built from the same sources (sha256 of KERNEL_SOURCES
    recorded in the JSON), and every launch matched its algorithmic bytes;
    else (None, reason)."""
    path = os.path.join(ROOT, PMC_JSON_BLOCK if block else PMC_JSON)
    if (m, d) != (200, 4):
        return None, "no PMC passes for this workload"
    if not os.path.exists(path):
        return None, "no PMC passes committed (%s)" % (PMC_JSON_BLOCK if block else PMC_JSON)
    rec = json.load(open(path))
    if bool(rec.get("block_basis", False)) != bool(block):
        return None, "PMC passes taken in another CG basis"
    if rec.get("recurrence") != recurrence or rec.get("fusion_layout", 0) != fusion:
        return None, "PMC passes taken with another recurrence / fusion layout"
    if rec.get("fold_mask", 0) != fold_mask:
        return None, "PMC passes taken with another fold state"
    if int(rec.get("x_deferred", 0)) != int(xdefer) or int(rec.get("x_window", 0)) != int(xwin):
        return None, "PMC passes taken with another x-update schedule"
    if bool(rec.get("r_derived", False)) != bool(rderive):
        return None, "PMC passes taken with another r source"
    if int(rec.get("rq_identity", 0)) != int(rq):
        return None, "PMC passes taken with another r.q source"
    if rec.get("source_sha256") != kernel_source_hash():
        return None, "stale: the kernel sources changed since the PMC passes (%s)" % (PMC_JSON_BLOCK if block else PMC_JSON)
    if not rec.get("calibrated_on_own_pattern"):
        return None, "PMC bytes did not match the algorithmic bytes of every launch"
    per = {pp["position"]: pp["traffic_bytes"] for pp in rec.get("per_position", [])}
    if not all(i in per for i in positions):
        return None, "PMC passes miss a launch position"
    return float(np.mean([per[i] for i in positions])), PMC_JSON_BLOCK if block else PMC_JSON


# ---------------------------------------------------------------- CPU leg
def _lscpu():
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
    except Exception:  # noqa: BLE001
        return {}
    kv = {}
    for line in out.splitlines():
        if ":" in line:
            k, v = line.split(":", 1)
            kv[k.strip()] = v.strip()
    return kv


def cpu_model():
    return _lscpu().get("Model name")


def cpu_share():
    """Host threads the CPU baseline may use on this box, and why: the
    process's affinity mask, the cgroup CPU quota (cpu.max) and the
    harness's OMP_NUM_THREADS share, whichever is smallest, beside the
    machine's physical core count (BASELINE.md section 4 asks for all
    physical cores; a leased GPU box confines a process to its share)."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(path).read().split()[:2]
            if q != "max":
                quota = float(q) / float(per)
        except Exception:  # noqa: BLE001
            pass
    omp = os.environ.get("OMP_NUM_THREADS")
    kv = _lscpu()
    phys = None
    try:
        phys = int(kv["Core(s) per socket"]) * int(kv.get("Socket(s)", "1"))
    except Exception:  # noqa: BLE001
        pass
    limits = {"affinity_mask": aff}
    if quota is not None:
        limits["cgroup_cpu_quota"] = max(1, int(quota))
    if omp and omp.isdigit() and int(omp) > 0:
        limits["OMP_NUM_THREADS"] = int(omp)
    by = min(limits, key=limits.get)
    return limits[by], {"affinity_cpus": aff, "cgroup_cpu_quota": quota,
                        "omp_num_threads": omp, "physical_cores": phys,
                        "logical_cpus": os.cpu_count(), "limited_by": by}


def cpu_baseline(F, sigma2, iters):
    """Textbook CG (oracle.cg_solve) on the full grid with the reference's BLAS
    call sequence for the operator (oracle.kron_matvec_dsymm, restating
    kron_matrix.py:74-96), 1 warm-up + `iters` timed iterations."""
    import oracle
    threads, share = cpu_share()
    try:
        from threadpoolctl import threadpool_limits
        ctx = threadpool_limits(limits=threads)
    except Exception:  # pragma: no cover
        ctx = None
    m, d = F[0].shape[0], len(F)
    n = m ** d
    rng = np.random.default_rng(1)
    block = rng.standard_normal(m ** min(d, 3))
    b = np.tile(block, n // block.size)
    mv = lambda v: oracle.kron_matvec_dsymm(F, v) + sigma2 * v
    stamps = [time.perf_counter()]
    oracle.cg_solve(mv, b, rtol=0.0, maxiter=1 + iters,
                    callback=lambda x: stamps.append(time.perf_counter()))
    del b
    if ctx is not None:
        ctx.__exit__(None, None, None)
    per_it = np.diff(stamps)              # [warm-up, timed...]
    timed = per_it[1:]
    return {"value": 1.0 / float(np.mean(timed)), "unit": "CG iters/s", "cores": threads,
            "kind": "port",
            "host_cpu_count": os.cpu_count(), "host_cpu_model": cpu_model(),
            "cpu_share": share,
            "iteration_s": [float(v) for v in per_it],
            "fidelity": "profiles/r02_cpu_fidelity.json",
            "sample": "textbook CG on the full %d^%d grid, operator = the reference's dsymm "
                      "sequence restated (oracle.kron_matvec_dsymm), %d threads (limited by "
                      "%s; affinity mask %d CPUs, %s physical cores on the host), 1 warm-up "
                      "iteration (%.1f s) + %d timed (mean %.1f s)"
                      % (m, d, threads, share["limited_by"], share["affinity_cpus"],
                         share["physical_cores"], per_it[0], iters, float(np.mean(timed)))}


def grief_leg(names, torch, cpu, dist=None, world=1, rank=0):
    """P2 beside the headline: one cold GPGriefModel fit per config through the
    public API, stage-timed with HIP events (bench_grief.run_config: best of
    2), the Gram's MFMA and the Phi writer's HBM fractions, and for C2 the
    oracle's NumPy fit (oracle/grief.py) on the host as its CPU baseline.
    world > 1: data rows sharded over the ranks (bench_grief.rows_of), the
    Gram and Phi^T y all-reduced, times the max over ranks."""
    import bench_grief
    import gp_grief_amd as gg
    import gp_grief_amd.grid  # noqa: F401
    import gp_grief_amd.kern  # noqa: F401
    import gp_grief_amd.models  # noqa: F401
    ctx = bench_grief.Ctx(torch, dist if world > 1 else None, world, rank)
    out = {}
    for name in names:
        r = bench_grief.run_config(gg, ctx, name, 2, cpu and name == "C2", False)
        keep = {k: r[k] for k in ("fit_ms", "stage_ms", "gram", "phi", "lml") if k in r}
        keep["n_gpus"] = world
        keep["parallelism"] = r["config"]["parallelism"]
        keep["rows_per_rank"] = r["config"]["rows_per_rank"]
        keep["workload"] = r["config"]
        if "cpu_baseline" in r:
            keep["cpu_baseline"] = r["cpu_baseline"]
        out[name] = keep
        torch.cuda.empty_cache()
    return out


def lanczos_passes(d, block=False):
    """8-byte passes over N per fused Lanczos step by launch position
    (gg_vec.hip gg_lanczos_probe; grid basis: d mode products, even d; block
    basis: d - 1 launches, round 6): the first launch's prologue reads the
    previous output Y, u and u_prev and writes w = cy Y + cu u + cp u_prev
    over u_prev (+3 beyond the plain 2); the last (the epilogue / the pair
    launch) reads w for shift * w and w.(K w + shift w) (+1)."""
    L = d - 1 if block else d
    passes = [2.0] * L
    passes[0] += 3.0
    passes[L - 1] += 1.0
    return passes


def time_lanczos(K, s, steps, torch, n, m, d, fold_mask):
    """`steps` Lanczos steps of one probe on the same operator (the SLQ leg of
    C3).  The 4N workspace is allocated (and the allocator warmed) before
    anything is timed; the library records HIP events at every step boundary on
    the stream it launches on (gg_lanczos_probe_timed: after the probe is drawn,
    before the tridiagonal is copied back) and around every mode product, so
    ms_per_step is the mean of the per-step event times; the closing pass
    after the last step (beta_{k-1}: one streaming pass, once per probe) is
    closing_ms.  bracket_ms (events around the whole call, workspace already
    resident) is reported beside them."""
    from gp_grief_amd import device as gdev
    from gp_grief_amd import linalg
    t0 = time.perf_counter()
    work = gdev.empty(4 * n)
    work.zero_()
    torch.cuda.synchronize()
    alloc_s = time.perf_counter() - t0
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    e0.record()
    a, b, step_ms, launch_ms = linalg.lanczos_tridiag(K, s, steps, seed=0, probe=0, work=work,
                                                      timed=True)
    closing = linalg.lanczos_tridiag.closing_ms
    e1.record()
    torch.cuda.synchronize()
    bracket = e0.elapsed_time(e1)
    del work
    k = int(a.size)
    st = step_ms[:k]
    ms = float(np.mean(st))
    steady = float(np.mean(st[1:])) if k > 1 else ms
    block, L = linalg.lanczos_info(K)
    passes = lanczos_passes(d, block) if (block or d % 2 == 0) else None
    out = {"steps": k, "ms_per_step": ms, "steps_per_s": 1e3 / ms,
           "steady_ms_per_step": steady, "first_step_ms": st[0],
           "step_ms_min": float(np.min(st)), "step_ms_max": float(np.max(st)),
           "ms_source": "mean of per-step HIP events the library records on its stream "
                        "(gg_lanczos_probe_timed); workspace allocated before timing; the "
                        "once-per-probe closing pass (the last beta's streaming pass after "
                        "the last step) is closing_ms, as the CG leg's closing update",
           "closing_ms": closing,
           "probe_ms": float(np.sum(st)) + (closing or 0.0),
           "basis": "block" if block else "grid", "launches_per_step": L,
           "mode_product_ms_by_position": [t / steps for t in launch_ms[:L]],
           "bracket_ms": bracket, "bracket_ms_per_step": bracket / max(k, 1),
           "workspace_alloc_s": alloc_s}
    if passes is not None and k > 1:
        byts = 8.0 * n * sum(passes)
        flop = (sum(block_launch_flops(n, m, d)) if block else
                sum((1.0 if (fold_mask >> i) & 1 else 2.0) * n * m for i in range(d)))
        out["roofline"] = {
            "passes_per_step": sum(passes), "passes_by_position": passes,
            "algorithmic_bytes_per_step": byts, "flop_per_step": flop,
            "achieved_gbs": byts / (steady * 1e-3) / 1e9,
            "frac_hbm": byts / (steady * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "achieved_tflops": flop / (steady * 1e-3) / 1e12,
            "frac_mfma": flop / (steady * 1e-3) / 1e12 / FP64_MFMA_PEAK_TFLOPS,
            "basis": "steady steps (2..k): the fused step with the update pass as the "
                     "first launch's prologue" + (" (parity-block basis: the probe folded "
                                                  "once, d - 1 launches per step)" if block
                                                  else "")}
    return out


def time_matvec(K, n, m, d, fold_mask, torch, dev, reps=5):
    """The north star's literal Kron-matvec: y = K x (no shift, no CG fusion)
    on the 200^4 operator, inputs resident, reps back-to-back matvecs after one
    warm-up, HIP events around every mode product on the library's stream
    (gg_kron_matvec_timed).  Roofline: 2 passes (X read, Y written) per mode
    product = 16 N bytes; n m MFMA FLOP per folded factor (2 n m dense)."""
    dk = K._device()
    x = grid_rhs_device(m, d, torch, dev)
    y = torch.empty_like(x)
    dk.matvec(x, out=y)          # warm-up (and the scratch allocation)
    torch.cuda.synchronize()
    per, tot = dk.matvec_timed(x, y, reps)
    del x, y
    ms = tot / reps
    byts = 16.0 * n * d
    flop = sum((1.0 if (fold_mask >> i) & 1 else 2.0) * n * m for i in range(d))
    pos = [t / reps for t in per]
    return {"reps": reps, "ms": ms, "mode_product_ms_by_position": pos,
            "ms_source": "HIP events around every mode product on the library's stream "
                         "(gg_kron_matvec_timed)",
            "algorithmic_bytes": byts, "passes": 2 * d, "flop": flop,
            "achieved_gbs": byts / (ms * 1e-3) / 1e9,
            "frac_hbm": byts / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "achieved_tflops": flop / (ms * 1e-3) / 1e12,
            "frac_mfma": flop / (ms * 1e-3) / 1e12 / FP64_MFMA_PEAK_TFLOPS,
            "dense_equivalent_tflops": d * 2.0 * n * m / (ms * 1e-3) / 1e12,
            "launch_frac_hbm": [16.0 * n / (t * 1e-3) / 1e9 / HBM_PEAK_GBS for t in pos]}


def time_block_matvec(K, n, m, d, torch, dev, reps=5):
    """The same operator in the parity-block basis (what the CG iterations
    apply): y_b = (P K P^T) x_b with x_b resident in
    the block layout, d - 1 launches (gg_kron_block_matvec_timed, HIP events
    per launch).  Bytes: 2 passes per launch (in place; the pair launch reads
    its slab once and writes it once) = 16 N (d - 1); FLOP n m per h x h
    factor applied (the same MFMA work as the folded grid-basis matvec)."""
    dk = K._device()
    x = grid_rhs_device(m, d, torch, dev)
    y = torch.empty_like(x)
    dk.block_matvec(x, out=y)    # warm-up (and the scratch allocation)
    torch.cuda.synchronize()
    per, tot = dk.block_matvec_timed(x, y, reps)
    del x, y
    dk.release_work()
    L = d - 1
    ms = tot / reps
    byts = 16.0 * n * L
    flop = float(sum(block_launch_flops(n, m, d)))
    pos = [t / reps for t in per]
    return {"reps": reps, "ms": ms, "launch_ms": pos, "launches": L,
            "ms_source": "HIP events around every launch on the library's stream "
                         "(gg_kron_block_matvec_timed)",
            "algorithmic_bytes": byts, "passes": 2 * L, "flop": flop,
            "achieved_gbs": byts / (ms * 1e-3) / 1e9,
            "frac_hbm": byts / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
            "achieved_tflops": flop / (ms * 1e-3) / 1e12,
            "frac_mfma": flop / (ms * 1e-3) / 1e12 / FP64_MFMA_PEAK_TFLOPS,
            "launch_frac_mfma": [f / (t * 1e-3) / 1e12 / FP64_MFMA_PEAK_TFLOPS
                                 for f, t in zip(block_launch_flops(n, m, d), pos)],
            "launch_frac_hbm": [16.0 * n / (t * 1e-3) / 1e9 / HBM_PEAK_GBS for t in pos]}


# ---------------------------------------------------------------- the box
class ClockSampler(object):
    """GPU 0's clocks, temperatures and power sampled by amdsmi every
    `period` s on a background thread (the timed CG region; VERDICT r05 item 2:
    every bench line explains its box).  Reports min / mean / max per field
    and the board's identity; {"error": ...} where amdsmi is unavailable."""

    def __init__(self, period=0.05):
        import threading
        self.period = period
        self.samples = []
        self.error = None
        self.ident = {}
        self._stop = threading.Event()
        self._thr = None
        try:
            import amdsmi
            amdsmi.amdsmi_init()
            self.smi = amdsmi
            self.h = amdsmi.amdsmi_get_processor_handles()[0]
            try:
                self.ident["bdf"] = amdsmi.amdsmi_get_gpu_device_bdf(self.h)
            except Exception:  # noqa: BLE001
                pass
            try:
                self.ident["serial"] = amdsmi.amdsmi_get_gpu_board_info(self.h).get(
                    "product_serial")
            except Exception:  # noqa: BLE001
                pass
        except Exception as e:  # noqa: BLE001
            self.smi = None
            self.error = "%s: %s" % (type(e).__name__, e)

    def sample(self):
        smi, h = self.smi, self.h
        rec = {}
        for key, typ in (("gfx_mhz", "GFX"), ("mem_mhz", "MEM"), ("fclk_mhz", "DF")):
            try:
                rec[key] = float(smi.amdsmi_get_clock_info(h, getattr(smi.AmdSmiClkType, typ))
                                 ["clk"])
            except Exception:  # noqa: BLE001
                pass
        for key, typ in (("temp_hotspot_c", "HOTSPOT"), ("temp_mem_c", "VRAM")):
            try:
                rec[key] = float(smi.amdsmi_get_temp_metric(
                    h, getattr(smi.AmdSmiTemperatureType, typ),
                    smi.AmdSmiTemperatureMetric.CURRENT))
            except Exception:  # noqa: BLE001
                pass
        try:
            p = smi.amdsmi_get_power_info(h)
            v = p.get("socket_power", p.get("current_socket_power"))
            if v not in (None, "N/A"):
                rec["power_w"] = float(v)
        except Exception:  # noqa: BLE001
            pass
        return rec

    def _run(self):
        while not self._stop.is_set():
            self.samples.append(self.sample())
            self._stop.wait(self.period)

    def __enter__(self):
        if self.smi is not None:
            import threading
            self._thr = threading.Thread(target=self._run, daemon=True)
            self._thr.start()
        return self

    def __exit__(self, *exc):
        if self._thr is not None:
            self._stop.set()
            self._thr.join()
        return False

    def report(self):
        if self.smi is None:
            return {"error": self.error}
        out = {"samples": len(self.samples), "period_s": self.period, "gpu": self.ident,
               "source": "amdsmi on GPU 0 during the timed CG iterations"}
        keys = sorted({k for s in self.samples for k in s})
        for k in keys:
            v = [s[k] for s in self.samples if k in s]
            out[k] = {"min": min(v), "mean": float(np.mean(v)), "max": max(v)}
        return out


# ---------------------------------------------------------------- main
def main():
    a = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and a.gpus > 1:
        sys.exit(launch_ranks(a))
    world = int(world_env or 1)
    if world != a.gpus:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE=%d" % (a.gpus, world))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    backend = os.environ.get("GG_BENCH_BACKEND", "nccl")
    # gloo-gpu (rehearsal on a box with fewer GPUs than ranks): the ranks'
    # work on the GPUs (rank % count), their collectives over gloo
    on_gpu = backend in ("nccl", "gloo-gpu")
    if world > 1:
        import torch.distributed as dist
        if on_gpu:
            torch.cuda.set_device(local % max(torch.cuda.device_count(), 1))
        dist.init_process_group("gloo" if backend == "gloo-gpu" else backend)
        dev = torch.device("cuda", torch.cuda.current_device()) if on_gpu \
            else torch.device("cpu")
        res = run_sharded(a, world, rank, torch, dev, dist, on_gpu, backend)
        if on_gpu and a.grief != "off":
            # P2 beside it: BASELINE C4 is the 4-GPU GRIEF config, C5 the
            # 8-GPU one -- data rows sharded, Gram / Phi^T y all-reduced
            names = {4: ["C4"], 8: ["C5"]}.get(world, [])
            torch.cuda.empty_cache()
            res["grief"] = grief_leg(names, torch, False, dist=dist, world=world, rank=rank) \
                if names else {"skipped": "the sharded GRIEF leg runs C4 at N = 4 and C5 at "
                                          "N = 8 (BASELINE configs[3], [4])"}
        if rank == 0:
            print(json.dumps(res), flush=True)
        dist.destroy_process_group()
        return

    dev = torch.device("cuda", torch.cuda.current_device())
    import gp_grief_amd as gg
    m, d, s = a.grid, a.dims, a.sigma2
    K, F = grid_factors(m, d)
    n = m ** d
    y = grid_rhs_device(m, d, torch, dev)
    solver = gg.linalg.KronCG(K, s, recurrence=a.recurrence,
                              fusion=a.fusion if a.recurrence == "fused" else None)
    solver.start(y, rtol=0.0, atol=0.0)   # never "converges": exactly the steps asked for
    torch.cuda.synchronize()
    # this box's memory floor for the prologue launch: its six streams alone
    # over the same buffers (gg_cg_calibrate), before any iteration
    cal_ms, cal_off = solver.calibrate(5)

    # ---- CG: warmup, then exactly `steps` iterations bracketed by sync.  The
    # recurrence stays open across the two calls (steady state, as inside a
    # long solve: the timed iterations continue the warm-up's, each doing its
    # full share of the vector work); the closing update -- the last r update
    # and the deferred x steps, once per solve -- runs after the timed region
    # and is reported beside it (closing_ms)
    solver.iterate(a.warmup, check_every=0, close=False)
    torch.cuda.synchronize()
    # live kernel timing: HIP events around every mode product of the timed
    # iterations, recorded by the library on the stream the kernels run on
    solver.profile(True)
    torch.cuda.synchronize()
    clocks = ClockSampler()
    with clocks:
        t0 = time.perf_counter()
        solver.iterate(a.steps, check_every=0, close=False)
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    n_mv, mode_ms = solver.profile_read()
    solver.profile(False)
    assert n_mv == a.steps, (n_mv, a.steps)
    c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    c0.record()
    solver.close()
    c1.record()
    torch.cuda.synchronize()
    closing_ms = c0.elapsed_time(c1)
    it, conv, res, tol = solver.status()
    assert it == a.warmup + a.steps, (it, a.warmup, a.steps)
    assert np.isfinite(res)

    ms_per_step = 1e3 * dt / a.steps
    per_pos = [t / n_mv for t in mode_ms]
    fold_mask = K._device().fold_mask()
    block = solver.basis == "block"
    roof, extra = roofline_report(per_pos, n, m, d, solver.recurrence, ms_per_step,
                                  solver.fusion, fold_mask, solver.xdefer, solver.rq, block,
                                  solver.xwin, solver.rderive)
    # the block basis has no per-factor fold state (tools/pmc_block.py records 0)
    traffic, src = pmc_traffic(m, d, roof["positions"], solver.recurrence, solver.fusion or 0,
                               0 if block else fold_mask, solver.xdefer, solver.rq, block,
                               solver.xwin, solver.rderive)
    roof["traffic"], roof["traffic_source"] = traffic, src
    result = {
        "metric": METRIC,
        "value": a.steps / dt,
        "unit": "CG iters/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic",
        "config": {"workload": "4D RBF grid %d^%d, CG on (K + %g I) x = y, N = %d"
                               % (m, d, s, n),
                   "grid": m, "dims": d, "sigma2": s, "n": n,
                   "cg_recurrence": solver.recurrence,
                   "cg_fusion_layout": solver.fusion,
                   "cg_x_deferred": solver.xdefer,
                   "cg_x_window": solver.xwin,
                   "cg_r_derived": solver.rderive,
                   "cg_rq_identity": solver.rq,
                   "cg_basis": solver.basis,
                   "launches_per_iteration": solver.launches(),
                   "fold_mask": fold_mask,
                   "timed_region": "exactly `steps` fused CG iterations continuing the "
                                   "warm-up's open recurrence; the once-per-solve closing "
                                   "update (gg_cg_close) after it, timed as closing_ms",
                   "parallelism": "single-gpu"},
        "roofline": roof,
        "closing_ms": closing_ms,
    }
    result.update(extra)
    # the box: the prologue's streams alone on these
    # buffers -- the launch's memory floor here -- beside the launch itself
    rd = bool(getattr(solver, "rderive", False))
    cal_bytes = (5.0 if rd else 6.0) * 8.0 * n
    result["prologue_calibration_gbs"] = cal_bytes / (cal_ms * 1e-3) / 1e9
    result["prologue_calibration"] = {
        "ms": cal_ms, "bytes": cal_bytes,
        "pattern": ("read p_old, p_{j-2}, q; write p_new, q (the derived-r prologue's five "
                    "streams" if rd else
                    "read p_old, r, q; write r, p_new, q (the fused prologue's six streams") +
                   ", its non-temporal mask, no MFMA work; gg_cg_calibrate: a plain "
                   "grid-stride stream kernel, 2 untimed + 5 timed passes -- a reference "
                   "rate for this box, not a bound)",
        "buffer_offsets_mod_2MiB": dict(zip(["r" if not rd else "p_{j-2}", "p_old", "p_new",
                                             "q"], cal_off)),
        "buffers_256B_aligned": all(v % 256 == 0 for v in cal_off),
        "prologue_launch_ms": per_pos[0],
        "prologue_launch_vs_streams": per_pos[0] / cal_ms}
    result["box"] = clocks.report()
    del solver, y
    torch.cuda.empty_cache()
    if a.matvec > 0:
        result["matvec"] = time_matvec(K, n, m, d, fold_mask, torch, dev, a.matvec)
        torch.cuda.empty_cache()
        if K._device().block_info()[0]:
            result["block_matvec"] = time_block_matvec(K, n, m, d, torch, dev, a.matvec)
            torch.cuda.empty_cache()
    if a.lanczos > 0:
        result["lanczos"] = time_lanczos(K, s, a.lanczos, torch, n, m, d, fold_mask)
        torch.cuda.empty_cache()
    if a.grief != "off":
        result["grief"] = grief_leg([c.strip() for c in a.grief.split(",") if c.strip()], torch,
                                    a.cpu_baseline == "auto")
    if a.cpu_baseline == "auto":
        result["cpu_baseline"] = cpu_baseline(F, s, a.cpu_iters)
    print(json.dumps(result), flush=True)


if __name__ == "__main__":
    main()
