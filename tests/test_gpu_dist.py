"""Sharded Kronecker CG with the HIP engine on one MI355X.

Virtual ranks: G ranks run as threads of one process, each with its own
gg_kron_dist handle, exchanging through tests/dist_helpers.ThreadExchange
(all-to-all mode) or storing straight into each other's buffers (push mode,
plain device pointers).  Process ranks: two processes share the GPU, learn
each other's exchange buffers by IPC handle (the path a one-process-per-GPU
run takes) and synchronise over gloo.  Both check the device phases and
their address maps (OutMap) against the oracle.
"""
import os
import socket

import numpy as np
import pytest

import oracle
from conftest import ROOT
from dist_helpers import ThreadExchange, reference_factors, run_threads

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("fold", ["dense", "fold"])
@pytest.mark.parametrize("mode", ["push", "a2a"])
@pytest.mark.parametrize("world,m,d", [(2, 8, 2), (2, 12, 3), (4, 16, 4), (8, 24, 3),
                                       (4, 40, 3), (2, 200, 2)])
def test_sharded_matvec_and_cg_virtual_ranks(gpu, monkeypatch, world, m, d, mode, fold):
    """fold: every factor on the centrosymmetric split (GG_KRON_FOLD_MIN=8) --
    identity and OutMap (all-to-all order / peer push) epilogues, with and
    without the textbook CG prologue; m = 200 with the 4x4x4 tails."""
    import torch
    from gp_grief_amd.distributed import (DistKronCG, HipEngine, gather_global,
                                          scatter_global)
    if fold == "fold":
        monkeypatch.setenv("GG_KRON_FOLD_MIN", "8")
    else:
        monkeypatch.setenv("GG_KRON_FOLD", "0")
    F = reference_factors(m, d)
    xg = np.random.default_rng(3).standard_normal(m ** d)
    shift = 0.05
    ex = ThreadExchange(world)
    engines = [HipEngine(F, world, g) for g in range(world)]
    assert engines[0].fold_mask == ((1 << d) - 1 if fold == "fold" else 0)

    def body(g):
        ex.bind(g)
        e = engines[g]
        cg = DistKronCG(e, ex, shift, mode=mode)
        assert cg.mode == mode
        xl = torch.from_numpy(scatter_global(xg, [m] * d, world, g).copy()).cuda()
        yl = e.empty()
        cg.apply(xl.clone(), yl)
        x, info = cg.solve(xl, rtol=1e-10, maxiter=3000, check_every=25)
        torch.cuda.synchronize()
        return yl.cpu().numpy(), x.cpu().numpy(), info, cg.status()[0]

    res = run_threads(world, body)
    y = gather_global([r[0] for r in res], [m] * d)
    ref = oracle.kron_matvec(F, xg)
    assert np.linalg.norm(y - ref) / np.linalg.norm(ref) < 1e-12
    x = gather_global([r[1] for r in res], [m] * d)
    xs, info, it = oracle.cg_solve(lambda v: oracle.kron_matvec(F, v) + shift * v, xg,
                                   rtol=1e-10)
    assert all(r[2] == 0 for r in res)
    assert len({r[3] for r in res}) == 1
    # finite-precision CG drifts with summation order: at 750 iterations
    # (m = 200, d = 2) the folded product and the oracle's dense one differ
    # by a few %, as the single-GPU fused / textbook comparison allows
    # (test_gpu_kron); the dense cases keep the 2 % bound
    slack = 0.05 if (fold == "fold" and m == 200) else 0.02
    assert abs(res[0][3] - it) <= max(2, slack * it)
    assert np.linalg.norm(x - xs) / np.linalg.norm(xs) < 1e-8


@pytest.mark.parametrize("recurrence", ["fused", "textbook"])
@pytest.mark.parametrize("mode", ["push", "a2a"])
@pytest.mark.parametrize("world,m,d,shift", [(2, 16, 4, 0.05), (4, 16, 4, 0.05),
                                             (8, 16, 4, 0.05), (2, 12, 5, 0.05),
                                             (4, 32, 4, 1.0)])
def test_sharded_fused_cg_virtual_ranks(gpu, monkeypatch, world, m, d, shift, mode, recurrence):
    """The fused sharded recurrence (gg_kron_dist_phase1_fused + gg_cgs_fused_*:
    CG prologue and deferred x side job inside phase 1, one 5-double
    all-reduce per iteration) against the oracle's CG and the textbook
    sharded recurrence; check_every 7 leaves and re-enters it mid-solve.
    32^4 takes the larger shift: at 0.05 it needs more than 3000 iterations
    (24^4 already 2994 in the oracle)."""
    import torch
    from gp_grief_amd.distributed import DistKronCG, HipEngine, gather_global, scatter_global
    monkeypatch.setenv("GG_KRON_FOLD_MIN", "8")
    F = reference_factors(m, d)
    xg = np.random.default_rng(5).standard_normal(m ** d)
    ex = ThreadExchange(world)
    engines = [HipEngine(F, world, g) for g in range(world)]
    assert all(e.supports_fused for e in engines)

    def body(g):
        ex.bind(g)
        e = engines[g]
        cg = DistKronCG(e, ex, shift, mode=mode, recurrence=recurrence)
        assert cg.recurrence == recurrence
        b = torch.from_numpy(scatter_global(xg, [m] * d, world, g).copy()).cuda()
        x, info = cg.solve(b, rtol=1e-10, maxiter=3000, check_every=7)
        torch.cuda.synchronize()
        return x.cpu().numpy(), info, cg.status()[0]

    res = run_threads(world, body)
    x = gather_global([r[0] for r in res], [m] * d)
    xs, info, it = oracle.cg_solve(lambda v: oracle.kron_matvec(F, v) + shift * v, xg,
                                   rtol=1e-10)
    assert all(r[1] == 0 for r in res)
    assert len({r[2] for r in res}) == 1
    assert abs(res[0][2] - it) <= max(2, 0.02 * it)
    assert np.linalg.norm(x - xs) / np.linalg.norm(xs) < 1e-8


def test_fused_recurrence_default_and_refusal(gpu, monkeypatch):
    """recurrence "auto" picks the fused one exactly where the engine supports
    it (d >= 4, factors 1..d-1 folded); asking for it elsewhere is an error."""
    from gp_grief_amd.distributed import DistKronCG, HipEngine
    ex = ThreadExchange(1)
    ex.bind(0)
    monkeypatch.setenv("GG_KRON_FOLD_MIN", "8")
    e4 = HipEngine(reference_factors(16, 4), 2, 0)
    assert DistKronCG(e4, ex, 0.1).recurrence == "fused"
    assert DistKronCG(e4, ex, 0.1, recurrence="textbook").recurrence == "textbook"
    e3 = HipEngine(reference_factors(16, 3), 2, 0)
    assert DistKronCG(e3, ex, 0.1).recurrence == "textbook"
    with pytest.raises(ValueError):
        DistKronCG(e3, ex, 0.1, recurrence="fused")
    monkeypatch.setenv("GG_KRON_FOLD", "0")
    monkeypatch.delenv("GG_KRON_FOLD_MIN")
    e4d = HipEngine(reference_factors(16, 4), 2, 0)
    assert DistKronCG(e4d, ex, 0.1).recurrence == "textbook"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _ipc_worker(rank, world, port, m, d, out_dir):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from dist_helpers import bind_device, reference_factors
    bind_device(rank)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gp_grief_amd.distributed import DistKronCG, HipEngine, TorchExchange, scatter_global
    F = reference_factors(m, d)
    xg = np.random.default_rng(11).standard_normal(m ** d)
    eng = HipEngine(F, world, rank)
    cg = DistKronCG(eng, TorchExchange(), 0.05, mode="push")
    xl = torch.from_numpy(scatter_global(xg, [m] * d, world, rank).copy()).cuda()
    yl = eng.empty()
    for _ in range(3):  # repeated: the buffers are reused across matvecs
        cg.apply(xl.clone(), yl)
    x, info = cg.solve(xl, rtol=1e-10, maxiter=3000, check_every=25)
    torch.cuda.synchronize()
    np.savez(os.path.join(out_dir, "rank%d.npz" % rank), y=yl.cpu().numpy(),
             x=x.cpu().numpy(), info=info, iters=cg.status()[0])
    dist.barrier()
    del cg, eng
    dist.destroy_process_group()


@pytest.mark.parametrize("world,m,d,fold", [(2, 16, 3, False), (4, 24, 3, True),
                                            (2, 16, 4, True)])
def test_push_exchange_over_ipc_processes(gpu, tmp_path, monkeypatch, world, m, d, fold):
    """One process per rank (one GPU each on a multi-GPU node, else all on
    cuda:0): exchange buffers shared by IPC handle (gg_ipc_handle /
    gg_kron_dist_set_peers), barriers over gloo; fold: the ranks' factors on
    the centrosymmetric split (the environment is inherited by the ranks);
    d = 4 folded runs the fused recurrence over the peer exchange."""
    import torch.multiprocessing as mp
    from gp_grief_amd.distributed import gather_global
    monkeypatch.setenv("GG_KRON_FOLD_MIN", "8" if fold else "1000")
    port = _free_port()
    mp.start_processes(_ipc_worker, args=(world, port, m, d, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    res = [np.load(os.path.join(tmp_path, "rank%d.npz" % g)) for g in range(world)]
    F = reference_factors(m, d)
    xg = np.random.default_rng(11).standard_normal(m ** d)
    y = gather_global([r["y"] for r in res], [m] * d)
    ref = oracle.kron_matvec(F, xg)
    assert np.linalg.norm(y - ref) / np.linalg.norm(ref) < 1e-12
    x = gather_global([r["x"] for r in res], [m] * d)
    xs, info, it = oracle.cg_solve(lambda v: oracle.kron_matvec(F, v) + 0.05 * v, xg,
                                   rtol=1e-10)
    assert all(int(r["info"]) == 0 for r in res)
    assert np.linalg.norm(x - xs) / np.linalg.norm(xs) < 1e-8


@pytest.mark.parametrize("world,m,d,shift", [(2, 16, 4, 0.05), (4, 16, 4, 0.05),
                                             (8, 16, 4, 0.05), (8, 24, 3, 0.05),
                                             (4, 32, 4, 1.0), (2, 200, 2, 0.05)])
def test_parity_sharded_cg_virtual_ranks(gpu, world, m, d, shift):
    """The parity-sharded CG (ParityShardCG on ParityHipEngine: each rank's
    even / odd block as a resident fused CG split at its one all-reduce,
    gg_cg_*_partial / _finish) on virtual ranks: the blocks' matvecs unfold to
    the oracle's K x, the solution to the oracle CG's (iterations within 2 %,
    x to 1e-8)."""
    import torch
    from gp_grief_amd.distributed import ParityShardCG, parity_fold, parity_unfold
    F = reference_factors(m, d)
    xg = np.random.default_rng(9).standard_normal(m ** d)
    ex = ThreadExchange(world)
    cgs = [ParityShardCG(F, world, g, ex, shift) for g in range(world)]
    bl = parity_fold(xg, [m] * d, world)

    def body(g):
        ex.bind(g)
        cg = cgs[g]
        b = torch.from_numpy(bl[g].copy()).cuda()
        y = cg.e.empty()
        cg.apply(b, y)
        x, info = cg.solve(b, rtol=1e-10, maxiter=4000, check_every=9)
        torch.cuda.synchronize()
        return y.cpu().numpy(), x.cpu().numpy(), info, cg.status()[0]

    res = run_threads(world, body)
    y = parity_unfold([r[0] for r in res], [m] * d)
    ref = oracle.kron_matvec(F, xg)
    assert np.linalg.norm(y - ref) / np.linalg.norm(ref) < 1e-12
    x = parity_unfold([r[1] for r in res], [m] * d)
    xs, info, it = oracle.cg_solve(lambda v: oracle.kron_matvec(F, v) + shift * v, xg,
                                   rtol=1e-10)
    assert all(r[2] == 0 for r in res)
    assert len({r[3] for r in res}) == 1
    # m = 200, d = 2 (ill-conditioned, ~750 iterations): the fused
    # recurrence's beta (|r - alpha q|^2 expanded, r.q by conjugacy) drifts
    # from the textbook's in finite precision -- its NumPy restatement takes
    # 771 iterations against the oracle's 739 (4.3 %) on this system
    slack = 0.07 if m == 200 else 0.02
    assert abs(res[0][3] - it) <= max(2, slack * it)
    assert np.linalg.norm(x - xs) / np.linalg.norm(xs) < 1e-8


def _parity_worker(rank, world, port, m, d, out_dir):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch
    import torch.distributed as dist
    from dist_helpers import bind_device, reference_factors
    bind_device(rank)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gp_grief_amd.distributed import ParityShardCG, TorchExchange, parity_fold
    F = reference_factors(m, d)
    xg = np.random.default_rng(13).standard_normal(m ** d)
    cg = ParityShardCG(F, world, rank, TorchExchange(), 0.05)
    b = torch.from_numpy(parity_fold(xg, [m] * d, world)[rank].copy()).cuda()
    x, info = cg.solve(b, rtol=1e-10, maxiter=3000, check_every=11)
    torch.cuda.synchronize()
    np.savez(os.path.join(out_dir, "rank%d.npz" % rank), x=x.cpu().numpy(), info=info,
             iters=cg.status()[0])
    dist.barrier()
    del cg
    dist.destroy_process_group()


@pytest.mark.parametrize("world,m,d", [(2, 16, 3), (4, 12, 3)])
def test_parity_sharded_cg_processes(gpu, tmp_path, world, m, d):
    """One process per rank (rank g on device g % count), the five-double
    all-reduce through TorchExchange (gloo here; RCCL on a multi-GPU node)."""
    import torch.multiprocessing as mp
    from gp_grief_amd.distributed import parity_unfold
    port = _free_port()
    mp.start_processes(_parity_worker, args=(world, port, m, d, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    res = [np.load(os.path.join(tmp_path, "rank%d.npz" % g)) for g in range(world)]
    F = reference_factors(m, d)
    xg = np.random.default_rng(13).standard_normal(m ** d)
    x = parity_unfold([r["x"] for r in res], [m] * d)
    xs, info, it = oracle.cg_solve(lambda v: oracle.kron_matvec(F, v) + 0.05 * v, xg,
                                   rtol=1e-10)
    assert all(int(r["info"]) == 0 for r in res)
    assert len({int(r["iters"]) for r in res}) == 1
    assert abs(int(res[0]["iters"]) - it) <= max(2, 0.02 * it)
    assert np.linalg.norm(x - xs) / np.linalg.norm(xs) < 1e-8


# ---------------------------------------------------------------- block sharding
@pytest.mark.parametrize("ms,blk0,nblk", [((6, 12, 40, 40), 4, 4), ((8, 72, 72), 2, 2),
                                          ((40, 40, 40, 40), 15, 1), ((6, 12, 40, 40), 0, 16)])
def test_block_fold_and_matvec_range_vs_oracle(gpu, ms, blk0, nblk):
    """gg_kron_block_fold_range / gg_kron_block_matvec_range: a rank's blocks
    of P b, of (P K P^T + s I) x_b, and its contribution to P^T x_b, against
    oracle.kron.block_fold / block_matvec (kron_matrix.py:52-97 restated)."""
    import gp_grief_amd as gg
    F = reference_factors_ms(ms)
    K = gg.tensors.KronMatrix(F, sym=True)
    dk = K._device()
    n = int(np.prod(ms))
    nb = n >> len(ms)
    b = np.random.default_rng(21).standard_normal(n)
    full = oracle.kron.block_fold(b, ms)
    loc = gg.device.to_host(dk.block_fold_range(gg.device.to_device(b), blk0, nblk))
    want = full[blk0 * nb:(blk0 + nblk) * nb]
    assert np.linalg.norm(loc - want) <= 1e-15 * np.linalg.norm(want) + 1e-300
    y = gg.device.to_host(dk.block_matvec_range(gg.device.to_device(want), blk0, nblk,
                                                shift=0.05))
    ref = (oracle.kron.block_matvec(F, full) + 0.05 * full)[blk0 * nb:(blk0 + nblk) * nb]
    assert np.linalg.norm(y - ref) / np.linalg.norm(ref) < 1e-13
    part = np.zeros(n)
    part[blk0 * nb:(blk0 + nblk) * nb] = want
    back = gg.device.to_host(dk.block_fold_range(gg.device.to_device(want), blk0, nblk,
                                                 inverse=True))
    ref = oracle.kron.block_fold(part, ms, inverse=True)
    assert np.linalg.norm(back - ref) <= 1e-15 * np.linalg.norm(ref) + 1e-300


def reference_factors_ms(ms):
    g = [np.linspace(0, 1, m) for m in ms]
    return [oracle.cov_1d("RBF", x, x, 1.0, 0.15 * (1 + 0.1 * k)) + 1e-12 * np.eye(len(x))
            for k, x in enumerate(g)]


@pytest.mark.parametrize("world,ms,shift,solution", [
    (2, (6, 12, 40, 40), 0.05, "gather"), (4, (6, 12, 40, 40), 0.05, "gather"),
    (8, (40, 40, 40, 40), 0.5, "gather"), (16, (6, 12, 40, 40), 0.05, "gather"),
    (4, (8, 72, 72), 0.2, "gather"), (2, (40, 8, 72, 72), 0.1, "gather"),
    (4, (8, 72, 72), 0.2, "reduce"), (8, (40, 40, 40, 40), 0.5, "reduce"),
    # padded pair axes (h = 32 / 24 in slabs of 36 / 36): the shares and the
    # whole block vector carry the zero padding through both routes
    (2, (6, 64, 64), 0.05, "gather"), (4, (4, 8, 48, 48), 0.1, "gather"),
    (4, (4, 8, 48, 48), 0.1, "reduce")])
def test_block_sharded_cg_virtual_ranks(gpu, monkeypatch, world, ms, shift, solution):
    """distributed.solve, block decomposition: each virtual rank (a thread)
    runs the block kernels on its 2^d / G blocks (gg_cg_create_blocks,
    gg_cg_*_partial / _finish), folds b on the device and gets x back by an
    all-gather of the shares + the whole device unfold (default) or by its
    own unfold summed in an all-reduce (GG_DIST_SOLUTION=reduce).  Every
    rank's x equals the oracle CG's (1e-8),
    the iteration count the oracle's and the single-GPU block CG's within 2 %
    (the restart vs repair of a cancelled beta, and the summation order:
    test_restart_penalty_single_gpu separates the two)."""
    import gp_grief_amd as gg
    from gp_grief_amd.distributed import solve
    monkeypatch.setenv("GG_DIST_SOLUTION", solution)
    F = reference_factors_ms(ms)
    K = gg.tensors.KronMatrix(F, sym=True)
    n = int(np.prod(ms))
    b = np.random.default_rng(22).standard_normal(n)
    ex = ThreadExchange(world)

    def body(g):
        ex.bind(g)
        x, info, it, how = solve(K, b, shift, ex, rtol=1e-10, maxiter=20000, check_every=9)
        return gg.device.to_host(x), info, it, how

    res = run_threads(world, body)
    xs, info, it = oracle.cg_solve(lambda v: oracle.kron_matvec(F, v) + shift * v, b,
                                   rtol=1e-10)
    assert all(r[3] == "block" and r[1] == 0 for r in res)
    assert len({r[2] for r in res}) == 1
    assert abs(res[0][2] - it) <= max(2, 0.02 * it)
    for r in res:
        assert np.linalg.norm(r[0] - xs) / np.linalg.norm(xs) < 1e-8
    # against the single-GPU block CG: the sharded recurrence restarts a
    # cancelled beta (p = r) where the single-GPU one repairs it with a true
    # r.r, and its dot products sum in another order -- (6, 12, 40, 40) at
    # 0.05: 1732 vs 1725 iterations with row-major slabs, 1737 vs 1716 with
    # k-step tiled ones (the same arithmetic, other rounding)
    x1, i1 = gg.linalg.cg(K, b[:, None], shift=shift, rtol=1e-10, maxiter=20000)
    assert abs(gg.linalg.cg.last.iters - res[0][2]) <= max(2, 0.02 * res[0][2])


@pytest.mark.parametrize("ms,shift", [((6, 12, 40, 40), 0.05), ((40, 8, 72, 72), 0.02),
                                      ((8, 8, 200, 200), 0.01)])
def test_restart_penalty_single_gpu(gpu, monkeypatch, ms, shift):
    """The restart penalty by itself: gg_cg_iterate repairs a cancelled beta
    with a true r.r (a second pass over r); a sharded rank restarts (p = r)
    to keep one all-reduce per iteration.  GG_CG_RESTART=1 makes the
    single-GPU CG restart too, everything else equal (same layout, same
    kernels, same summation order).  Both solutions equal the oracle's (1e-8);
    the restart's iteration count stays within 2 % of the repair's.  The
    counts are printed (DESIGN.md section 6 quotes them)."""
    import gp_grief_amd as gg
    F = reference_factors_ms(ms)
    K = gg.tensors.KronMatrix(F, sym=True)
    n = int(np.prod(ms))
    b = np.random.default_rng(23).standard_normal(n)
    xs, info, it = oracle.cg_solve(lambda v: oracle.kron_matvec(F, v) + shift * v, b,
                                   rtol=1e-10) if n <= 2_000_000 else (None, 0, None)
    out = {}
    for flag in ("0", "1"):
        monkeypatch.setenv("GG_CG_RESTART", flag)
        cg = gg.linalg.KronCG(K, shift)
        cg.start(gg.device.to_device(b), rtol=1e-10)
        while True:
            cg.iterate(50)
            k, conv, res, tol = cg.status()
            if conv or k >= 20000:
                break
        assert conv
        out[flag] = (k, cg.cancels(), gg.device.to_host(cg.x))
    for flag, (k, c, x) in out.items():
        if xs is not None:
            assert np.linalg.norm(x - xs) / np.linalg.norm(xs) < 1e-8
    (k0, c0, x0), (k1, c1, x1) = out["0"], out["1"]
    print("restart penalty %s shift %g: repair %d iterations (%d cancelled), restart %d (%d)"
          % (ms, shift, k0, c0, k1, c1))
    assert np.linalg.norm(x1 - x0) / np.linalg.norm(x0) < 1e-7
    if c0 == 0:
        assert k1 == k0
    assert abs(k1 - k0) <= max(2, 0.02 * k0)


def test_forced_cancellations_restart_vs_repair(gpu, monkeypatch):
    """Both branches of a cancelled beta, made frequent: GG_CG_CANCEL_TOL=0.3
    counts every step whose |r_{j+1}|^2 expansion is below 0.3 rho_j as
    cancelled (24 of the ~1714 steps of this solve have beta < 0.3; none is
    below the production threshold 1e-6).  The single-GPU CG repairs (true r.r, textbook beta), the
    single-GPU CG with GG_CG_RESTART=1 and a block-sharded solve over two
    virtual ranks restart (p = r).  All three converge to the oracle's x
    (1e-8) with cancellations counted; the iteration counts are the restart
    penalty at that rate (printed)."""
    import gp_grief_amd as gg
    from gp_grief_amd.distributed import solve
    ms, shift = (6, 12, 40, 40), 0.05
    F = reference_factors_ms(ms)
    K = gg.tensors.KronMatrix(F, sym=True)
    b = np.random.default_rng(25).standard_normal(int(np.prod(ms)))
    xs, info, it = oracle.cg_solve(lambda v: oracle.kron_matvec(F, v) + shift * v, b,
                                   rtol=1e-10)
    monkeypatch.setenv("GG_CG_CANCEL_TOL", "0.3")
    out = {}
    for flag in ("0", "1"):
        monkeypatch.setenv("GG_CG_RESTART", flag)
        cg = gg.linalg.KronCG(K, shift)
        cg.start(gg.device.to_device(b), rtol=1e-10)
        while True:
            cg.iterate(50)
            k, conv, res, tol = cg.status()
            if conv or k >= 20000:
                break
        assert conv
        out["restart" if flag == "1" else "repair"] = (k, cg.cancels(), gg.device.to_host(cg.x))
    monkeypatch.setenv("GG_CG_RESTART", "0")
    ex = ThreadExchange(2)

    def body(g):
        ex.bind(g)
        x, info, k, how = solve(K, b, shift, ex, rtol=1e-10, maxiter=20000, check_every=10,
                                decomposition="block")
        assert info == 0 and how == "block"
        return k, solve.last_cancels, gg.device.to_host(x)

    out["sharded"] = run_threads(2, body)[0]
    print("forced cancellations (tol 0.3), oracle %d iterations: %s"
          % (it, ", ".join("%s %d (%d cancelled)" % (n, v[0], v[1]) for n, v in out.items())))
    for n, (k, c, x) in out.items():
        assert c > 0, n
        assert np.linalg.norm(x - xs) / np.linalg.norm(xs) < 1e-8, n
        assert k <= 2 * it, n


@pytest.mark.parametrize("how", ["block", "parity", "transpose"])
def test_ill_conditioned_decompositions_virtual_ranks(gpu, how):
    """(6, 12, 40, 40) at shift 0.05 (cond ~ 1e3, about 1700 iterations to
    1e-10) over 2 virtual ranks in each decomposition: x equals the oracle
    CG's (1e-8) and the iteration count is within 2 % of the oracle's."""
    import gp_grief_amd as gg
    from gp_grief_amd.distributed import solve
    ms, shift, world = (6, 12, 40, 40), 0.05, 2
    F = reference_factors_ms(ms)
    K = gg.tensors.KronMatrix(F, sym=True)
    b = np.random.default_rng(24).standard_normal(int(np.prod(ms)))
    ex = ThreadExchange(world)

    def body(g):
        ex.bind(g)
        x, info, it, got = solve(K, b, shift, ex, rtol=1e-10, maxiter=20000, check_every=11,
                                 decomposition=how)
        return gg.device.to_host(x), info, it, got, solve.last_cancels

    res = run_threads(world, body)
    xs, info, it = oracle.cg_solve(lambda v: oracle.kron_matvec(F, v) + shift * v, b,
                                   rtol=1e-10)
    assert all(r[3] == how and r[1] == 0 for r in res)
    assert len({r[2] for r in res}) == 1
    print("%s: %d iterations (oracle %d), cancelled betas %s" % (how, res[0][2], it, res[0][4]))
    assert abs(res[0][2] - it) <= max(2, 0.02 * it)
    for r in res:
        assert np.linalg.norm(r[0] - xs) / np.linalg.norm(xs) < 1e-8


def test_cg_comm_api_virtual_ranks(gpu):
    """The drop-in entry point: linalg.cg(K, y, comm=...) on every rank
    returns the whole solution (host in, host out), sharded underneath."""
    import gp_grief_amd as gg
    ms, shift, world = (6, 12, 40, 40), 0.05, 4
    F = reference_factors_ms(ms)
    K = gg.tensors.KronMatrix(F, sym=True)
    y = np.random.default_rng(23).standard_normal((int(np.prod(ms)), 1))
    ex = ThreadExchange(world)

    def body(g):
        ex.bind(g)
        x, info = gg.linalg.cg(K, y, shift=shift, rtol=1e-10, comm=ex)
        return x, info, gg.linalg.cg.last.decomposition

    res = run_threads(world, body)
    xs, _, _ = oracle.cg_solve(lambda v: oracle.kron_matvec(F, v) + shift * v, y[:, 0],
                               rtol=1e-10)
    for x, info, how in res:
        assert info == 0 and how == "block" and x.shape == y.shape
        assert np.linalg.norm(x[:, 0] - xs) / np.linalg.norm(xs) < 1e-8


def _block_worker(rank, world, port, out_dir):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from dist_helpers import bind_device
    bind_device(rank)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import gp_grief_amd as gg
    ms = (6, 12, 40, 40)
    F = reference_factors_ms(ms)
    K = gg.tensors.KronMatrix(F, sym=True)
    y = np.random.default_rng(24).standard_normal(int(np.prod(ms)))
    x, info = gg.linalg.cg(K, y, shift=0.05, rtol=1e-10, comm=True)
    np.savez(os.path.join(out_dir, "rank%d.npz" % rank), x=x, info=info,
             iters=gg.linalg.cg.last.iters, how=gg.linalg.cg.last.decomposition)
    dist.barrier()
    dist.destroy_process_group()


def test_block_sharded_cg_processes(gpu, tmp_path):
    """Two processes (rank g on device g % count), linalg.cg(comm=True) over
    the default process group (gloo here; RCCL on a multi-GPU node)."""
    import torch.multiprocessing as mp
    port = _free_port()
    mp.start_processes(_block_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True,
                       start_method="spawn")
    res = [np.load(os.path.join(tmp_path, "rank%d.npz" % g)) for g in range(2)]
    ms = (6, 12, 40, 40)
    F = reference_factors_ms(ms)
    y = np.random.default_rng(24).standard_normal(int(np.prod(ms)))
    xs, _, it = oracle.cg_solve(lambda v: oracle.kron_matvec(F, v) + 0.05 * v, y, rtol=1e-10)
    for r in res:
        assert str(r["how"]) == "block" and int(r["info"]) == 0
        assert abs(int(r["iters"]) - it) <= max(2, 0.02 * it)
        assert np.linalg.norm(r["x"] - xs) / np.linalg.norm(xs) < 1e-8


@pytest.mark.parametrize("m,world", [((10, 12, 9), 2), ((8, 6, 12, 5), 4), ((6, 4, 8), 8)])
def test_device_parity_and_shard0_folds_vs_host(gpu, m, world):
    """gg_parity_fold / gg_shard0_fold (round 6: the parity and transpose
    decompositions' fold / unfold on the device) against the host
    restatements parity_fold / parity_unfold and scatter_global /
    gather_global, every rank; the unfold contributions sum to the vector."""
    import gp_grief_amd as gg
    from gp_grief_amd import distributed as D
    n = int(np.prod(m))
    x = np.random.default_rng(31).standard_normal(n)
    xd = gg.device.to_device(x)
    host = D.parity_fold(x, m, world)
    acc = np.zeros(n)
    for g in range(world):
        loc = gg.device.to_host(D.device_parity_fold(xd, m, world, g))
        assert np.allclose(loc, host[g], rtol=0, atol=1e-14)
        acc += gg.device.to_host(D.device_parity_fold(gg.device.to_device(loc), m, world, g,
                                                      inverse=True))
    assert np.allclose(acc, x, rtol=0, atol=1e-13)
    if m[0] % world == 0:
        acc = np.zeros(n)
        for g in range(world):
            loc = gg.device.to_host(D.device_shard0_fold(xd, m, world, g))
            assert np.array_equal(loc, D.scatter_global(x, m, world, g))
            acc += gg.device.to_host(D.device_shard0_fold(gg.device.to_device(loc), m, world, g,
                                                          inverse=True))
        assert np.array_equal(acc, x)


def _fallback_worker(rank, world, port, out_dir, how):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from dist_helpers import bind_device
    bind_device(rank)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import gp_grief_amd as gg
    from gp_grief_amd.distributed import block_shard_ok
    ms, F = _fallback_problem(how)
    K = gg.tensors.KronMatrix(F, sym=True)
    assert not block_shard_ok(K, world)
    y = np.random.default_rng(25).standard_normal(int(np.prod(ms)))
    x, info = gg.linalg.cg(K, y, shift=0.05, rtol=1e-10, comm=True)
    np.savez(os.path.join(out_dir, "rank%d.npz" % rank), x=x, info=info,
             iters=gg.linalg.cg.last.iters, how=gg.linalg.cg.last.decomposition)
    dist.barrier()
    dist.destroy_process_group()


def _fallback_problem(how):
    """A grid where the block decomposition does not exist: an odd order
    (parity sharding on the even factor 0), or factor 0 not centrosymmetric
    (the transpose decomposition)."""
    ms = (10, 12, 9) if how == "parity" else (10, 8, 12)
    F = reference_factors_ms(ms)
    if how == "transpose":
        F[0] = F[0] + np.diag(np.linspace(0.0, 0.2, ms[0]))   # breaks J F J = F
    return ms, F


@pytest.mark.parametrize("how", ["parity", "transpose"])
def test_fallback_decompositions_processes(gpu, tmp_path, how):
    """linalg.cg(comm=True) over two gloo processes on a grid without the
    block basis: the 'auto' decomposition falls back to parity / transpose
    sharding, whose fold and unfold now run on the device (one all-reduce of
    the grid vector instead of gathered host arrays) -- x against the oracle."""
    import torch.multiprocessing as mp
    port = _free_port()
    mp.start_processes(_fallback_worker, args=(2, port, str(tmp_path), how), nprocs=2,
                       join=True, start_method="spawn")
    res = [np.load(os.path.join(tmp_path, "rank%d.npz" % g)) for g in range(2)]
    ms, F = _fallback_problem(how)
    y = np.random.default_rng(25).standard_normal(int(np.prod(ms)))
    xs, _, it = oracle.cg_solve(lambda v: oracle.kron_matvec(F, v) + 0.05 * v, y, rtol=1e-10)
    for r in res:
        assert str(r["how"]) == how and int(r["info"]) == 0
        assert abs(int(r["iters"]) - it) <= max(2, 0.02 * it)
        assert np.linalg.norm(r["x"] - xs) / np.linalg.norm(xs) < 1e-8
