"""Parity sharding of the Kronecker CG (gp_grief_amd/distributed.py): the
even / odd basis change, the block-diagonal operator, and the sharded CG
over gloo (world 2 and 4) with the NumPy rank engine against the oracle's
single-process CG."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from conftest import ROOT


def test_centro_split_block_diagonalises():
    from dist_helpers import reference_factors
    from gp_grief_amd.distributed import centro_split
    F = reference_factors(12, 1)[0]
    S, T = centro_split(F)
    m, h = 12, 6
    P = np.zeros((m, m))
    for i in range(h):
        P[i, i] = P[i, m - 1 - i] = np.sqrt(0.5)
        P[h + i, i], P[h + i, m - 1 - i] = np.sqrt(0.5), -np.sqrt(0.5)
    M = P @ F @ P.T
    assert np.abs(M[:h, :h] - S).max() < 1e-14 and np.abs(M[h:, h:] - T).max() < 1e-14
    assert np.abs(M[:h, h:]).max() < 1e-14
    assert np.allclose(S, S.T) and np.allclose(T, T.T)
    assert centro_split(np.random.default_rng(0).random((6, 6))) is None   # not centrosymmetric
    assert centro_split(reference_factors(7, 1)[0]) is None                 # odd order


@pytest.mark.parametrize("world,m,d", [(2, 8, 3), (4, 6, 3), (8, 4, 4), (4, 10, 2)])
def test_parity_fold_roundtrip_and_blocks(world, m, d):
    """unfold(fold(x)) == x; the blocks' local Kronecker products reproduce
    K x (fold(K x) == local K_g fold(x) for every rank)."""
    from dist_helpers import reference_factors
    from gp_grief_amd.distributed import parity_fold, parity_local_factors, parity_unfold
    F = reference_factors(m, d)
    x = np.random.default_rng(1).standard_normal(m ** d)
    loc = parity_fold(x, [m] * d, world)
    assert sum(v.size for v in loc) == x.size
    assert np.abs(parity_unfold(loc, [m] * d) - x).max() < 1e-14
    y = oracle.kron_matvec(F, x)
    yl = parity_fold(y, [m] * d, world)
    for g in range(world):
        Fg = parity_local_factors(F, world, g)
        assert np.abs(oracle.kron_matvec(Fg, loc[g]) - yl[g]).max() < 1e-13 * np.abs(y).max()


def test_parity_ok_rules():
    from dist_helpers import reference_factors
    from gp_grief_amd.distributed import parity_ok
    F = reference_factors(8, 3)
    assert parity_ok(F, 1) and parity_ok(F, 2) and parity_ok(F, 8)
    assert not parity_ok(F, 3) and not parity_ok(F, 16)
    G = list(F)
    G[1] = np.random.default_rng(2).random((8, 8))
    assert parity_ok(G, 2) and not parity_ok(G, 4)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, m, d, shift, out_dir):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gp_grief_amd.distributed import ParityShardCG, TorchExchange, parity_fold
    from dist_helpers import ParityNumpyEngine, reference_factors
    F = reference_factors(m, d)
    xg = np.random.default_rng(7).standard_normal(m ** d)
    eng = ParityNumpyEngine(F, world, rank, shift)
    cg = ParityShardCG(F, world, rank, TorchExchange(), shift, engine=eng)
    b = torch.from_numpy(parity_fold(xg, [m] * d, world)[rank].copy())
    x, info = cg.solve(b, rtol=1e-10, maxiter=5000, check_every=7)
    np.savez(os.path.join(out_dir, "rank%d.npz" % rank), x=x.numpy(), info=info,
             iters=cg.status()[0])
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,m,d", [(2, 8, 3), (4, 8, 3), (2, 6, 2)])
def test_parity_sharded_cg_gloo(tmp_path, world, m, d):
    from dist_helpers import reference_factors
    from gp_grief_amd.distributed import parity_unfold
    shift = 0.05
    port = _free_port()
    mp.start_processes(_worker, args=(world, port, m, d, shift, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    res = [np.load(os.path.join(tmp_path, "rank%d.npz" % g)) for g in range(world)]
    F = reference_factors(m, d)
    xg = np.random.default_rng(7).standard_normal(m ** d)
    x = parity_unfold([r["x"] for r in res], [m] * d)
    xs, info, it = oracle.cg_solve(lambda v: oracle.kron_matvec(F, v) + shift * v, xg,
                                   rtol=1e-10)
    assert all(int(r["info"]) == 0 for r in res)
    iters = {int(r["iters"]) for r in res}
    assert len(iters) == 1 and abs(iters.pop() - it) <= max(2, 0.02 * it)
    assert np.linalg.norm(x - xs) / np.linalg.norm(xs) < 1e-8
