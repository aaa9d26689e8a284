"""Sharded Kronecker CG on CPU: world_size 2 (and 4) over gloo.

The orchestration (gp_grief_amd.distributed.DistKronCG, its exchange order and
local layouts) runs unchanged; the arithmetic is the NumPy test engine
(tests/dist_helpers.py).  Checks: the sharded matvec equals the oracle's
global matvec; the sharded CG reproduces the single-process CG, with the
textbook recurrence and with the fused one (one 5-double all-reduce per
iteration, deferred x updates over rotating direction buffers).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle
from conftest import ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, m, d, shift, out_dir, recurrence):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from gp_grief_amd.distributed import DistKronCG, TorchExchange, scatter_global
    from dist_helpers import NumpyEngine, reference_factors
    F = reference_factors(m, d)
    rng = np.random.default_rng(7)
    xg = rng.standard_normal(m ** d)
    eng = NumpyEngine(F, world, rank)
    cg = DistKronCG(eng, TorchExchange(), shift, recurrence=recurrence)
    assert cg.recurrence == recurrence
    xl = torch.from_numpy(scatter_global(xg, [m] * d, world, rank).copy())
    yl = eng.empty()
    cg.apply(xl.clone(), yl)
    b = torch.from_numpy(scatter_global(xg, [m] * d, world, rank).copy())
    # check_every 7: the fused recurrence is left (closing update) and
    # re-entered mid-solve, with the x deferral's pair at every phase
    x, info = cg.solve(b, rtol=1e-10, maxiter=5000, check_every=7)
    it = cg.status()[0]
    np.savez(os.path.join(out_dir, "rank%d.npz" % rank), y=yl.numpy(), x=x.numpy(),
             info=info, iters=it)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("recurrence", ["textbook", "fused"])
@pytest.mark.parametrize("world,m,d", [(2, 8, 3), (2, 6, 2), (4, 8, 4)])
def test_sharded_cg_gloo(tmp_path, world, m, d, recurrence):
    from gp_grief_amd.distributed import gather_global
    from dist_helpers import reference_factors
    shift = 0.05
    port = _free_port()
    mp.start_processes(_worker, args=(world, port, m, d, shift, str(tmp_path), recurrence), nprocs=world,
                       join=True, start_method="spawn")
    res = [np.load(os.path.join(tmp_path, "rank%d.npz" % g)) for g in range(world)]
    F = reference_factors(m, d)
    xg = np.random.default_rng(7).standard_normal(m ** d)
    y = gather_global([r["y"] for r in res], [m] * d)
    ref = oracle.kron_matvec(F, xg)
    assert np.linalg.norm(y - ref) / np.linalg.norm(ref) < 1e-13
    x = gather_global([r["x"] for r in res], [m] * d)
    xs, info, it = oracle.cg_solve(lambda v: oracle.kron_matvec(F, v) + shift * v, xg,
                                   rtol=1e-10)
    assert all(int(r["info"]) == 0 for r in res)
    iters = {int(r["iters"]) for r in res}
    assert len(iters) == 1 and abs(iters.pop() - it) <= max(2, 0.02 * it)
    assert np.linalg.norm(x - xs) / np.linalg.norm(xs) < 1e-8


def test_local_index_map_is_a_partition():
    from gp_grief_amd.distributed import local_index_map
    m = [8, 4, 3]
    idx = np.concatenate([local_index_map(m, 4, g) for g in range(4)])
    assert np.array_equal(np.sort(idx), np.arange(96))
