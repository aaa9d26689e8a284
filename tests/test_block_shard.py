"""Block sharding of the P1 CG (gp_grief_amd/distributed.py, DESIGN.md section
6): the operator in its parity-block basis is block diagonal over the 2^d
parity patterns; rank g of G = 2^K owns blocks [g 2^d / G, (g + 1) 2^d / G)
and the ranks exchange nothing but the five-double all-reduce of each
iteration.  CPU tests: the orchestration (distributed.solve, ParityShardCG)
over gloo processes with the NumPy restatement of the rank engine
(tests/dist_helpers.BlockNumpyEngine), the solution against the oracle CG on
the reference's operator (kron_matrix.py:52-97, oracle.kron_matvec)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_block_range_partitions_the_blocks():
    from gp_grief_amd.distributed import block_range
    for d in (3, 4, 5):
        for world in (1, 2, 4, 8):
            if world > 1 << d:
                continue
            seen = []
            for g in range(world):
                b0, nb = block_range(d, world, g)
                assert nb == (1 << d) // world
                seen += list(range(b0, b0 + nb))
            assert seen == list(range(1 << d))


@pytest.mark.parametrize("world", [2, 4])
def test_rank_blocks_are_the_parity_blocks(world):
    """Rank g's blocks have factor k's parity bit = bit k of g for k < K: the
    same split as parity sharding of factors 0..K-1 (distributed.parity_fold),
    so the rank's operator is its parity block's."""
    from gp_grief_amd.distributed import block_range
    d = 3
    K = world.bit_length() - 1
    for g in range(world):
        b0, nb = block_range(d, world, g)
        for b in range(b0, b0 + nb):
            for k in range(K):
                assert (b >> (d - 1 - k)) & 1 == (g >> (K - 1 - k)) & 1


def test_block_engine_unfold_all_equals_sum_of_rank_unfolds():
    """The all-gather route: the whole unfold of the concatenated shares is
    the sum of the ranks' own unfolds (the all-reduce route), bit for bit up
    to the order of the sum."""
    from dist_helpers import BlockNumpyEngine, reference_factors
    from gp_grief_amd.tensors import KronMatrix
    ms, world = (6, 8, 10), 4
    F = [reference_factors(m, 1)[0] for m in ms]
    Kh = KronMatrix(F, sym=True)
    b = np.random.default_rng(5).standard_normal(int(np.prod(ms)))
    engs = [BlockNumpyEngine(Kh, world, g, 0.1) for g in range(world)]
    shares = [e.fold(b) for e in engs]
    via_gather = engs[0].unfold_all(torch.cat(shares)).numpy()
    via_reduce = sum(e.unfold(x).numpy() for e, x in zip(engs, shares))
    assert np.linalg.norm(via_gather - via_reduce) < 1e-14 * np.linalg.norm(b)
    assert np.linalg.norm(via_gather - b) < 1e-13 * np.linalg.norm(b)


def test_block_engine_fold_unfold_sum_over_ranks():
    """The ranks' unfold contributions sum to P^T of the whole block vector,
    and their folds tile P b."""
    from dist_helpers import BlockNumpyEngine, reference_factors
    from gp_grief_amd.tensors import KronMatrix
    ms, world = (8, 6, 10), 4
    F = [reference_factors(m, 1)[0] for m in ms]
    Kh = KronMatrix(F, sym=True)
    b = np.random.default_rng(3).standard_normal(int(np.prod(ms)))
    engs = [BlockNumpyEngine(Kh, world, g, 0.1) for g in range(world)]
    xb = np.concatenate([e.fold(b).numpy() for e in engs])
    assert np.allclose(xb, oracle.kron.block_fold(b, ms), atol=1e-14, rtol=0)
    back = sum(e.unfold(e.fold(b)).numpy() for e in engs)
    assert np.linalg.norm(back - b) < 1e-13 * np.linalg.norm(b)
    # the ranks' operators are the block operator's diagonal blocks
    y = np.concatenate([e._Kb(e.fold(b).numpy()) for e in engs])
    assert np.allclose(y, oracle.kron.block_matvec(F, oracle.kron.block_fold(b, ms)),
                       atol=1e-12, rtol=0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, ms, shift, out_dir, solution="gather"):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      GG_DIST_SOLUTION=solution)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from dist_helpers import BlockNumpyEngine, reference_factors
    from gp_grief_amd.distributed import TorchExchange, solve
    from gp_grief_amd.tensors import KronMatrix
    F = [reference_factors(m, 1)[0] for m in ms]
    Kh = KronMatrix(F, sym=True)
    b = np.random.default_rng(11).standard_normal(int(np.prod(ms)))
    x, info, it, how = solve(Kh, b, shift, TorchExchange(), rtol=1e-10, maxiter=5000,
                             check_every=7, decomposition="block", engine=BlockNumpyEngine)
    np.savez(os.path.join(out_dir, "rank%d.npz" % rank), x=np.asarray(x), info=info, iters=it,
             how=how)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,ms,solution", [(2, (8, 6, 10), "gather"),
                                               (2, (8, 6, 10), "reduce"),
                                               (4, (6, 8, 8, 6), "gather"),
                                               (8, (6, 6, 8), "gather"),
                                               (8, (6, 6, 8), "reduce")])
def test_block_sharded_solve_gloo(tmp_path, world, ms, solution):
    """distributed.solve over gloo processes: every rank gets the whole x,
    equal to the oracle CG's on the reference operator (x to 1e-8, iteration
    counts within 2 %; the sharded fused recurrence restarts a cancelled
    beta instead of repairing it).  The solution comes back by an all-gather
    of the block shares + the whole unfold (default) or by each rank's
    unfold summed in an all-reduce (GG_DIST_SOLUTION=reduce)."""
    from dist_helpers import reference_factors
    shift = 0.05
    port = _free_port()
    mp.start_processes(_worker, args=(world, port, ms, shift, str(tmp_path), solution),
                       nprocs=world, join=True, start_method="spawn")
    res = [np.load(os.path.join(tmp_path, "rank%d.npz" % g)) for g in range(world)]
    F = [reference_factors(m, 1)[0] for m in ms]
    b = np.random.default_rng(11).standard_normal(int(np.prod(ms)))
    xs, info, it = oracle.cg_solve(lambda v: oracle.kron_matvec(F, v) + shift * v, b,
                                   rtol=1e-10)
    assert all(str(r["how"]) == "block" and int(r["info"]) == 0 for r in res)
    iters = {int(r["iters"]) for r in res}
    assert len(iters) == 1 and abs(iters.pop() - it) <= max(2, 0.02 * it)
    for r in res:
        assert np.linalg.norm(r["x"] - xs) / np.linalg.norm(xs) < 1e-8
