"""Sharded Kronecker CG with the HIP engine on one MI355X: G virtual ranks run as
threads, each with its own gg_kron_dist handle, exchanging through
tests/dist_helpers.ThreadExchange.  Exercises the device phases and their
all-to-all address maps (OutMap) against the single-GPU operator and the oracle.
"""
import numpy as np
import pytest

import oracle
from dist_helpers import ThreadExchange, reference_factors, run_threads

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("world,m,d", [(2, 8, 2), (2, 12, 3), (4, 16, 4), (8, 24, 3),
                                       (4, 40, 3)])
def test_sharded_matvec_and_cg_virtual_ranks(gpu, world, m, d):
    import torch
    from gp_grief_amd.distributed import (DistKronCG, HipEngine, gather_global,
                                          scatter_global)
    F = reference_factors(m, d)
    xg = np.random.default_rng(3).standard_normal(m ** d)
    shift = 0.05
    ex = ThreadExchange(world)
    engines = [HipEngine(F, world, g) for g in range(world)]

    def body(g):
        ex.bind(g)
        e = engines[g]
        cg = DistKronCG(e, ex, shift)
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
    assert abs(res[0][3] - it) <= max(2, 0.02 * it)
    assert np.linalg.norm(x - xs) / np.linalg.norm(xs) < 1e-8
