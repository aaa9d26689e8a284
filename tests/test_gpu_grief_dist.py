"""P2 (GRIEF) sharded over data rows: G virtual ranks (threads on one MI355X),
each holding its rows of X / Y and its own replica of the basis, reduce the
Gram, the Phi^T v products and the scalars through
tests/dist_helpers.ThreadExchange (the stand-in for RCCL all-reduce).  Every
rank must reproduce the reference-generated fixture values that the
unsharded model matches (LML, gradient, predictive mean and covariance, to
the north star's 1e-6 relative)."""
import numpy as np
import pytest

from conftest import golden
from dist_helpers import ThreadExchange, run_threads

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = np.asarray(a, dtype=np.float64).reshape(-1)
    b = np.asarray(b, dtype=np.float64).reshape(-1)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


@pytest.mark.parametrize("case,world", [("3d", 2), ("6d", 3), ("8d", 4)])
def test_grief_row_sharded_matches_fixture(gpu, case, world):
    import gp_grief_amd as gg
    import gp_grief_amd.grid  # noqa: F401
    import gp_grief_amd.kern  # noqa: F401
    import gp_grief_amd.models  # noqa: F401
    z = golden("grief_small_%s.npz" % case)
    d = z["x"].shape[1]
    n = z["x"].shape[0]
    kind = str(z["kind"])
    bounds = np.linspace(0, n, world + 1).astype(int)  # uneven shards allowed
    ex = ThreadExchange(world)

    def body(g):
        ex.bind(g)
        kl = [getattr(gg.kern, kind)(1, variance=1.0, lengthscale=float(l))
              for l in z["lengthscales"]]
        grid = gg.grid.InducingGrid(xg=[np.linspace(0, 1, int(z["m"])).reshape(-1, 1)
                                        for _ in range(d)])
        kern = gg.kern.GriefKernel(kern_list=kl, grid=grid, n_eigs=int(z["p"]))
        lo, hi = bounds[g], bounds[g + 1]
        m = gg.models.GPGriefModel(z["x"][lo:hi], z["y"][lo:hi].reshape(-1, 1), kern,
                                   noise_var=float(z["sigma2"]), comm=ex)
        assert m.num_data == n
        ll, grad = m.log_likelihood(return_gradient=True)
        mean, var = m.predict(z["xtest"])
        return float(ll[0, 0]), grad.copy(), mean, var

    res = run_threads(world, body)
    p = int(z["p"])
    for ll, grad, mean, var in res:
        assert abs(ll - z["lml"]) < 1e-6 * abs(z["lml"])
        assert rel(mean[:, 0], z["pred_mean"]) < 1e-6
        assert rel(var, z["pred_var"]) < 1e-6
        assert rel(grad[-p:], z["grad"][-p:]) < 1e-6
        assert abs(grad[0] - z["grad"][0]) < 1e-6 * abs(z["grad"][0])
    # every rank holds the same answer
    assert max(abs(r[0] - res[0][0]) for r in res) <= 1e-9 * abs(res[0][0])


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _grief_rank(rank, world, port, case, solver, out_dir):
    """One process per rank (one GPU each on a multi-GPU node, all on cuda:0
    on one GPU): GPGriefModel(comm=TorchExchange()) over a real
    torch.distributed group."""
    import os
    import sys
    from conftest import ROOT
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from dist_helpers import bind_device
    bind_device(rank)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import gp_grief_amd as gg
    import gp_grief_amd.grid  # noqa: F401
    import gp_grief_amd.kern  # noqa: F401
    import gp_grief_amd.models  # noqa: F401
    from gp_grief_amd.distributed import TorchExchange
    z = golden("grief_small_%s.npz" % case)
    d, n = z["x"].shape[1], z["x"].shape[0]
    kl = [getattr(gg.kern, str(z["kind"]))(1, variance=1.0, lengthscale=float(l))
          for l in z["lengthscales"]]
    grid = gg.grid.InducingGrid(xg=[np.linspace(0, 1, int(z["m"])).reshape(-1, 1)
                                    for _ in range(d)])
    kern = gg.kern.GriefKernel(kern_list=kl, grid=grid, n_eigs=int(z["p"]))
    lo, hi = np.linspace(0, n, world + 1).astype(int)[rank:rank + 2]
    m = gg.models.GPGriefModel(z["x"][lo:hi], z["y"][lo:hi].reshape(-1, 1), kern,
                               noise_var=float(z["sigma2"]), comm=TorchExchange(),
                               p_solver=solver)
    ll, grad = m.log_likelihood(return_gradient=True)
    mean, var = m.predict(z["xtest"])
    np.savez(os.path.join(out_dir, "rank%d.npz" % rank), ll=float(ll[0, 0]), grad=grad,
             mean=mean, var=var, n=m.num_data)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("case,world,solver", [("3d", 2, "chol"), ("8d", 2, "cg")])
def test_grief_row_sharded_processes(gpu, tmp_path, case, world, solver):
    """The sharded GRIEF fit across real processes (torch.distributed, gloo;
    the driver's multi-GPU runs use the same code over RCCL): every rank
    reproduces the fixture at 1e-6."""
    import os
    import torch.multiprocessing as mp
    port = _free_port()
    mp.start_processes(_grief_rank, args=(world, port, case, solver, str(tmp_path)),
                       nprocs=world, join=True, start_method="spawn")
    z = golden("grief_small_%s.npz" % case)
    p = int(z["p"])
    for g in range(world):
        r = np.load(os.path.join(tmp_path, "rank%d.npz" % g))
        assert int(r["n"]) == z["x"].shape[0]
        assert abs(float(r["ll"]) - z["lml"]) < 1e-6 * abs(z["lml"])
        assert rel(r["mean"][:, 0], z["pred_mean"]) < 1e-6
        assert rel(r["var"], z["pred_var"]) < 1e-6
        assert rel(r["grad"][-p:], z["grad"][-p:]) < 1e-6
