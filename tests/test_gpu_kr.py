"""Off-grid P1: the device Khatri-Rao contraction (gg_kr_contract) and
GPGridModel.predict against the oracle (oracle.kr_contract,
oracle.grid_offgrid_predict) and the reference-generated fixture
grid_offgrid.npz (GridKernel.cov_kr KhatriRaoMatrix * alpha; dense variance)."""
import numpy as np
import pytest

import oracle
from conftest import golden

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = np.asarray(a, dtype=np.float64).reshape(-1)
    b = np.asarray(b, dtype=np.float64).reshape(-1)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


@pytest.fixture(scope="module")
def gg(gpu):
    import gp_grief_amd
    import gp_grief_amd.kern  # noqa: F401
    import gp_grief_amd.models  # noqa: F401
    return gp_grief_amd


@pytest.mark.parametrize("ms,M", [([13], 5), ([7, 9], 37), ([5, 6, 7], 300),
                                  ([4, 3, 5, 6], 1), ([3, 4, 2, 5, 3], 129),
                                  ([2, 3, 2, 2, 3, 2, 2, 3], 65),        # d = 8: fused, NF = 7
                                  ([2, 3, 2, 2, 3, 2, 2, 2, 3], 70),     # d = 9: two-pass path
                                  ([300, 1, 130], 200)])
def test_kr_contract_vs_oracle(gg, ms, M):
    rng = np.random.default_rng(len(ms) * 100 + M)
    blocks = [rng.standard_normal((M, m)) for m in ms]
    c = rng.standard_normal(int(np.prod(ms)))
    KR = gg.tensors.KhatriRaoMatrix(blocks, partition=0)
    assert KR.shape == (M, int(np.prod(ms)))
    y = KR * c.reshape(-1, 1)
    assert y.shape == (M, 1)
    assert rel(y, oracle.kr_contract(blocks, c)) < 1e-13


def test_kr_contract_chunked_equals_single(gg):
    """A scratch of the minimum size forces several GEMM chunks on the
    two-pass path (d > 8); results agree and repeated runs are bitwise
    identical (fixed-order reductions)."""
    import torch
    rng = np.random.default_rng(5)
    ms, M = [3, 3, 3, 3, 3, 3, 3, 3, 2], 70      # d = 9: the chunked two-pass path
    blocks = [rng.standard_normal((M, m)) for m in ms]
    c = rng.standard_normal(int(np.prod(ms)))
    KR = gg.tensors.KhatriRaoMatrix(blocks, partition=0)
    cd = torch.from_numpy(c).cuda()
    a = KR.contract(cd).cpu().numpy()
    b = KR.contract(cd, work_elems=1).cpu().numpy()
    b2 = KR.contract(cd, work_elems=1).cpu().numpy()
    assert np.array_equal(b, b2)
    assert rel(a, b) < 1e-14
    f1 = KR.contract(cd).cpu().numpy()
    assert np.array_equal(a, f1)


def test_kr_contract_fused_deterministic(gg):
    import torch
    rng = np.random.default_rng(6)
    ms, M = [37, 41, 29], 333
    blocks = [rng.standard_normal((M, m)) for m in ms]
    c = torch.from_numpy(rng.standard_normal(int(np.prod(ms)))).cuda()
    KR = gg.tensors.KhatriRaoMatrix(blocks, partition=0)
    a = KR.contract(c).cpu().numpy()
    assert np.array_equal(a, KR.contract(c).cpu().numpy())
    assert rel(a, oracle.kr_contract(blocks, c.cpu().numpy())) < 1e-13


def test_kr_wrong_shape_raises(gg):
    KR = gg.tensors.KhatriRaoMatrix([np.ones((3, 4)), np.ones((3, 5))], partition=0)
    with pytest.raises(ValueError):
        KR * np.ones((21, 1))
    with pytest.raises(NotImplementedError):
        gg.tensors.KhatriRaoMatrix([np.ones((3, 4))], partition=1)


def _grid_model(gg, z, tag, solver):
    ms, ls = z[tag + "_m"], z[tag + "_ls"]
    kerns = [gg.kern.RBF(1, variance=1.0, lengthscale=float(l)) for l in ls]
    xg = [np.linspace(0.0, 1.0, int(m)).reshape(-1, 1) for m in ms]
    gk = gg.kern.GridKernel(kerns)
    return gg.models.GPGridModel(xg, z[tag + "_y"].reshape(-1, 1), gk,
                                 noise_var=float(z[tag + "_sigma2"]), solver=solver)


@pytest.mark.parametrize("tag", ["a", "b"])
@pytest.mark.parametrize("solver", ["exact", "cg"])
def test_grid_predict_offgrid_fixture(gg, tag, solver):
    z = golden("grid_offgrid.npz")
    m = _grid_model(gg, z, tag, solver)
    mean, var = m.predict(z[tag + "_xs"])
    assert mean.shape == var.shape == (len(z[tag + "_xs"]), 1)
    tol = 1e-11 if solver == "exact" else 1e-7
    assert rel(mean, z[tag + "_mean"]) < tol
    s = float(z[tag + "_sigma2"])
    assert rel(var - s, z[tag + "_var_latent"]) < 1e-9
    mean2, none = m.predict(z[tag + "_xs"], compute_var=False)
    assert none is None and rel(mean2, mean) < 1e-15


def test_grid_predict_on_grid_points_matches_predict_grid(gg):
    """At the grid nodes the off-grid path equals predict_grid (K alpha and the
    eigen-streamed variance)."""
    z = golden("grid_offgrid.npz")
    m = _grid_model(gg, z, "a", "exact")
    ms = [int(v) for v in z["a_m"]]
    xg = [np.linspace(0.0, 1.0, k) for k in ms]
    idx = np.random.default_rng(0).integers(0, int(np.prod(ms)), 40)
    # flat index -> per-dimension grid coordinates, input dim 0 fastest
    coords = np.stack([xg[i][(idx // int(np.prod(ms[:i]))) % ms[i]] for i in range(len(ms))], 1)
    mean, var = m.predict(coords)
    gm, gv = m.predict_grid()
    assert rel(mean[:, 0], gm[idx, 0]) < 1e-10
    assert rel(var[:, 0], gv[idx, 0]) < 1e-8


def test_grid_predict_offgrid_larger(gg):
    """48^4 grid (5.3M points), 64 test points: mean and variance vs the oracle."""
    rng = np.random.default_rng(9)
    m, d, s = 48, 4, 0.01
    ls = [0.15 * (1 + 0.05 * i) for i in range(d)]
    g = np.linspace(0.0, 1.0, m)
    kerns = [gg.kern.RBF(1, variance=1.0, lengthscale=l) for l in ls]
    gk = gg.kern.GridKernel(kerns)
    y = rng.standard_normal((m ** d, 1))
    model = gg.models.GPGridModel([g.reshape(-1, 1)] * d, y, gk, noise_var=s)
    xs = rng.uniform(0, 1, (64, d))
    mean, var = model.predict(xs)
    factors = [oracle.cov_1d("RBF", g, g, 1.0, ls[d - 1 - f]) + 1e-12 * np.eye(m)
               for f in range(d)]
    blocks = [oracle.cov_1d("RBF", xs[:, d - 1 - f], g, 1.0, ls[d - 1 - f]) for f in range(d)]
    Q, t = oracle.factor_eigh(factors)
    lam = t[0]
    for ti in t[1:]:
        lam = np.multiply.outer(lam, ti).reshape(-1)
    alpha = oracle.solve_schur(Q, lam, y[:, 0], s)
    mo, vo = oracle.grid_offgrid_predict(factors, blocks, np.ones(64), alpha, s)
    assert rel(mean, mo) < 1e-9
    assert rel(var - s, vo) < 1e-8
