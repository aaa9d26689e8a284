"""The persistent LDS-DMA ring version of the folded mode product
(gg_kron_ring.hip, GG_FOLD_RING=<variant>) on the MI355X.

Same arithmetic as mode_product_fold_kernel -- the same u / v operands, the
same fragment order and k-step order, the same tail handling -- so the plain
matvec must agree BITWISE with the chunked folded kernel (and with the dense
oracle, kron_matrix.py:52-97's product, at 1e-13) for every ring variant:
partial last blocks, M not a multiple of the block, a workgroup walking many
blocks (the ring running across block boundaries), the factor at any mode
position, the transposed operator of a centrosymmetric non-symmetric factor.
"""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

VARIANTS = ["1"]   # the ring (one configuration since round 5); "0" is the chunked kernel


def rel(a, b):
    a = np.asarray(a, dtype=np.float64).reshape(-1)
    b = np.asarray(b, dtype=np.float64).reshape(-1)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


@pytest.fixture(scope="module")
def gg(gpu):
    import gp_grief_amd
    return gp_grief_amd


def grid_factor(m, ell=0.15, kind="RBF"):
    g = np.linspace(0.0, 1.0, m)
    return oracle.cov_1d(kind, g, g, 1.0, ell) + 1e-12 * np.eye(m)


def run(gg, monkeypatch, F, x, variant, transpose=False, sym=True):
    import torch
    monkeypatch.setenv("GG_FOLD_RING", variant)
    K = gg.tensors.KronMatrix(F, sym=sym)
    dk = K._device()
    xd = torch.from_numpy(np.ascontiguousarray(x)).cuda()
    y = dk.matvec(xd, transpose=transpose)
    torch.cuda.synchronize()
    return y.cpu().numpy()


@pytest.mark.parametrize("dims", [(200, 40, 36), (36, 200, 40), (40, 36, 200), (200, 7, 3)])
def test_ring_matches_fold_kernel(gg, monkeypatch, dims):
    F = [grid_factor(m, 0.1 + 0.02 * k) if m != 200 else grid_factor(200, 0.1 + 0.02 * k)
         for k, m in enumerate(dims)]
    n = int(np.prod(dims))
    x = np.random.default_rng(n).standard_normal(n)
    y0 = run(gg, monkeypatch, F, x, "0")
    ref = oracle.kron_matvec(F, x)
    assert rel(y0, ref) < 1e-13
    for v in VARIANTS:
        y = run(gg, monkeypatch, F, x, v)
        assert np.array_equal(y, y0), (v, rel(y, y0))


def test_ring_many_blocks_per_workgroup(gg, monkeypatch):
    """200^3 x 4: M = 160000 rows b for each 200-factor, about five blocks per
    workgroup -- the ring crosses block boundaries with epilogues in the
    counted window."""
    dims = (200, 200, 200, 4)
    F = [grid_factor(200, 0.1), grid_factor(200, 0.13), grid_factor(200, 0.2, "Matern52"),
         grid_factor(4, 0.5)]
    n = int(np.prod(dims))
    x = np.random.default_rng(1).standard_normal(n)
    y0 = run(gg, monkeypatch, F, x, "0")
    for v in VARIANTS:
        y = run(gg, monkeypatch, F, x, v)
        assert np.array_equal(y, y0), (v, rel(y, y0))
    # a sampled check against the oracle's entry formula
    rng = np.random.default_rng(2)
    idx = rng.integers(0, n, 64)
    Kd = [np.asarray(f) for f in F]
    xs = x.reshape(dims)
    for g in idx[:8]:
        i = np.unravel_index(int(g), dims)
        row = Kd[0][i[0]][:, None, None, None] * Kd[1][i[1]][None, :, None, None] * \
            Kd[2][i[2]][None, None, :, None] * Kd[3][i[3]][None, None, None, :]
        assert abs(float(np.sum(row * xs)) - y0[g]) <= 1e-12 * np.abs(row * xs).sum()


def test_ring_transposed_nonsymmetric(gg, monkeypatch):
    rng = np.random.default_rng(4)
    C = rng.standard_normal((200, 200))
    Fc = C + C[::-1, ::-1]
    F = [Fc, grid_factor(30)]
    x = rng.standard_normal(6000)
    for tr in (False, True):
        y0 = run(gg, monkeypatch, F, x, "0", transpose=tr, sym=False)
        ref = oracle.kron_matvec([f.T for f in F] if tr else F, x)
        assert rel(y0, ref) < 1e-13
        for v in VARIANTS:
            y = run(gg, monkeypatch, F, x, v, transpose=tr, sym=False)
            assert np.array_equal(y, y0), (v, tr)


def test_ring_lanczos_unchanged(gg, monkeypatch):
    """Lanczos (its middle mode products are plain launches) gives the same
    tridiagonal with and without the ring."""
    F = [grid_factor(200, 0.1), grid_factor(40, 0.13), grid_factor(200, 0.2), grid_factor(6)]
    out = []
    for v in ("0", "1"):
        monkeypatch.setenv("GG_FOLD_RING", v)
        K = gg.tensors.KronMatrix(F, sym=True)
        out.append(gg.linalg.lanczos_tridiag(K, 0.02, 10, seed=5, probe=0))
    assert np.array_equal(out[0][0], out[1][0]) and np.array_equal(out[0][1], out[1][1])


