"""CPU checks of the oracle's parity-block restatement (test infrastructure
for tests/test_gpu_block.py): the padded layout of round 6 (pair axes padded
to 16 TF + 4, oracle.kron.block_fold(pad=True)) is the unpadded one with zero
rows / columns inserted, the fold stays orthogonal, and the block operator
through the fold is the reference's product (kron_matrix.py:52-97 restated by
oracle.kron_matvec)."""
import numpy as np
import pytest

import oracle


def factors(ms):
    return [oracle.cov_1d("RBF", np.linspace(0, 1, m), np.linspace(0, 1, m), 1.0,
                          0.15 + 0.02 * k) + 1e-12 * np.eye(m) for k, m in enumerate(ms)]


@pytest.mark.parametrize("h,hp", [(4, 20), (16, 20), (20, 20), (24, 36), (32, 36), (36, 36),
                                  (48, 52), (50, 52), (64, 68), (100, 100)])
def test_block_pad_extent(h, hp):
    assert oracle.kron.block_pad(h) == hp


@pytest.mark.parametrize("ms", [(6, 64, 64), (4, 6, 48, 48), (8, 72, 72), (10, 32, 32)])
def test_padded_fold_is_orthogonal_and_zero_padded(ms):
    n = int(np.prod(ms))
    x = np.random.default_rng(0).standard_normal(n)
    xb = oracle.kron.block_fold(x, ms, pad=True)
    es = oracle.kron.block_extents(ms, pad=True)
    assert xb.size == int(np.prod(es)) << len(ms)
    assert np.isclose(np.linalg.norm(xb), np.linalg.norm(x), rtol=1e-14)
    assert np.allclose(oracle.kron.block_fold(xb, ms, inverse=True, pad=True), x,
                       rtol=0, atol=1e-14)
    # the padding holds exactly zeros: as many as the padded minus the real extents
    assert int(np.sum(xb == 0.0)) >= xb.size - n


@pytest.mark.parametrize("ms", [(6, 64, 64), (4, 6, 48, 48), (2, 4, 100, 100)])
def test_padded_block_matvec_is_the_reference_product(ms):
    F = factors(ms)
    n = int(np.prod(ms))
    x = np.random.default_rng(1).standard_normal(n)
    yb = oracle.kron.block_matvec(F, oracle.kron.block_fold(x, ms, pad=True), pad=True)
    y = oracle.kron.block_fold(yb, ms, inverse=True, pad=True)
    ref = oracle.kron_matvec(F, x)
    assert np.linalg.norm(y - ref) <= 1e-13 * np.linalg.norm(ref)
