"""KronMatrix.eig_vals / schur / svd on non-symmetric factors: the
factor-sized host path (kron_matrix.py:161-200, 355-366 call scipy's real
Schur form and numpy's eigvals / svd per factor; so does this build for
factors that are not symmetric), against tests/golden/kron_nonsym.npz, which
the reference itself produced (tests/golden/make_golden.py f10).  No GPU: a
non-symmetric factor never reaches the device eigensolver."""
import numpy as np
import pytest

from conftest import golden


@pytest.fixture(scope="module")
def z():
    return golden("kron_nonsym.npz")


def _kron(z):
    from gp_grief_amd.tensors import KronMatrix
    return KronMatrix([z["F%d" % i] for i in range(3)], sym=False)


def test_eig_vals_match_reference(z):
    e = _kron(z).eig_vals()
    assert e.ndim == 1 and e.n == 3
    for i in range(3):
        np.testing.assert_allclose(np.asarray(e.K[i]), z["eig%d" % i], rtol=1e-12, atol=1e-13)


def test_schur_matches_reference(z):
    Q, T = _kron(z).schur()
    for i in range(3):
        F = z["F%d" % i]
        q, t = np.asarray(Q.K[i]), np.asarray(T.K[i])
        np.testing.assert_allclose(q, z["schurQ%d" % i], rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(t, z["schurT%d" % i], rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(q.dot(t).dot(q.T), F, atol=1e-12)
        np.testing.assert_allclose(np.tril(t, -2), 0.0)      # quasi upper triangular


def test_svd_matches_reference(z):
    U, S = _kron(z).svd()
    for i in range(3):
        np.testing.assert_allclose(np.asarray(S.K[i]), z["svdS%d" % i], rtol=1e-12)
        np.testing.assert_allclose(np.abs(np.asarray(U.K[i])), np.abs(z["svdU%d" % i]),
                                   atol=1e-12)


def test_eig_vals_of_the_kron_product(z):
    """The Kronecker product's spectrum is the outer product of the factors'."""
    F = [z["F%d" % i] for i in range(3)]
    e = _kron(z).eig_vals().expand()
    full = np.linalg.eigvals(np.kron(np.kron(F[0], F[1]), F[2]))
    key = lambda v: (np.round(v.real, 8), np.round(v.imag, 8))   # noqa: E731
    np.testing.assert_allclose(sorted(e, key=key), sorted(full, key=key), atol=1e-9)
