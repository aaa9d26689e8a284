"""WEB models (GPwebModel, GPwebTransformedModel) on the MI355X against the
reference-generated fixture web.npz (tests/golden/make_golden.py f7_web) and
the oracle (oracle/web.py); replays the reference tests
test_gp_web_model.py / test_gp_web_transformed_model.py (dense mvn logpdf,
checkgrad)."""
import numpy as np
import pytest
from scipy.stats import multivariate_normal as mvn

import oracle
from conftest import golden

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = np.asarray(a, dtype=np.float64).reshape(-1)
    b = np.asarray(b, dtype=np.float64).reshape(-1)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


@pytest.fixture(scope="module")
def models(gpu):
    import gp_grief_amd.models
    return gp_grief_amd.models


@pytest.mark.parametrize("tag", ["t", "b"])
@pytest.mark.parametrize("cls", ["GPwebModel", "GPwebTransformedModel"])
def test_web_fixture(models, tag, cls):
    z = golden("web.npz")
    key = "web" if cls == "GPwebModel" else "tr"
    X, Y, prm, Xn = z[tag + "_X"], z[tag + "_Y"], z[tag + "_params"], z[tag + "_Xnew"]
    m = getattr(models, cls)(Phi=X, y=Y)
    m.parameters = prm.copy()
    ll = m.log_likelihood()
    assert abs(float(ll) - float(z["%s_%s_lml" % (tag, key)])) <= \
        1e-9 * abs(float(z["%s_%s_lml" % (tag, key)]))
    ll2, g = m.log_likelihood(return_gradient=True)
    assert rel(g, z["%s_%s_grad" % (tag, key)]) < 1e-8
    mean, var = m.predict(Xn)
    assert mean.shape == (Xn.shape[0], 1) and var.shape == (Xn.shape[0],) * 2
    assert rel(mean, z["%s_%s_mean" % (tag, key)]) < 1e-8
    assert rel(var, z["%s_%s_var" % (tag, key)]) < 1e-10
    if cls == "GPwebTransformedModel":
        assert rel(m.singular_vals, z[tag + "_tr_singular"]) < 1e-10
        assert m.p == m.p_orig == X.shape[1]


def test_web_reference_test_replay(models):
    """test_gp_web_model.py:12-33: LML equals the dense mvn logpdf; checkgrad."""
    np.random.seed(0)
    X = np.random.randn(100, 4)
    X[:, 0] = 1.
    Y = np.dot(X, [0.5, 0.1, 0.25, 1.]) + 0.1 * np.random.randn(X.shape[0])
    m = models.GPwebModel(Phi=X, y=Y)
    m.parameters = np.random.rand(*m.parameters.shape) + 1e-6
    ll = m.log_likelihood()
    w = m.kern.parameters
    K = X.dot(np.diag(w)).dot(X.T) + m.noise_var * np.identity(X.shape[0])
    ll_exact = mvn.logpdf(Y, mean=np.zeros(X.shape[0]), cov=K)
    np.testing.assert_array_almost_equal(ll, ll_exact)
    assert np.ndim(ll) == 0
    m.checkgrad()


def test_web_transformed_reference_test_replay(models):
    """test_gp_web_transformed_model.py:12-33."""
    np.random.seed(0)
    X = np.random.randn(100, 4)
    X[:, 0] = 1.
    Y = np.dot(X, [0.5, 0.1, 0.25, 1.]) + 0.1 * np.random.randn(X.shape[0])
    m = models.GPwebTransformedModel(Phi=X, y=Y)
    m.parameters = np.random.rand(*m.parameters.shape) + 1e-6
    ll = m.log_likelihood()
    w = m.kern.parameters
    Phit = np.linalg.svd(X, full_matrices=False)[0]
    K = Phit.dot(np.diag(w)).dot(Phit.T) + m.noise_var * np.identity(X.shape[0])
    ll_exact = mvn.logpdf(Y, mean=np.zeros(X.shape[0]), cov=K)
    np.testing.assert_array_almost_equal(ll, ll_exact)
    m.checkgrad()


def test_web_vs_oracle_and_optimize(models):
    """A 4000 x 96 basis: LML / gradient / predictions vs the oracle, then a
    few L-BFGS steps through the device likelihood increase the LML."""
    rng = np.random.default_rng(11)
    X = rng.standard_normal((4000, 96)) / 10.0
    Y = np.cos(X[:, :5].sum(axis=1) * 4.0) + 0.05 * rng.standard_normal(4000)
    prm = np.concatenate(([0.02], rng.uniform(0.3, 3.0, 96)))
    m = models.GPwebModel(Phi=X, y=Y)
    m.parameters = prm.copy()
    ll, g = m.log_likelihood(return_gradient=True)
    ll_o, g_o = oracle.web_lml_grad(X, Y, prm)
    assert abs(float(ll) - ll_o) <= 1e-10 * abs(ll_o)
    assert rel(g, g_o) < 1e-8
    mean, var = m.predict(X[:50])
    mo, vo = oracle.web_predict(X, Y, prm, X[:50])
    assert rel(mean, mo) < 1e-9 and rel(var, vo) < 1e-11
    ll0 = float(m.log_likelihood())
    m.optimize(max_iters=5)
    assert float(m.log_likelihood()) > ll0


def test_web_shape_asserts(models):
    X = np.random.default_rng(0).standard_normal((30, 5))
    with pytest.raises(AssertionError):
        models.GPwebModel(Phi=X, y=np.ones(29))
    m = models.GPwebModel(Phi=X, y=np.ones(30))
    with pytest.raises(AssertionError):
        m.predict(np.ones((3, 4)))


@pytest.mark.parametrize("case", ["wide", "rank_deficient"])
def test_web_transformed_basis_count_matches_lapack(models, case):
    """The kept basis count and the LML follow the reference's LAPACK thin SVD
    (gp_web_transformed_model.py:31-38: singular values > 1e-7, at most
    min(n, p)) when p_orig > n and when Phi is rank deficient.  (The
    reference's own log message for p < p_orig has a format bug and raises;
    the arithmetic is what is compared here.)"""
    rng = np.random.default_rng(8)
    if case == "wide":
        n, p = 30, 60
        Phi = rng.standard_normal((n, p))
    else:
        n, p = 200, 40
        Phi = rng.standard_normal((n, p))
        Phi[:, 20:] = Phi[:, :20]
    y = rng.standard_normal(n)
    U, S, VT = np.linalg.svd(Phi, full_matrices=False)
    keep = S > 1e-7
    S, U = S[keep], U[:, keep]
    m = models.GPwebTransformedModel(Phi, y, noise_var=0.3)
    assert m.p == S.size == (30 if case == "wide" else 20)
    np.testing.assert_allclose(m.singular_vals, S, rtol=1e-8)
    w = np.linspace(0.5, 2.0, m.p)
    m.kern.parameters = w
    c2 = (U.T.dot(y)) ** 2
    Pd = 0.3 / w + 1.0
    ll_ref = -0.5 * (np.sum(np.log(Pd)) + np.sum(np.log(w)) + (n - m.p) * np.log(0.3)
                     + (y.dot(y) - np.sum(c2 / Pd)) / 0.3 + n * np.log(2 * np.pi))
    assert abs(float(np.squeeze(m.log_likelihood())) - ll_ref) < 1e-9 * abs(ll_ref)


@pytest.mark.parametrize("smin", [1e-3, 1e-5, 2e-7])
def test_web_transformed_ill_conditioned_full_rank(models, smin):
    """A full-rank Phi with singular values from 300 down to smin (> 1e-7):
    the reference's LAPACK SVD keeps every basis, and so does the device
    CholeskyQR3 route -- singular values to LAPACK's accuracy, LML and
    predictions to 1e-8 (the Gram spectrum alone dropped every
    direction below ~1e-3 here)."""
    import oracle
    rng = np.random.default_rng(21)
    n, p = 1500, 40
    U, _ = np.linalg.qr(rng.standard_normal((n, p)))
    Vq, _ = np.linalg.qr(rng.standard_normal((p, p)))
    S = np.logspace(np.log10(300.0), np.log10(smin), p)
    Phi = (U * S).dot(Vq.T)
    y = Phi.dot(rng.standard_normal(p)) * 1e-3 + 0.1 * rng.standard_normal(n)
    st = oracle.web.web_transformed_setup(Phi, y)
    m = models.GPwebTransformedModel(Phi, y, noise_var=0.3)
    assert m.p == st["p"] == p
    # both SVDs carry an absolute error ~ p eps s_max
    np.testing.assert_allclose(m.singular_vals, st["sv"], rtol=1e-10, atol=1e-10)
    params = np.concatenate([[0.3], np.linspace(0.5, 2.0, p)])
    m.kern.parameters = params[1:]
    ll_ref, g_ref = oracle.web.web_transformed_lml_grad(st, params)
    assert abs(float(np.squeeze(m.log_likelihood())) - ll_ref) < 1e-8 * abs(ll_ref)
    Pn = rng.standard_normal((7, p))
    mean, var = m.predict(Pn)
    mo, vo = oracle.web.web_transformed_predict(st, params, Pn)
    # the mean divides by the singular values: singular-vector angle errors
    # (~ p eps s_max / gap in either SVD) grow by s_max / smin
    tol = 2e-13 * (300.0 / smin) + 1e-9
    assert np.linalg.norm(mean - mo) < tol * np.linalg.norm(mo) + 1e-12
    assert np.linalg.norm(var - vo) < 1e-8 * np.linalg.norm(vo)


@pytest.mark.parametrize("smin", [1e-3, 2e-7])
def test_web_transformed_wide_ill_conditioned(models, smin):
    """a wide Phi (n < p) takes the CholeskyQR3 route on Phi^T,
    so its singular values keep LAPACK accuracy down to 1e-7 (the Gram
    spectrum alone loses everything below ~sqrt(eps) s_max): the kept basis
    count, singular values and LML match the oracle's LAPACK thin SVD (the
    reference's algorithm, gp_web_transformed_model.py:27-38).  Parity
    unpinned beyond the oracle: the reference has no wide fixture."""
    import oracle
    rng = np.random.default_rng(23)
    n, p = 40, 600
    U, _ = np.linalg.qr(rng.standard_normal((n, n)))
    Vq, _ = np.linalg.qr(rng.standard_normal((p, n)))
    S = np.logspace(np.log10(300.0), np.log10(smin), n)
    Phi = (U * S).dot(Vq.T)
    y = Phi.dot(rng.standard_normal(p)) * 1e-3 + 0.1 * rng.standard_normal(n)
    st = oracle.web.web_transformed_setup(Phi, y)
    m = models.GPwebTransformedModel(Phi, y, noise_var=0.3)
    assert m.p == st["p"] == n
    np.testing.assert_allclose(m.singular_vals, st["sv"], rtol=1e-10, atol=1e-10)
    params = np.concatenate([[0.3], np.linspace(0.5, 2.0, n)])
    m.kern.parameters = params[1:]
    ll_ref, _ = oracle.web.web_transformed_lml_grad(st, params)
    assert abs(float(np.squeeze(m.log_likelihood())) - ll_ref) < 1e-8 * abs(ll_ref)
