"""The reference's remaining import-surface pieces on the MI355X, against
NumPy restatements of the reference arithmetic:
  expand_SKC            tensors.py:97-128 (logged: sign before zeros -> 1)
  GPRegressionModel     gpr_model.py:14-127 (dense exact GP; LML via Cholesky)
  RBF_RFF.Phi           rbf_rff.py:33-54
  TensorProduct / BlockMatrix over device KronMatrix operands."""
import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu


def rel(a, b):
    a = np.asarray(a, dtype=np.float64).reshape(-1)
    b = np.asarray(b, dtype=np.float64).reshape(-1)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


@pytest.fixture(scope="module")
def gp(gpu):
    import gp_grief
    return gp_grief


def expand_skc_ref(S, K, C, logged):
    """tensors.py:97-128 restated (test-local)."""
    log_prod, sign, prod = 0., 1, 1.
    for s, k, c in zip(S, K, C):
        xu = k[s.unique, :].dot(c)
        if logged:
            sign = sign * np.int32(np.sign(xu))[s.unique_inverse]
            xu[xu == 0] = 1.
            log_prod = log_prod + np.log(np.abs(xu))[s.unique_inverse]
        else:
            prod = prod * xu[s.unique_inverse]
    return (log_prod, sign) if logged else prod


@pytest.mark.parametrize("logged", [True, False])
def test_expand_skc(gp, logged):
    from gp_grief.tensors import expand_SKC, SelectionMatrixSparse
    rng = np.random.default_rng(1)
    d, n, p = 3, 1000, 40
    ms = [7, 9, 5]
    S, K, C = [], [], []
    for m in ms:
        S.append(SelectionMatrixSparse((rng.integers(0, m, p), m)))
        K.append(rng.standard_normal((m, m)))
        c = rng.standard_normal((m, n))
        c[:, 3] = 0.0                     # exact zeros: sign 0, log counted as 0
        C.append(c)
    got = expand_SKC(S, K, C, logged=logged)
    ref = expand_skc_ref(S, K, C, logged)
    if logged:
        assert got[0].shape == (p, n) and got[1].dtype == np.int32
        assert rel(got[0], ref[0]) < 1e-13
        np.testing.assert_array_equal(got[1], ref[1])
        assert np.all(got[1][:, 3] == 0)
    else:
        assert rel(got, ref) < 1e-13


def test_expand_skc_reproduces_grief_phi(gp):
    """Phi = sign^T exp(log^T - log_lam / 2) from expand_SKC on the GRIEF
    selection equals the oracle's Phi (grief_kernel.py:96-104)."""
    from gp_grief.tensors import expand_SKC, SelectionMatrixSparse
    rng = np.random.default_rng(2)
    d, m, p, n = 3, 16, 30, 500
    specs = [("RBF", 1.0, 0.2 + 0.02 * i) for i in range(d)]
    xg = [np.linspace(0, 1, m) for _ in range(d)]
    x = rng.random((n, d))
    ind = oracle.grief_inducing(specs, xg, p)
    S = [SelectionMatrixSparse((ind["eig_pos"][:, f], m)) for f in range(d)]
    K = [q.T for q in ind["Q"]]
    C = [oracle.cov_1d(specs[d - 1 - f][0], xg[d - 1 - f], x[:, d - 1 - f], 1.0,
                       specs[d - 1 - f][2]) for f in range(d)]
    lg, sg = expand_SKC(S, K, C, logged=True)
    Phi = sg.T * np.exp(lg.T - 0.5 * ind["log_lam"].reshape(1, -1))
    assert rel(Phi, oracle.grief_phi(x, specs, xg, ind)) < 1e-12


def test_gp_regression_model(gp):
    rng = np.random.default_rng(3)
    n, d = 300, 2
    x = rng.random((n, d))
    y = (np.sin(4 * x).sum(1) + 0.1 * rng.standard_normal(n)).reshape(-1, 1)
    k = gp.kern.RBF(d, variance=1.3, lengthscale=0.4)
    m = gp.models.GPRegressionModel(x, y, k, noise_var=0.05)
    d2 = ((x[:, None, :] - x[None, :, :]) ** 2).sum(-1)
    Kd = 1.3 * np.exp(-0.5 * d2 / 0.16) + 0.05 * np.eye(n)
    sign, ld = np.linalg.slogdet(Kd)
    a = np.linalg.solve(Kd, y)
    ll_ref = -0.5 * (ld + float(y[:, 0].dot(a[:, 0])) + n * np.log(2 * np.pi))
    ll = m.log_likelihood()
    assert abs(float(np.squeeze(ll)) - ll_ref) < 1e-9 * abs(ll_ref)
    xt = rng.random((20, d))
    dt = ((xt[:, None, :] - x[None, :, :]) ** 2).sum(-1)
    Ks = 1.3 * np.exp(-0.5 * dt / 0.16)
    mean_ref = Ks.dot(a)
    dtt = ((xt[:, None, :] - xt[None, :, :]) ** 2).sum(-1)
    var_ref = 1.3 * np.exp(-0.5 * dtt / 0.16) + 0.05 * np.eye(20) - Ks.dot(np.linalg.solve(Kd, Ks.T))
    mean, var = m.predict(xt, compute_var='full')
    assert rel(mean, mean_ref) < 1e-10 and rel(var, var_ref) < 1e-8
    mean2, vd = m.predict(xt, compute_var='diag')
    assert vd.shape == (20, 1) and rel(vd[:, 0], np.diag(var_ref)) < 1e-8
    assert m.predict(xt).shape == (20, 1)
    ll0, g = m.log_likelihood(return_gradient=True)
    assert g.shape == (3,) and np.all(np.isfinite(g))


def test_rbf_rff_features(gp):
    np.random.seed(0)
    f = gp.kern.RBF_RFF(3, log_lengthscale=np.log([0.5, 1.0, 2.0]), n_rffs=64)
    x = np.random.default_rng(4).random((50, 3))
    Phi = f.Phi(x)
    Xf = x.dot(f.freq_weights / np.exp(f.log_ell))
    ref = np.concatenate([np.cos(Xf), np.sin(Xf)], axis=1) / np.sqrt(64)
    assert Phi.shape == (50, 128) and rel(Phi, ref) < 1e-13


def test_tensor_product_of_device_kron(gp):
    from gp_grief.tensors import KronMatrix, TensorProduct, TensorSum, Array
    rng = np.random.default_rng(5)
    F = [rng.standard_normal((4, 4)) for _ in range(3)]
    G = [rng.standard_normal((4, 4)) for _ in range(3)]
    A, B = KronMatrix(F), KronMatrix(G)
    x = rng.standard_normal((64, 1))
    dA, dB = oracle.kron_expand(F), oracle.kron_expand(G)
    assert rel(TensorProduct([A, B]) * x, dA.dot(dB).dot(x)) < 1e-12
    assert rel(TensorSum([A, B, Array(np.eye(64))]) * x, (dA + dB + np.eye(64)).dot(x)) < 1e-12
