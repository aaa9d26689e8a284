"""P2 (GRIEF) parity on the MI355X: covariances, MFMA GEMM, Cholesky, Phi, and
the GPGriefModel API against the reference-generated fixtures and the oracle."""
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
    import gp_grief_amd.grid  # noqa: F401
    return gp_grief_amd


# ------------------------------------------------------------------ kernels
@pytest.mark.parametrize("kind", ["RBF", "Exponential", "Matern32", "Matern52"])
def test_cov_1d_vs_oracle(gg, kind):
    rng = np.random.default_rng(0)
    x = rng.random((37, 1))
    z = rng.random((23, 1))
    k = getattr(gg.kern, kind)(1, variance=1.7, lengthscale=0.31)
    K = k.cov(x, z)
    assert K.shape == (37, 23)
    assert rel(K, oracle.cov_1d(kind, x[:, 0], z[:, 0], 1.7, 0.31)) < 1e-14
    Kxx = k.cov(x)
    assert np.allclose(Kxx, Kxx.T)


def test_cov_multidim_product_and_sum(gg):
    rng = np.random.default_rng(1)
    x = rng.random((11, 2))
    k = gg.kern.RBF(2, variance=2.0, lengthscale=0.5) * gg.kern.Matern52(2, lengthscale=0.7)
    d2 = ((x[:, None, :] - x[None, :, :]) ** 2).sum(-1)
    r = np.sqrt(d2) / 0.7
    ref = 2.0 * np.exp(-0.5 * d2 / 0.25) * (1 + np.sqrt(5) * r + 5.0 / 3 * r ** 2) * \
        np.exp(-np.sqrt(5) * r)
    assert rel(k.cov(x), ref) < 1e-13
    k2 = gg.kern.RBF(2) + gg.kern.Exponential(2)
    ref2 = np.exp(-0.5 * d2) + np.exp(-np.sqrt(d2))
    assert rel(k2.cov(x), ref2) < 1e-13


# ------------------------------------------------------------------ GEMM / GEMV
@pytest.mark.parametrize("shape", [(1, 1, 1), (7, 5, 3), (128, 128, 16), (130, 257, 33),
                                   (300, 40, 5000), (64, 64, 100000)])
@pytest.mark.parametrize("ta", [False, True])
@pytest.mark.parametrize("tb", [False, True])
def test_gemm_vs_numpy(gg, shape, ta, tb):
    import torch
    from gp_grief_amd import dense
    M, N, K = shape
    rng = np.random.default_rng(M + N + K)
    A = rng.standard_normal((K, M) if ta else (M, K))
    B = rng.standard_normal((N, K) if tb else (K, N))
    C0 = rng.standard_normal((M, N))
    opA = A.T if ta else A
    opB = B.T if tb else B
    Ad, Bd = torch.from_numpy(A).cuda(), torch.from_numpy(B).cuda()
    C = dense.matmul(Ad, Bd, ta=ta, tb=tb, alpha=0.5, beta=-2.0,
                     C=torch.from_numpy(C0.copy()).cuda())
    ref = 0.5 * opA.dot(opB) - 2.0 * C0
    assert rel(C.cpu().numpy(), ref) < 1e-13


def test_gemm_triangle(gg):
    import torch
    from gp_grief_amd import dense
    rng = np.random.default_rng(3)
    R = rng.standard_normal((500, 300))
    Rd = torch.from_numpy(R).cuda()
    C = torch.zeros((300, 300), dtype=torch.float64, device="cuda")
    dense.matmul(Rd, Rd, ta=True, C=C, beta=0.0, uplo=1)
    ref = R.T.dot(R)
    Ch = C.cpu().numpy()
    assert rel(np.tril(Ch), np.tril(ref)) < 1e-13
    assert np.all(np.triu(Ch, 1) == 0)


@pytest.mark.parametrize("S", ["2", "3", "8"])
@pytest.mark.parametrize("uplo", [0, 1])
def test_gemm_tn_splitk(gg, monkeypatch, S, uplo):
    """The TN kernel split over K (GG_GEMM_SPLITK forces S): partial slabs +
    reduce, with alpha / beta and the lower-triangle mode of the Gram."""
    import ctypes
    import torch
    from gp_grief_amd import dense, native
    monkeypatch.setenv("GG_GEMM_SPLITK", S)
    native.knobs_reload()
    try:
        _splitk_case(native, dense, S, uplo)
    finally:
        monkeypatch.delenv("GG_GEMM_SPLITK")
        native.knobs_reload()


def _splitk_case(native, dense, S, uplo):
    import ctypes
    import torch
    rng = np.random.default_rng(int(S) + 10 * uplo)
    K, M = 20000, 258
    R = rng.standard_normal((K, M))
    C0 = rng.standard_normal((M, M))
    need = ctypes.c_int64()
    native.check(native.lib().gg_gemm_workspace_elems(1, 0, M, M, K, uplo, ctypes.byref(need)))
    assert need.value == int(S) * M * M
    Rd = torch.from_numpy(R).cuda()
    C = dense.matmul(Rd, Rd, ta=True, alpha=0.5, beta=-2.0,
                     C=torch.from_numpy(C0.copy()).cuda(), uplo=uplo).cpu().numpy()
    ref = 0.5 * R.T.dot(R) - 2.0 * C0
    if uplo == 1:
        assert rel(np.tril(C), np.tril(ref)) < 1e-13
        assert np.array_equal(np.triu(C, 1), np.triu(C0, 1))
    else:
        assert rel(C, ref) < 1e-13


def test_gemm_tn_splitk_model(gg):
    """The Gram (K = n >> p) is split 8-way over K, 16-way up to p = 2000
    (gg_dense.hip tn_splitk, whole groups of 8 slabs for the XCD-slab grid);
    a small-K product is not split."""
    import ctypes
    from gp_grief_amd import native
    need = ctypes.c_int64()
    native.check(native.lib().gg_gemm_workspace_elems(1, 0, 5000, 5000, 100000, 1,
                                                      ctypes.byref(need)))
    assert need.value == 8 * 5000 * 5000
    native.check(native.lib().gg_gemm_workspace_elems(1, 0, 1000, 1000, 100000, 1,
                                                      ctypes.byref(need)))
    assert need.value == 16 * 1000 * 1000
    native.check(native.lib().gg_gemm_workspace_elems(1, 0, 5000, 5000, 256, 1,
                                                      ctypes.byref(need)))
    assert need.value == 0


@pytest.mark.parametrize("R,C", [(1, 1), (1000, 37), (100000, 300), (33, 5000)])
def test_gemv(gg, R, C):
    import torch
    from gp_grief_amd import dense
    rng = np.random.default_rng(R + C)
    A = rng.standard_normal((R, C))
    x = rng.standard_normal(R)
    v = rng.standard_normal(C)
    Ad = torch.from_numpy(A).cuda()
    yt = dense.matvec(Ad, torch.from_numpy(x).cuda(), trans=True).cpu().numpy()
    assert rel(yt, A.T.dot(x)) < 1e-13
    yn = dense.matvec(Ad, torch.from_numpy(v).cuda()).cpu().numpy()
    assert rel(yn, A.dot(v)) < 1e-13


# ------------------------------------------------------------------ Cholesky
@pytest.mark.parametrize("n", [1, 5, 64, 65, 129, 300, 1000, 2500, 4099])
def test_cholesky_solve_logdet(gg, n):
    import torch
    from gp_grief_amd import dense
    rng = np.random.default_rng(n)
    G = rng.standard_normal((n, n + 10))
    P = G.dot(G.T) / n + 0.1 * np.eye(n)
    ch = dense.Cholesky(torch.from_numpy(P).cuda())
    assert abs(ch.logdet - np.linalg.slogdet(P)[1]) < 1e-10 * max(1, abs(ch.logdet))
    L = np.tril(ch.L.cpu().numpy())
    assert rel(L.dot(L.T), P) < 1e-13
    B = rng.standard_normal((n, 3))
    X = ch.solve(torch.from_numpy(B).cuda(), which=3).cpu().numpy()
    assert rel(X, np.linalg.solve(P, B)) < 1e-10
    b = rng.standard_normal(n)
    x = ch.solve(torch.from_numpy(b).cuda(), which=3).cpu().numpy()
    assert rel(x, np.linalg.solve(P, b)) < 1e-10
    dinv = ch.inverse_diag().cpu().numpy()
    assert rel(dinv, np.diag(np.linalg.inv(P))) < 1e-10
    # the two triangular halves separately, and L^-1 of the identity
    X1 = ch.solve(torch.from_numpy(B).cuda(), which=1).cpu().numpy()
    assert rel(L.dot(X1), B) < 1e-12
    X2 = ch.solve(torch.from_numpy(B).cuda(), which=2).cpu().numpy()
    assert rel(L.T.dot(X2), B) < 1e-12
    Li = ch.solve(torch.eye(n, dtype=torch.float64).cuda(), which=5).cpu().numpy()
    assert rel(np.tril(Li), np.linalg.inv(L)) < 1e-10
    # recursive triangular inverse (gg_trtri), strict upper triangle untouched
    Xi = ch.inverse().cpu().numpy()
    assert rel(Xi, np.linalg.inv(L)) < 1e-10
    assert np.all(np.triu(Xi, 1) == 0)


def test_cholesky_lookahead_streams_bitwise(gg, monkeypatch):
    """The look-ahead schedule (factor chain and wide trailing updates on two
    priority streams) gives the factor of the serial schedule
    (GG_POTRF_LOOKAHEAD=0, every launch on the caller's stream): the same
    kernels on the same operands in a dependency-equivalent order, bitwise."""
    import torch
    from gp_grief_amd import dense
    n = 4500   # 512-column panels: several wide updates
    rng = np.random.default_rng(7)
    G = rng.standard_normal((n, n + 10))
    P = torch.from_numpy(G.dot(G.T) / n + 0.1 * np.eye(n)).cuda()
    monkeypatch.delenv("GG_POTRF_LOOKAHEAD", raising=False)
    ref = dense.Cholesky(P.clone())
    monkeypatch.setenv("GG_POTRF_LOOKAHEAD", "0")
    gg.native.knobs_reload()
    try:
        ch = dense.Cholesky(P.clone())
    finally:
        monkeypatch.delenv("GG_POTRF_LOOKAHEAD", raising=False)
        gg.native.knobs_reload()
    assert torch.equal(torch.tril(ch.L), torch.tril(ref.L))
    assert ch.logdet == ref.logdet


def test_cholesky_not_spd_raises(gg):
    import torch
    from gp_grief_amd import dense
    P = np.eye(70)
    P[40, 40] = -1.0
    with pytest.raises(np.linalg.LinAlgError):
        dense.Cholesky(torch.from_numpy(P).cuda())


# ------------------------------------------------------------------ GRIEF model
def _grief_test_model(gg, z):
    d = z["x"].shape[1]
    grid = gg.grid.InducingGrid(z["x"])
    np.testing.assert_allclose(np.stack([g[:, 0] for g in grid.xg]), z["xg"])
    kern = gg.kern.RBF(1, lengthscale=0.5)
    kern = gg.kern.GriefKernel(kern_list=[kern] * d, grid=grid, n_eigs=50)
    return gg.models.GPGriefModel(z["x"], z["y"].reshape(-1, 1), kern, noise_var=0.1)


def test_grief_test_fixture_model(gg):
    """The reference's own test (test_gp_grief_model.py) with the in-house RBF."""
    z = golden("grief_test.npz")
    m = _grief_test_model(gg, z)
    np.testing.assert_allclose(m.parameters, z["params"])
    lml = m._compute_log_likelihood(m.parameters)
    assert lml.shape == (1, 1)
    assert abs(lml[0, 0] - z["lml"]) < 1e-8 * abs(z["lml"])
    np.testing.assert_allclose(m.kern._log_lam, z["log_lam"], rtol=1e-10, atol=1e-12)
    Kd = m._mv_cov(np.identity(z["x"].shape[0]))
    assert rel(Kd, z["cov_dense"]) < 1e-10
    alp = m._mv_cov_inv(z["y"].reshape(-1, 1))
    assert rel(alp, z["alpha"]) < 1e-8
    assert rel(alp, np.linalg.solve(Kd, z["y"])) < 1e-6
    assert abs(m._cov_log_det() - z["logdet"]) < 1e-8 * abs(z["logdet"])
    ll, grad = m.log_likelihood(return_gradient=True)
    g = z["grad"]
    free = ~np.isnan(g)
    np.testing.assert_array_equal(np.isnan(grad), np.isnan(g))
    np.testing.assert_allclose(grad[free], g[free], rtol=1e-6, atol=1e-9)
    mean, var = m.predict(z["x"][:7])
    assert rel(mean[:, 0], z["pred_mean"]) < 1e-8
    assert rel(var, z["pred_var"]) < 1e-8
    Phi = m.kern.cov(z["x"])[0]
    assert rel(np.abs(Phi), np.abs(z["phi_signnorm"])) < 1e-9


@pytest.mark.parametrize("case", ["3d", "6d", "8d"])
def test_grief_small_fixtures_model(gg, case):
    z = golden("grief_small_%s.npz" % case)
    d = z["x"].shape[1]
    kind = str(z["kind"])
    kl = [getattr(gg.kern, kind)(1, variance=1.0, lengthscale=float(l)) for l in z["lengthscales"]]
    grid = gg.grid.InducingGrid(xg=[np.linspace(0, 1, int(z["m"])).reshape(-1, 1)
                                    for _ in range(d)])
    kern = gg.kern.GriefKernel(kern_list=kl, grid=grid, n_eigs=int(z["p"]))
    m = gg.models.GPGriefModel(z["x"], z["y"].reshape(-1, 1), kern, noise_var=float(z["sigma2"]))
    ll, grad = m.log_likelihood(return_gradient=True)
    # north-star bar: LML, posterior mean and variance to 1e-6 relative
    assert abs(ll[0, 0] - z["lml"]) < 1e-6 * abs(z["lml"])
    np.testing.assert_allclose(m.kern._log_lam, z["log_lam"], rtol=1e-9, atol=1e-10)
    mean, var = m.predict(z["xtest"])
    assert rel(mean[:, 0], z["pred_mean"]) < 1e-6
    assert rel(var, z["pred_var"]) < 1e-6
    assert rel(grad[-int(z["p"]):], z["grad"][-int(z["p"]):]) < 1e-6
    assert abs(grad[0] - z["grad"][0]) < 1e-6 * abs(z["grad"][0])


def test_automobile_optimize(gg):
    """Type-II tutorial case: L-BFGS with finite-difference gradients over the
    device LML; parameters, LML and test RMSE after 5 iterations."""
    z = golden("automobile.npz")
    x, y, itr = z["x"], z["y"].reshape(-1, 1), z["i_train"]
    grid = gg.grid.InducingGrid(x=x)
    np.testing.assert_allclose(np.concatenate([g[:, 0] for g in grid.xg]), z["xg_cat"])
    kern = gg.kern.GriefKernel(kern_list=[gg.kern.RBF(1, lengthscale=1.0)] * x.shape[1],
                               grid=grid, n_eigs=100, reweight_eig_funs=False,
                               opt_kernel_params=True)
    m = gg.models.GPGriefModel(X=x[itr], Y=y[itr], kern=kern, noise_var=1.0)
    np.testing.assert_allclose(m.parameters, z["params0"])
    assert abs(float(np.squeeze(m.log_likelihood())) - z["lml0"]) < 1e-8 * abs(z["lml0"])
    m.optimize(max_iters=5)
    np.testing.assert_allclose(m.parameters, z["params_opt"], rtol=1e-4)
    assert abs(float(np.squeeze(m.log_likelihood())) - z["lml_opt"]) < 1e-5 * abs(z["lml_opt"])
    mean, var = m.predict(Xnew=x[~itr])
    rmse = np.linalg.norm((mean[:, 0] - y[~itr, 0]) * z["y_scale"]) / np.sqrt(mean.size)
    assert abs(rmse - z["rmse"]) < 1e-4 * z["rmse"]


def test_fd_gradient_batched_eigs_equal_sequential(gg):
    """opt_kernel_params: the finite-difference gradient with the perturbed
    bases' eigendecompositions batched into one launch equals the sequential
    one (distinct kernels per dim, and the shared-kernel-object case)."""
    rng = np.random.default_rng(4)
    d, m, n, p = 3, 20, 400, 60
    x = rng.random((n, d))
    y = (np.sin(6 * x).sum(axis=1) + 0.1 * rng.standard_normal(n)).reshape(-1, 1)
    for shared in (False, True):
        grads = []
        for batched in (True, False):
            if shared:
                kl = [gg.kern.RBF(1, variance=1.0, lengthscale=0.3)] * d
            else:
                kl = [gg.kern.RBF(1, variance=1.0, lengthscale=0.2 + 0.05 * i) for i in range(d)]
            grid = gg.grid.InducingGrid(xg=[np.linspace(0, 1, m).reshape(-1, 1)] * d)
            kern = gg.kern.GriefKernel(kern_list=kl, grid=grid, n_eigs=p,
                                       reweight_eig_funs=False, opt_kernel_params=True)
            if not batched:
                kern.prefetch_eigs = lambda sets: 0
            model = gg.models.GPGriefModel(x, y, kern, noise_var=0.05)
            ll, g = model.log_likelihood(return_gradient=True)
            if batched:
                assert len(kern._eig_cache) >= 1
            grads.append((float(np.squeeze(ll)), g.copy(), model.parameters.copy()))
        (l1, g1, p1), (l2, g2, p2) = grads
        assert np.array_equal(p1, p2)
        assert abs(l1 - l2) <= 1e-12 * abs(l2)
        assert np.allclose(g1, g2, rtol=1e-6, atol=1e-8), (g1, g2)


@pytest.mark.parametrize("case", ["3d", "6d", "8d"])
def test_grief_p_system_cg_matches_cholesky(gg, case):
    """p_solver='cg' (Jacobi PCG on P = Phi^T Phi + diag(s/w), one p-vector
    all-reduce per iteration when sharded) reproduces the Cholesky solve:
    alpha and the predictive mean, and the fixture LML / mean at 1e-6."""
    z = golden("grief_small_%s.npz" % case)
    d = z["x"].shape[1]
    kind = str(z["kind"])

    def build(solver):
        kl = [getattr(gg.kern, kind)(1, variance=1.0, lengthscale=float(l))
              for l in z["lengthscales"]]
        grid = gg.grid.InducingGrid(xg=[np.linspace(0, 1, int(z["m"])).reshape(-1, 1)
                                        for _ in range(d)])
        kern = gg.kern.GriefKernel(kern_list=kl, grid=grid, n_eigs=int(z["p"]))
        return gg.models.GPGriefModel(z["x"], z["y"].reshape(-1, 1), kern,
                                      noise_var=float(z["sigma2"]), p_solver=solver)

    mc, mg = build('chol'), build('cg')
    mc.fit()
    mg.fit()
    assert mg._A is None and mg._Pchol is None      # alpha needed no Gram / factorisation
    assert len(mg.cg_iters) == 1 and 0 < mg.cg_iters[0] < int(z["p"])
    ac, ag = gg.dense.host(mc._alpha), gg.dense.host(mg._alpha)
    assert rel(ag, ac) < 1e-9
    mean_g, _ = mg.predict(z["xtest"])
    assert rel(mean_g[:, 0], z["pred_mean"]) < 1e-6
    ll = float(np.squeeze(mg.log_likelihood()))
    assert abs(ll - z["lml"]) < 1e-6 * abs(z["lml"])
    # an LML needs chol(P) for its log det: a fresh 'cg' model solves alpha
    # with that factor rather than running PCG beside it
    m2 = build('cg')
    ll2 = float(np.squeeze(m2.log_likelihood()))
    assert m2.cg_iters == [] and abs(ll2 - z["lml"]) < 1e-6 * abs(z["lml"])


# ------------------------------------------------ eigensolver subset path
def _grid_factor(m, ls, var=1.0, noise=1e-12):
    g = np.linspace(0, 1, m)
    return var * np.exp(-0.5 * (g[:, None] - g[None, :]) ** 2 / ls ** 2) + noise * np.eye(m)


@pytest.mark.parametrize("m,ls,k", [(128, 0.1, 20), (200, 0.05, 30), (32, 0.2, 8), (5, 0.5, 5)])
def test_eig_subset_vs_full(gg, m, ls, k):
    """Bisection eigenvalues and inverse-iteration eigenvectors of the
    tridiagonalised factor (the GRIEF setup's subset path) against the full
    QL decomposition and numpy's LAPACK eigh: eigenvalues to 1e-13 ||K||,
    the top-k eigenvectors to 1e-9 (up to sign), orthonormal to 1e-12."""
    from gp_grief_amd.tensors import (device_sym_eig, device_sym_eig_tridiag,
                                      device_sym_eig_tridiag_vectors)
    F = [_grid_factor(m, ls), _grid_factor(m, 1.3 * ls, var=2.0)]
    lam, h = device_sym_eig_tridiag(F)
    Q, lamq = device_sym_eig(F)
    for f in range(len(F)):
        ln = np.linalg.eigvalsh(F[f])
        scale = np.abs(ln).max()
        assert np.all(np.diff(lam[f]) >= 0)
        assert np.abs(lam[f] - ln).max() <= 1e-13 * scale * m
        assert np.abs(lam[f] - lamq[f]).max() <= 1e-13 * scale * m
    sel = [np.arange(m - k, m), np.arange(m - k // 2, m)]
    V = device_sym_eig_tridiag_vectors(h, sel)
    for f in range(len(F)):
        Vh = V[f].cpu().numpy()
        assert Vh.shape == (sel[f].size, m)
        assert np.abs(Vh @ Vh.T - np.eye(sel[f].size)).max() < 1e-12
        Qs = Q[f][:, sel[f]].T
        signs = np.sign(np.sum(Vh * Qs, axis=1)).reshape(-1, 1)
        assert np.abs(Vh - signs * Qs).max() < 1e-9
        # eigen-residual against the input factor
        lv = lam[f][sel[f]]
        assert np.abs(Vh @ F[f] - lv[:, None] * Vh).max() < 1e-12 * np.abs(lam[f]).max()


def test_grief_subset_setup_matches_full(gg, monkeypatch):
    """GPGriefModel on the subset setup (default) and on the full QL setup
    (GG_EIG_SUBSET=0): same selection, LML to 1e-10, predictions to 1e-9."""
    rng = np.random.default_rng(7)
    d, m, n, p = 3, 48, 3000, 300
    x = rng.random((n, d))
    y = (np.sin(5 * x).sum(axis=1) + 0.1 * rng.standard_normal(n)).reshape(-1, 1)
    xt = rng.random((200, d))
    out = []
    for flag in ("1", "0"):
        monkeypatch.setenv("GG_EIG_SUBSET", flag)
        kl = [gg.kern.RBF(1, variance=1.0, lengthscale=0.15 + 0.03 * i) for i in range(d)]
        grid = gg.grid.InducingGrid(xg=[np.linspace(0, 1, m).reshape(-1, 1)] * d)
        kern = gg.kern.GriefKernel(kern_list=kl, grid=grid, n_eigs=p)
        model = gg.models.GPGriefModel(x, y, kern, noise_var=0.05)
        ll = float(np.squeeze(model.log_likelihood()))
        mean = np.asarray(model.predict(xt)[0]).reshape(-1)
        subset = kern._Quu_full is None
        out.append((ll, mean, kern._log_lam.copy(), subset))
    (l1, m1, g1, s1), (l0, m0, g0, s0) = out
    assert s1 and not s0
    assert np.allclose(g1, g0, rtol=1e-11, atol=1e-11)
    assert abs(l1 - l0) <= 1e-10 * abs(l0)
    assert rel(m1, m0) < 1e-9


@pytest.mark.parametrize("m,ls", [(128, 0.1), (64, 0.2), (200, 0.05), (32, 0.3)])
def test_centro_halves_eigenpairs(gg, m, ls):
    """A centrosymmetric grid factor's spectrum from its two half-order
    problems (tensors.centro_halves / centro_merge / centro_expand) against
    numpy's LAPACK eigh: eigenvalues to 1e-13 m ||K||, selected eigenvectors
    to 1e-9 up to sign, orthonormal to 1e-12; odd m and a perturbed
    (non-centrosymmetric) factor are refused."""
    import torch
    from gp_grief_amd.tensors import (centro_expand, centro_halves, centro_merge,
                                      device_sym_eig_tridiag, device_sym_eig_tridiag_vectors)
    F = _grid_factor(m, ls, noise=1e-8)
    Fd = torch.tensor(F, device="cuda")
    Ke, Ko = centro_halves(Fd)
    (le, lo), h = device_sym_eig_tridiag([Ke, Ko])
    lam, half, idx = centro_merge(le, lo)
    ln, Qn = np.linalg.eigh(F)
    scale = np.abs(ln).max()
    assert np.abs(lam - ln).max() <= 1e-13 * scale * m
    k = min(12, m // 4)   # well-separated top eigenpairs (vectors to 1e-9)
    sel = np.arange(m - k, m)
    se, so = np.sort(idx[sel][half[sel] == 0]), np.sort(idx[sel][half[sel] == 1])
    Vh = device_sym_eig_tridiag_vectors(h, [se, so])
    V = centro_expand(Vh, [m // 2], [se.size], [so.size])[0].cpu().numpy()
    # rows: the even half's selected indices, then the odd half's
    where = {(int(hh), int(i)): kk for kk, (hh, i) in enumerate(zip(half, idx))}
    full = [where[(0, int(v))] for v in se] + [where[(1, int(v))] for v in so]
    assert np.abs(V @ V.T - np.eye(k)).max() < 1e-12
    Qs = Qn[:, full].T
    signs = np.sign(np.sum(V * Qs, axis=1)).reshape(-1, 1)
    assert np.abs(V - signs * Qs).max() < 1e-9
    assert np.abs(V @ F - lam[full][:, None] * V).max() < 1e-12 * scale
    assert centro_halves(torch.tensor(_grid_factor(m + 1, ls), device="cuda")) is None
    Fp = F.copy()
    Fp[0, 1] += 1e-6
    Fp[1, 0] += 1e-6
    assert centro_halves(torch.tensor(Fp, device="cuda")) is None


def test_grief_centro_setup_matches_unsplit(gg, monkeypatch):
    monkeypatch.setenv("GG_EIG_CENTRO_MIN", "16")
    _centro_setup_cases(gg, monkeypatch)


def _centro_setup_cases(gg, monkeypatch):
    """The GRIEF setup with the factors split into half-order problems
    (default) and without (GG_EIG_CENTRO=0): same eigenvalue selection, LML to
    1e-10, predictions to 1e-9, Matern-5/2 and RBF factors of even and odd
    order (odd ones stay unsplit)."""
    rng = np.random.default_rng(9)
    d, n, p = 3, 3000, 300
    x = rng.random((n, d))
    y = (np.sin(5 * x).sum(axis=1) + 0.1 * rng.standard_normal(n)).reshape(-1, 1)
    xt = rng.random((200, d))
    for ms, kind in (((48, 40, 56), "RBF"), ((48, 40, 56), "Matern52"), ((47, 40, 56), "RBF")):
        out = []
        for flag in ("1", "0"):
            monkeypatch.setenv("GG_EIG_CENTRO", flag)
            kl = [getattr(gg.kern, kind)(1, variance=1.0, lengthscale=0.15 + 0.03 * i)
                  for i in range(d)]
            grid = gg.grid.InducingGrid(xg=[np.linspace(0, 1, m).reshape(-1, 1) for m in ms])
            kern = gg.kern.GriefKernel(kern_list=kl, grid=grid, n_eigs=p)
            model = gg.models.GPGriefModel(x, y, kern, noise_var=0.05)
            ll = float(np.squeeze(model.log_likelihood()))
            mean = np.asarray(model.predict(xt)[0]).reshape(-1)
            out.append((ll, mean, kern._log_lam.copy(), kern._Quu_full is None))
        (l1, m1, g1, s1), (l0, m0, g0, s0) = out
        assert s1 and s0
        assert np.allclose(g1, g0, rtol=1e-11, atol=1e-11)
        assert abs(l1 - l0) <= 1e-10 * abs(l0)
        assert rel(m1, m0) < 1e-9


def test_grief_subset_falls_back_on_clusters(gg, monkeypatch):
    """A factor with a clustered spectrum (a kernel so short that K ~ I) fails
    the separation test: the setup takes the full QL path and stays correct."""
    monkeypatch.setenv("GG_EIG_SUBSET", "1")
    rng = np.random.default_rng(8)
    d, m, n, p = 2, 24, 800, 40
    x = rng.random((n, d))
    y = rng.standard_normal((n, 1))
    kl = [gg.kern.RBF(1, variance=1.0, lengthscale=1e-4) for _ in range(d)]
    grid = gg.grid.InducingGrid(xg=[np.linspace(0, 1, m).reshape(-1, 1)] * d)
    kern = gg.kern.GriefKernel(kern_list=kl, grid=grid, n_eigs=p)
    kern._setup_inducing_cov()
    assert kern._Quu_full is not None


@pytest.mark.parametrize("d,kind", [(3, "RBF"), (6, "Matern52")])
def test_grief_phi_value_table_matches_log_table(gg, monkeypatch, d, kind):
    """Phi from the value table (default: gg_grief_tables_all / gg_grief_phi
    with stab NULL) against the log / sign tables of the reference's
    expand_SKC (GG_GRIEF_LOGTAB=1), row-major and transposed: the same numbers
    up to the exp(log|X|) rounding, 1e-13 relative."""
    import torch
    rng = np.random.default_rng(3)
    n, m, p = 2000, 24, 200
    x = rng.random((n, d))
    out = []
    for flag in ("0", "1"):
        monkeypatch.setenv("GG_GRIEF_LOGTAB", flag)
        kl = [getattr(gg.kern, kind)(1, variance=1.0, lengthscale=0.2 + 0.02 * i)
              for i in range(d)]
        grid = gg.grid.InducingGrid(xg=[np.linspace(0, 1, m).reshape(-1, 1)] * d)
        kern = gg.kern.GriefKernel(kern_list=kl, grid=grid, n_eigs=p)
        P = kern.phi_device(x).cpu().numpy()
        PT = kern.phi_device(x, transposed=True).cpu().numpy()
        torch.cuda.synchronize()
        out.append((P, PT))
    (P0, T0), (P1, T1) = out
    assert np.abs(T0 - P0.T).max() == 0.0
    assert rel(P0, P1) < 1e-13 and rel(T0, T1) < 1e-13


@pytest.mark.parametrize("kind", ["RBF", "Matern52"])
def test_d_yhat_d_x_matches_finite_differences(gg, kind):
    """GPGriefModel.d_Yhat_d_x (gp_grief_model.py:127-134 via
    GriefKernel.cov_grad, on the fit's own eigenvector basis) against central
    differences of the predictive mean.  The reference needs GPy kernels for
    it (grid_kernel.py:196-199): parity unpinned, checked by differences."""
    rng = np.random.default_rng(11)
    d, m, n, p = 2, 32, 600, 60
    x = rng.random((n, d))
    y = (np.sin(5 * x).sum(axis=1) + 0.05 * rng.standard_normal(n)).reshape(-1, 1)
    kl = [getattr(gg.kern, kind)(1, variance=1.0, lengthscale=0.2 + 0.05 * i) for i in range(d)]
    grid = gg.grid.InducingGrid(xg=[np.linspace(0, 1, m).reshape(-1, 1)] * d)
    kern = gg.kern.GriefKernel(kern_list=kl, grid=grid, n_eigs=p)
    model = gg.models.GPGriefModel(x, y, kern, noise_var=0.01)
    xt = 0.1 + 0.8 * rng.random((40, d))
    h = 1e-5
    for dim in range(d):
        g = np.asarray(model.d_Yhat_d_x(xt, dim))
        assert g.shape == (40, 1)
        e = np.zeros(d)
        e[dim] = h
        fp = np.asarray(model.predict(xt + e)[0])
        fm = np.asarray(model.predict(xt - e)[0])
        fd = (fp - fm) / (2 * h)
        assert np.abs(g - fd).max() < 1e-5 * max(1.0, np.abs(fd).max())
