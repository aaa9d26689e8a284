"""Generate the golden fixtures under tests/golden/ from the reference itself.

Runs ONLY in the build container, where the read-only reference checkout lives
at /root/reference.  It is never run on the GPU box and nothing it imports is
shipped: the committed outputs are plain .npz data (inputs + expected
outputs), each well under 1 MB.

The reference imports GPy at module import time (gp_grief/kern/basekernel.py:3,
gp_grief/kern/gpy_kernel.py:2).  GPy is not installed in this image and the
GPy-backed kernel (GPyKernel) is never exercised here, so a minimal module
object is placed in sys.modules purely so that `import gp_grief` succeeds; every
fixture below uses the reference's own in-house kernels (stationary.py RBF /
Matern52).  numpy>=2 removed np.product, which gp_grief/grid.py:15 uses; it is
aliased to np.prod.

Fixtures:
  kron_matvec.npz    K*x for the reference test factors (sym 5^3), a non-square
                     case (test_kron_eigenvalues.py:104-127) and an RBF 12^4 grid
  kron_eig.npz       find_extremum_eigs (test_kron_eigenvalues.py:11-92 setup)
  grid_gp.npz        8^4 RBF grid GP: solve_schur alpha, mean, latent var, exact
                     log det / LML, scipy-cg restatement history
  grief_test.npz     test_gp_grief_model.py setting with the in-house RBF
  grief_small_*.npz  3-D / 6-D (Matern-5/2) / 8-D GRIEF fits with distinct
                     lengthscales and the p-boundary eigen-gap recorded
  automobile.npz     Type-II tutorial automobile case after optimize(max_iters=5)
  grid_offgrid.npz   off-grid prediction of the grid GP: KhatriRaoMatrix(cov_kr)
                     times alpha, and the dense predictive variance, on a
                     7 x 9 x 8 (mixed sizes) and a 6^4 RBF grid
  rowcol_kr.npz      RowColKhatriRaoMatrix(R, K, C): matvec, transposed matvec,
                     expand and logged expand (test_RowColKhatriRaoMatrix.py
                     setting, plus a 300 x 800 case)
  web.npz            GPwebModel / GPwebTransformedModel: the reference tests'
                     setting (test_gp_web_model.py:12-31) and a 1200 x 48 case
  kron_nonsym.npz    KronMatrix.eig_vals / schur / svd of non-symmetric factors
                     (kron_matrix.py:161-200, 355-366: scipy schur, numpy
                     eigvals / svd per factor) and the SPD sym=True/False log det
                     of test_kron_eigenvalues.py:95-102

Usage:  python tests/golden/make_golden.py [--ref /root/reference]
"""
import argparse
import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def import_reference(ref_root):
    """Import the reference package with GPy absent (see module docstring)."""
    gpy = types.ModuleType("GPy")
    gpy_kern = types.ModuleType("GPy.kern")

    class _Kern(object):  # never instantiated by the fixtures
        pass

    gpy_kern.Kern = _Kern
    gpy_kern.src = types.SimpleNamespace(
        stationary=types.SimpleNamespace(Stationary=_Kern))
    gpy.kern = gpy_kern
    sys.modules.setdefault("GPy", gpy)
    sys.modules.setdefault("GPy.kern", gpy_kern)
    if not hasattr(np, "product"):
        np.product = np.prod
    sys.path.insert(0, ref_root)
    import gp_grief  # noqa: F401
    import logging
    logging.getLogger().setLevel(logging.WARNING)
    return gp_grief


def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    size = os.path.getsize(path)
    assert size < 1 << 20, (name, size)
    print("wrote %-28s %8d bytes" % (name, size))


def rbf_grid(gg, m_list, ls_list, kind="RBF"):
    """The 1-D kernels + per-dim grids used by the grid fixtures."""
    kerns = []
    for ls in ls_list:
        if kind == "RBF":
            kerns.append(gg.kern.RBF(1, variance=1.0, lengthscale=ls))
        else:
            kerns.append(gg.kern.Matern52(1, variance=1.0, lengthscale=ls))
    xg = np.empty(len(m_list), dtype=object)
    for i, m in enumerate(m_list):
        xg[i] = np.linspace(0.0, 1.0, m).reshape((-1, 1))
    return kerns, xg


def grid_targets(xg):
    """y on the grid, dimension 0 fastest (KronMatrix order)."""
    d = len(xg)
    shape = [xg[i].shape[0] for i in range(d)]
    vals = np.zeros(shape[::-1])  # C order, dim d-1 slowest
    for i in range(d):
        f = np.sin(6.0 * xg[i][:, 0])
        bshape = [1] * d
        bshape[d - 1 - i] = shape[i]
        vals = vals + f.reshape(bshape)
    return vals.reshape(-1)


# ---------------------------------------------------------------- F1
def f1_kron_matvec(gg):
    from gp_grief.tensors import KronMatrix
    out = {}
    # reference test setup, tests/test_tensors/test_kron_matrix_sym.py:11-25
    np.random.seed(0)
    d, n = 3, 5
    A = [np.array(np.random.rand(n, n), order="F") for _ in range(d)]
    A = [np.array(a.dot(a.T) + 1e-6 * np.identity(n), order="F") for a in A]
    K = KronMatrix(A, sym=True)
    x = np.random.rand(n ** d, 1)
    out["sym5_factors"] = np.stack(A)
    out["sym5_x"] = x[:, 0]
    out["sym5_y"] = (K * x)[:, 0]
    Q, T = K.schur()
    out["sym5_solve_shift"] = np.float64(1e-3)
    out["sym5_y_solve"] = Q.solve_schur(T, x, shift=1e-3)[:, 0]
    out["sym5_logdet"] = np.float64(K.eig_vals().log_det())

    # non-square case, tests/test_tensors/test_kron_eigenvalues.py:104-127
    np.random.seed(0)
    shapes = [(2, 3), (2, 2), (5, 2)]
    Kn = KronMatrix([np.random.rand(*s) for s in shapes])
    xn = np.random.rand(int(Kn.shape[1]), 1)
    for i, Ki in enumerate(Kn.K):
        out["nonsq_factor%d" % i] = np.asarray(Ki)
    out["nonsq_x"] = xn[:, 0]
    out["nonsq_y"] = (Kn * xn)[:, 0]
    out["nonsq_yT"] = (Kn.T * np.random.RandomState(7).rand(int(Kn.shape[0]), 1))[:, 0]
    out["nonsq_xT"] = np.random.RandomState(7).rand(int(Kn.shape[0]), 1)[:, 0]

    # RBF 12^4 grid with distinct lengthscales
    m = 12
    ls = [0.1 * (1 + 0.05 * i) for i in range(4)]
    kerns, xg = rbf_grid(gg, [m] * 4, ls)
    Kg = gg.kern.GridKernel(kerns).cov_grid(xg, dim_noise_var=1e-12)
    xr = np.random.default_rng(3).standard_normal((m ** 4, 1))
    out["rbf12_factors"] = np.stack([np.asarray(k) for k in Kg.K])
    out["rbf12_lengthscales"] = np.array(ls)
    out["rbf12_x"] = xr[:, 0]
    out["rbf12_y"] = (Kg * xr)[:, 0]
    save("kron_matvec.npz", **out)


# ---------------------------------------------------------------- F2
def f2_kron_eig(gg):
    from gp_grief.tensors import KronMatrix
    out = {}
    np.random.seed(1)  # tests/test_tensors/test_kron_eigenvalues.py:11-17
    d, n, p = 10, 3, 5
    eigs = KronMatrix([np.random.rand(n) for _ in range(d)])
    out["eig_factors"] = np.stack(eigs.K)
    out["n_eigs"] = np.int64(p)
    for mode in ("largest", "smallest"):
        for log in (False, True):
            loc, vals, gloc = eigs.find_extremum_eigs(
                p, mode=mode, log_expand=log, sort=True, compute_global_loc=True)
            tag = "%s_%s" % (mode, "log" if log else "lin")
            out[tag + "_loc"] = np.asarray(loc, dtype=np.int64)
            out[tag + "_vals"] = np.asarray(vals)
            out[tag + "_global"] = np.asarray(gloc, dtype=np.int64)
    # log det of a 2-factor SPD Kron (test_log_det, :94-102)
    np.random.seed(0)
    A = [np.random.rand(5, 5) + np.eye(5) for _ in range(2)]
    A = [a.dot(a.T) + 1e-6 * np.eye(5) for a in A]
    Ak = KronMatrix(A, sym=True)
    out["logdet_factors"] = np.stack(A)
    out["logdet_value"] = np.float64(Ak.eig_vals().log_det())
    # log_kron, tests/test_linalg.py:8-12
    from gp_grief.linalg import log_kron
    np.random.seed(1)
    a = np.random.rand(10)
    b = np.random.rand(4)
    out["logkron_a"] = a
    out["logkron_b"] = b
    out["logkron_ab"] = log_kron(a, b)
    save("kron_eig.npz", **out)


# ---------------------------------------------------------------- F3
class _CGRecorder(object):
    def __init__(self, A, b):
        self.A, self.b, self.hist = A, b, []

    def __call__(self, xk):
        r = self.b - self.A.matvec(xk)
        self.hist.append(np.linalg.norm(r))


def f3_grid_gp(gg):
    from gp_grief.tensors import KronMatrix
    from scipy.sparse.linalg import LinearOperator, cg
    out = {}
    m, d, sig2 = 8, 4, 0.01
    ls = [0.1 * (1 + 0.05 * i) for i in range(d)]
    kerns, xg = rbf_grid(gg, [m] * d, ls)
    K = gg.kern.GridKernel(kerns).cov_grid(xg, dim_noise_var=1e-12)
    N = m ** d
    y = grid_targets(xg) + 0.1 * np.random.default_rng(1).standard_normal(N)
    y = y.reshape((-1, 1))
    Q, T = K.schur()
    t = T.diag().expand()
    alpha = Q.solve_schur(t, y, shift=sig2)
    mean = K * alpha
    Q2 = KronMatrix([np.asarray(q) ** 2 for q in Q.K])
    var_latent = Q2 * (t * sig2 / (t + sig2)).reshape((-1, 1))
    logdet = np.sum(np.log(t + sig2))
    lml = -0.5 * (float(y[:, 0].dot(alpha[:, 0])) + logdet + N * np.log(2 * np.pi))
    out.update(factors=np.stack([np.asarray(k) for k in K.K]), lengthscales=np.array(ls),
               sigma2=np.float64(sig2), y=y[:, 0], alpha=alpha[:, 0], mean=mean[:, 0],
               var_latent=var_latent[:, 0], logdet=np.float64(logdet),
               logdet_unshifted=np.float64(T.diag().log_det()), lml=np.float64(lml),
               eigvals_sorted=np.sort(t))
    A = LinearOperator((N, N), matvec=lambda v: (K * v.reshape((-1, 1)))[:, 0] + sig2 * v,
                       dtype=np.float64)
    rec = _CGRecorder(A, y[:, 0])
    x50, _ = cg(A, y[:, 0], rtol=1e-30, maxiter=50, callback=rec)
    out["cg50_x"] = x50
    out["cg50_true_resid"] = np.array(rec.hist)
    rec2 = _CGRecorder(A, y[:, 0])
    xs, info = cg(A, y[:, 0], rtol=1e-10, callback=rec2)
    out["cg_rtol"] = np.float64(1e-10)
    out["cg_x"] = xs
    out["cg_info"] = np.int64(info)
    out["cg_iters"] = np.int64(len(rec2.hist))
    save("grid_gp.npz", **out)


# ---------------------------------------------------------------- F4
def factor_eigs(kern):
    """Per-factor eigenvalues in the reference's own (gees) order."""
    Kuu = kern.cov_grid(kern.grid.xg, dim_noise_var=kern.dim_noise_var)
    _, T = Kuu.schur()
    lam = [np.asarray(t) for t in T.diag().K]
    return dict(lam_cat=np.concatenate(lam),
                lam_len=np.array([l.size for l in lam], dtype=np.int64))


def phi_signnorm(Phi):
    """Phi is only defined up to per-column sign: fix the sign of each column."""
    Phi = np.array(Phi)
    idx = np.argmax(np.abs(Phi), axis=0)
    s = np.sign(Phi[idx, np.arange(Phi.shape[1])])
    s[s == 0] = 1.0
    return Phi * s


def f4_grief_test(gg):
    from gp_grief.grid import InducingGrid
    from gp_grief.kern import GriefKernel, RBF
    from gp_grief.models import GPGriefModel
    np.random.seed(0)  # tests/test_models/test_gp_grief_model.py:14-21
    d, n = 5, 100
    x = np.random.rand(n, d)
    y = np.random.rand(n, 1)
    grid = InducingGrid(x)
    kern = RBF(1, lengthscale=0.5)
    kern = GriefKernel(kern_list=[kern] * d, grid=grid, n_eigs=50)
    m = GPGriefModel(x, y, kern, noise_var=0.1)
    lml = m._compute_log_likelihood(m.parameters)
    Kd = m._mv_cov(np.identity(n))
    alp = m._mv_cov_inv(y)
    logdet = m._cov_log_det()
    ll, grad = m.log_likelihood(return_gradient=True)
    mean, var = m.predict(x[:7])
    out = dict(x=x, y=y[:, 0], xg=np.stack([g[:, 0] for g in grid.xg]),
               params=m.parameters, alpha=alp[:, 0], alpha_dense=np.linalg.solve(Kd, y)[:, 0],
               logdet=np.float64(logdet), lml=np.float64(np.squeeze(lml)),
               lml_grad_call=np.float64(np.squeeze(ll)), grad=grad,
               pred_mean=mean[:, 0], pred_var=var, log_lam=kern._log_lam,
               eig_pos=np.stack([s.indicies for s in kern._Sp], axis=1).astype(np.int64),
               phi_signnorm=phi_signnorm(m._Phi), A_gram=m._A,
               cov_dense=Kd)
    out.update(factor_eigs(kern))
    save("grief_test.npz", **out)


# ---------------------------------------------------------------- F5
def grief_case(gg, name, d, m, p, kind, n=1000, M=40, sig2=0.01):
    from gp_grief.grid import InducingGrid
    from gp_grief.kern import GriefKernel, RBF, Matern52
    from gp_grief.models import GPGriefModel
    from gp_grief.tensors import KronMatrix
    ls = [0.2 * (1 + 0.05 * i) for i in range(d)]
    if kind == "RBF":
        kl = [RBF(1, variance=1.0, lengthscale=l) for l in ls]
    else:
        kl = [Matern52(1, variance=1.0, lengthscale=l) for l in ls]
    xg = [np.linspace(0.0, 1.0, m).reshape((-1, 1)) for _ in range(d)]
    grid = InducingGrid(xg=xg)
    kern = GriefKernel(kern_list=kl, grid=grid, n_eigs=p)
    x = np.random.default_rng(0).random((n, d))
    y = (np.sin(6.0 * x).sum(axis=1) + 0.1 * np.random.default_rng(1).standard_normal(n))
    y = y.reshape((-1, 1))
    xt = np.random.default_rng(2).random((M, d))
    mdl = GPGriefModel(x, y, kern, noise_var=sig2)
    ll, grad = mdl.log_likelihood(return_gradient=True)
    mean, var = mdl.predict(xt)
    # p-boundary gap: the (p+1)-th largest Kron log-eigenvalue
    Kuu = kern.cov_grid(kern.grid.xg, dim_noise_var=kern.dim_noise_var)
    _, T = Kuu.schur()
    ev = T.diag()
    _, lv, _ = ev.find_extremum_eigs(n_eigs=p + 1, mode="largest", log_expand=True)
    gap = lv[p - 1] - lv[p]
    assert gap > 1e-8, (name, gap)
    out = dict(x=x, y=y[:, 0], xtest=xt, lengthscales=np.array(ls), m=np.int64(m),
               p=np.int64(p), kind=np.array(kind), sigma2=np.float64(sig2),
               lml=np.float64(np.squeeze(ll)), grad=grad, alpha=mdl._alpha[:, 0],
               logdet=np.float64(mdl._cov_log_det()), pred_mean=mean[:, 0],
               pred_var=var, log_lam=kern._log_lam,
               eig_pos=np.stack([s.indicies for s in kern._Sp], axis=1).astype(np.int64),
               boundary_gap=np.float64(gap),
               A_diag=np.diag(mdl._A).copy())
    out.update(factor_eigs(kern))
    save(name, **out)


def f5_grief_small(gg):
    grief_case(gg, "grief_small_3d.npz", d=3, m=32, p=200, kind="RBF")
    grief_case(gg, "grief_small_6d.npz", d=6, m=8, p=500, kind="Matern52")
    grief_case(gg, "grief_small_8d.npz", d=8, m=6, p=1000, kind="RBF")


# ---------------------------------------------------------------- F6
def f6_automobile(gg, ref_root):
    from sklearn.preprocessing import StandardScaler
    from gp_grief.grid import InducingGrid
    from gp_grief.kern import GriefKernel, RBF
    from gp_grief.models import GPGriefModel
    # tutorials/Type-II example with GRIEF kernel.ipynb, cells 9 and 11, with
    # the fork's in-house RBF and GPGriefModel
    np.random.seed(0)
    data = np.loadtxt(os.path.join(ref_root, "tutorials", "automobile.csv"), delimiter=",")
    i_train = np.random.rand(data.shape[0]) < 0.9
    xs, ys = StandardScaler(), StandardScaler()
    x = xs.fit_transform(data[:, :-1])
    y = ys.fit_transform(data[:, (-1,)])
    grid = InducingGrid(x=x)
    kern = GriefKernel(kern_list=[RBF(1, lengthscale=1.0)] * x.shape[1], grid=grid,
                       n_eigs=100, reweight_eig_funs=False, opt_kernel_params=True)
    mdl = GPGriefModel(X=x[i_train], Y=y[i_train], kern=kern, noise_var=1.0)
    p0 = mdl.parameters
    lml0 = float(np.squeeze(mdl.log_likelihood()))
    opt = mdl.optimize(max_iters=5)
    mean, var = mdl.predict(Xnew=x[~i_train])
    rmse = np.linalg.norm(ys.inverse_transform(mean) - ys.inverse_transform(y[~i_train])) \
        / np.sqrt(mean.size)
    out = dict(x=x, y=y[:, 0], i_train=i_train, y_scale=ys.scale_, y_mean=ys.mean_,
               params0=p0, lml0=np.float64(lml0),
               params_opt=mdl.parameters, lml_opt=np.float64(np.squeeze(mdl.log_likelihood())),
               pred_mean=mean[:, 0], pred_var_diag=np.diag(var).copy(),
               rmse=np.float64(rmse), n_funcalls=np.int64(opt["funcalls"]),
               xg_cat=np.concatenate([g[:, 0] for g in grid.xg]),
               xg_len=np.array([g.shape[0] for g in grid.xg], dtype=np.int64))
    save("automobile.npz", **out)


def f7_web(gg):
    """GPwebModel / GPwebTransformedModel (gp_web_model.py:14-130,
    gp_web_transformed_model.py:13-127): LML, adjoint gradient and predictions.
    Case 't' replays test_gp_web_model.py:12-23 exactly (seed 0, intercept
    column, rand + 1e-6 parameters); case 'b' is a 1200 x 48 Gaussian Phi."""
    from gp_grief.models import GPwebModel, GPwebTransformedModel
    out = {}
    for tag in ("t", "b"):
        if tag == "t":
            np.random.seed(0)
            X = np.random.randn(100, 4)
            X[:, 0] = 1.
            Y = np.dot(X, [0.5, 0.1, 0.25, 1.]) + 0.1 * np.random.randn(X.shape[0])
            params = np.random.rand(5) + 1e-6
        else:
            rng = np.random.default_rng(7)
            X = rng.standard_normal((1200, 48)) / 7.0
            Y = np.sin(X.sum(axis=1) * 3.0) + 0.1 * rng.standard_normal(1200)
            params = np.concatenate(([0.05], rng.uniform(0.5, 2.0, 48)))
        Xnew = X[:7] + 0.01
        out[tag + "_X"] = X
        out[tag + "_Y"] = Y
        out[tag + "_params"] = params
        out[tag + "_Xnew"] = Xnew
        for cls, key in ((GPwebModel, "web"), (GPwebTransformedModel, "tr")):
            m = cls(Phi=X, y=Y)
            m.parameters = params.copy()
            ll, g = m._adjoint_gradient(m.parameters)
            out["%s_%s_lml" % (tag, key)] = np.asarray(ll, dtype=np.float64)
            out["%s_%s_grad" % (tag, key)] = g
            yh, yv = m.predict(Xnew)
            out["%s_%s_mean" % (tag, key)] = yh
            out["%s_%s_var" % (tag, key)] = yv
            if key == "tr":
                out[tag + "_tr_singular"] = m.singular_vals
                out[tag + "_tr_PhitTy2"] = m.PhitT_y_2
    save("web.npz", **out)


def f8_grid_offgrid(gg):
    """Off-grid posterior of a full-grid GP: mean = K(X*, grid) alpha with
    K(X*, grid) = GridKernel.cov_kr(X*, xg) (grid_kernel.py:148-179), a
    row-partitioned KhatriRaoMatrix (khatri_rao_matrix.py:7-50) applied by
    BlockMatrix.__mul__; latent variance k** - k*^T (K + s I)^-1 k* from the
    expanded Khatri-Rao rows and KronMatrix.solve_schur (kron_matrix.py:328-352)."""
    out = {}
    for tag, ms, ls, M in (("a", [7, 9, 8], [0.15, 0.2, 0.25], 23),
                           ("b", [6, 6, 6, 6], [0.2, 0.22, 0.24, 0.26], 17)):
        d, sig2 = len(ms), 0.01
        kerns, xg = rbf_grid(gg, ms, ls)
        gk = gg.kern.GridKernel(kerns)
        K = gk.cov_grid(xg, dim_noise_var=1e-12)
        N = int(np.prod(ms))
        y = (grid_targets(xg) + 0.1 * np.random.default_rng(3).standard_normal(N)).reshape(-1, 1)
        Q, T = K.schur()
        t = T.diag().expand()
        alpha = Q.solve_schur(t, y, shift=sig2)
        xs = np.random.default_rng(4).uniform(-0.05, 1.05, (M, d))
        # cov_kr(form_kr=True) hands a ragged list to np.ndim, which numpy>=2
        # rejects (khatri_rao_matrix.py:25); the same blocks as an object array:
        blocks = gk.cov_kr(xs, xg, form_kr=False)
        A = np.empty(len(blocks), dtype=object)
        for i, b in enumerate(blocks):
            A[i] = b
        Kxz = gg.tensors.KhatriRaoMatrix(A=A, partition=0)
        mean = Kxz * alpha
        Kd = Kxz.expand()
        quad = np.array([float(Kd[j].dot(Q.solve_schur(t, Kd[j].reshape(-1, 1), shift=sig2)[:, 0]))
                         for j in range(M)])
        kss = np.array([float(gk.cov(xs[(j,), :])[0, 0]) for j in range(M)])
        out.update({tag + "_m": np.array(ms), tag + "_ls": np.array(ls),
                    tag + "_sigma2": np.float64(sig2), tag + "_y": y[:, 0],
                    tag + "_alpha": alpha[:, 0], tag + "_xs": xs, tag + "_mean": mean[:, 0],
                    tag + "_var_latent": kss - quad})
    save("grid_offgrid.npz", **out)


def f9_rowcol_kr(gg):
    """RowColKhatriRaoMatrix (khatri_rao_matrix.py:53-178) and the Transposed
    variant (:181-210): A[a, b] = prod_i (R_i K_i C_i)[a, b]."""
    from gp_grief.tensors import RowColKhatriRaoMatrix, RowColKhatriRaoMatrixTransposed
    out = {}
    for tag in ("t", "b"):
        if tag == "t":   # test_RowColKhatriRaoMatrix.py:9-22, same draws
            np.random.seed(0)
            N, p, d = 5, 6, 3
            grid_shape = np.random.randint(low=2, high=15, size=d)
            R = [np.random.rand(p, m) - 0.5 for m in grid_shape]
            K = [np.random.rand(m, m) - 0.5 for m in grid_shape]
            C = [np.random.rand(m, N) - 0.5 for m in grid_shape]
            for i in range(d):
                R[i][0, :] = 0.
            vec = np.random.rand(N, 1) - 0.5
            vecT = np.random.rand(p, 1) - 0.5
        else:
            rng = np.random.default_rng(12)
            N, p, grid_shape = 800, 300, np.array([17, 9, 23])
            d = 3
            R = [rng.random((p, m)) - 0.5 for m in grid_shape]
            K = [rng.random((m, m)) - 0.5 for m in grid_shape]
            C = [rng.random((m, N)) - 0.5 for m in grid_shape]
            R[1][:7, :] = 0.
            vec = rng.random((N, 1)) - 0.5
            vecT = rng.random((p, 1)) - 0.5
        def objarr(L):
            a = np.empty(len(L), dtype=object)
            for i, x in enumerate(L):
                a[i] = x
            return a
        A = RowColKhatriRaoMatrix(R=objarr(R), K=objarr(K), C=objarr(C))
        AT = RowColKhatriRaoMatrixTransposed(R=objarr(R), K=objarr(K), C=objarr(C))
        log_A, sign = A.expand(logged=True)
        for i in range(d):
            out["%s_R%d" % (tag, i)] = R[i]
            out["%s_K%d" % (tag, i)] = K[i]
            out["%s_C%d" % (tag, i)] = C[i]
        out.update({tag + "_d": np.int64(d), tag + "_vec": vec, tag + "_vecT": vecT,
                    tag + "_Avec": A * vec, tag + "_ATvecT": A.T * vecT,
                    tag + "_ATT_vecT": AT * vecT,
                    # first 24 rows only (fixture size); the products cover the rest
                    tag + "_expand": A.expand()[:24], tag + "_log": log_A[:24],
                    tag + "_sign": np.asarray(sign, dtype=np.float64)[:24]})
    save("rowcol_kr.npz", **out)


def f10_kron_nonsym(gg):
    from gp_grief.tensors import KronMatrix
    out = {}
    np.random.seed(3)
    F = [np.random.rand(5, 5) + np.eye(5), np.random.rand(3, 3), np.random.rand(4, 4) - 0.5]
    K = KronMatrix(F, sym=False)
    eig = K.eig_vals()
    for i, e in enumerate(eig.K):
        out["eig%d" % i] = np.asarray(e)
    Q, T = K.schur()
    U, S = K.svd()
    for i in range(3):
        out["F%d" % i] = F[i]
        out["schurQ%d" % i] = np.asarray(Q.K[i])
        out["schurT%d" % i] = np.asarray(T.K[i])
        out["svdU%d" % i] = np.asarray(U.K[i])
        out["svdS%d" % i] = np.asarray(S.K[i])
    # test_kron_eigenvalues.py:95-102: SPD factors, sym True / False, log det
    for sym in (True, False):
        np.random.seed(0)
        A = [np.random.rand(5, 5) + np.eye(5) for _ in range(2)]
        A = [Ai.dot(Ai.T) + 1e-6 * np.eye(5) for Ai in A]
        KA = KronMatrix(A, sym=sym)
        tag = "spd_sym%d" % int(sym)
        out[tag + "_A0"], out[tag + "_A1"] = A
        out[tag + "_logdet"] = np.float64(KA.eig_vals().log_det())
        out[tag + "_slogdet"] = np.float64(np.linalg.slogdet(KA.expand())[1])
    save("kron_nonsym.npz", **out)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--only", default=None, help="comma list of fixture functions, e.g. f7_web")
    a = ap.parse_args()
    gg = import_reference(a.ref)
    if a.only:
        for name in a.only.split(","):
            globals()[name](gg)
        return
    f1_kron_matvec(gg)
    f2_kron_eig(gg)
    f3_grid_gp(gg)
    f4_grief_test(gg)
    f5_grief_small(gg)
    f6_automobile(gg, a.ref)
    f7_web(gg)
    f8_grid_offgrid(gg)
    f9_rowcol_kr(gg)
    f10_kron_nonsym(gg)


if __name__ == "__main__":
    main()
