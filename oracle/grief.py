"""GP-GRIEF fit / likelihood / predict -- CPU oracle (test infrastructure only).

Restates, for the in-house 1-D kernels:
  GriefKernel._setup_inducing_cov   kern/grief_kernel.py:168-190
  GriefKernel.cov + expand_SKC      kern/grief_kernel.py:68-111, tensors/tensors.py:97-128
  GPGriefModel._cov_setup/_mv_cov_inv/_cov_log_det/_compute_log_likelihood
                                    models/gp_grief_model.py:137-153, 228-245, 203-214
  GPGriefModel._adjoint_gradient    models/gp_grief_model.py:156-200
  GPGriefModel.predict              models/gp_grief_model.py:99-125
Factor order follows GridKernel (grid_kernel.py:109,174): factor f belongs to
input dimension d-1-f.
"""
import numpy as np
from scipy.linalg import cho_factor, cho_solve

from .kernels import cov_1d
from .kron import factor_eigh, find_extremum_eigs


def grief_inducing(kern_specs, xg, n_eigs, jitter=1e-12):
    """Per-factor eigenpairs and the top-p Kronecker eigen-selection.

    kern_specs: list over INPUT dims of (kind, variance, lengthscale).
    xg: list over input dims of 1-D grid arrays.
    Returns dict(Q=[factor order], lam=[...], eig_pos [p x d], log_lam [p]).
    """
    d = len(xg)
    K = []
    for f in range(d):
        i = d - 1 - f
        kind, var, ls = kern_specs[i]
        g = np.asarray(xg[i], dtype=np.float64).reshape(-1)
        K.append(cov_1d(kind, g, g, var, ls) + jitter * np.eye(g.size))
    Q, lam = factor_eigh(K)
    total = float(np.prod([float(k.shape[0]) for k in K]))   # grid size, as float (no overflow)
    p = int(min(n_eigs, total))
    pos, log_lam, _ = find_extremum_eigs(lam, p, mode='largest', log_expand=True)
    return dict(K=K, Q=Q, lam=lam, eig_pos=pos, log_lam=log_lam, p=p)


def grief_phi(x, kern_specs, xg, ind):
    """Phi (n x p): Phi[a, j] = prod_f (Q_f^T Kux_f)[pos_jf, a] / sqrt(prod lambda).

    Log-space product exactly as expand_SKC(logged=True) + the exp in
    GriefKernel.cov: the sign is taken before zeros are replaced by one.
    """
    x = np.asarray(x, dtype=np.float64)
    d = x.shape[1]
    pos = ind["eig_pos"]
    logp = 0.0
    sign = np.int32(1)
    for f in range(d):
        i = d - 1 - f
        kind, var, ls = kern_specs[i]
        kux = cov_1d(kind, np.asarray(xg[i]).reshape(-1), x[:, i], var, ls)  # m x n
        uniq, inv = np.unique(pos[:, f], return_inverse=True)
        xu = ind["Q"][f].T[uniq, :].dot(kux)
        sign = sign * np.int32(np.sign(xu))[inv]
        xu[xu == 0] = 1.0
        logp = logp + np.log(np.abs(xu))[inv]
    return sign.T * np.exp(logp.T - 0.5 * ind["log_lam"].reshape((1, -1)))


def grief_fit(Phi, w, y, sig2):
    """A = Phi^T Phi, P = A + diag(s/w), upper Cholesky, Woodbury alpha."""
    y = np.asarray(y, dtype=np.float64).reshape((-1, 1))
    A = Phi.T.dot(Phi)
    P = A + np.diag(sig2 / np.asarray(w, dtype=np.float64))
    Pc = cho_factor(P)
    alpha = (y - Phi.dot(cho_solve(Pc, Phi.T.dot(y)))) / sig2
    n, p = Phi.shape
    logdet = (2.0 * np.sum(np.log(np.diag(Pc[0]))) + np.sum(np.log(w))
              + float(n - p) * np.log(sig2))
    return dict(A=A, P=P, Pchol=Pc, alpha=alpha, logdet=logdet)


def grief_lml(fit, y):
    y = np.asarray(y, dtype=np.float64).reshape(-1)
    n = y.size
    return -0.5 * (float(y.dot(fit["alpha"][:, 0])) + fit["logdet"] + n * np.log(2 * np.pi))


def grief_adjoint_grad(Phi, fit, sig2, reweight=True, noise_free=True):
    """(dL/dsigma^2, dL/dw) of GPGriefModel._adjoint_gradient."""
    alpha = fit["alpha"]
    A = fit["A"]
    PinvA = cho_solve(fit["Pchol"], A)
    dw = None
    if reweight:
        data = 0.5 * (Phi.T.dot(alpha)[:, 0]) ** 2
        comp = -0.5 * (np.diag(A) - (A * PinvA).sum(axis=0)) / sig2
        dw = data + comp
    ds = None
    if noise_free:
        n = Phi.shape[0]
        ds = 0.5 * float(alpha[:, 0].dot(alpha[:, 0])) - 0.5 * (n - np.trace(PinvA)) / sig2
    return ds, dw


def grief_predict(Phi, fit, w, sig2, Phi_star):
    alpha_p = Phi.T.dot(fit["alpha"]) * np.asarray(w).reshape((-1, 1))
    mean = Phi_star.dot(alpha_p)
    var = sig2 * Phi_star.dot(cho_solve(fit["Pchol"], Phi_star.T)) \
        + sig2 * np.eye(Phi_star.shape[0])
    return mean, var
