"""Weighted-basis (WEB) GP models -- CPU oracle (test infrastructure only).

Restates, on a given basis matrix Phi (n x p) and weights w (the WEBKernel
parameters, kern/web_kernel.py:4-13):
  GPwebModel               models/gp_web_model.py:14-130
      _compute_log_likelihood  :51-69   (P = A + diag(s/w), Cholesky, datafit)
      _adjoint_gradient        :72-106
      predict                  :109-129
  GPwebTransformedModel    models/gp_web_transformed_model.py:13-127
      __init__ (thin SVD, keep s > 1e-7)  :19-50
      _compute_log_likelihood  :53-65
      _adjoint_gradient        :68-98
      predict                  :101-121
Parameters are [noise_var, w_1..w_p] (basemodel.py:150-184).
"""
import numpy as np
from scipy.linalg import cho_factor, cho_solve


def web_lml_grad(Phi, y, params):
    """(LML, gradient [s, w...]) of GPwebModel with dense p x p algebra."""
    y = np.asarray(y, dtype=np.float64).reshape(-1, 1)
    n, p = Phi.shape
    s = float(params[0])
    w = np.asarray(params[1:], dtype=np.float64)
    A = Phi.T.dot(Phi)
    r = Phi.T.dot(y)
    yTy = float(y.T.dot(y)[0, 0])
    Pc = cho_factor(A + np.diag(s / w))
    z = cho_solve(Pc, r)
    rz = float(r.T.dot(z)[0, 0])
    datafit = (yTy - rz) / s
    complexity = 2. * np.sum(np.log(np.diag(Pc[0]))) + np.sum(np.log(w)) + (n - p) * np.log(s)
    ll = -0.5 * (complexity + datafit + n * np.log(2. * np.pi))
    PinvA = cho_solve(Pc, A)
    g = np.zeros(p + 1)
    dfg = -((r - A.dot(z)) / s) ** 2
    cg = (A.diagonal() - (A * PinvA).sum(axis=0)) / s
    g[1:] = -0.5 * dfg.ravel() - 0.5 * cg
    dfs = -(yTy - 2. * rz + float(z.T.dot(A.dot(z))[0, 0])) / s ** 2
    cs = (n - np.trace(PinvA)) / s
    g[0] = -0.5 * (dfs + cs)
    return ll, g


def web_predict(Phi, y, params, Phi_new):
    y = np.asarray(y, dtype=np.float64).reshape(-1, 1)
    s = float(params[0])
    w = np.asarray(params[1:], dtype=np.float64).reshape(-1, 1)
    A = Phi.T.dot(Phi)
    r = Phi.T.dot(y)
    Pc = cho_factor(A + np.diag(s / w.ravel()))
    z = cho_solve(Pc, r)
    alpha_p = (r - A.dot(z)) * w / s
    mean = Phi_new.dot(alpha_p)
    var = s * Phi_new.dot(cho_solve(Pc, Phi_new.T)) + s * np.eye(Phi_new.shape[0])
    return mean, var


def web_transformed_setup(Phi, y):
    """Thin SVD of Phi, bases with singular value > 1e-7 kept."""
    y = np.asarray(y, dtype=np.float64).reshape(-1, 1)
    U, sv, VT = np.linalg.svd(Phi, full_matrices=False)
    keep = sv > 1e-7
    U, sv, VT = U[:, keep], sv[keep], VT[keep]
    PhitTy = U.T.dot(y).ravel()
    return dict(sv=sv, V=VT.T, PhitTy=PhitTy, PhitTy2=PhitTy ** 2,
                yTy=float((y ** 2).sum()), n=Phi.shape[0], p=int(keep.sum()))


def web_transformed_lml_grad(st, params):
    s = float(params[0])
    w = np.asarray(params[1:], dtype=np.float64)
    n, p = st["n"], st["p"]
    Pd = s / w + 1.
    datafit = (st["yTy"] - np.sum(st["PhitTy2"] / Pd)) / s
    complexity = np.sum(np.log(Pd)) + np.sum(np.log(w)) + (n - p) * np.log(s)
    ll = -0.5 * (complexity + datafit + n * np.log(2. * np.pi))
    g = np.zeros(p + 1)
    g[1:] = -0.5 * (-st["PhitTy2"] / (s + w) ** 2 + 1. / (s + w))
    dfs = (-st["yTy"] + np.sum(st["PhitTy2"] * w * (2. * s + w) / (s + w) ** 2)) / s ** 2
    cs = float(n - p) / s + np.sum(1. / (s + w))
    g[0] = -0.5 * (dfs + cs)
    return ll, g


def web_transformed_predict(st, params, Phi_new):
    s = float(params[0])
    w = np.asarray(params[1:], dtype=np.float64)
    Pd = s / w + 1.
    alpha_p = (st["PhitTy"] - st["PhitTy"] / Pd) * w / s
    mean = Phi_new.dot(st["V"].dot(alpha_p / st["sv"])).reshape(-1, 1)
    var = s * Phi_new.dot(Phi_new.T / Pd.reshape(-1, 1)) + s * np.eye(Phi_new.shape[0])
    return mean, var
