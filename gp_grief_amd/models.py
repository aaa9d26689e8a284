"""Models: drop-in mirror of gp_grief.models on the MI355X.

  BaseModel      gp_grief/models/basemodel.py:14-379 -- parameter vector, softplus
                 transforms, L-BFGS optimize, finite-difference gradient,
                 checkgrad, cache invalidation (host logic, same behaviour)
  GPGriefModel   gp_grief/models/gp_grief_model.py:15-245 -- Phi, the p x p
                 Gram, Cholesky, Woodbury solve, log det, LML, adjoint gradient,
                 predict: every O(n p) / O(p^3) step on the device
  GPwebModel     gp_grief/models/gp_web_model.py:14-130 -- WEB kernel GP, device
                 Gram / Cholesky / solves / predictions
  GPwebTransformedModel  gp_grief/models/gp_web_transformed_model.py:13-127 -- thin
                 SVD of Phi on the device (Gram + Jacobi), O(p) likelihood
  GPRegressionModel  gp_grief/models/gpr_model.py:14-127 -- dense exact GP,
                 device covariance and Cholesky (off the GRIEF hot path)
  GPGridModel    (new, the north star's P1 model) exact or CG grid GP on a full
                 Kronecker-structured grid: KronMatrix operator, device CG /
                 exact eigen-solve, exact or Lanczos (SLQ) log det, posterior
                 mean and latent variance on the grid.

Device state keeps the reference's attribute names (_Phi, _A, _P, _Pchol,
_alpha, _alpha_p) holding CUDA tensors (or small host arrays where the
reference keeps scalars/vectors).
"""
import logging
from traceback import format_exc

import numpy as np
from numpy.linalg import LinAlgError
from numpy.testing import assert_array_almost_equal
from scipy.optimize import fmin_l_bfgs_b

from . import dense
from . import device as dev
from .kern import GriefKernel, BaseKernel
from .linalg import solver_counter, LogexpTransformation

logger = logging.getLogger(__name__)


class BaseModel(object):
    """Parameter plumbing and optimisation (basemodel.py:14-379)."""
    param_shift = {'+ve': 1e-200, '-ve': -1e-200}
    _transformations = {'+ve': LogexpTransformation()}

    def __init__(self):
        logger.debug('Initializing %s model.' % self.__class__.__name__)
        self.dependent_attributes = ['_alpha', '_log_like', '_gradient', '_K', '_log_det']
        self._previous_parameters = None
        self.grad_method = None
        self.noise_var_constraint = '+ve'

    def log_likelihood(self, return_gradient=False):
        p = self.parameters
        if return_gradient and (self._gradient is None):
            if 'adjoint' in self.grad_method:
                (self._log_like, self._gradient) = self._adjoint_gradient(p)
            elif 'finite_difference' in self.grad_method:
                (self._log_like, self._gradient) = self._finite_diff_gradient(p)
            else:
                raise RuntimeError('unknown grad_method %s' % repr(self.grad_method))
        elif self._log_like is None:
            self._log_like = self._compute_log_likelihood(p)
        if return_gradient:
            return self._log_like, self._gradient
        return self._log_like

    def optimize(self, max_iters=1e3, messages=False, use_counter=False, factr=1e7,
                 pgtol=1e-05):
        logger.debug('Beginning MLE to optimize hyperparams. grad_method=%s' % self.grad_method)
        try:
            x0 = self._transform_parameters(self.parameters)
            assert np.all(np.isfinite(x0))
        except Exception:
            logger.error('Transformation failed for initial values. '
                         'Ensure constraints are met or the value is not too small.')
            raise
        free = np.logical_not(self._fixed_indicies)
        x0 = x0[free]
        self._counter = solver_counter(disp=True) if use_counter else None
        try:
            x_opt, f_opt, opt = fmin_l_bfgs_b(func=self._objective_grad, x0=x0, factr=factr,
                                              pgtol=pgtol, maxiter=max_iters, disp=messages)
        except (KeyboardInterrupt, IndexError):
            logger.info('Keyboard interrupt raised. Cleaning up...')
            if self._counter is not None and self._counter.backup is not None:
                self.parameters = self._counter.backup[1]
                logger.info('will return best parameter set with log-likelihood = %.4g'
                            % self._counter.backup[0])
            opt = None
        else:
            logger.info('Function Evals: %d. Exit status: %s' % (f_opt, opt['warnflag']))
            transformed = self._previous_parameters
            transformed[free] = x_opt
            self.parameters = self._untransform_parameters(transformed)
        return opt

    def checkgrad(self, decimal=3, raise_if_fails=True):
        grad_exact = self._finite_diff_gradient(self.parameters)[1]
        grad_exact[self._fixed_indicies] = 1
        grad_analytic = self.log_likelihood(return_gradient=True)[1].copy()
        grad_analytic[self._fixed_indicies] = 1
        protected_nan = np.logical_and(np.abs(grad_exact) < 1e-8, np.abs(grad_analytic) < 1e-8)
        protected_div0 = np.abs(grad_exact - grad_analytic) < 1e-5
        prot = np.logical_or(protected_nan, protected_div0)
        grad_exact[prot] = 1.
        grad_analytic[prot] = 1.
        try:
            assert_array_almost_equal(grad_exact / grad_analytic, np.ones(grad_exact.shape),
                                      decimal=decimal)
        except AssertionError:
            logger.info('Gradient check failed.')
            logger.debug('[[Finite-Diff Gradient], [Analytic Gradient]]:\n%s\n'
                         % repr(np.asarray([grad_exact, grad_analytic])))
            if raise_if_fails:
                raise
            logger.info(format_exc())
            return False
        logger.info('Gradient check passed.')
        return True

    @property
    def parameters(self):
        parameters = np.concatenate((np.ravel(self.noise_var), self.kern.parameters), axis=0)
        if not np.array_equal(parameters, self._previous_parameters):
            for attr in self.dependent_attributes:
                setattr(self, attr, None)
            self._previous_parameters = parameters.copy()
        return parameters.copy()

    @parameters.setter
    def parameters(self, parameters):
        self.noise_var = parameters[0]
        self.kern.parameters = parameters[1:]
        if not np.array_equal(parameters, self._previous_parameters):
            for attr in self.dependent_attributes:
                setattr(self, attr, None)
            self._previous_parameters = parameters.copy()

    @property
    def constraints(self):
        return np.concatenate((np.ravel(self.noise_var_constraint), self.kern.constraints),
                              axis=0)

    def predict(self, Xnew, compute_var=None):
        raise NotImplementedError('')

    def fit(self):
        raise NotImplementedError('')

    def _objective_grad(self, transformed_free_parameters):
        free = np.logical_not(self._fixed_indicies)
        transformed = self._previous_parameters
        transformed[free] = transformed_free_parameters
        try:
            self.parameters = self._untransform_parameters(transformed)
            (objective, gradient) = self.log_likelihood(return_gradient=True)
            objective = -objective
            gradient = -gradient
            if not np.isfinite(objective):
                logger.debug('objective is not finite')
            if not np.all(np.isfinite(gradient[free])):
                logger.debug('some derivatives are non-finite')
            gradient = self._transform_gradient(self.parameters, gradient)
        except (LinAlgError, ZeroDivisionError, ValueError):
            logger.error('numerical issue computing log-likelihood or gradient')
            raise
        free_gradient = gradient[free]
        if self._counter is not None:
            msg = 'log-likelihood=%.4g, gradient_norm=%.2g' % (-objective,
                                                              np.linalg.norm(gradient))
            if self._counter.backup is None or self._counter.backup[0] < -objective:
                self._counter(msg=msg, store=(-objective, self.parameters.copy()))
            else:
                self._counter(msg=msg)
        return objective, free_gradient

    @property
    def _fixed_indicies(self):
        return self.constraints == 'fixed'

    @property
    def _free_indicies(self):
        return np.logical_not(self._fixed_indicies)

    def _transform_parameters(self, parameters):
        constraints = self.constraints
        assert parameters.size == np.size(constraints)
        out = np.zeros(parameters.size)
        for i, (param, c) in enumerate(zip(parameters, constraints)):
            if c is None or c == 'fixed' or c == '':
                out[i] = param
            else:
                out[i] = self._transformations[c].transform(param - self.param_shift[c])
        if not np.all(np.isfinite(out)):
            logger.debug('transformation led to non-finite value')
        return out

    def _transform_gradient(self, parameters, gradients):
        constraints = self.constraints
        assert parameters.size == gradients.size == np.size(constraints)
        out = np.zeros(parameters.size)
        for i, (param, grad, c) in enumerate(zip(parameters, gradients, constraints)):
            if c is None or c == '':
                out[i] = grad
            elif c != 'fixed':
                out[i] = self._transformations[c].transform_grad(param - self.param_shift[c],
                                                                grad)
        if not np.all(np.isfinite(out)):
            logger.debug('transformation led to non-finite value')
        return out

    def _untransform_parameters(self, transformed_parameters):
        assert transformed_parameters.size == np.size(self.constraints)
        out = np.zeros(transformed_parameters.size)
        for i, (t, c) in enumerate(zip(transformed_parameters, self.constraints)):
            if c is None or c == 'fixed' or c == '':
                out[i] = t
            else:
                out[i] = self._transformations[c].inverse_transform(t) + self.param_shift[c]
        if not np.all(np.isfinite(out)):
            logger.debug('transformation led to non-finite value')
        return out

    def _finite_diff_gradient(self, parameters):
        """Forward differences, step 1e-6 (basemodel.py:328-361)."""
        assert isinstance(parameters, np.ndarray)
        free_inds = np.nonzero(np.logical_not(self._fixed_indicies))[0]
        step = 1e-6
        ll_fs = np.zeros(free_inds.size)
        for i, idx in enumerate(free_inds):
            p_fs = parameters.copy()
            p_fs[idx] += step
            ll_fs[i] = np.squeeze(self._compute_log_likelihood(p_fs))
        log_like = self._compute_log_likelihood(parameters)
        gradient = np.zeros(parameters.shape)
        gradient[free_inds] = (ll_fs - np.squeeze(log_like)) / step
        return log_like, gradient

    def _compute_log_likelihood(self, parameters):
        raise NotImplementedError('')

    def _adjoint_gradient(self, parameters):
        raise NotImplementedError('')


class GPRegressionModel(BaseModel):
    """Dense exact GP regression (gpr_model.py:14-127): the n x n covariance
    from the kernel's device cov, a device Cholesky of K + s I, alpha, the LML
    and predictions.  Outside the GRIEF hot path but part of
    the reference's model surface.  The reference's 'svd' / mvn branches are
    broken; this keeps its default 'finite_difference chol'
    route, and compute_var='diag' returns the diagonal as intended."""

    def __init__(self, X, Y, kernel, noise_var=1.):
        super(GPRegressionModel, self).__init__()
        assert X.ndim == 2
        assert Y.ndim == 2
        self.X = np.asarray(X)
        self.Y = np.asarray(Y)
        assert not np.any(np.isnan(Y))
        self.num_data, self.input_dim = self.X.shape
        if Y.shape[0] != self.num_data:
            raise ValueError('X and Y sizes are inconsistent')
        self.output_dim = self.Y.shape[1]
        if self.output_dim != 1:
            raise RuntimeError('this only deals with 1 response for now')
        assert isinstance(kernel, BaseKernel)
        self.kern = kernel
        self.noise_var = np.float64(noise_var)
        self.grad_method = 'finite_difference chol'
        self.dependent_attributes = list(self.dependent_attributes) + ['_chol']
        self._chol = None

    def _cov_dev(self, x, z=None):
        xd = dev.to_device(x).reshape(np.shape(x))
        zd = None if z is None else dev.to_device(z).reshape(np.shape(z))
        return self.kern.cov(xd, zd)

    def _factor(self):
        if self._chol is None:
            K = self._cov_dev(self.X)
            self._chol = dense.Cholesky(dense.add_diag(K, float(self.noise_var)))
        return self._chol

    def fit(self):
        self.parameters
        if self._alpha is None:
            self._alpha = self._factor().solve(dev.to_device(self.Y[:, 0]), which=3)

    def predict(self, Xnew, compute_var=None):
        """Yhat (M,1), and with compute_var 'diag' (M,1) / 'full' (M,M) the
        predictive covariance k** + s I - k*^T (K + s I)^-1 k*."""
        assert Xnew.ndim == 2
        assert Xnew.shape[1] == self.input_dim
        self.parameters
        self.fit()
        Khat = self._cov_dev(Xnew, self.X)                         # M x n
        yhat = dense.matvec(Khat, self._alpha)
        if compute_var is None:
            return dense.host(yhat).reshape((-1, 1))
        if compute_var not in ('diag', 'full'):
            raise ValueError('Unknown compute_var = %s' % repr(compute_var))
        V = self._factor().solve(Khat.t().contiguous(), which=1)  # L^-1 k*  (n x M)
        var = dense.matmul(V, V, ta=True, alpha=-1.0, beta=1.0,
                           C=dense.add_diag(self._cov_dev(Xnew), float(self.noise_var)))
        var = dense.host(var)
        if compute_var == 'diag':
            var = np.diag(var).reshape((-1, 1))
        return dense.host(yhat).reshape((-1, 1)), var

    def _compute_log_likelihood(self, parameters):
        self.parameters = parameters
        self.fit()
        yd = dev.to_device(self.Y[:, 0])
        return -0.5 * (dense.dot(yd, self._alpha) + self._factor().logdet
                       + self.num_data * np.log(np.pi * 2))


def _dev_2d(x):
    xd = dev.to_device(x)
    shape = tuple(x.shape)
    return xd.reshape(shape[0], shape[1] if len(shape) > 1 else 1)


class GPGriefModel(BaseModel):
    """GP-GRIEF (gp_grief_model.py:15-245) with every O(np), O(np^2), O(p^3)
    step on the MI355X (Phi build, SYRK Gram on FP64 MFMA, blocked Cholesky,
    Woodbury solves, GEMV / GEMM predictions).

    comm (optional, new): data-row sharding over GPUs.  Each
    rank passes ITS rows of X and Y; the basis (grid, eigen-selection) is
    replicated, Phi is built only for the local rows, and the three global
    reductions of the Woodbury algebra are all-reduces through comm
    (gp_grief_amd.distributed.TorchExchange = RCCL): the p x p Gram
    Phi^T Phi, the p-vector Phi^T v of every solve / prediction, and the
    scalars y.alpha, alpha.alpha and n.  The p x p Cholesky is replicated.
    Results are the unsharded model's on the concatenated data, on every rank.

    p_solver (new): how the Woodbury p-system P z = Phi^T v (P = A + diag(s/w),
    gp_grief_model.py:228-235) is solved.  'chol' (default, the reference's
    cho_solve): the p x p Gram and its Cholesky.  'cg': Jacobi-preconditioned
    CG whose operator P v = sum_g Phi_g^T (Phi_g v) + (s/w) v is two device
    GEMVs over the local rows and ONE all-reduce of p doubles per iteration
    (the "RCCL all-reduce CG" of config C5) -- no Gram, no
    factorisation for alpha and the predictive mean.  The log det (LML) and
    the predictive covariance still need P's Cholesky and build it on demand.
    """

    def __init__(self, X, Y, kern, noise_var=1., comm=None, p_solver='chol', cg_rtol=1e-12,
                 cg_maxiter=None):
        super(GPGriefModel, self).__init__()
        assert X.ndim == 2
        assert Y.ndim == 2
        self.X = np.asarray(X)
        self.Y = np.asarray(Y)
        assert not np.any(np.isnan(Y))
        self.comm = comm
        self._n_local, self.input_dim = self.X.shape
        if Y.shape[0] != self._n_local:
            raise ValueError('X and Y sizes are inconsistent')
        self.num_data = self._n_local if comm is None else \
            int(round(self._sum_scalar(float(self._n_local))))
        self.output_dim = self.Y.shape[1]
        if self.output_dim != 1:
            raise RuntimeError('this only deals with 1 response for now')
        assert isinstance(kern, GriefKernel)
        assert np.ndim(kern.kern_list) == 1
        for ki in kern.kern_list:
            assert isinstance(ki, BaseKernel)
            assert ki.n_dims == 1, "currently only 1-dimensional grids allowed"
        self.kern = kern
        self.noise_var = np.float64(noise_var)
        self.dependent_attributes = np.unique(np.concatenate(
            (self.dependent_attributes, ['_P', '_Pchol', '_alpha_p'])))
        if self.kern.opt_kernel_params:
            self.dependent_attributes = np.unique(np.concatenate(
                (self.dependent_attributes, ['_A', '_Phi', '_X_last_pred', '_Phi_last_pred'])))
        else:
            self._A = None
            self._Phi = None
            self._Phi_last_pred = None
            self._X_last_pred = None
        if self.kern.opt_kernel_params:
            self.grad_method = 'finite_difference'
        else:
            self.grad_method = ['adjoint', 'finite_difference'][0]
        self._Yd = None
        self._Xd = None
        self._Xd_src = None
        self._gram_uplo = 1   # A = Phi^T Phi is formed in its lower triangle only
        if p_solver not in ('chol', 'cg'):
            raise ValueError("p_solver must be 'chol' or 'cg'")
        self.p_solver = p_solver
        self.cg_rtol = float(cg_rtol)
        self.cg_maxiter = cg_maxiter
        self.cg_iters = []    # p-system CG iteration counts of the solves so far
        self._Adiag = None
        if self.kern.opt_kernel_params:
            self.dependent_attributes = np.unique(np.concatenate(
                (self.dependent_attributes, ['_Adiag'])))

    # ---- global sums over the data-row shards (identity without comm)
    def _sum(self, t):
        if self.comm is not None:
            self.comm.all_reduce(t)
        return t

    def _sum_scalar(self, v):
        if self.comm is None:
            return float(v)
        t = dev.torch().tensor([float(v)], dtype=dev.torch().float64, device=dev.device())
        self.comm.all_reduce(t)
        return float(t.item())

    def _y_dev(self):
        if self._Yd is None:
            self._Yd = dev.to_device(self.Y[:, 0])
        return self._Yd

    def _x_dev(self):
        """The training inputs on the device, uploaded once per content of X:
        Phi is rebuilt at every new kernel parameter (optimize), and the copy
        is reused while X (same array, same bytes -- an in-place edit changes
        the key) is unchanged."""
        key = _content_key(self.X)
        if self._Xd is None or self._Xd_src != key:
            self._Xd = dev.to_device(self.X)
            self._Xd_src = key
        return self._Xd

    def fit(self, **kwargs):
        self.parameters
        if self._alpha is not None:
            return
        if self.p_solver == 'chol':
            self._cov_setup()
        else:
            self._phi_setup()
        self._alpha = self._mv_cov_inv_dev(self._y_dev())

    def predict_precompute(self, Xnew):
        assert Xnew.ndim == 2
        assert Xnew.shape[1] == self.input_dim
        self.parameters
        if self._alpha is None:
            self.fit()
        if self._alpha_p is None:
            t = self._sum(dense.matvec(self._Phi, self._alpha, trans=True))
            self._alpha_p = dense.scale_rows(t, dev.to_device(self.kern.w), 0)

    def predict(self, Xnew):
        """(Yhat (M,1), Yhatvar (M,M)) with Var = s Phi* P^-1 Phi*^T + s I (:99-125)."""
        self.predict_precompute(Xnew)
        if self._Phi_last_pred is None or not np.array_equal(Xnew, self._X_last_pred):
            self._Phi_last_pred = self.kern.phi_device(Xnew, transposed=True)  # p x M
            self._X_last_pred = Xnew
        PhiT = self._Phi_last_pred
        yhat = dense.matvec(PhiT, self._alpha_p, trans=True)
        self._cov_setup()
        V = self._Pchol.solve(PhiT, which=1)                  # L^-1 Phi*^T  (p x M)
        var = dense.matmul(V, V, ta=True, alpha=float(self.noise_var))
        var = dense.add_diag(var, float(self.noise_var))
        return dense.host(yhat).reshape((-1, 1)), dense.host(var)

    def d_Yhat_d_x(self, Xnew, dim):
        """d Yhat / d Xnew[:, dim] (gp_grief_model.py:127-134): dPhi* alpha_p,
        dPhi* from GriefKernel.cov_grad on the fit's basis; a host array as
        the reference's dot product, (M, 1)."""
        self.predict_precompute(Xnew)
        dPhi = self.kern.cov_grad(Xnew, dim)
        return dPhi.dot(dense.host(self._alpha_p).reshape(-1, 1))

    def _phi_setup(self):
        self._w = self.kern.w
        if self._Phi is None:
            self._Phi = self.kern.phi_device(self._x_dev())   # n x p

    def _cov_setup(self):
        if self._P is not None:
            return
        self._w = self.kern.w
        if self._A is None:
            if self._Phi is None:
                self._Phi = self.kern.phi_device(self._x_dev())  # n x p
            self._A = self._gram()
        wd = dev.to_device(np.asarray(self._w, dtype=np.float64))
        self._P = dense.add_diag(self._A, float(self.noise_var), wd)
        self._Pchol = dense.Cholesky(self._P)

    def _gram(self):
        """A = Phi^T Phi (:148), summed over the data-row shards, in its lower
        triangle only: half the MFMA work of the full GEMM, and potrf and the
        adjoint gradient read nothing above the diagonal (the upper stays 0)."""
        t = dev.torch()
        p = int(self._Phi.shape[1])
        A = t.zeros((p, p), dtype=t.float64, device=self._Phi.device)
        return self._sum(dense.matmul(self._Phi, self._Phi, ta=True, C=A, uplo=self._gram_uplo))

    def _finite_diff_gradient(self, parameters):
        """Forward differences (basemodel.py:328-361).  With opt_kernel_params
        every perturbed base-kernel parameter needs its own eigen-basis: those
        eigendecompositions are batched into one device launch up front
        (GriefKernel.prefetch_eigs); the LMLs then run as in the reference."""
        if self.kern.opt_kernel_params:
            free_inds = np.nonzero(np.logical_not(self._fixed_indicies))[0]
            sets = [np.asarray(parameters[1:], dtype=np.float64)]
            for idx in free_inds:
                if idx == 0:
                    continue                       # the noise leaves the basis unchanged
                p_fs = np.array(parameters, dtype=np.float64)
                p_fs[idx] += 1e-6
                sets.append(p_fs[1:])
            self.kern.prefetch_eigs(sets)
        return super(GPGriefModel, self)._finite_diff_gradient(parameters)

    def _adjoint_gradient(self, parameters):
        """dL/dw and dL/dsigma^2 (:156-200) via diag(P^-1): with P = A + D,
        sum_i A_ij (P^-1 A)_ij = A_jj - d_j + d_j^2 (P^-1)_jj and
        tr(P^-1 A) = p - sum_j d_j (P^-1)_jj  (exact algebra, one triangular
        inverse instead of the reference's p x p cho_solve)."""
        assert isinstance(parameters, np.ndarray)
        free_inds = np.nonzero(np.logical_not(self._fixed_indicies))[0]
        gradient = np.zeros(parameters.shape) + np.nan
        log_like = self._compute_log_likelihood(parameters)
        s = float(self.noise_var)
        w = np.asarray(self._w, dtype=np.float64)
        dvec = s / w
        pinv_diag = None
        if self.kern.reweight_eig_funs or self.noise_var_constraint != 'fixed':
            pinv_diag = dense.host(self._Pchol.inverse_diag())
        if self.kern.reweight_eig_funs:
            phia = dense.host(self._sum(dense.matvec(self._Phi, self._alpha, trans=True)))
            data_fit_grad = 0.5 * phia ** 2
            complexity_grad = -0.5 * dvec * (1.0 - dvec * pinv_diag) / s
            gradient[-self.kern.n_eigs:] = data_fit_grad + complexity_grad
        if self.noise_var_constraint != 'fixed':
            data_fit = 0.5 * self._sum_scalar(dense.dot(self._alpha, self._alpha))
            tr = float(self.kern.n_eigs) - float(np.sum(dvec * pinv_diag))
            gradient[0] = data_fit - 0.5 * (float(self.num_data) - tr) / s
        if self.kern.opt_kernel_params:
            raise NotImplementedError("adjoint method not implemented for"
                                      "kernel parameter optimiszation, just weights")
        assert not np.any(np.isnan(gradient[free_inds])), "gradient missed!"
        return log_like, gradient

    def _compute_log_likelihood(self, parameters):
        self.parameters = parameters
        # the log det needs chol(P) whatever the p-solver: a p_solver='cg'
        # model factors first and solves alpha with the same factor (fit()
        # then takes it) instead of running PCG beside it
        if self.p_solver == 'cg':
            self._phi_setup()
            ld = self._cov_log_det()
            self.fit()
        else:
            self.fit()
            ld = self._cov_log_det()
        yd = self._y_dev()
        ll = -0.5 * (self._sum_scalar(dense.dot(yd, self._alpha)) + ld
                     + self.num_data * np.log(np.pi * 2))
        return np.array([[ll]])

    def _mv_cov(self, x):
        """(Phi W Phi^T + s I) x (:217-225)."""
        assert x.shape[0] == self._n_local
        assert self._Phi is not None, "cov has not been setup"
        xd = _dev_2d(x)
        t = self._sum(dense.matmul(self._Phi, xd, ta=True))
        dense.scale_rows(t, dev.to_device(np.asarray(self._w, dtype=np.float64)), 0)
        out = xd.clone()
        dense.matmul(self._Phi, t, alpha=1.0, beta=float(self.noise_var), C=out)
        return dense.host(out).reshape(np.shape(x))

    # ---- the p-system by preconditioned CG (p_solver='cg')
    def _p_matvec(self, v, dvec):
        """P v = sum_g Phi_g^T (Phi_g v) + (s / w) v: two local GEMVs and one
        all-reduce of the p-vector."""
        u = self._sum(dense.matvec(self._Phi, dense.matvec(self._Phi, v), trans=True))
        dv = dense.scale_rows(v.clone(), dvec, 0)
        return dense.axpby(1.0, dv, 1.0, u)

    def _jacobi_diag(self, dvec):
        """diag(P) = column sums of squares of Phi (all ranks) + s / w."""
        if self._Adiag is None:
            sq = dense.scale_rows(self._Phi.clone(), None, 2)
            ones = dev.torch().ones(int(sq.shape[0]), dtype=sq.dtype, device=sq.device)
            self._Adiag = self._sum(dense.matvec(sq, ones, trans=True))
            del sq
        return dense.axpby(1.0, dvec, 1.0, self._Adiag.clone())

    def solve_p_cg(self, b, rtol=None, maxiter=None):
        """z = P^-1 b by Jacobi-preconditioned CG (b: device p-vector, the
        same on every rank).  Stops when ||b - P z|| <= rtol ||b||
        (recursive residual); every p-sized scalar and vector stays replicated,
        so the only communication is the operator's all-reduce."""
        rtol = self.cg_rtol if rtol is None else float(rtol)
        p = int(b.numel())
        maxiter = (self.cg_maxiter or 10 * p) if maxiter is None else int(maxiter)
        dvec = dev.to_device(float(self.noise_var) / np.asarray(self._w, dtype=np.float64))
        minv = self._jacobi_diag(dvec)
        x = dev.zeros(p)
        r = b.clone()
        bnorm = np.sqrt(dense.dot(b, b))
        if bnorm == 0.0:
            self.cg_iters.append(0)
            return x
        z = dense.scale_rows(r.clone(), minv, 1)
        d = z.clone()
        rz = dense.dot(r, z)
        it = 0
        while it < maxiter:
            q = self._p_matvec(d, dvec)
            alpha = rz / dense.dot(d, q)
            dense.axpby(alpha, d, 1.0, x)
            dense.axpby(-alpha, q, 1.0, r)
            it += 1
            if np.sqrt(dense.dot(r, r)) <= rtol * bnorm:
                break
            z = dense.scale_rows(r.clone(), minv, 1)
            rz_new = dense.dot(r, z)
            dense.axpby(1.0, z, rz_new / rz, d)
            rz = rz_new
        self.cg_iters.append(it)
        if it >= maxiter:
            res = np.sqrt(dense.dot(r, r)) / bnorm
            if not res <= rtol:
                logger.warning("p-system PCG stopped at maxiter=%d with relative residual "
                               "%.3g > rtol=%.3g" % (maxiter, res, rtol))
                self.cg_converged = False
                return x
        self.cg_converged = True
        return x

    def _mv_cov_inv_dev(self, xd):
        """(x - Phi P^-1 Phi^T x) / s for a 1-D device vector."""
        t = self._sum(dense.matvec(self._Phi, xd, trans=True))
        if self.p_solver == 'cg' and self._Pchol is None:
            # no factor for these parameters: PCG (fit / predictive mean only)
            t = self.solve_p_cg(t)
        else:
            t = self._Pchol.solve(t, which=3)
        out = xd.clone()
        dense.matvec(self._Phi, t, alpha=-1.0, beta=1.0, y=out)
        dense.axpby(0.0, out, 1.0 / float(self.noise_var), out)
        return out

    def _mv_cov_inv(self, x):
        """(x - Phi cho_solve(P, Phi^T x)) / s (:228-235)."""
        assert x.shape[0] == self._n_local
        assert self._Phi is not None, "cov has not been setup"
        self._cov_setup()
        xd = _dev_2d(x)
        t = self._sum(dense.matmul(self._Phi, xd, ta=True))
        t = self._Pchol.solve(t, which=3)
        out = xd.clone()
        dense.matmul(self._Phi, t, alpha=-1.0, beta=1.0, C=out)
        flat = out.reshape(-1)
        dense.axpby(0.0, flat, 1.0 / float(self.noise_var), flat)
        return dense.host(out).reshape(np.shape(x))

    def _cov_log_det(self):
        """2 sum log diag chol(P) + sum log w + (n - p) log s (:238-245)."""
        assert self._Phi is not None or self._P is not None, "cov has not been setup"
        self._cov_setup()
        return (self._Pchol.logdet + np.sum(np.log(self._w))
                + float(self.num_data - self.kern.n_eigs) * np.log(self.noise_var))


class GPGridModel(BaseModel):
    """Gaussian process with Y observed on every point of a full Kronecker grid
    (P1, the north star's grid model).  The reference has no such class; it
    is composed from the reference's own primitives exactly as SURVEY 8c
    prescribes: K = GridKernel.cov_grid(xg) (grid_kernel.py:56-115, input
    dimension 0 fastest), the shifted solve KronMatrix.solve_schur
    (kron_matrix.py:328-352) or CG, the log det from the Kronecker eigenvalues
    (kron_matrix.py:466-474 extended to the shift) or stochastic Lanczos,
    posterior mean K alpha and latent variance (Q o Q)-Kron (t s / (t + s)).

    solver: 'exact' (per-factor eigendecomposition, two device Kron matvecs
    and a decoded divide) or 'cg' (device CG, linalg.KronCG).  logdet: 'exact'
    (streamed over the grid on the device) or 'slq'.  Y (N,1) numpy or CUDA
    tensor; results come back in the same kind.  grad_method is finite
    differences over (noise, kernel parameters) like the reference's
    kernel-parameter path.
    """

    def __init__(self, xg, Y, kern, noise_var=1., solver='exact', logdet='exact',
                 dim_noise_var=1e-12, cg_rtol=1e-10, slq_probes=8, slq_steps=50, seed=0):
        super(GPGridModel, self).__init__()
        from .kern import GridKernel
        assert isinstance(kern, GridKernel)
        if solver not in ('exact', 'cg'):
            raise ValueError("solver must be 'exact' or 'cg'")
        if logdet not in ('exact', 'slq'):
            raise ValueError("logdet must be 'exact' or 'slq'")
        self.xg = xg
        self.kern = kern
        self.num_data = int(np.prod([np.shape(g)[0] for g in xg]))
        if tuple(Y.shape) != (self.num_data, 1):
            raise ValueError('Y must be (%d,1), the flattened grid' % self.num_data)
        self._y_is_dev = dev.is_device_array(Y)
        self._yd = dev.to_device(Y)
        self.noise_var = np.float64(noise_var)
        self.solver, self.logdet = solver, logdet
        self.dim_noise_var = float(dim_noise_var)
        self.cg_rtol = float(cg_rtol)
        self.slq = (int(slq_probes), int(slq_steps), int(seed))
        self.grad_method = 'finite_difference'
        self._K = self._QT = self._kern_key = None
        self.dependent_attributes = list(self.dependent_attributes)
        self._alpha = self._log_like = self._gradient = self._log_det = None

    # ---- operator, cached on the kernel parameters (like grief_kernel.py:171-173)
    def _operator(self):
        key = np.asarray(self.kern.parameters).copy()
        if self._K is None or not np.array_equal(key, self._kern_key):
            self._K = self.kern.cov_grid(self.xg, dim_noise_var=self.dim_noise_var)
            self._QT = None
            self._kern_key = key
        return self._K

    def _schur(self):
        K = self._operator()
        if self._QT is None:
            self._QT = K.schur()
        return self._QT

    def fit(self):
        self.parameters
        if self._alpha is not None:
            return
        s = float(self.noise_var)
        y = self._yd.reshape(-1, 1)
        if self.solver == 'exact':
            Q, T = self._schur()
            self._alpha = Q.solve_schur(T, y, shift=s).reshape(-1)
        else:
            from .linalg import cg
            x, info = cg(self._operator(), y, shift=s, rtol=self.cg_rtol)
            if info != 0:
                logger.info('CG did not converge in %d iterations' % info)
            self._alpha = x.reshape(-1)

    def _cov_log_det(self):
        if self._log_det is None:
            s = float(self.noise_var)
            if self.logdet == 'exact':
                Q, T = self._schur()
                self._log_det = T.diag().log_det_shifted(s)
            else:
                from .linalg import slq_logdet
                probes, steps, seed = self.slq
                self._log_det = slq_logdet(self._operator(), s, probes=probes, steps=steps,
                                           seed=seed)[0]
        return self._log_det

    def _compute_log_likelihood(self, parameters):
        self.parameters = parameters
        self.fit()
        ll = -0.5 * (dense.dot(self._yd, self._alpha) + self._cov_log_det()
                     + self.num_data * np.log(2 * np.pi))
        return np.array([[ll]])

    def _out(self, vd):
        return vd.reshape(-1, 1) if self._y_is_dev else dev.to_host(vd).reshape(-1, 1)

    def predict_grid(self, compute_var=True):
        """Posterior mean K alpha on the grid and the predictive variance
        diag(K - K (K + s I)^-1 K) + s (the latent variance from the
        eigenpairs, streamed on the device)."""
        from . import native
        from .tensors import KronMatrix
        self.fit()
        K = self._operator()
        mean = K.matvec_device(self._alpha)
        if not compute_var:
            return self._out(mean), None
        s = float(self.noise_var)
        Q, T = self._schur()
        lam = [np.asarray(e, dtype=np.float64).reshape(-1) for e in T.diag().K]
        lamd = dev.to_device(np.concatenate(lam))
        v = dev.empty(self.num_data)
        native.check(native.lib().gg_kron_diag_scale(
            len(lam), native.i64_array([l.size for l in lam]), native.dptr(lamd), s,
            native.GG_DIAG_POSTVAR, None, native.dptr(v), native.stream_ptr()),
            "gg_kron_diag_scale")
        Q2 = KronMatrix([np.asarray(q) ** 2 for q in Q.K])
        var = Q2.matvec_device(v)
        var += s
        return self._out(mean), self._out(var)

    def predict(self, Xnew, compute_var=True):
        """Posterior at off-grid points Xnew (M x d): mean K(X*, grid) alpha
        and the predictive variance k** - k*^T (K + s I)^-1 k* + s, both (M,1).

        K(X*, grid) is GridKernel.cov_kr's row-partitioned Khatri-Rao matrix
        (grid_kernel.py:148-179, khatri_rao_matrix.py:7-50), applied on the
        device (gg_kr_contract).  The quadratic form uses the per-factor
        eigenpairs K_f = Q_f T_f Q_f^T: Q^T k* = kron_f(Q_f^T k_f(x*)), so
        k*^T (K + s I)^-1 k* = sum_g c[g] prod_f V_f[j, g_f]^2 with
        V_f = K_f(X*, xg_f) Q_f (device GEMM) and c = 1 / (prod t + s) decoded
        on the device -- the same Khatri-Rao contraction as the mean."""
        from . import native
        assert Xnew.ndim == 2 and Xnew.shape[1] == len(self.xg)
        self.fit()
        Kxz = self.kern.cov_kr(np.asarray(Xnew, dtype=np.float64), self.xg)
        mean = Kxz.contract(self._alpha)
        if not compute_var:
            return dense.host(mean).reshape(-1, 1), None
        s = float(self.noise_var)
        Q, T = self._schur()
        V2 = []
        for Af, Qf in zip(Kxz.A, Q.K):
            V = dense.matmul(_dev_matrix(Af), _dev_matrix(np.asarray(Qf)))
            V2.append(dense.scale_rows(V.reshape(-1), None, 2).reshape(V.shape))
        lam = [np.asarray(e, dtype=np.float64).reshape(-1) for e in T.diag().K]
        lamd = dev.to_device(np.concatenate(lam))
        ones = dev.torch().ones(self.num_data, dtype=dev.torch().float64, device=lamd.device)
        c = dev.empty(self.num_data)
        native.check(native.lib().gg_kron_diag_scale(
            len(lam), native.i64_array([l.size for l in lam]), native.dptr(lamd), s,
            native.GG_DIAG_DIVIDE, native.dptr(ones), native.dptr(c), native.stream_ptr()),
            "gg_kron_diag_scale")
        del ones
        from .tensors import KhatriRaoMatrix
        quad = KhatriRaoMatrix(V2, partition=0).contract(c)
        kss = float(self.kern.diag_val)
        var = kss - dense.host(quad) + s
        return dense.host(mean).reshape(-1, 1), var.reshape(-1, 1)


def _content_key(a):
    """A cheap content key of a host array: identity, shape, dtype and a
    64-bit hash of its bytes (xxh3 when importable, else blake2b)."""
    a = np.ascontiguousarray(a)
    try:
        import xxhash
        h = xxhash.xxh3_64_intdigest(memoryview(a).cast("B"))
    except ImportError:  # pragma: no cover
        import hashlib
        h = hashlib.blake2b(memoryview(a).cast("B"), digest_size=8).hexdigest()
    return (a.shape, a.dtype.str, h)


def _dev_matrix(Phi):
    """Row-major float64 device copy of a 2-D basis matrix (or the tensor itself)."""
    t = dev.torch()
    if isinstance(Phi, t.Tensor):
        Pd = Phi.detach()
        if Pd.dtype != t.float64:
            Pd = Pd.to(t.float64)
        if not Pd.is_cuda:
            Pd = Pd.to(dev.device())
        return Pd.contiguous()
    arr = np.ascontiguousarray(np.asarray(Phi, dtype=np.float64))
    return t.from_numpy(arr).to(dev.device())


class GPwebModel(BaseModel):
    """GP with the weighted basis-function (WEB) kernel Phi W Phi^T + s I and
    O(p^3) algebra (gp_web_model.py:14-130).  The O(n p^2) Gram A = Phi^T Phi
    (lower triangle, FP64 MFMA), r = Phi^T y, the p x p Cholesky, the solves and
    the predictions run on the MI355X.

    The adjoint gradient avoids the reference's p x p cho_solve(P, A) with the
    exact identities of P = A + D, D = diag(s/w), z = P^-1 r:
      r - A z = D z,   colsum(A o P^-1 A)_j = A_jj - d_j + d_j^2 (P^-1)_jj,
      tr(P^-1 A) = p - sum_j d_j (P^-1)_jj,   z^T A z = r^T z - sum_j d_j z_j^2,
    so only diag(P^-1) (one triangular inverse, p^3/3) is needed; and the
    posterior weights (r - A z) w / s = z exactly.
    """

    def __init__(self, Phi, y, noise_var=1.):
        super(GPwebModel, self).__init__()
        self.n = y.shape[0]
        yd = dev.to_device(y)
        assert yd.numel() == self.n
        assert Phi.shape[0] == self.n
        self.p = int(Phi.shape[1])
        self._Phid = _dev_matrix(Phi)
        self._r = dense.matvec(self._Phid, yd, trans=True)               # Phi^T y
        self.yTy = np.array([[dense.dot(yd, yd)]])
        t = dev.torch()
        A = t.zeros((self.p, self.p), dtype=t.float64, device=self._Phid.device)
        self._A_lower = dense.matmul(self._Phid, self._Phid, ta=True, C=A, uplo=1)
        self.noise_var = np.float64(noise_var)
        from .kern import WEBKernel
        self.kern = WEBKernel(initial_weights=np.ones(self.p))
        self.grad_method = 'adjoint'
        self.dependent_attributes = np.unique(np.concatenate(
            (self.dependent_attributes, ['_P', '_Pchol', '_Pinv_r', '_alpha_p'])))

    @property
    def r(self):
        return dense.host(self._r).reshape((-1, 1))

    @property
    def A(self):
        """Phi^T Phi as a full symmetric host array (device keeps the lower triangle)."""
        L = dense.host(self._A_lower)
        return np.tril(L) + np.tril(L, -1).T

    def _compute_log_likelihood(self, parameters):
        self.parameters = parameters
        w = self.kern.parameters
        s = float(self.noise_var)
        if self._P is None:
            wd = dev.to_device(np.asarray(w, dtype=np.float64))
            self._P = dense.add_diag(self._A_lower, s, wd)
            self._Pchol = dense.Cholesky(self._P)
            self._Pinv_r = self._Pchol.solve(self._r, which=3)
        datafit = (float(self.yTy[0, 0]) - dense.dot(self._r, self._Pinv_r)) / s
        complexity = (self._Pchol.logdet + np.sum(np.log(w))
                      + float(self.n - self.p) * np.log(s))
        return np.array(-0.5 * (complexity + datafit + self.n * np.log(2. * np.pi)))

    def _adjoint_gradient(self, parameters):
        assert isinstance(parameters, np.ndarray)
        free_inds = np.nonzero(np.logical_not(self._fixed_indicies))[0]
        gradient = np.zeros(parameters.shape) + np.nan
        log_like = self._compute_log_likelihood(parameters)
        w = np.asarray(self.kern.parameters, dtype=np.float64)
        s = float(self.noise_var)
        dvec = s / w
        z = dense.host(self._Pinv_r)
        rz = dense.dot(self._r, self._Pinv_r)
        pinv_diag = dense.host(self._Pchol.inverse_diag())
        data_fit_grad = -(z / w) ** 2                            # -((r - A z)/s)^2
        complexity_grad = (dvec - dvec ** 2 * pinv_diag) / s
        gradient[1:] = -0.5 * data_fit_grad - 0.5 * complexity_grad
        data_fit_grad = -(float(self.yTy[0, 0]) - rz - np.sum(dvec * z ** 2)) / s ** 2
        complexity_grad = (float(self.n) - (float(self.p) - np.sum(dvec * pinv_diag))) / s
        gradient[0] = -0.5 * (data_fit_grad + complexity_grad)
        assert not np.any(np.isnan(gradient[free_inds])), "gradient missed!"
        return log_like, gradient

    def predict(self, Phi_new):
        """(Yhat (M,1), Var (M,M)) = Phi* alpha_p, s Phi* P^-1 Phi*^T + s I (:109-129)."""
        assert Phi_new.ndim == 2
        assert Phi_new.shape[1] == self.p
        parameters = self.parameters
        if self._alpha_p is None:
            if self._Pinv_r is None:
                self._compute_log_likelihood(parameters)
            self._alpha_p = self._Pinv_r                           # (r - A z) w / s = z
        Pn = _dev_matrix(Phi_new)
        yhat = dense.matvec(Pn, self._alpha_p)
        V = self._Pchol.solve(Pn.t().contiguous(), which=1)         # L^-1 Phi*^T (p x M)
        var = dense.matmul(V, V, ta=True, alpha=float(self.noise_var))
        var = dense.add_diag(var, float(self.noise_var))
        return dense.host(yhat).reshape((-1, 1)), dense.host(var)


def _gram_svd(Pd):
    """Right singular vectors / values of Phi from the device eigensolver on
    A = Phi^T Phi (descending); returns (sv, V, eigenvalues of A)."""
    A = dense.host(dense.matmul(Pd, Pd, ta=True))
    A = 0.5 * (A + A.T)
    from .tensors import device_sym_eig
    Qs, lams = device_sym_eig([A])
    lam, V = lams[0], Qs[0]
    order = np.argsort(-lam, kind='stable')
    lam, V = lam[order], V[:, order]
    return np.sqrt(np.maximum(lam, 0.0)), V, lam


def _cholqr3_svd(Pd, left=False):
    """Singular values (descending) and right singular vectors of the n x p
    device matrix Phi (n >= p) by shifted CholeskyQR3: A1 = Phi^T Phi + s I
    (s = 11 (n p + p (p + 1)) eps ||A||_F), Q1 = Phi L1^-T, then CholeskyQR2 on
    Q1 -- R = L3^T L2^T L1^T with Phi = Q3 R -- and the SVD of the p x p R on
    the host.  left=True also returns the left singular vectors Q3 U_R (n x p,
    host).  None when a Gram is not numerically positive definite beyond the
    shift's reach (rank deficiency): the caller falls back."""
    n, p = int(Pd.shape[0]), int(Pd.shape[1])
    none = (None, None, None) if left else (None, None)
    eps = np.finfo(np.float64).eps
    A = dense.matmul(Pd, Pd, ta=True)
    fro = float(np.sqrt(max(dense.dot(A.reshape(-1), A.reshape(-1)), 0.0)))
    if not fro > 0.0:
        return none
    shift = 11.0 * (n * p + p * (p + 1)) * eps * fro
    R = np.eye(p)
    Q = Pd
    try:
        for stage in range(3):
            if stage > 0:
                A = dense.matmul(Q, Q, ta=True)
            C = dense.Cholesky(dense.add_diag(A, shift) if stage == 0 else A)
            L = np.tril(dense.host(C.L))
            d = np.diag(L)
            # a near-singular Gram after the shifted first stage means a null
            # direction of Phi (its singular value is far below 1e-7)
            if stage > 0 and not np.min(d) ** 2 > 1e3 * eps * np.max(d) ** 2:
                return none
            R = L.T.dot(R)
            if stage < 2 or left:
                Q = dense.matmul(Q, C.inverse(), tb=True)   # Q L^-T
    except np.linalg.LinAlgError:
        return none
    UR, sv, VT = np.linalg.svd(R)
    if left:
        U = dense.host(dense.matmul(Q, dev.to_device(np.ascontiguousarray(UR)).reshape(p, p)))
        return sv, np.ascontiguousarray(VT.T), np.asarray(U).reshape(n, p)
    return sv, np.ascontiguousarray(VT.T)


def _thin_svd(Pd):
    """(singular values, right singular vectors) of the n x p device matrix
    Phi by shifted CholeskyQR3 at LAPACK accuracy: on Phi itself when n >= p,
    on Phi^T (p x n) when n < p -- Phi^T = Q3 R, R = U_R S W^T gives Phi =
    W S (Q3 U_R)^T, so the right singular vectors are Q3 U_R (p x n).
    (None, None) when the CholeskyQR3 test finds Phi numerically rank
    deficient."""
    n, p = int(Pd.shape[0]), int(Pd.shape[1])
    if n >= p:
        return _cholqr3_svd(Pd)
    sv, _, U = _cholqr3_svd(Pd.t().contiguous(), left=True)
    return sv, U


class GPwebTransformedModel(BaseModel):
    """WEB GP with the basis rotated to Phi's left singular vectors so that the
    likelihood and gradient are O(p) (gp_web_transformed_model.py:13-127).

    The thin SVD: Phi = Q R by shifted CholeskyQR3 on the MI355X (three Grams
    and two Q L^-T products on FP64 MFMA, three device Cholesky factors; Q is
    orthonormal to working precision for cond(Phi) up to ~1/eps), then the
    small p x p SVD R = U_R S V^T on the host (factor-sized, LAPACK), so S and
    V carry the accuracy of LAPACK's SVD of Phi; Phit^T y = S^-1 V^T (Phi^T y).
    Bases with singular value <= 1e-7 are dropped as in the reference
    (:27-35).  A wide Phi (n < p) takes the same route on Phi^T (its left
    singular vectors are Phi's right ones).  A numerically rank-deficient Phi
    falls back to the Gram spectrum A = V S^2 V^T with a floor at its rounding
    level, logged.
    The O(p) likelihood / gradient stay on the host, as in the reference;
    predictions are device GEMV / GEMM.
    """

    def __init__(self, Phi, y, noise_var=1.):
        super(GPwebTransformedModel, self).__init__()
        self.n = y.shape[0]
        yd = dev.to_device(y)
        assert yd.numel() == self.n
        assert Phi.shape[0] == self.n
        self.p_orig = int(Phi.shape[1])
        Pd = _dev_matrix(Phi)
        sv, V = _thin_svd(Pd)

        if sv is not None:
            ikeep = sv > 1e-7
        else:
            logger.warning("Phi is numerically rank deficient: its singular values come "
                           "from the Gram spectrum (accurate to ~sqrt(eps) s_max)")
            sv, V, lam = _gram_svd(Pd)
            # The reference keeps LAPACK singular values above 1e-7 (at most
            # min(n, p) of them).  Gram eigenvalues carry an absolute error of
            # ~eps * s_max^2, so null directions surface as ~sqrt(eps) * s_max
            # "singular values": drop eigenvalues under the Gram's own rounding
            # floor, and never keep more than min(n, p_orig) bases.
            floor = max(self.n, self.p_orig) * np.finfo(np.float64).eps * max(float(lam[0]), 0.0)
            ikeep = (sv > 1e-7) & (lam > floor)
            dropped = int(np.sum((sv > 1e-7) & ~(lam > floor)))
            if dropped:
                logger.warning("%d Gram directions with apparent singular value > 1e-7 lie "
                               "under the Gram rounding floor and were dropped" % dropped)
        ikeep &= np.arange(sv.size) < min(self.n, self.p_orig)
        self.singular_vals = sv[ikeep]
        self.V = np.ascontiguousarray(V[:, ikeep])
        self.p = int(self.singular_vals.size)
        if self.p < self.p_orig:
            logger.info("Num Bases decreased from p=%d to p=%d. Only a subspace can now be "
                        "searched." % (self.p_orig, self.p))
        PhiTy = dense.host(dense.matvec(Pd, yd, trans=True))
        self.PhitT_y = self.V.T.dot(PhiTy) / self.singular_vals
        self.PhitT_y_2 = np.power(self.PhitT_y, 2)
        self.yTy = dense.dot(yd, yd)
        self.noise_var = np.float64(noise_var)
        from .kern import WEBKernel
        self.kern = WEBKernel(initial_weights=np.ones(self.p))
        self.grad_method = 'adjoint'

    def _compute_log_likelihood(self, parameters):
        self.parameters = parameters
        w = self.kern.parameters
        sig2 = self.noise_var
        Pdiag = sig2 / w + 1.
        datafit = (self.yTy - np.sum(self.PhitT_y_2 / Pdiag)) / sig2
        complexity = np.sum(np.log(Pdiag)) + np.sum(np.log(w)) + (self.n - self.p) * np.log(sig2)
        return -0.5 * (complexity + datafit + self.n * np.log(2. * np.pi))

    def _adjoint_gradient(self, parameters):
        assert isinstance(parameters, np.ndarray)
        free_inds = np.nonzero(np.logical_not(self._fixed_indicies))[0]
        gradient = np.zeros(parameters.shape) + np.nan
        log_like = self._compute_log_likelihood(parameters)
        w = self.kern.parameters
        sig2 = self.noise_var
        gradient[1:] = -0.5 * (-self.PhitT_y_2 / np.power(sig2 + w, 2) + 1. / (sig2 + w))
        data_fit_grad = (-self.yTy + np.sum(self.PhitT_y_2 * w * (sig2 * 2. + w)
                                            / np.power(sig2 + w, 2))) / sig2 ** 2
        complexity_grad = float(self.n - self.p) / sig2 + np.sum(1. / (sig2 + w))
        gradient[0] = -0.5 * (data_fit_grad + complexity_grad)
        assert not np.any(np.isnan(gradient[free_inds])), "gradient missed!"
        return log_like, gradient

    def predict(self, Phi_new):
        """Yhat = Phi* V (alpha_p / S); Var = s Phi* diag(1/Pdiag) Phi*^T + s I (:101-121)."""
        assert Phi_new.ndim == 2
        assert Phi_new.shape[1] == self.p_orig
        self.parameters
        w = self.kern.parameters
        sig2 = float(self.noise_var)
        Pdiag = sig2 / w + 1.
        alpha_p = (self.PhitT_y - self.PhitT_y / Pdiag) * w / sig2
        coef = dev.to_device(self.V.dot(alpha_p / self.singular_vals))
        Pn = _dev_matrix(Phi_new)
        yhat = dense.matvec(Pn, coef)
        if Pdiag.size != self.p_orig:
            raise ValueError("the predictive variance needs every basis kept (p == p_orig)")
        B = Pn.t().contiguous()
        dense.scale_rows(B, dev.to_device(Pdiag), 1)                  # Phi*^T / Pdiag
        var = dense.matmul(Pn, B, alpha=sig2)
        var = dense.add_diag(var, sig2)
        return dense.host(yhat).reshape((-1, 1)), dense.host(var)
