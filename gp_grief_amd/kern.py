"""Kernels: drop-in mirror of gp_grief.kern with device evaluation.

  BaseKernel           gp_grief/kern/basekernel.py:8-204   (parameters, constraints,
                                                           * / + composition, copy)
  RBF, Exponential,
  Matern32, Matern52   gp_grief/kern/stationary.py:79-258  (cov on the device, gg_cov)
  GridKernel           gp_grief/kern/grid_kernel.py:11-259 (cov_grid -> KronMatrix,
                                                           cov, cov_kr, parameters)
  GriefKernel          gp_grief/kern/grief_kernel.py:12-190 (device eigensolve of the
                                                           grid factors, top-p selection,
                                                           Phi built on the device)
  WEBKernel            gp_grief/kern/web_kernel.py:4-13     (weights of the WEB models)
  RBF_RFF              gp_grief/kern/rbf_rff.py:8-54        (random Fourier features)
  GPyKernel            gp_grief/kern/gpy_kernel.py:10-141   (only when GPy is importable)
Parameter / constraint bookkeeping is host logic identical in behaviour to the
reference (including the shared-kernel-object quirk of GridKernel's setter,
grid_kernel.py:233-239).  Every covariance evaluation and the eigenfunction
matrix Phi run on the MI355X.  GPy is not part of this stack (SURVEY 2, row
10): GPyKernel raises ImportError at construction unless GPy is importable.
"""
import ctypes
import logging
import os
from copy import deepcopy

import numpy as np

from . import device as dev
from . import native
from .grid import InducingGrid
from .tensors import (KronMatrix, KhatriRaoMatrix, SelectionMatrixSparse, centro_expand,
                      centro_halves_host, centro_merge, device_sym_eig, device_sym_eig_tridiag,
                      device_sym_eig_tridiag_vectors)

logger = logging.getLogger(__name__)


class BaseKernel(object):
    """Base of all kernels (basekernel.py:8-204)."""

    def __init__(self, n_dims, active_dims, name):
        self.n_dims = n_dims
        if active_dims is None:
            active_dims = np.arange(self.n_dims)
        else:
            active_dims = np.ravel(active_dims)
            assert 'int' in active_dims.dtype.type.__name__
            assert active_dims.min() >= 0
            assert active_dims.max() < self.n_dims
        self.active_dims = active_dims
        self.name = self.__class__.__name__ if name is None else name
        self.parameter_list = None
        self.constraint_map = None
        self._children = []

    def cov(self, x, z=None):
        x, z = self._process_cov_inputs(x, z)
        raise NotImplementedError('Not implemented')

    @property
    def parameters(self):
        if self.parameter_list is None:
            raise NotImplementedError('Need to specify kern.parameter_list')
        parts = [np.ravel(getattr(self, nm)) for nm in self.parameter_list]
        parts += [child.parameters for _, child in self._children]
        return np.concatenate(parts, axis=0) if parts else np.array([])

    @parameters.setter
    def parameters(self, value):
        assert isinstance(value, np.ndarray)
        assert value.ndim == 1
        i0 = 0
        for nm in self.parameter_list:
            old = getattr(self, nm)
            setattr(self, nm, value[i0:i0 + np.size(old)].reshape(np.shape(old)))
            i0 += np.size(old)
        for _, child in self._children:
            old = child.parameters
            child.parameters = value[i0:i0 + np.size(old)].reshape(np.shape(old))
            i0 += np.size(old)

    @property
    def constraints(self):
        if self.constraint_map is None:
            raise NotImplementedError('Need to specify kern.constraint_map')
        parts = [np.ravel(self.constraint_map[nm]) for nm in self.parameter_list]
        parts += [child.constraints for _, child in self._children]
        return np.concatenate(parts, axis=0) if parts else np.array([])

    def is_stationary(self):
        return isinstance(self, Stationary)

    def _process_cov_inputs(self, x, z):
        assert x.ndim == 2
        assert x.shape[1] == self.n_dims
        if z is None:
            z = x
        else:
            assert z.ndim == 2
            assert z.shape[1] == self.n_dims, "should be %d dims, not %d" % (self.n_dims,
                                                                             z.shape[1])
        return x, z

    def __mul__(k1, k2):
        assert isinstance(k2, BaseKernel)
        assert k2.n_dims == k1.n_dims
        parent, child = k1.copy(), k2.copy()
        if np.size(child.constraint_map['variance']) > 1:
            child.constraint_map['variance'][0] = 'fixed'
        else:
            child.constraint_map['variance'] = 'fixed'
        parent._children.append(('mul', child))
        return parent

    def __add__(k1, k2):
        assert isinstance(k2, BaseKernel), 'k2 must be a kernel'
        parent, child = k1.copy(), k2.copy()
        parent._children.append(('add', child))
        return parent

    def copy(self):
        c = deepcopy(self)
        c._children = [(deepcopy(op), ch.copy()) for op, ch in c._children]
        return c


def _stationary_host(kind, var, ls, d2):
    """k(r^2) on the host, the same formulas as the device kernels
    (gg_grief.hip stationary(); the reference's stationary.py:108-258)."""
    if kind == "RBF":
        if ls < 1e-6:
            return np.where(d2 == 0.0, var, 0.0)
        return var * np.exp(-0.5 * d2 / (ls * ls))
    r = np.sqrt(d2) / ls
    if kind == "Exponential":
        return var * np.exp(-r)
    if kind == "Matern32":
        s3 = 1.7320508075688772
        return var * (1.0 + s3 * r) * np.exp(-s3 * r)
    if kind == "Matern52":
        s5 = 2.23606797749979
        return var * (1.0 + s5 * r + (5.0 / 3) * r * r) * np.exp(-s5 * r)
    raise NotImplementedError(kind)


def _stationary_grad_host(kind, var, ls, diff):
    """d k(x, z) / d x for 1-D inputs, diff = x - z: the analytic gradients of
    _stationary_host (the reference takes them from GPy's gradients_X,
    grid_kernel.py:196-199; its native kernels have none)."""
    if kind == "RBF":
        if ls < 1e-6:
            return np.zeros_like(diff)
        return -diff / (ls * ls) * var * np.exp(-0.5 * diff * diff / (ls * ls))
    r = np.abs(diff) / ls
    if kind == "Exponential":
        return -var * np.exp(-r) * np.sign(diff) / ls
    if kind == "Matern32":
        s3 = 1.7320508075688772
        return -3.0 * var * np.exp(-s3 * r) * diff / (ls * ls)
    if kind == "Matern52":
        s5 = 2.23606797749979
        return -(5.0 / 3) * var * (1.0 + s5 * r) * np.exp(-s5 * r) * diff / (ls * ls)
    raise NotImplementedError(kind)


class Stationary(BaseKernel):
    """Stationary kernels evaluated on the device (stationary.py:9-76)."""
    _kind = None

    def cov_grad_x(self, x, z):
        """(N, M) matrix of d k(x_a, z_j) / d x_a for a 1-D kernel (host) --
        GPy's gradients_X(1, x, z_j) column by column in the reference."""
        if self._children or self.active_dims.size != 1:
            raise NotImplementedError("input gradients need a plain 1-D stationary kernel")
        x = np.asarray(x, dtype=np.float64).reshape(-1, self.n_dims)[:, self.active_dims]
        z = np.asarray(z, dtype=np.float64).reshape(-1, self.n_dims)[:, self.active_dims]
        return _stationary_grad_host(self._kind, float(np.asarray(self.variance).reshape(-1)[0]),
                                     float(np.asarray(self.lengthscale).reshape(-1)[0]),
                                     x[:, :1] - z[:, 0][None, :])

    def _device_cov(self, x, z, mode, out, lengthscale=None):
        """Evaluate into the device matrix `out` (N x M); mode 0/1/2 = set/mul/add."""
        x = np.asarray(x, dtype=np.float64)[:, self.active_dims] if not dev.is_device_array(x) \
            else x[:, self.active_dims.tolist()]
        z = np.asarray(z, dtype=np.float64)[:, self.active_dims] if not dev.is_device_array(z) \
            else z[:, self.active_dims.tolist()]
        ls = float(np.asarray(self.lengthscale).reshape(-1)[0])
        if lengthscale is not None:
            lsv = np.asarray(lengthscale, dtype=np.float64).reshape(-1)
            assert len(lsv) == self.active_dims.size
            x = x / lsv
            z = z / lsv
            ls = 1.0
        xd = dev.to_device(x)
        zd = dev.to_device(z)
        D = int(self.active_dims.size)
        native.check(native.lib().gg_cov(native.GG_KERN[self._kind],
                                         float(np.asarray(self.variance).reshape(-1)[0]), ls, D,
                                         native.dptr(xd), xd.numel() // D, native.dptr(zd),
                                         zd.numel() // D, int(mode), native.dptr(out),
                                         native.stream_ptr()), "gg_cov")

    def _cov_into(self, x, z, out, mode=0, lengthscale=None):
        self._device_cov(x, z, mode, out, lengthscale)
        for op, child in self._children:
            if not isinstance(child, Stationary):
                raise NotImplementedError("device composition needs stationary children")
            child._cov_into(x, z, out, mode=1 if op == 'mul' else 2)

    def cov(self, x, z=None, lengthscale=None):
        """Covariance matrix (N, M); numpy in, numpy out (CUDA tensors stay on device)."""
        on_dev = dev.is_device_array(x)
        x, z = self._process_cov_inputs(x, z)
        out = dev.empty(int(x.shape[0]) * int(z.shape[0]))
        if lengthscale is not None and self._kind != "RBF":
            raise TypeError("per-dimension lengthscales are an RBF option")
        self._cov_into(x, z, out, lengthscale=lengthscale)
        out = out.reshape(int(x.shape[0]), int(z.shape[0]))
        return out if on_dev else dev.to_host(out)


def _stationary_init(self, n_dims, variance, lengthscale, active_dims, name, check_size):
    Stationary.__init__(self, n_dims=n_dims, active_dims=active_dims, name=name)
    logger.debug('Initializing %s kernel.' % self.name)
    if check_size:
        assert np.size(variance) == 1
        assert np.size(lengthscale) == 1
    self.variance = np.float64(variance)
    self.lengthscale = np.float64(lengthscale)
    self.parameter_list = ['variance', 'lengthscale']
    self.constraint_map = {'variance': '+ve', 'lengthscale': '+ve'}


class RBF(Stationary):
    """Squared exponential (stationary.py:79-134)."""
    _kind = "RBF"

    def __init__(self, n_dims, variance=1., lengthscale=1., active_dims=None, name=None):
        _stationary_init(self, n_dims, variance, lengthscale, active_dims, name, True)


class Exponential(Stationary):
    """stationary.py:137-175."""
    _kind = "Exponential"

    def __init__(self, n_dims, variance=1., lengthscale=1., active_dims=None, name=None):
        _stationary_init(self, n_dims, variance, lengthscale, active_dims, name, False)


class Matern32(Stationary):
    """stationary.py:178-216."""
    _kind = "Matern32"

    def __init__(self, n_dims, variance=1., lengthscale=1., active_dims=None, name=None):
        _stationary_init(self, n_dims, variance, lengthscale, active_dims, name, False)


class Matern52(Stationary):
    """stationary.py:219-258."""
    _kind = "Matern52"

    def __init__(self, n_dims, variance=1., lengthscale=1., active_dims=None, name=None):
        _stationary_init(self, n_dims, variance, lengthscale, active_dims, name, False)


class GridKernel(object):
    """Product of 1-D kernels on a grid (grid_kernel.py:11-259)."""

    def __init__(self, kern_list, radial_kernel=False):
        self.kern_list = kern_list
        self.grid_dim = len(kern_list)
        assert isinstance(radial_kernel, bool)
        self.radial_kernel = radial_kernel
        if self.radial_kernel:
            for kern in self.kern_list:
                assert kern.n_dims == self.kern_list[0].n_dims, \
                    "number of grid dims must be equal for all slices"
            self.kern_list = [self.kern_list[0], ] * np.size(kern_list)
        else:
            for i in range(1, self.grid_dim):
                if hasattr(self.kern_list[i], 'fix_variance'):
                    self.kern_list[i].fix_variance()
                elif np.size(self.kern_list[i].constraint_map['variance']) > 1:
                    logger.info("Multiple variance parameters found in the kernel, "
                                "will only fix the first")
                    self.kern_list[i].constraint_map['variance'][0] = 'fixed'
                else:
                    self.kern_list[i].constraint_map['variance'] = 'fixed'
        self.n_dims = np.sum([kern.n_dims for kern in self.kern_list])

    def cov_grid(self, x, z=None, dim_noise_var=None, use_toeplitz=False):
        """Per-dimension covariances as a KronMatrix, input dims reversed (:56-115)."""
        assert dim_noise_var is not None, "dim_noise_var must be specified"
        if isinstance(use_toeplitz, bool):
            use_toeplitz = [use_toeplitz, ] * self.grid_dim
        else:
            assert np.size(use_toeplitz) == self.grid_dim
        if np.any(use_toeplitz):
            raise NotImplementedError("no kernel implements cov_toeplitz (reference neither)")
        assert len(x) == self.grid_dim
        cross = z is not None
        if not cross:
            z = [None, ] * self.grid_dim
        else:
            assert len(z) == self.grid_dim
        K = [kern.cov(x=x[i], z=z[i]) for i, kern in enumerate(self.kern_list)]
        K = KronMatrix(K[::-1], sym=(z[0] is None))
        if dim_noise_var != 0.:
            assert not cross, "not implemented for cross covariances yet"
            K = K.sub_shift(shift=dim_noise_var)
        return K

    def cov(self, x, z=None, dim_noise_var=None):
        """Dense Hadamard product over dimensions (:118-145), on the device."""
        assert dim_noise_var is None, "currenly no way to add dim_noise_var"
        on_dev = dev.is_device_array(x)
        zz = x if z is None else z
        out = dev.empty(int(x.shape[0]) * int(zz.shape[0]))
        i_cur = 0
        for i, kern in enumerate(self.kern_list):
            sl = slice(i_cur, i_cur + kern.n_dims)
            i_cur += kern.n_dims
            xi = x[:, sl]
            zi = zz[:, sl]
            if not isinstance(kern, Stationary):
                raise NotImplementedError("device GridKernel.cov needs stationary kernels")
            kern._cov_into(xi, zi, out, mode=0 if i == 0 else 1)
        out = out.reshape(int(x.shape[0]), int(zz.shape[0]))
        return out if on_dev else dev.to_host(out)

    def cov_kr(self, x, z, dim_noise_var=None, form_kr=True):
        """Row-partitioned Khatri-Rao cross covariance (:148-179), factors reversed."""
        assert dim_noise_var is None, "currenly no way to add dim_noise_var"
        (N, d) = x.shape
        assert self.grid_dim == d, "currently only works for 1-dimensional grids"
        Kxz = [kern.cov(x=x[:, (i,)], z=z[i]) for i, kern in enumerate(self.kern_list)]
        Kxz = Kxz[::-1]
        if form_kr:
            Kxz = KhatriRaoMatrix(A=Kxz, partition=0)   # row partitioned
        return Kxz

    def cov_kr_grad(self, x, z, grad_dim):
        """Gradient of cov_kr w.r.t. x[:, grad_dim] (grid_kernel.py:181-209):
        the grad_dim factor replaced by d k / d x (analytic for the stationary
        kernels; the reference needs GPy kernels here), factors reversed."""
        (N, d) = x.shape
        assert self.grid_dim == d
        Kxz = []
        for i, kern in enumerate(self.kern_list):
            if i == grad_dim:
                Kxz.append(kern.cov_grad_x(x[:, (i,)], np.asarray(z[i])))
            else:
                Kxz.append(kern.cov(x=x[:, (i,)], z=z[i]))
        return Kxz[::-1]

    @property
    def parameters(self):
        if self.radial_kernel:
            return np.ravel(self.kern_list[0].parameters)
        return np.concatenate([np.ravel(k.parameters) for k in self.kern_list], axis=0)

    @parameters.setter
    def parameters(self, value):
        assert isinstance(value, np.ndarray)
        assert value.ndim == 1
        if self.radial_kernel:
            self.kern_list[0].parameters = value
            self.kern_list = [self.kern_list[0], ] * np.size(self.kern_list)
        else:
            i0 = 0
            for kern in self.kern_list:
                old = kern.parameters
                kern.parameters = value[i0:i0 + np.size(old)].reshape(np.shape(old))
                i0 += np.size(old)

    @property
    def constraints(self):
        if self.radial_kernel:
            return np.ravel(self.kern_list[0].constraints)
        return np.concatenate([np.ravel(k.constraints) for k in self.kern_list], axis=0)

    @property
    def diag_val(self):
        return self.cov(np.zeros((1, self.n_dims))).squeeze()


class GriefKernel(GridKernel):
    """GRId-structured EIgenFunctions kernel (grief_kernel.py:12-190).

    cov(x) returns (Phi, w, Phi) with Phi = (n x p) numpy; the models keep Phi
    on the device through phi_device().
    """

    def __init__(self, kern_list, grid, n_eigs=1000, reweight_eig_funs=True,
                 opt_kernel_params=False, w=1., dim_noise_var=1e-12, log_KRrowcol=True,
                 **kwargs):
        self.reweight_eig_funs = bool(reweight_eig_funs)
        self.opt_kernel_params = bool(opt_kernel_params)
        super(GriefKernel, self).__init__(kern_list=kern_list, **kwargs)
        assert isinstance(grid, InducingGrid), "must be an InducingGrid"
        assert grid.input_dim == self.n_dims, "number of dimensions do not match"
        self.grid = grid
        self.dim_noise_var = float(dim_noise_var)
        self.n_eigs = int(min(n_eigs, self.grid.num_data))
        if not self.opt_kernel_params:
            for i, kern in enumerate(self.kern_list):
                for key in kern.constraint_map:
                    self.kern_list[i].constraint_map[key] = \
                        np.tile('fixed', np.shape(kern.constraint_map[key]))
        label = '+ve' if self.reweight_eig_funs else 'fixed'
        self.w_constraints = np.array([label, ] * self.n_eigs, dtype='|S10')
        if np.isscalar(w) and w == 1.:
            self.w = np.ones(self.n_eigs)
        else:
            w = np.asarray(w, dtype=np.float64)
            assert w.shape == (self.n_eigs,)
            assert np.all(w > 0.), "w's must be positive"
            self.w = w
        self._old_base_kern_params = None
        self.log_KRrowcol = log_KRrowcol
        self._dev_basis = None
        self._eig_cache = {}   # base-kernel parameters -> per-factor (Q, lambda)

    # ------------------------------------------------------------------ Phi
    def cov(self, x, z=None):
        assert x.shape[1] == self.n_dims
        if z is not None:
            Phi_L = self.cov(x=x)[0]
            Phi_R = self.cov(x=z)[0]
            return Phi_L, self.w, Phi_R
        Phi = dev.to_host(self.phi_device(x))
        return Phi, self.w, Phi

    def phi_device(self, x, transposed=False):
        """Phi (n x p) row-major -- or Phi^T (p x n) -- as a CUDA tensor."""
        self._setup_inducing_cov()
        B = self._dev_basis
        xd = dev.to_device(x)
        n = xd.numel() // self.grid_dim
        d = self.grid_dim
        L = native.lib()
        # the value table X (gg_grief_tables_all with stab NULL): one double per
        # entry, where the log / sign pair of the reference's expand_SKC costs
        # two -- Phi takes the product of the values, the same numbers up to
        # rounding (GG_GRIEF_LOGTAB=1: the log / sign tables, A/B)
        ltab = dev.empty(max(n * B["U"], 1))
        stab = dev.empty(max(n * B["U"], 1)) if os.environ.get("GG_GRIEF_LOGTAB") == "1" \
            else None
        # every dimension's table in one launch (factor f reads input dim d-1-f);
        # the host argument arrays are built once per basis
        a = B.get("tab_args")
        if a is None:
            a = self._table_args()
            B["tab_args"] = a
        native.check(L.gg_grief_tables_all(d, a["kinds"], a["var"], a["ls"], native.dptr(xd), d,
                                           a["xoff"], n, a["xgp"], a["ms"], a["qsp"], a["us"],
                                           native.dptr(ltab),
                                           native.dptr(stab) if stab is not None else None,
                                           B["U"], a["c0"],
                                           native.stream_ptr()), "gg_grief_tables_all")
        p = self.n_eigs
        phi = dev.empty(n * p)
        native.check(L.gg_grief_phi(native.dptr(ltab),
                                    native.dptr(stab) if stab is not None else None, B["U"], n,
                                    native.dptr(B["cidx"]), d, native.dptr(B["log_lam"]), p,
                                    int(bool(transposed)), native.dptr(phi),
                                    native.stream_ptr()), "gg_grief_phi")
        return phi.reshape(p, n) if transposed else phi.reshape(n, p)

    def _table_args(self):
        """ctypes arrays of gg_grief_tables_all for the current basis."""
        B = self._dev_basis
        d = self.grid_dim
        a = dict(kinds=(ctypes.c_int * d)(), var=(ctypes.c_double * d)(),
                 ls=(ctypes.c_double * d)(), xoff=(ctypes.c_int64 * d)(),
                 xgp=(ctypes.c_void_p * d)(), qsp=(ctypes.c_void_p * d)(),
                 ms=(ctypes.c_int * d)(*[int(v) for v in B["m"]]),
                 us=(ctypes.c_int * d)(*[int(v) for v in B["u"]]),
                 c0=(ctypes.c_int * d)(*[int(v) for v in B["col0"]]))
        for f in range(d):
            i = d - 1 - f
            kern = self.kern_list[i]
            if not isinstance(kern, Stationary) or kern._children:
                raise NotImplementedError("GRIEF device basis needs plain stationary kernels")
            a["kinds"][f] = native.GG_KERN[kern._kind]
            a["var"][f] = float(np.asarray(kern.variance).reshape(-1)[0])
            a["ls"][f] = float(np.asarray(kern.lengthscale).reshape(-1)[0])
            a["xoff"][f] = i
            a["xgp"][f] = native.dptr(B["xg"][f])
            a["qsp"][f] = native.dptr(B["qsel"][f])
        return a

    def cov_grad(self, x, grad_dim):
        """d Phi_L / d x[:, grad_dim] (grief_kernel.py:113-126), n x p (host),
        on the SAME selected eigenvectors as Phi (the device basis: qsel,
        cidx, log_lam), so it pairs with the fit's alpha.  Per factor f the
        selected rows X_f = Qsel_f K_ux,f (d k / d x for the input dimension
        grad_dim), Phi_jk = prod_f X_f[c_jf] exp(-log_lam_j / 2)."""
        self._setup_inducing_cov()
        B = self._dev_basis
        x = np.asarray(x, dtype=np.float64)
        n, d = x.shape
        assert d == self.grid_dim
        rows = []
        for f in range(d):
            i = d - 1 - f                      # factor f = input dimension d - 1 - f
            kern = self.kern_list[i]
            xg = np.asarray(self.grid.xg[i], dtype=np.float64).reshape(-1, 1)
            if i == grad_dim:
                Kux = kern.cov_grad_x(x[:, (i,)], xg).T
            else:
                Kux = np.asarray(kern.cov(x=x[:, (i,)], z=xg)).T
            rows.append(dev.to_host(B["qsel"][f]).reshape(int(B["u"][f]), -1).dot(Kux))
        X = np.concatenate(rows, axis=0)       # U x n, factor f's rows from col0_f
        cidx = dev.to_host(B["cidx"]).reshape(self.n_eigs, d)
        dPhi = np.exp(-0.5 * np.asarray(self._log_lam, dtype=np.float64)).reshape(-1, 1) * \
            np.prod(np.stack([X[cidx[:, f], :] for f in range(d)]), axis=0)
        return np.ascontiguousarray(dPhi.T)

    # ------------------------------------------------------------ parameters
    @property
    def parameters(self):
        return np.concatenate([super(GriefKernel, self).parameters, self.w], axis=0)

    @parameters.setter
    def parameters(self, value):
        n_theta = value.size - self.n_eigs
        GridKernel.parameters.fset(self, value[:n_theta])
        self.w = value[n_theta:]

    @property
    def constraints(self):
        return np.concatenate([super(GriefKernel, self).constraints, self.w_constraints],
                              axis=0)

    @property
    def diag_val(self):
        raise NotImplementedError('')

    # ------------------------------------------------- inducing eigen-basis
    def _setup_inducing_cov(self):
        """Factors, device eigendecomposition, top-p selection (:168-190).

        Cached on the base-kernel parameters like the reference.  Every factor
        eigenvalue enters the selection, but Phi needs only the eigenvectors of
        the selected indices: on a cache miss the factors are tridiagonalised,
        their eigenvalues found by bisection, and only the selected
        eigenvectors computed (inverse iteration + the reflectors) -- unless a
        selected eigenvalue is not separated from its neighbours (relative gap
        below _SUBSET_GAP), then the full QL decomposition is used.  With
        opt_kernel_params the finite-difference gradient compares LMLs of
        perturbed bases, which must all come from the same eigensolver (the
        batched prefetch is the full one): those kernels always take the full
        path.  GG_EIG_SUBSET=0 forces the full path.
        """
        base = super(GriefKernel, self).parameters
        if self._old_base_kern_params is not None and \
                np.array_equal(self._old_base_kern_params, base):
            return
        key = np.asarray(base, dtype=np.float64).tobytes()
        hit = self._eig_cache.get(key)
        qsel_dev = None
        qperm = None
        # optional stage marks (bench_grief.py: HIP events between the parts)
        mark = getattr(self, "_stage_mark", None) or (lambda name: None)
        if hit is None and not self.opt_kernel_params and \
                os.environ.get("GG_EIG_SUBSET", "1") != "0":
            factors = self._grid_factors_host()
            if factors is None:
                factors = self._grid_factors_device()
            mark("setup_factors")
            # centrosymmetric factors (evenly spaced grids): two half-order
            # problems each (tensors.centro_halves); GG_EIG_CENTRO=0 disables
            # (from m = 96: below it the halves' saving is under the extra
            # bookkeeping, profiles/r03/aa_centro_setup.jsonl)
            halves = None
            cmin = int(os.environ.get("GG_EIG_CENTRO_MIN", "96"))
            if os.environ.get("GG_EIG_CENTRO", "1") != "0" and \
                    not dev.is_device_array(factors[0]) and \
                    min(int(F.shape[0]) for F in factors) >= cmin:
                halves = [centro_halves_host(F) for F in factors]
                if any(hv is None for hv in halves):
                    halves = None
            split = halves is not None
            if split:
                lamh, handle = device_sym_eig_tridiag([M for hv in halves for M in hv])
                merged = [centro_merge(lamh[2 * f], lamh[2 * f + 1]) for f in range(len(factors))]
                lam = [mg[0] for mg in merged]
            else:
                lam, handle = device_sym_eig_tridiag(factors)
            mark("setup_eigvals")
            eig_pos, log_lam = self._select(lam)
            Sp = [SelectionMatrixSparse((col, lam[i].shape[0])) for i, col in enumerate(eig_pos.T)]
            mark("setup_select")
            if self._separated(lam, [S.unique for S in Sp]):
                if split:
                    qsel_dev, qperm = self._centro_vectors(handle, merged,
                                                           [S.unique for S in Sp])
                else:
                    qsel_dev = device_sym_eig_tridiag_vectors(handle, [S.unique for S in Sp])
                self._Quu_factors = factors
                self._Quu_full = None
                mark("setup_vectors")
        if qsel_dev is None:
            Q, lam = self._factor_eigs(base)
            eig_pos, log_lam = self._select(lam)
            Sp = [SelectionMatrixSparse((col, Q[i].shape[0])) for i, col in enumerate(eig_pos.T)]
            self._Quu_full = KronMatrix(Q)
        self._log_lam = log_lam
        self._Sp = Sp
        self._old_base_kern_params = base
        self._build_device_basis(qsel_dev, qperm)

    def _grid_factors_host(self):
        """The inducing-grid factors K_f + dim_noise_var I on the host, in
        KronMatrix order (input dims reversed, grid_kernel.py:56-115), for
        plain stationary kernels (the reference's own formulas,
        stationary.py:108-258; m x m, cheaper here than per-factor device
        launches and copies); None for composed kernels."""
        if not all(isinstance(k, Stationary) and not k._children for k in self.kern_list):
            return None
        host = []
        for i, kern in enumerate(self.kern_list):
            g = np.asarray(self.grid.xg[i], dtype=np.float64).reshape(-1)
            d2 = (g[:, None] - g[None, :]) ** 2
            Fi = _stationary_host(kern._kind, float(np.asarray(kern.variance).reshape(-1)[0]),
                                  float(np.asarray(kern.lengthscale).reshape(-1)[0]), d2)
            if self.dim_noise_var != 0.:
                Fi[np.diag_indices_from(Fi)] += float(self.dim_noise_var)
            host.append(Fi)
        return host[::-1]

    def _grid_factors_device(self):
        """The grid factors on the device (composed kernels: the device cov)."""
        t = dev.torch()
        F = []
        for i, kern in enumerate(self.kern_list):
            xg = np.asarray(self.grid.xg[i], dtype=np.float64)
            xd = t.from_numpy(np.ascontiguousarray(xg.reshape(xg.shape[0], -1))).to(dev.device())
            Fi = kern.cov(xd)
            if self.dim_noise_var != 0.:
                Fi = Fi + float(self.dim_noise_var) * t.eye(Fi.shape[0], dtype=t.float64,
                                                             device=dev.device())
            F.append(Fi)
        return F[::-1]

    @staticmethod
    def _centro_vectors(handle, merged, uniques):
        """Selected eigenvector rows of each factor from its halves' problems
        (tensors.centro_halves): inverse iteration on the half tridiagonals
        for the selected indices of each half, then [y; +-J y] / sqrt 2 in one
        launch (gg_centro_expand).  The rows come even-half first; returns them
        and, per factor, the row of each selected index (unique order)."""
        sel_h, hs, kes, kos, perms = [], [], [], [], []
        for f, (lamf, half, idx) in enumerate(merged):
            u = np.asarray(uniques[f], dtype=np.int64).reshape(-1)
            hr, ir = half[u], idx[u]
            se, so = np.sort(ir[hr == 0]), np.sort(ir[hr == 1])
            sel_h += [se, so]
            hs.append(lamf.size // 2)
            kes.append(se.size)
            kos.append(so.size)
            perms.append(np.where(hr == 0, np.searchsorted(se, ir),
                                  se.size + np.searchsorted(so, ir)).astype(np.int64))
        Vh = device_sym_eig_tridiag_vectors(handle, sel_h)
        return centro_expand(Vh, hs, kes, kos), perms

    # inverse iteration converges by eps ||T|| / gap per step and the Cholesky
    # QR restores orthogonality: a gap of 1e-10 ||T|| leaves each vector within
    # ~2e-6 of the true one -- the same bound any backward-stable solver (QL,
    # LAPACK) has at that gap
    _SUBSET_GAP = 1e-10

    def _select(self, lam):
        all_eig_vals = KronMatrix(lam)
        n_eigs = int(min(self.n_eigs, all_eig_vals.shape[0]))
        return all_eig_vals.find_extremum_eigs(n_eigs=n_eigs, mode='largest',
                                               log_expand=True)[:2]

    def _separated(self, lam, selections):
        """Every selected eigenvalue at least _SUBSET_GAP * max|lambda| away from
        its neighbours (inverse iteration then gives orthogonal vectors)."""
        for l, sel in zip(lam, selections):
            l = np.asarray(l)
            if l.size < 2:
                continue
            tol = self._SUBSET_GAP * np.abs(l).max()
            gaps = np.diff(l)
            for k in np.asarray(sel).reshape(-1):
                if (k > 0 and gaps[k - 1] < tol) or (k < l.size - 1 and gaps[k] < tol):
                    return False
        return True

    @property
    def _Quu(self):
        """Per-factor eigenvectors (KronMatrix); after a subset setup the full
        decomposition is computed on first access."""
        if getattr(self, "_Quu_full", None) is None and getattr(self, "_Quu_factors", None):
            Q, _ = device_sym_eig([dev.to_host(F) if dev.is_device_array(F) else F
                                   for F in self._Quu_factors])
            self._Quu_full = KronMatrix(Q)
        return self._Quu_full

    _EIG_CACHE_MAX = 64

    def _factor_eigs(self, base):
        """Per-factor eigenpairs for the base-kernel parameters `base` (the
        state the kernel objects hold now), from the cache or the device."""
        key = np.asarray(base, dtype=np.float64).tobytes()
        hit = self._eig_cache.get(key)
        if hit is None:
            Kuu = self.cov_grid(self.grid.xg, dim_noise_var=self.dim_noise_var)
            hit = device_sym_eig([np.asarray(k) for k in Kuu.K])
            self._cache_put(key, hit)
        return hit

    def _cache_put(self, key, value):
        while len(self._eig_cache) >= self._EIG_CACHE_MAX:
            self._eig_cache.pop(next(iter(self._eig_cache)))
        self._eig_cache[key] = value

    def prefetch_eigs(self, parameter_sets):
        """Eigendecompose the grid factors of several kernel parameter vectors
        (GriefKernel.parameters layout) in ONE batched device launch and cache
        them, so the finite-difference gradient of opt_kernel_params
        (basemodel.py:328-361, one basis per perturbed parameter) pays one
        eigensolver latency instead of one per perturbation.  Each vector is
        applied through the parameters setter -- so the shared-kernel-object
        rule (grid_kernel.py:233-239) decides the effective factors exactly as
        in the sequential path -- and the kernel state is restored."""
        saved = self.parameters.copy()
        keys, mats, d = [], [], self.grid_dim
        try:
            for v in parameter_sets:
                self.parameters = np.asarray(v, dtype=np.float64).copy()
                key = np.asarray(super(GriefKernel, self).parameters,
                                 dtype=np.float64).tobytes()
                if key in self._eig_cache or key in keys:
                    continue
                Kuu = self.cov_grid(self.grid.xg, dim_noise_var=self.dim_noise_var)
                keys.append(key)
                mats.extend(np.asarray(k) for k in Kuu.K)
        finally:
            self.parameters = saved
        if not mats:
            return 0
        Q, lam = device_sym_eig(mats)
        for i, key in enumerate(keys):
            self._cache_put(key, (Q[i * d:(i + 1) * d], lam[i * d:(i + 1) * d]))
        return len(keys)

    def _build_device_basis(self, qsel_dev=None, qperm=None):
        """Device basis tables; qsel_dev (subset setup): the selected
        eigenvector rows Q_f^T[unique_f, :] already on the device, row
        qperm[f][r] holding unique index r when qperm is given."""
        d = self.grid_dim
        qsel, xg, us, ms, col0 = [], [], [], [], []
        cidx = np.zeros((self.n_eigs, d), dtype=np.int32)
        c = 0
        for f in range(d):
            i = d - 1 - f
            S = self._Sp[f]
            if qsel_dev is not None:
                qsel.append(qsel_dev[f].contiguous())
                ms.append(int(qsel_dev[f].shape[1]))
            else:
                Qf = np.asarray(self._Quu.K[f])
                qsel.append(dev.to_device(np.ascontiguousarray(Qf.T[S.unique, :])))
                ms.append(int(Qf.shape[0]))
            xg.append(dev.to_device(np.asarray(self.grid.xg[i], dtype=np.float64).reshape(-1)))
            us.append(int(S.unique.size))
            col0.append(c)
            inv = np.asarray(S.unique_inverse).reshape(-1)
            cidx[:, f] = c + (inv if qperm is None else qperm[f][inv])
            c += int(S.unique.size)
        t = dev.torch()
        self._dev_basis = dict(
            qsel=qsel, xg=xg, u=us, m=ms, col0=col0, U=c,
            cidx=t.from_numpy(cidx.reshape(-1)).to(dev.device()),
            log_lam=dev.to_device(self._log_lam))


class WEBKernel(object):
    """Weighted basis-function kernel parametrisation (web_kernel.py:4-13): the
    p weights are the parameters, each constrained '+ve'."""

    def __init__(self, initial_weights):
        assert isinstance(initial_weights, np.ndarray)
        assert np.ndim(initial_weights) == 1
        self.p = np.size(initial_weights)
        self.parameters = initial_weights
        self.constraints = ['+ve', ] * self.p


class GPyKernel(BaseKernel):
    """A GPy kernel behind the BaseKernel interface (gpy_kernel.py:10-141).

    GPy is not part of this stack (no network, not
    installed), so construction raises ImportError unless GPy is importable;
    then the covariance is GPy's own (host) and composes like the reference's.
    The in-house device kernels (RBF, Matern52, ...) cover every config."""

    def __init__(self, n_dims, kernel=None, name=None, **kwargs):
        try:
            import GPy  # noqa: F401
        except ImportError as exc:
            raise ImportError("GPyKernel needs GPy, which is not installed; use the "
                              "device kernels gp_grief.kern.RBF / Matern52 / ...") from exc
        import GPy
        if isinstance(kernel, str):
            name = "GPy - " + kernel if name is None else name
            BaseKernel.__init__(self, n_dims=n_dims, active_dims=None, name=name)
            self.kern = getattr(GPy.kern, kernel)(input_dim=n_dims, **kwargs)
        elif isinstance(kernel, GPy.kern.Kern):
            name = "GPy - " + repr(kernel) if name is None else name
            BaseKernel.__init__(self, n_dims=n_dims, active_dims=None, name=name)
            self.kern = kernel
        else:
            raise TypeError("must specify kernel as str or a GPy kernel object")
        self.constraint_list = [['+ve'] * np.size(p.values)
                                for p in self.kern.flattened_parameters]

    def cov(self, x, z=None):
        K = self.kern.K(x, z)
        for op, child in self._children:
            K = K * child.cov(x, z) if op == 'mul' else K + child.cov(x, z)
        return K

    @property
    def parameters(self):
        parts = [np.ravel(p.values) for p in self.kern.flattened_parameters]
        parts += [child.parameters for _, child in self._children]
        return np.concatenate(parts, axis=0) if parts else np.array([])

    @parameters.setter
    def parameters(self, value):
        assert isinstance(value, np.ndarray) and value.ndim == 1
        i0 = 0
        for p in self.kern.flattened_parameters:
            p[:] = value[i0:i0 + np.size(p)].reshape(np.shape(p))
            i0 += np.size(p)
        for _, child in self._children:
            old = child.parameters
            child.parameters = value[i0:i0 + np.size(old)].reshape(np.shape(old))
            i0 += np.size(old)

    @property
    def constraints(self):
        parts = [np.ravel(c) for c in self.constraint_list]
        parts += [child.constraints for _, child in self._children]
        return np.concatenate(parts, axis=0) if parts else np.array([])

    def fix_variance(self):
        i_var = np.where(['variance' in p._name.lower()
                          for p in self.kern.flattened_parameters])[0]
        if np.size(i_var) == 0:
            raise RuntimeError("No variance parameter found")
        self.constraint_list[i_var[0]][0] = 'fixed'


class RBF_RFF(object):
    """Random Fourier features of an ARD RBF kernel (rbf_rff.py:8-54):
    Phi(x) = [cos(x W / ell), sin(x W / ell)] / sqrt(n_rffs), W ~ N(0, 1)^(d x
    n_rffs) drawn from numpy's global generator as the reference does.  The
    (n x d)(d x n_rffs) product runs on FP64 MFMA; cos / sin on the device."""

    def __init__(self, d, log_lengthscale=0, n_rffs=1000, dtype=np.float64, tune_len=True):
        logger.info("initializing RBF kernel")
        self.d = int(d)
        self.n_rffs = int(n_rffs)
        self.n_features = 2 * n_rffs
        self.dtype = dtype
        self.freq_weights = np.asarray(np.random.normal(size=(self.d, self.n_rffs), loc=0,
                                                        scale=1.), dtype=self.dtype)
        self.bf_scale = 1. / np.sqrt(self.n_rffs)
        if np.size(log_lengthscale) == 1 and log_lengthscale == 0:
            log_lengthscale = np.zeros((d, 1), dtype=self.dtype)
        else:
            log_lengthscale = np.asarray(log_lengthscale, dtype=self.dtype).reshape((d, 1))
        self.log_ell = log_lengthscale

    def Phi(self, x):
        """(n, 2 n_rffs) basis matrix at the inputs x (n, d)."""
        from . import dense
        t = dev.torch()
        on_dev = dev.is_device_array(x)
        xd = dev.to_device(x).reshape(-1, self.d)
        W = dev.to_device(self.freq_weights / np.exp(self.log_ell)).reshape(self.d, self.n_rffs)
        F = dense.matmul(xd, W)
        out = t.cat([t.cos(F), t.sin(F)], dim=1).mul_(self.bf_scale)
        return out if on_dev else dev.to_host(out)
