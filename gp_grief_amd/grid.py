"""Inducing grids (gp_grief/grid.py): host metadata only, O(d * m) numbers.

InducingGrid mirrors grid.py:48-165 (constructor semantics, attributes xg,
grid_dim, grid_shape, grid_sub_dim, input_dim, num_data as float, eq).
nd_grid / grid2mat mirror grid.py:8-45 (C order, last dimension fastest).
"""
import logging

import numpy as np

logger = logging.getLogger(__name__)


def nd_grid(*xg):
    grid_shape = [np.shape(g)[0] for g in xg]
    d = len(grid_shape)
    mesh = np.empty(d, dtype=object)
    for i, g in enumerate(xg):
        if np.ndim(g) > 1:
            assert np.shape(g)[1] == 1, "currently supports 1d grid dims"
        slice_shape = np.ones(d, dtype=int)
        slice_shape[i] = np.shape(g)[0]
        reps = np.array(grid_shape)
        reps[i] = 1
        mesh[i] = np.tile(np.asarray(g).reshape(slice_shape), reps)
    return mesh


def grid2mat(*xg):
    mesh = nd_grid(*xg)
    x = np.zeros((mesh[0].size, mesh.shape[0]))
    for i, X1d in enumerate(mesh):
        x[:, i] = X1d.reshape(-1, order='C')
    return x


class InducingGrid(object):
    """Inducing point grid from scattered data (mbar points per dim) or from xg."""

    def __init__(self, x=None, mbar=10, eq=True, mbar_min=1, xg=None, beyond_domain=None):
        k, k_min = mbar, mbar_min
        if xg is None:
            assert isinstance(x, np.ndarray)
            assert x.ndim == 2
            self.eq = eq
            if not isinstance(k, (tuple, list, np.ndarray)):
                k = (k,) * x.shape[1]
            n_train, self.grid_dim = x.shape
            self.grid_sub_dim = np.ones(self.grid_dim, dtype=int)
            self.input_dim = np.sum(self.grid_sub_dim)
            self.grid_shape = np.zeros(self.grid_dim, dtype=int)
            lo, hi = np.amin(x, axis=0), np.amax(x, axis=0)
            span = np.ptp(x, axis=0)
            n_unq = np.array([np.unique(x[:, i]).size for i in range(self.grid_dim)])
            if not np.all(n_unq >= 2):
                logger.debug('some dimension have < 2 unique points')
            for i, ki in enumerate(k):
                if ki <= 1:
                    self.grid_shape[i] = np.int32(np.maximum(np.ceil(ki * n_unq[i]), k_min))
                else:
                    assert np.mod(ki, 1) == 0, "if k > 1 then k must be integer"
                    self.grid_shape[i] = np.int32(np.maximum(np.minimum(ki, n_unq[i]), k_min))
            self.num_data = np.prod(np.float64(self.grid_shape))
            if beyond_domain is not None:
                assert np.all(self.grid_shape >= 2), "need >=2 points per dim"
                inner = InducingGrid(x=x, mbar=tuple(self.grid_shape - 2), eq=eq, mbar_min=0)
                xg = np.empty(self.grid_dim, dtype=object)
                for i in range(self.grid_dim):
                    xg[i] = np.vstack((lo[i] - beyond_domain * span[i], inner.xg[i],
                                       hi[i] + beyond_domain * span[i]))
            else:
                on_unique = self.grid_shape == n_unq
                self.xg = np.empty(self.grid_dim, dtype=object)
                for i in range(self.grid_dim):
                    if on_unique[i]:
                        self.xg[i] = np.unique(x[:, i]).reshape((-1, 1))
                    elif self.eq:
                        self.xg[i] = np.linspace(lo[i], hi[i],
                                                 num=self.grid_shape[i]).reshape((-1, 1))
                    elif self.grid_shape[i] == 2:
                        self.xg[i] = np.array([lo[i], hi[i]]).reshape((-1, 1))
                    else:
                        raise NotImplementedError
        if xg is not None:
            arr = np.empty(len(xg), dtype=object)
            for i, X in enumerate(xg):
                arr[i] = X
            self.xg = arr
            self.grid_dim = self.xg.shape[0]
            self.grid_shape = np.zeros(self.grid_dim, dtype=int)
            self.grid_sub_dim = np.zeros(self.grid_dim, dtype=int)
            for i, X in enumerate(self.xg):
                assert X.ndim == 2, "each element in xg must be a 2d array"
                self.grid_sub_dim[i] = X.shape[1]
                self.grid_shape[i] = X.shape[0]
            self.input_dim = np.sum(self.grid_sub_dim)
            self.num_data = np.prod(np.float64(self.grid_shape))
            self.eq = None

    def __getitem__(self, key):
        return self.xg[key]

    def __setitem__(self, key, value):
        self.xg[key] = value
