"""1-D stationary covariance functions -- CPU oracle (test infrastructure only).

Restates /root/reference/gp_grief/kern/stationary.py for one input dimension
(the only case GridKernel / GriefKernel use, grid_kernel.py:148-179):
  RBF        stationary.py:108-134
  Exponential stationary.py:161-175
  Matern32   stationary.py:202-216
  Matern52   stationary.py:243-258
"""
import numpy as np

_KINDS = ("RBF", "Exponential", "Matern32", "Matern52")


def cov_1d(kind, x, z, variance, lengthscale):
    """k(x_a, z_b) for column vectors x (N,) and z (M,) -> (N, M)."""
    if kind not in _KINDS:
        raise ValueError("unknown kernel %r" % (kind,))
    x = np.asarray(x, dtype=np.float64).reshape((-1, 1))
    z = np.asarray(z, dtype=np.float64).reshape((1, -1))
    d2 = (x - z) ** 2
    if kind == "RBF":
        if lengthscale < 1e-6:
            return variance * (d2 == 0)
        return variance * np.exp(-0.5 * d2 / lengthscale ** 2)
    if kind == "Matern52":
        r2 = d2 / lengthscale ** 2
        r = np.sqrt(r2)
        return variance * (1.0 + np.sqrt(5.0) * r + (5.0 / 3) * r2) * np.exp(-np.sqrt(5.0) * r)
    r = np.sqrt(d2) / lengthscale
    if kind == "Exponential":
        return variance * np.exp(-r)
    return variance * (1.0 + np.sqrt(3.0) * r) * np.exp(-np.sqrt(3.0) * r)
