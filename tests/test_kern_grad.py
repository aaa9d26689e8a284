"""Analytic input gradients of the 1-D stationary kernels (kern.py
_stationary_grad_host, used by GridKernel.cov_kr_grad / GriefKernel.cov_grad)
against central differences of the kernel values.  The reference takes these
from GPy (grid_kernel.py:196-199; GPy is not importable here): parity
unpinned, checked against the kernels' own formulas."""
import numpy as np
import pytest


@pytest.mark.parametrize("kind", ["RBF", "Exponential", "Matern32", "Matern52"])
def test_stationary_grad_matches_finite_differences(kind):
    from gp_grief_amd.kern import _stationary_grad_host, _stationary_host
    rng = np.random.default_rng(0)
    x = rng.random(200)
    z = rng.random(30)
    diff = x[:, None] - z[None, :]
    diff = np.where(np.abs(diff) < 1e-3, 1e-3, diff)   # Exponential: no kink at 0
    var, ls, h = 1.3, 0.17, 1e-6
    g = _stationary_grad_host(kind, var, ls, diff)
    fd = (_stationary_host(kind, var, ls, (diff + h) ** 2) -
          _stationary_host(kind, var, ls, (diff - h) ** 2)) / (2 * h)
    assert np.abs(g - fd).max() < 1e-7 * max(1.0, np.abs(fd).max())
