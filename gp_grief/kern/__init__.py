"""gp_grief.kern -> gp_grief_amd.kern (reference: gp_grief/kern/__init__.py:2-9)."""
import sys as _sys

from gp_grief_amd.kern import (BaseKernel, GPyKernel, Stationary, RBF, Exponential,  # noqa: F401
                               Matern32, Matern52, GridKernel, GriefKernel, WEBKernel, RBF_RFF)
from .._alias import register as _register

_register(_sys.modules[__name__], {
    "basekernel": ["BaseKernel"],
    "gpy_kernel": ["GPyKernel"],
    "stationary": ["Stationary", "RBF", "Exponential", "Matern32", "Matern52"],
    "grid_kernel": ["GridKernel"],
    "grief_kernel": ["GriefKernel"],
    "web_kernel": ["WEBKernel"],
    "rbf_rff": ["RBF_RFF"],
})
