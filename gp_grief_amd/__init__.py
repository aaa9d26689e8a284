"""gp_grief_amd: the gp_grief Kronecker / GRIEF GP hot path, native on MI355X.

Drop-in mirror of the reference package's API (scwolof/gp_grief):
    gp_grief_amd.tensors.KronMatrix, SelectionMatrixSparse
    gp_grief_amd.linalg  (log_kron, solver_counter, LogexpTransformation, + device cg / slq)
    gp_grief_amd.kern    (RBF, Exponential, Matern32, Matern52, GridKernel, GriefKernel)
    gp_grief_amd.grid    (InducingGrid)
    gp_grief_amd.models  (BaseModel, GPGriefModel, GPwebModel, GPwebTransformedModel, GPGridModel)
The arithmetic runs in libgpgrief.so (hand-written HIP for gfx950) through the
C ABI in include/gp_grief_amd.h; see DESIGN.md.
"""
import logging as _logging

from . import native
from . import linalg
from . import tensors

__version__ = "0.1.0"

_logging.getLogger(__name__).addHandler(_logging.NullHandler())


def __getattr__(name):
    # kern / grid / models import lazily (they pull in scipy.optimize)
    if name in ("kern", "grid", "models"):
        import importlib
        mod = importlib.import_module("." + name, __name__)
        globals()[name] = mod
        return mod
    raise AttributeError(name)
