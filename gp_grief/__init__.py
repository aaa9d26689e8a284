"""gp_grief: the reference package's import path, served by gp_grief_amd.

`from gp_grief.models import GPGriefModel`, `from gp_grief.kern import
GriefKernel, RBF`, `from gp_grief.tensors import KronMatrix` and
`from gp_grief.tensors.kron_matrix import KronMatrix`-style imports resolve to
the MI355X implementation (gp_grief_amd), so caller code switches by putting
this tree on sys.path instead of the reference.  Mirrors the reference's
package layout and its import-time behaviour (gp_grief/__init__.py:1-34):
submodules imported eagerly, debug(), and root logging at INFO on stdout.
"""
import logging
import sys

from . import kern
from . import models
from . import tensors
from . import linalg
from . import grid

__version__ = '1.0+'


def debug():
    """Reset the root logger to DEBUG on stdout (gp_grief/__init__.py:9-22)."""
    for handler in logging.root.handlers[:]:
        logging.root.removeHandler(handler)
    logging.basicConfig(stream=sys.stdout, level=logging.DEBUG,
                        format='%(asctime)s %(name)s %(levelname)s: %(message)s',
                        datefmt='[ %H:%M:%S ]')


__all__ = [s for s in dir() if not s.startswith('_')]

logging.basicConfig(stream=sys.stdout, level=logging.INFO,
                    format='%(asctime)s %(name)s %(levelname)s: %(message)s',
                    datefmt='[ %H:%M:%S ]')
