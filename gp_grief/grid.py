"""gp_grief.grid -> gp_grief_amd.grid (reference: gp_grief/grid.py)."""
from gp_grief_amd.grid import *  # noqa: F401,F403
from gp_grief_amd.grid import InducingGrid  # noqa: F401
