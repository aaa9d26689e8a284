"""gp_grief.linalg -> gp_grief_amd.linalg (reference: gp_grief/linalg.py)."""
from gp_grief_amd.linalg import *  # noqa: F401,F403
from gp_grief_amd.linalg import (solve_schur, solve_chol, solver_counter, log_kron, uniquetol,  # noqa: F401
                                 LogexpTransformation, cg, slq_logdet, KronCG)
