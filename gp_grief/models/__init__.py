"""gp_grief.models -> gp_grief_amd.models (reference: gp_grief/models/__init__.py:2-6)."""
import sys as _sys

from gp_grief_amd.models import (BaseModel, GPRegressionModel, GPGriefModel,  # noqa: F401
                                 GPwebModel, GPwebTransformedModel, GPGridModel)
from .._alias import register as _register

_register(_sys.modules[__name__], {
    "basemodel": ["BaseModel"],
    "gpr_model": ["GPRegressionModel"],
    "gp_grief_model": ["GPGriefModel"],
    "gp_web_model": ["GPwebModel"],
    "gp_web_transformed_model": ["GPwebTransformedModel"],
})
