"""ame_amd — MI355X (gfx950) implementation of the temporal-AME structured /
naive mean-field VI update loop (drop-in for Alfieriek/Python-Temporal-AME-SVI's
``TemporalAMEStructuredMFVI`` / ``TemporalAMENaiveMFVI``).

    from ame_amd.models import TemporalAMEModel
    from ame_amd.inference import TemporalAMEStructuredMFVI
"""
from .models import TemporalAMEModel
from .inference import (BaseTemporalVariationalInference, BaseVariationalInference,
                        TemporalAMENaiveMFVI, TemporalAMEStructuredMFVI)

__all__ = ["TemporalAMEModel", "TemporalAMEStructuredMFVI", "TemporalAMENaiveMFVI",
           "BaseVariationalInference", "BaseTemporalVariationalInference"]
__version__ = "0.1.0"
