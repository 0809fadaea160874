"""Model containers for the VI hot path (reference: src/models/__init__.py:36-43)."""
from .temporal_ame import TemporalAMEModel

__all__ = ["TemporalAMEModel"]
