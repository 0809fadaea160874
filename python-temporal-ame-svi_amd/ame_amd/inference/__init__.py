"""Inference classes (reference import surface: src/inference/__init__.py:45-56)."""
from .base import BaseVariationalInference, BaseTemporalVariationalInference
from .structured_mf import TemporalAMEStructuredMFVI
from .naive_mf import TemporalAMENaiveMFVI

__all__ = ["BaseVariationalInference", "BaseTemporalVariationalInference",
           "TemporalAMEStructuredMFVI", "TemporalAMENaiveMFVI"]
