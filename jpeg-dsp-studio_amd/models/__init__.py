"""Data models (drop-in for the reference's models/__init__.py:1-7)."""

from .compression_params import CompressionParams
from .compression_result import CompressionResult
from .intermediate_data import IntermediateData

__all__ = ['CompressionParams', 'CompressionResult', 'IntermediateData']
