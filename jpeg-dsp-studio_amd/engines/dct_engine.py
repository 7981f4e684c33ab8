"""DCT/IDCT operations with level shift (engines/dct_engine.py:1-27).

Orthonormal 8x8 DCT-II / DCT-III on the GPU (csrc/jds_dct8.hpp), bit-identical
to scipy.fft.dctn / idctn(type=2, norm='ortho').  Accepts one 8x8 block or a
stack (..., 8, 8) of blocks (each transformed independently)."""

import numpy as np

from jds import codec


def dct2(block: np.ndarray) -> np.ndarray:
    """2D DCT-II with orthonormal normalization."""
    return codec.stage_block(block, 0)


def idct2(coeffs: np.ndarray) -> np.ndarray:
    """2D inverse DCT (Type-III)."""
    return codec.stage_block(coeffs, 1)


def encode_block(block: np.ndarray) -> np.ndarray:
    """Level shift (-128) then DCT."""
    return codec.stage_block(block, 2)


def decode_block(coeffs: np.ndarray) -> np.ndarray:
    """IDCT then reverse level shift (+128), clip to [0,255]."""
    return codec.stage_block(coeffs, 3)
