"""Quantization operations (engines/quantizer.py:1-29)."""

import numpy as np

from jds import codec
from utils.constants import JPEG_LUMA_Q50  # noqa: F401  (re-exported like the reference)


def scale_quant_matrix(base_matrix: np.ndarray, quality: int) -> np.ndarray:
    """Scale quantization matrix by quality factor (1-100), IJG formula.

    Host-side table setup (64 entries), evaluated with the reference's NumPy
    expression so the GPU receives the identical doubles."""
    quality = np.clip(quality, 1, 100)
    if quality < 50:
        scale = 5000.0 / quality
    else:
        scale = 200.0 - 2.0 * quality
    q = np.floor((base_matrix * scale + 50.0) / 100.0)
    q = np.clip(q, 1, 255)
    return q.astype(np.float64)


def quantize(dct_coeffs: np.ndarray, Q_matrix: np.ndarray) -> np.ndarray:
    """int16(round-half-even(c / Q)) on the GPU."""
    return codec.stage_quant(dct_coeffs, Q_matrix, dequant=False)


def dequantize(quantized: np.ndarray, Q_matrix: np.ndarray) -> np.ndarray:
    """float64(q) * Q on the GPU."""
    return codec.stage_quant(quantized, Q_matrix, dequant=True)
