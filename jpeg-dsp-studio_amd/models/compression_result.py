"""Compression result (models/compression_result.py:7-30 of the reference)."""

from dataclasses import dataclass

import numpy as np


@dataclass
class CompressionResult:
    """Results of compress_reconstruct.

    encode_time_ms / decode_time_ms hold the forward / inverse HIP kernel times
    (hipEvents) of this call.  The reference timed only rgb_to_ycbcr and
    ycbcr_to_rgb with perf_counter (engines/pipeline.py:28,89-94).
    """

    original_image: np.ndarray
    reconstructed_image: np.ndarray

    # Quality metrics
    psnr_y: float
    ssim_y: float
    psnr_rgb: float
    ssim_rgb: float

    # Compression stats
    bpp: float
    compression_ratio: float
    nonzero_coeffs: int
    total_coeffs: int

    # Runtime
    encode_time_ms: float
    decode_time_ms: float

    bitrate_label: str = "Estimated (no entropy coding)"
