"""Metrics: PSNR, SSIM, bitrate estimation (utils/metrics.py:1-92 of the reference).

PSNR / SSIM run on the GPU (jds_psnr_ssim, csrc/jds_ssim.hip) and reproduce
skimage.metrics' values bit for bit, including NumPy's reduction order.
"""

import time
from typing import Dict

import numpy as np

from jds.codec import psnr_ssim_raw


def psnr_from_mse(mse, data_range: int = 255) -> float:
    """skimage peak_signal_noise_ratio tail: 10 * log10(R**2 / mse) in NumPy float64."""
    with np.errstate(divide='ignore'):
        return float(10 * np.log10((data_range ** 2) / np.float64(mse)))


def compute_psnr_ssim(original_rgb: np.ndarray, reconstructed_rgb: np.ndarray) -> Dict[str, float]:
    """Compute PSNR and SSIM on RGB and Y channel (utils/metrics.py:9-28)."""
    r = psnr_ssim_raw(original_rgb, reconstructed_rgb)
    ssim_rgb = np.array(r[:3]).mean()  # skimage: mean of the per-channel SSIMs
    return {
        'psnr_rgb': psnr_from_mse(r[5]),
        'ssim_rgb': float(ssim_rgb),
        'psnr_y': psnr_from_mse(r[4]),
        'ssim_y': float(r[3]),
    }


class Timer:
    """Simple timer for encode/decode runtime (utils/metrics.py:31-48)."""

    def __init__(self):
        self.encode_time_ms = 0.0
        self.decode_time_ms = 0.0

    def measure_encode(self, func, *args, **kwargs):
        start = time.perf_counter()
        result = func(*args, **kwargs)
        self.encode_time_ms = (time.perf_counter() - start) * 1000.0
        return result

    def measure_decode(self, func, *args, **kwargs):
        start = time.perf_counter()
        result = func(*args, **kwargs)
        self.decode_time_ms = (time.perf_counter() - start) * 1000.0
        return result


def _bitrate_tail(coeff_bits, nonzero: int, total_coeffs: int, original_shape: tuple, block_size: int) -> Dict:
    """utils/metrics.py:62-70 and :83-92: block overhead, totals and the dict,
    with `coeff_bits` kept in whatever NumPy type the caller's sum produced
    (the reference's promotion decides the float32 / float64 result)."""
    h, w = original_shape
    num_pixels = h * w
    original_bits = num_pixels * 3 * 8
    padded_h = ((h + block_size - 1) // block_size) * block_size
    padded_w = ((w + block_size - 1) // block_size) * block_size
    num_blocks = (padded_h // block_size) * (padded_w // block_size)
    block_overhead_bits = num_blocks * 2
    estimated_bits = block_overhead_bits + coeff_bits
    return {
        'estimated_bits': int(estimated_bits),
        'bpp': float(estimated_bits / num_pixels),
        'compression_ratio': float(original_bits / max(estimated_bits, 1)),
        'nonzero_count': int(nonzero),
        'total_coeffs': int(total_coeffs),
        'label': 'Estimated (no entropy coding)',
    }


def bitrate_from_counts(nonzero: int, magnitude_bits, total_coeffs: int, original_shape: tuple,
                        block_size: int = 8) -> Dict:
    """The tail of estimate_bitrate_no_entropy (utils/metrics.py:62-92) from the
    pipeline's GPU counts.

    The pipeline's coefficients are int16, for which the reference sums
    ceil(log2(|q|+1)) + 1 as float32 (np.log2 of int16 is float32):
    `magnitude_bits` is that float32 sum (k_mag_f32 reproduces NumPy's buffered
    pairwise float32 reduction; below 2**24 it equals the exact integer).
    Evaluating the reference's expression with that np.float32 scalar reproduces
    its NumPy-version-dependent promotion (float32 under NumPy >= 2, float64
    under 1.x)."""
    coeff_bits = 6 * int(nonzero) + np.float32(magnitude_bits) if nonzero > 0 else 0
    return _bitrate_tail(coeff_bits, nonzero, total_coeffs, original_shape, block_size)


def estimate_bitrate_no_entropy(quantized_coeffs: np.ndarray, original_shape: tuple, block_size: int = 8) -> Dict:
    """Estimate compressed size WITHOUT entropy coding (utils/metrics.py:51-92).

    Per nonzero coefficient: 6 position bits + ceil(log2(|c|+1)) + 1 magnitude
    bits; plus 2 bits per luma block.  A standalone host utility on a NumPy
    array (the pipeline itself uses the GPU counts, bitrate_from_counts): the
    magnitude sum is the reference's own NumPy expression on the caller's
    array, so its dtype rules hold -- float32 accumulation (pairwise order) for
    int8/int16 input, float64 for int32/int64, wrap-around of |int16 min|."""
    q = np.asarray(quantized_coeffs)
    mask = q != 0
    nz = q[mask]
    if len(nz) > 0:
        mags = np.abs(nz)
        coeff_bits = 6 * len(nz) + np.sum(np.ceil(np.log2(mags + 1)) + 1)
    else:
        coeff_bits = 0
    return _bitrate_tail(coeff_bits, int(np.sum(mask)), int(q.size), original_shape, block_size)
