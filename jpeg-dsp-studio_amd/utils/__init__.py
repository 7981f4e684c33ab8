"""Shared utilities (drop-in for the reference's utils/__init__.py:3-18)."""

from .constants import JPEG_LUMA_Q50, ZIGZAG_ORDER
from .metrics import compute_psnr_ssim, Timer, estimate_bitrate_no_entropy
from .test_images import generate_colored_checkerboard, generate_thin_stripes
from .image_io import load_image, save_image

__all__ = [
    'JPEG_LUMA_Q50',
    'ZIGZAG_ORDER',
    'compute_psnr_ssim',
    'Timer',
    'estimate_bitrate_no_entropy',
    'generate_colored_checkerboard',
    'generate_thin_stripes',
    'load_image',
    'save_image',
]
