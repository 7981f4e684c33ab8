"""Color space conversion and chroma subsampling (engines/color_space.py:1-66).

GPU kernels: csrc/jds_stages.hip (same fp64 operation order as NumPy / OpenCV)."""

from typing import Literal, Tuple

import numpy as np

from jds import codec


def rgb_to_ycbcr(rgb: np.ndarray) -> np.ndarray:
    """RGB to YCbCr using ITU-R BT.601 (color_space.py:8-14)."""
    return codec.stage_rgb_ycbcr(rgb, inverse=False)


def ycbcr_to_rgb(ycbcr: np.ndarray) -> np.ndarray:
    """YCbCr to RGB using ITU-R BT.601, clipped to [0, 255] (color_space.py:17-24)."""
    return codec.stage_rgb_ycbcr(ycbcr, inverse=True)


def subsample_chroma(
    cb: np.ndarray,
    cr: np.ndarray,
    mode: Literal['4:4:4', '4:2:2', '4:2:0'],
    use_prefilter: bool = False
) -> Tuple[np.ndarray, np.ndarray]:
    """Subsample chroma channels according to mode (color_space.py:27-53):
    optional 3x3 Gaussian (sigma 0.75) prefilter, then 2x / 2x2 area average."""
    if mode == '4:4:4':
        return cb.copy(), cr.copy()
    if mode not in ('4:2:2', '4:2:0'):
        raise ValueError(f"Unknown subsampling mode: {mode}")
    return codec.stage_subsample(cb, cr, mode, use_prefilter)


def upsample_chroma(
    cb_sub: np.ndarray,
    cr_sub: np.ndarray,
    target_shape: Tuple[int, int],
    method: str = 'bilinear'
) -> Tuple[np.ndarray, np.ndarray]:
    """Upsample chroma channels to target resolution (color_space.py:56-66)."""
    nearest = method != 'bilinear'
    h, w = int(target_shape[0]), int(target_shape[1])
    return codec.stage_resize(cb_sub, h, w, nearest), codec.stage_resize(cr_sub, h, w, nearest)
