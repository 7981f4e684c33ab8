"""jds — the MI355X-native backend under the drop-in engines.* API.

libjds.so (HIP for gfx950, built from ../csrc by jds.build) does all the work;
this package is its ctypes binding (``_abi``) and thin NumPy marshalling
(``codec``).  See include/jds.h for the C-ABI.
"""
from ._abi import (JDSError, Context, Plan, FrameStats, Geometry, Params, STATS_DTYPE, MODE_CODES, RUN_SSE,
                   check, context, device_count, geometry, lib, make_params)
from .codec import compress_reconstruct_raw, gaussian_kernel3, psnr_ssim_raw

__all__ = ['JDSError', 'Context', 'Plan', 'FrameStats', 'Geometry', 'Params', 'STATS_DTYPE', 'MODE_CODES',
           'RUN_SSE', 'check', 'context', 'device_count', 'geometry', 'lib', 'make_params',
           'compress_reconstruct_raw', 'gaussian_kernel3', 'psnr_ssim_raw']
