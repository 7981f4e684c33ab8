#!/usr/bin/env python3
"""Where the drop-in engines.compress_reconstruct spends a 1080p call (not product code):
wall time per call and with maps off; run under rocprofv3 --kernel-trace --stats for kernels."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'jpeg-dsp-studio_amd'), ROOT]
import numpy as np  # noqa: E402
from engines import compress_reconstruct  # noqa: E402
from models import CompressionParams  # noqa: E402
from jds import codec  # noqa: E402
from engines.quantizer import scale_quant_matrix  # noqa: E402
from utils.constants import JPEG_LUMA_Q50  # noqa: E402

img = np.random.default_rng(5).integers(0, 256, (1080, 1920, 3), dtype=np.uint8)
prm = CompressionParams(quality=50, subsampling_mode='4:2:0', use_prefilter=True)
compress_reconstruct(img, prm)
for name, fn in (('drop-in', lambda: compress_reconstruct(img, prm)),
                 ('raw+maps', lambda: codec.compress_reconstruct_raw(img, 50, scale_quant_matrix(JPEG_LUMA_Q50, 50),
                                                                     '4:2:0', True, maps=True)),
                 ('raw-nomaps', lambda: codec.compress_reconstruct_raw(img, 50, scale_quant_matrix(JPEG_LUMA_Q50, 50),
                                                                       '4:2:0', True, maps=False)),
                 ('psnr_ssim', lambda: codec.psnr_ssim_raw(img, img))):
    fn()
    t0 = time.perf_counter()
    for _ in range(5):
        fn()
    print(f'{name:12s} {(time.perf_counter() - t0) / 5 * 1e3:8.2f} ms', flush=True)
