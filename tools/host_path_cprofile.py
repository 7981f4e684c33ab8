#!/usr/bin/env python3
"""cProfile of the drop-in engines.compress_reconstruct on one 1080p frame (not product code)."""
import cProfile
import os
import pstats
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'jpeg-dsp-studio_amd'), ROOT]
import numpy as np  # noqa: E402
from engines import compress_reconstruct  # noqa: E402
from models import CompressionParams  # noqa: E402

img = np.random.default_rng(5).integers(0, 256, (1080, 1920, 3), dtype=np.uint8)
prm = CompressionParams(quality=50, subsampling_mode='4:2:0', use_prefilter=True)
for _ in range(3):
    compress_reconstruct(img, prm)
pr = cProfile.Profile()
pr.enable()
for _ in range(10):
    compress_reconstruct(img, prm)
pr.disable()
pstats.Stats(pr).sort_stats('tottime').print_stats(14)
