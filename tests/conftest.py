"""Test configuration: the `gpu` marker and import paths.

`jpeg-dsp-studio_amd/` holds the drop-in packages (`engines`, `models`,
`utils`, `jds`) at top level, exactly like the reference repo root, so tests
import them the same way the reference's own tests do.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, 'jpeg-dsp-studio_amd')
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs an MI355X (HIP device) — runs on the GPU box')
