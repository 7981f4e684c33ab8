"""The A/B-only kernel variants still compile (they are left out of the product
library): k_inv_fast6, the transpose-free 4:2:0 inverse measured in round 6
(DESIGN.md §4 "Round 6"), built by tools/build_variant.py with -DJDS_INV6."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'jpeg-dsp-studio_amd'))
from jds import build as B  # noqa: E402


@pytest.mark.skipif(not os.path.exists(B.HIPCC), reason='hipcc not installed')
@pytest.mark.parametrize('unit', ['jds_inv_fast.hip', 'jds_abi.hip'])
def test_inv6_variant_compiles(tmp_path, unit):
    cmd = [B.HIPCC, '-std=c++17', '-O1', f'--offload-arch={B.ARCH}', '--cuda-device-only' if unit != 'jds_abi.hip'
           else '-fPIC', '-c', '-fno-slp-vectorize', '-ffp-contract=off', '-w', '-DJDS_INV6', f'-I{B.INCLUDE}',
           f'-I{B.CSRC}', '-o', str(tmp_path / 'v.o'), os.path.join(B.CSRC, unit)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
