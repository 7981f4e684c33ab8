"""In-tree build of the HIP library (libjds.so) for gfx950.

Called by __graft_entry__.build() and by the test suite.  hipcc cross-compiles
gfx950 code objects without a GPU.  The product is built with FP contraction
off: the codec's fp64 arithmetic must round exactly like NumPy / pocketfft /
OpenCV (no FMA).
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.dirname(HERE)
REPO = os.path.dirname(PKG)
CSRC = os.path.join(PKG, 'csrc')
INCLUDE = os.path.join(REPO, 'include')
LIB = os.path.join(HERE, 'libjds.so')
HIPCC = os.environ.get('HIPCC', '/opt/rocm/bin/hipcc')
ARCH = os.environ.get('JDS_OFFLOAD_ARCH', 'gfx950')

SOURCES = ['jds_codec.hip', 'jds_b16.hip', 'jds_inv.hip', 'jds_fast.hip', 'jds_stages.hip', 'jds_ssim.hip', 'jds_entropy.hip', 'jds_abi.hip']
HEADERS = ['jds_dct8.hpp', 'jds_dct16.hpp', 'jds_internal.hpp', 'jds_device.hpp']


def _inputs():
    files = [os.path.join(CSRC, s) for s in SOURCES + HEADERS if os.path.exists(os.path.join(CSRC, s))]
    return files + [os.path.join(INCLUDE, 'jds.h')]


def up_to_date() -> bool:
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(f) <= t for f in _inputs())


def build(force: bool = False, verbose: bool = False) -> str:
    if not force and up_to_date():
        return LIB
    srcs = [os.path.join(CSRC, s) for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]
    cmd = [HIPCC, '-std=c++17', '-O3', f'--offload-arch={ARCH}', '-fPIC', '-shared', '-fno-slp-vectorize',
           '-ffp-contract=off', '-Wall', '-Wno-unused-function', f'-I{INCLUDE}', f'-I{CSRC}',
           '-o', LIB + '.tmp'] + srcs
    if verbose:
        print(' '.join(cmd), file=sys.stderr)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f'hipcc failed ({r.returncode}):\n{r.stderr[-6000:]}')
    os.replace(LIB + '.tmp', LIB)
    return LIB


if __name__ == '__main__':
    print(build(force='--force' in sys.argv, verbose=True))
