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

SOURCES = ['jds_codec.hip', 'jds_gen.hip', 'jds_b16.hip', 'jds_inv.hip', 'jds_inv_fast.hip', 'jds_fast.hip', 'jds_fast16.hip', 'jds_stages.hip', 'jds_ssim.hip', 'jds_ssim_band.hip', 'jds_entropy.hip', 'jds_abi.hip']


def headers():
    """Every header under csrc/ is a build input (tests/test_abi_cpu.py checks
    that each #include "..." of the sources resolves to one of them)."""
    return sorted(f for f in os.listdir(CSRC) if f.endswith('.hpp'))


def _inputs():
    files = [os.path.join(CSRC, s) for s in SOURCES + headers() if os.path.exists(os.path.join(CSRC, s))]
    return files + [os.path.join(INCLUDE, 'jds.h')]


def up_to_date() -> bool:
    if not os.path.exists(LIB):
        return False
    t = os.path.getmtime(LIB)
    return all(os.path.getmtime(f) <= t for f in _inputs())


def _compile(src, obj, verbose):
    cmd = [HIPCC, '-std=c++17', '-O3', f'--offload-arch={ARCH}', '-fPIC', '-c', '-fno-slp-vectorize',
           '-ffp-contract=off', '-Wall', '-Wno-unused-function', f'-I{INCLUDE}', f'-I{CSRC}', '-o', obj, src]
    if verbose:
        print(' '.join(cmd), file=sys.stderr)
    return subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)


def build(force: bool = False, verbose: bool = False) -> str:
    """Each translation unit compiles on its own (in parallel; no device code is
    shared across units), then one host link makes libjds.so."""
    if not force and up_to_date():
        return LIB
    srcs = [os.path.join(CSRC, s) for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]
    objdir = os.path.join(HERE, '_obj')
    os.makedirs(objdir, exist_ok=True)
    jobs = max(1, min(len(srcs), int(os.environ.get('MAX_JOBS', os.cpu_count() or 4))))
    objs, errs, pending = [], [], []
    for src in srcs:
        obj = os.path.join(objdir, os.path.basename(src) + '.o')
        objs.append(obj)
        pending.append((src, obj))
    running = []
    while pending or running:
        while pending and len(running) < jobs:
            src, obj = pending.pop(0)
            running.append((src, _compile(src, obj, verbose)))
        src, pr = running.pop(0)
        _, err = pr.communicate()
        if pr.returncode != 0:
            errs.append(f'{os.path.basename(src)}:\n{err[-4000:]}')
    if errs:
        raise RuntimeError('hipcc failed:\n' + '\n'.join(errs))
    cmd = [HIPCC, f'--offload-arch={ARCH}', '-shared', '-fPIC', '-o', LIB + '.tmp'] + objs
    if verbose:
        print(' '.join(cmd), file=sys.stderr)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f'hipcc link failed ({r.returncode}):\n{r.stderr[-6000:]}')
    os.replace(LIB + '.tmp', LIB)
    return LIB


if __name__ == '__main__':
    print(build(force='--force' in sys.argv, verbose=True))
