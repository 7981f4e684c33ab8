#!/usr/bin/env python3
"""Build an A/B variant of libjds.so: the listed translation units recompiled
with extra flags (e.g. -DJDS_PROBE_STAGE1), linked with the current objects of
the others, into tools/bin/ab/libjds_<name>.so (load it with JDS_LIB_PATH).
Usage: tools/build_variant.py NAME "FLAGS" file.hip[=alt/path.hip] ...
(file.hip=alt/path.hip compiles another version of that unit, e.g. one taken
from git history, in its place)"""
import os
import shlex
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'jpeg-dsp-studio_amd'))
from jds import build as B  # noqa: E402

name, flags = sys.argv[1], shlex.split(sys.argv[2])
alt = dict((a.split('=', 1) + [None])[:2] for a in sys.argv[3:])
files = list(alt)
B.build()
objdir = os.path.join(B.HERE, '_obj')
out = os.path.join(ROOT, 'tools', 'bin', 'ab')
os.makedirs(out, exist_ok=True)
objs = []
for s in B.SOURCES:
    o = os.path.join(objdir, s + '.o')
    if s in files:
        o = os.path.join(out, f'{name}_{s}.o')
        cmd = [B.HIPCC, '-std=c++17', '-O3', f'--offload-arch={B.ARCH}', '-fPIC', '-c', '-fno-slp-vectorize',
               '-ffp-contract=off', '-w', f'-I{B.INCLUDE}', f'-I{B.CSRC}', *flags, '-o', o,
               alt[s] or os.path.join(B.CSRC, s)]
        subprocess.run(cmd, check=True)
    objs.append(o)
subprocess.run([B.HIPCC, f'--offload-arch={B.ARCH}', '-shared', '-fPIC', '-o', os.path.join(out, f'libjds_{name}.so'),
                *objs], check=True)
print(os.path.join(out, f'libjds_{name}.so'))
