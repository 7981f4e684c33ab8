#!/usr/bin/env python3
"""Per-kernel VGPR / SGPR / spill / LDS / occupancy table for one HIP source
(hipcc -Rpass-analysis=kernel-resource-usage).  Usage: tools/kres.py file.hip [filter]"""
import re, subprocess, sys, os
src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ''
inc = os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'include')
# the library's own flags (jds/build.py), plus KRES_FLAGS (e.g. "-DJDS_Q16_GLOBAL")
extra = os.environ.get('KRES_FLAGS', '').split()
r = subprocess.run(['/opt/rocm/bin/hipcc', '-std=c++17', '-O3', '--offload-arch=gfx950', '-fPIC', '-c', src,
                    '-fno-slp-vectorize', '-ffp-contract=off', '-o', '/tmp/_kres.o', '-I', inc,
                    '-I', os.path.dirname(os.path.abspath(src)), *extra, '-Rpass-analysis=kernel-resource-usage'],
                   capture_output=True, text=True)
if r.returncode:
    print(r.stderr[-4000:]); sys.exit(1)
rows, cur = [], None
for line in r.stderr.splitlines():
    m = re.search(r'remark: (.*?): (.*) \[-Rpass', line) or re.search(r'remark:\s+(\w[\w /\[\]]*?): (.*?) \[', line)
    if 'Function Name:' in line:
        cur = {'name': line.split('Function Name:')[1].split('[')[0].strip()}
        rows.append(cur)
    elif cur is not None:
        for key in ('VGPRs', 'AGPRs', 'TotalSGPRs', 'VGPRs Spill', 'SGPRs Spill', 'LDS Size [bytes/block]', 'Occupancy [waves/SIMD]'):
            mm = re.search(re.escape(key) + r': (\d+)', line)
            if mm and key + ':' in line:
                cur[key] = mm.group(1)
dem = subprocess.run(['c++filt'], input='\n'.join(r_['name'] for r_ in rows), capture_output=True, text=True).stdout.split('\n')
for r_, d in zip(rows, dem):
    d = d.split('(')[0]
    if flt and flt not in d:
        continue
    print(f"{d[:48]:48s} v={r_.get('VGPRs','?'):>4} s={r_.get('TotalSGPRs','?'):>4} vsp={r_.get('VGPRs Spill','?'):>3} "
          f"ssp={r_.get('SGPRs Spill','?'):>3} lds={r_.get('LDS Size [bytes/block]','?'):>6} occ={r_.get('Occupancy [waves/SIMD]','?')}")
