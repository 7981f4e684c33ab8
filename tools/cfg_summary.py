#!/usr/bin/env python3
"""Copy one tools/profile_cfg.sh result into profiles/ and record its HBM traffic.

    python tools/cfg_summary.py TAG [PROFILE_NAME] [TRAFFIC_KEY]

Reads gpurun_out/cfg/TAG/{bench.json, stats/run_kernel_stats.csv,
fetch/run_counter_collection.csv, write/run_counter_collection.csv} and writes
  profiles/PROFILE_NAME_bench.json         the bench line
  profiles/PROFILE_NAME_kernel_stats.csv   rocprofv3 --stats summary
  profiles/PROFILE_NAME_pmc.json           mean FETCH_SIZE / WRITE_SIZE (KB) per kernel launch
and adds the configuration's key to profiles/pmc_traffic.json (bytes per launch
of the bench's two phases), which bench.py reports as roofline.traffic.

HBM bytes (MI355X_MICROARCH.md, HBM/rocprofv3 section): FETCH_SIZE and WRITE_SIZE
come from separate --pmc passes, in KB.  Forward phase = every forward launch
(k_fwd32i / k_fwd32 / k_fix_fwd / k_fwd_reduce_fix); its 8-byte-per-lane RGB
loads were calibrated at face value in round 1 (k_fwd32i FETCH = 1.00x its RGB
bytes).  Inverse = the inverse kernels: FETCH x2 for their 16-byte-per-lane
coefficient reads (128-B requests tallied at 64 B on gfx950), WRITE as is."""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
tag = sys.argv[1]
name = sys.argv[2] if len(sys.argv) > 2 else tag
src = os.path.join(ROOT, 'gpurun_out', 'cfg', tag)
prof = os.path.join(ROOT, 'profiles')

bench = json.loads(open(os.path.join(src, 'bench.json')).read().strip().splitlines()[-1])
json.dump(bench, open(os.path.join(prof, f'{name}_bench.json'), 'w'), indent=1)
shutil.copy(os.path.join(src, 'stats', 'run_kernel_stats.csv'), os.path.join(prof, f'{name}_kernel_stats.csv'))

def mark_name(k):
    """rocprofv3's kernel name -> the plan's launch-mark name (jds_plan_profile):
    'void jds::k_fwd32i<2, true, false>' -> 'k_fwd32i<2,1>'."""
    k = k.replace('void ', '').replace('jds::', '').replace(' ', '').replace('true', '1').replace('false', '0')
    if '<' not in k:
        return k
    base, args = k.split('<', 1)
    a = args.rstrip('>').split(',')
    if base in ('k_fwd32i', 'k_fwd32') and len(a) == 3:
        a = a[:2] + (['mq'] if a[2] == '1' else [])
    if base == 'k_fwd_reduce_rows' and len(a) == 2 and a[1] == '0':
        a = a[:1]
    return f'{base}<{",".join(a)}>'


FWD = ('k_fwd32i', 'k_fwd32<', 'k_fix_fwd', 'k_fwd_reduce', 'k_fwd16', 'k_fwd<', 'k_fwdq', 'k_quant_mq')
INV = ('k_inv2', 'k_inv<', 'k_inv_fast', 'k_inv16', 'k_chroma16', 'k_inv32', 'k_fix_inv')
pmc = collections.defaultdict(dict)
for ctr in ('fetch', 'write'):
    path = os.path.join(src, ctr, 'run_counter_collection.csv')
    if not os.path.exists(path):
        continue
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        agg[r['Kernel_Name'].split('(')[0]].append(float(r['Counter_Value']))
    for k, v in agg.items():
        if 'jds::' in k:
            pmc[k][ctr.upper() + '_SIZE_KB'] = sum(v) / len(v)
json.dump(pmc, open(os.path.join(prof, f'{name}_pmc.json'), 'w'), indent=1)

if pmc:
    fwd = inv = 0.0
    for k, m in pmc.items():
        f, w = m.get('FETCH_SIZE_KB', 0.0), m.get('WRITE_SIZE_KB', 0.0)
        if any(t in k for t in FWD):
            fwd += (f + w) * 1024
        elif any(t in k for t in INV):
            inv += (2 * f + w) * 1024
    per_kernel = {}
    for k, m in pmc.items():
        f, w = m.get('FETCH_SIZE_KB', 0.0), m.get('WRITE_SIZE_KB', 0.0)
        inv_k = any(t in k for t in INV)
        per_kernel[mark_name(k)] = int(((2 * f if inv_k else f) + w) * 1024)
    cfg = bench['config']
    key = sys.argv[3] if len(sys.argv) > 3 else cfg.get('traffic_key')
    if key:
        tf = os.path.join(prof, 'pmc_traffic.json')
        rec = json.load(open(tf)) if os.path.exists(tf) else {}
        rec[key] = {'k_fwd': int(fwd), 'k_inv': int(inv), 'kernels': per_kernel,
                    'method': __doc__.split('\n\n', 2)[2].replace('\n', ' '),
                    'source': f'profiles/{name}_pmc.json'}
        json.dump(rec, open(tf, 'w'), indent=1)
    print(f'{name}: fwd {fwd / 1e6:.1f} MB/launch, inv {inv / 1e6:.1f} MB/launch')
print(json.dumps({k: bench[k] for k in ('value', 'ms_per_step', 'kernels_ms') if k in bench}))
