#!/usr/bin/env python3
"""Merge a tools/valu_roofline.py result (gpurun_out/<tag>/valu_roofline.json) into
profiles/pmc_valu.json under a bench configuration key, as per-launch VALU issue
cycles of the bench's two phases (forward = k_fwd32i / k_fwd32 / k_fwd444w +
k_fwd_reduce* + k_fix_fwd; inverse = k_inv_fast / k_inv2 / k_inv_fast444), which
bench.py turns into roofline.valu (issue cycles / (1024 SIMDs x 2.4 GHz x launch time)).
usage: valu_to_profiles.py gpurun_out/<tag> KEY SOURCE_NOTE"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src, key, note = sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else ''
d = json.load(open(os.path.join(src, 'valu_roofline.json')))
ph = {'k_fwd': {'lo': 0.0, 'hi': 0.0, 'kernels': []}, 'k_inv': {'lo': 0.0, 'hi': 0.0, 'kernels': []}}
for k, v in d.items():
    name = k.replace('void ', '')
    if any(s in name for s in ('k_fwd32', 'k_fwd444w', 'k_fwd_reduce', 'k_fix_fwd', 'k_fwd16', 'k_fix_fwd16')):
        p = 'k_fwd'
    elif any(s in name for s in ('k_inv_fast', 'k_inv2', 'k_inv16')):
        p = 'k_inv'
    else:
        continue
    ph[p]['lo'] += v['issue_cycles_lo']
    ph[p]['hi'] += v['issue_cycles_hi']
    ph[p]['kernels'].append({'kernel': name, 'valu_insts': v['valu_insts'], 'f64_insts': v['f64_insts'],
                             'int32_insts': v['int32_insts'], 'valu_per_wave': round(v['valu_per_wave'], 1),
                             'issue_cycles_lo': v['issue_cycles_lo'], 'issue_cycles_hi': v['issue_cycles_hi'],
                             'valu_frac_profiled_lo': round(v['valu_frac_lo'], 4),
                             'valu_frac_profiled_hi': round(v['valu_frac_hi'], 4)})
out = os.path.join(ROOT, 'profiles', 'pmc_valu.json')
rec = json.load(open(out)) if os.path.exists(out) else {}
rec[key] = {'k_fwd': {'issue_cycles_lo': ph['k_fwd']['lo'], 'issue_cycles_hi': ph['k_fwd']['hi'],
                      'kernels': ph['k_fwd']['kernels']},
            'k_inv': {'issue_cycles_lo': ph['k_inv']['lo'], 'issue_cycles_hi': ph['k_inv']['hi'],
                      'kernels': ph['k_inv']['kernels']},
            'method': 'per-launch SQ_INSTS_VALU by class (SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64/F32, _CVT, _INT32, '
                      '_INT64; the rest unclassified) x the class issue cost measured on gfx950 '
                      '(profiles/r03_gfx950_op_rates.txt; INT32 and unclassified at their cheap 2.4 and dear 4.5 '
                      'cycle ends = lo / hi); tools/r4_pmc.sh + tools/valu_roofline.py',
            'source': note}
json.dump(rec, open(out, 'w'), indent=1)
print(key, {p: (round(v['lo'] / 2.4576e12 * 1e6, 1), round(v['hi'] / 2.4576e12 * 1e6, 1)) for p, v in ph.items()},
      'us of issue at 1024 SIMDs x 2.4 GHz')
