#!/usr/bin/env python3
"""Per-kernel issue, wave-cycle and traffic records from a tools/r6_pmc.sh run
(VERDICT r05 item 1), merged into profiles/pmc_valu.json and
profiles/pmc_traffic.json under a bench-configuration key.

VALU issue fraction that cannot exceed 1: every class of VALU instruction is
priced at its MINIMUM issue cost per wave64 instruction on gfx950 -- the
peak-rate cost (fp32 add/mul/fma and the simple int32 class: 2 cycles, the
157.3 TF/s fp32 vector peak; fp64: 4 cycles, the 78.6 TF/s fp64 peak; cvt /
int64: 4; transcendental: 8) and the unclassified rest (moves, selects,
compares, DPP, permutes) at 2 -- over the SIMD-cycles of the same profiled
launches (1024 SIMDs x GRBM_GUI_ACTIVE / 8, the per-XCD cycle count; no clock
assumption).  A lower bound on the VALU-busy fraction, <= 1 by construction;
`frac_upper` prices int32 and the rest at the slow class (4 cycles).
Wave-cycle split (MI355X_MICROARCH.md: SQ_WAIT_ANY + SQ_WAIT_INST_ANY +
SQ_ACTIVE_INST_ANY ~ SQ_WAVE_CYCLES, disjoint): parked (s_waitcnt / barrier),
issue-stalled (dependency / pipe), active; LDS-issue stalls (SQ_WAIT_INST_LDS)
and the bank-conflict share of LDS cycles.  HBM bytes per launch: 2 x
FETCH_SIZE (calibrated: tools/microbench/fetch_cal.hip, 0.50 of the true bytes
for the forward's 24-B / lane, the inverse's 2-B column and 16-B / lane
streams alike) + WRITE_SIZE (face value).
usage: r6_valu.py gpurun_out/<pmc dir> KEY SOURCE [--frames B]"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MIN_COST = {'SQ_INSTS_VALU_ADD_F64': 4, 'SQ_INSTS_VALU_MUL_F64': 4, 'SQ_INSTS_VALU_FMA_F64': 4,
            'SQ_INSTS_VALU_TRANS_F64': 8, 'SQ_INSTS_VALU_ADD_F32': 2, 'SQ_INSTS_VALU_MUL_F32': 2,
            'SQ_INSTS_VALU_FMA_F32': 2, 'SQ_INSTS_VALU_TRANS_F32': 8, 'SQ_INSTS_VALU_CVT': 4,
            'SQ_INSTS_VALU_INT64': 4, 'SQ_INSTS_VALU_INT32': 2}
UPPER = {'SQ_INSTS_VALU_INT32': 4}
REST_MIN, REST_UP = 2, 4


def load(root):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(f'{root}/p*/run_counter_collection.csv')):
        for r in csv.DictReader(open(f)):
            k = r['Kernel_Name'].split('(')[0].replace('void ', '')
            per[k][r['Counter_Name']].append(float(r['Counter_Value']))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in per.items()}


def record(m):
    valu = m.get('SQ_INSTS_VALU', 0.0)
    known = sum(m.get(c, 0.0) for c in MIN_COST)
    rest = max(0.0, valu - known)
    lo = sum(m.get(c, 0.0) * w for c, w in MIN_COST.items()) + rest * REST_MIN
    up = lo + sum(m.get(c, 0.0) * (UPPER[c] - MIN_COST[c]) for c in UPPER) + rest * (REST_UP - REST_MIN)
    simd_cycles = 1024.0 * m['GRBM_GUI_ACTIVE'] / 8.0
    wc = m.get('SQ_WAVE_CYCLES', 0.0) or 1.0
    lds = m.get('SQ_LDS_IDX_ACTIVE', 0.0) or 1.0
    return {
        'valu_insts': valu, 'valu_per_wave': valu / max(1.0, m.get('SQ_WAVES', 1.0)),
        'f64_insts': sum(m.get(c, 0.0) for c in MIN_COST if c.endswith('F64')),
        'issue_cycles_min': lo, 'issue_cycles_upper': up, 'simd_cycles': simd_cycles,
        'valu_frac': lo / simd_cycles, 'valu_frac_upper': up / simd_cycles,
        'wave_split': {'parked_waitcnt_barrier': m.get('SQ_WAIT_ANY', 0.0) / wc,
                       'issue_stalled_dependency_pipe': m.get('SQ_WAIT_INST_ANY', 0.0) / wc,
                       'active': m.get('SQ_ACTIVE_INST_ANY', 0.0) / wc,
                       'lds_issue_stalled': m.get('SQ_WAIT_INST_LDS', 0.0) / wc,
                       'valu_active': m.get('SQ_ACTIVE_INST_VALU', 0.0) / wc,
                       'lds_active': m.get('SQ_ACTIVE_INST_LDS', 0.0) / wc},
        'lds_conflict_share': m.get('SQ_LDS_BANK_CONFLICT', 0.0) / lds,
        'lds_cycles_per_simd_cycle_x4': lds / max(1.0, simd_cycles / 4.0),
        'hbm_bytes': (2.0 * m.get('FETCH_SIZE', 0.0) + m.get('WRITE_SIZE', 0.0)) * 1024.0,
        'fetch_raw_bytes': m.get('FETCH_SIZE', 0.0) * 1024.0, 'write_bytes': m.get('WRITE_SIZE', 0.0) * 1024.0,
    }


def main():
    src, key, note = sys.argv[1], sys.argv[2], sys.argv[3]
    d = load(src)
    recs = {k: record(m) for k, m in d.items() if k.startswith('jds::') and m.get('SQ_INSTS_VALU') and
            m.get('GRBM_GUI_ACTIVE')}
    out = os.path.join(ROOT, 'profiles', 'pmc_valu.json')
    rec = json.load(open(out)) if os.path.exists(out) else {}
    rec[key] = {'kernels': recs, 'method': __doc__.split('\n\n', 1)[1].split('usage:')[0].replace('\n', ' '),
                'source': note}
    json.dump(rec, open(out, 'w'), indent=1)
    tout = os.path.join(ROOT, 'profiles', 'pmc_traffic.json')
    trec = json.load(open(tout)) if os.path.exists(tout) else {}
    trec[key] = {'kernels': {k: int(v['hbm_bytes']) for k, v in recs.items()},
                 'method': '2 x FETCH_SIZE + WRITE_SIZE per launch (FETCH calibrated on the kernels\' own load shapes, '
                           'profiles/r06_fetch_cal.json)', 'source': note}
    json.dump(trec, open(tout, 'w'), indent=1)
    for k, v in recs.items():
        print(f"{k:42s} valu {v['valu_frac']:.3f}..{v['valu_frac_upper']:.3f}  split park/stall/active "
              f"{v['wave_split']['parked_waitcnt_barrier']:.2f}/{v['wave_split']['issue_stalled_dependency_pipe']:.2f}/"
              f"{v['wave_split']['active']:.2f}  lds conflict {v['lds_conflict_share']:.2f}  hbm {v['hbm_bytes'] / 1e6:.1f} MB")


if __name__ == '__main__':
    main()
