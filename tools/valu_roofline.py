#!/usr/bin/env python3
"""VALU issue roofline of each kernel from rocprofv3 PMC passes (tools/r4_pmc.sh).

Dynamic instruction counts per launch by class (SQ_INSTS_VALU_*) times the
measured issue cost of that class on gfx950 (cycles per wave instruction per
SIMD at 8 waves/SIMD, profiles/r03_gfx950_op_rates.txt), over the SIMD-cycles
the launch had (1024 SIMDs x effective clock x launch time):

    valu_frac = sum_c count_c * cost_c / (1024 * f_clk * t_launch)

f_clk = GRBM_GUI_ACTIVE / 8 / t (MI355X_MICROARCH.md, DVFS give-back; the sum over
the 8 XCDs) when collected, else the 2.4 GHz peak.  INT32 and the unclassified
rest (moves, selects, compares, DPP) mix cheap (~2.5 cycles) and dear (~4.4)
forms, so frac is reported at both ends and the midpoint.  Writes
<dir>/valu_roofline.json and prints one line per kernel."""
import collections
import csv
import glob
import json
import sys

COST = {  # cycles per wave instruction (profiles/r03_gfx950_op_rates.txt)
    'SQ_INSTS_VALU_ADD_F64': (4.91, 4.91), 'SQ_INSTS_VALU_MUL_F64': (4.99, 4.99),
    'SQ_INSTS_VALU_FMA_F64': (5.04, 5.04), 'SQ_INSTS_VALU_TRANS_F64': (8.0, 8.0),
    'SQ_INSTS_VALU_ADD_F32': (2.64, 2.64), 'SQ_INSTS_VALU_MUL_F32': (2.53, 2.53),
    'SQ_INSTS_VALU_FMA_F32': (2.48, 2.73), 'SQ_INSTS_VALU_TRANS_F32': (8.0, 8.0),
    'SQ_INSTS_VALU_CVT': (4.23, 4.35), 'SQ_INSTS_VALU_INT64': (4.43, 4.68),
    'SQ_INSTS_VALU_INT32': (2.41, 4.53),
}
REST = (2.38, 4.53)  # unclassified VALU: v_mov_b32 .. v_cndmask / v_cmp / DPP


def main(root):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(list)
    for f in sorted(glob.glob(f'{root}/p*/run_counter_collection.csv')):
        for r in csv.DictReader(open(f)):
            k = r['Kernel_Name'].split('(')[0]
            per[k][r['Counter_Name']].append(float(r['Counter_Value']))
    for f in sorted(glob.glob(f'{root}/p*/run_kernel_trace.csv')):
        for r in csv.DictReader(open(f)):
            k = r['Kernel_Name'].split('(')[0]
            dur[k].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) * 1e-9)
    out = {}
    for k, d in per.items():
        if 'jds::' not in k or not dur.get(k):
            continue
        m = {c: sum(v) / len(v) for c, v in d.items()}
        t = sorted(dur[k])[len(dur[k]) // 2]  # median launch (profiled passes run slower: ratios only)
        valu = m.get('SQ_INSTS_VALU', 0.0)
        if not valu:
            continue
        lo = hi = 0.0
        known = 0.0
        for c, (a, b) in COST.items():
            n = m.get(c, 0.0)
            known += n
            lo += n * a
            hi += n * b
        rest = max(0.0, valu - known)
        lo += rest * REST[0]
        hi += rest * REST[1]
        clk = m['GRBM_GUI_ACTIVE'] / 8.0 / t if m.get('GRBM_GUI_ACTIVE') else 2.4e9
        clk = min(clk, 2.4e9)
        cap = 1024 * clk * t
        rec = {'valu_insts': valu, 'f64_insts': sum(m.get(c, 0.0) for c in COST if c.endswith('F64')),
               'int32_insts': m.get('SQ_INSTS_VALU_INT32', 0.0), 'unclassified_insts': rest,
               'launch_s_profiled': t, 'clock_hz': clk,
               'issue_cycles_lo': lo, 'issue_cycles_hi': hi,
               'valu_frac_lo': lo / cap, 'valu_frac_hi': hi / cap, 'valu_frac_mid': (lo + hi) / 2 / cap,
               'valu_per_wave': valu / max(1.0, m.get('SQ_WAVES', 1.0))}
        out[k] = rec
        print(f"{k:60s} VALU {valu:.3g} (f64 {rec['f64_insts']:.3g}, int32 {rec['int32_insts']:.3g}) "
              f"clk {clk / 1e9:.2f} GHz  valu_frac {rec['valu_frac_lo']:.2f}..{rec['valu_frac_hi']:.2f}")
    json.dump(out, open(f'{root}/valu_roofline.json', 'w'), indent=1)


if __name__ == '__main__':
    main(sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/pmcv')
