#!/usr/bin/env python3
"""Per-kernel mean PMC counters from tools/pmc.sh output (gpurun_out/pmc/p*/run_counter_collection.csv),
plus derived figures: HBM bytes per launch (FETCH_SIZE x2 for 16-B/lane streaming reads per
MI355X_MICROARCH.md, WRITE_SIZE as is), wave-cycle split and LDS conflict share."""
import collections, csv, glob, json, sys
root = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/pmc'
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(f'{root}/p*/run_counter_collection.csv')):
    for r in csv.DictReader(open(f)):
        agg[r['Kernel_Name'].split('(')[0]][r['Counter_Name']].append(float(r['Counter_Value']))
out = {}
for k, d in agg.items():
    if not k.startswith('void jds::') and not k.startswith('jds::'):
        continue
    m = {c: sum(v) / len(v) for c, v in d.items()}
    out[k] = m
    wc = m.get('SQ_WAVE_CYCLES', 0) or 1
    print(f'{k}')
    print('   ' + '  '.join(f'{c}={m[c]:.4g}' for c in sorted(m)))
    print(f"   wait_any={m.get('SQ_WAIT_ANY', 0) / wc:.2f} wait_inst={m.get('SQ_WAIT_INST_ANY', 0) / wc:.2f} "
          f"active={m.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f} lds_conflict={m.get('SQ_LDS_BANK_CONFLICT', 0) / max(1, m.get('SQ_LDS_IDX_ACTIVE', 1)):.2f} "
          f"fetch_MB(raw)={m.get('FETCH_SIZE', 0) / 1024:.1f} write_MB={m.get('WRITE_SIZE', 0) / 1024:.1f} "
          f"valu_per_wave={m.get('SQ_INSTS_VALU', 0) / max(1, m.get('SQ_WAVES', 1)):.0f}")
json.dump(out, open(f'{root}/summary.json', 'w'), indent=1)
