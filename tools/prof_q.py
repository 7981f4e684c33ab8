"""Per-quality kernel durations from a rocprofv3 kernel trace of tools/sweep_probe.py
(SETS of six equal qualities, NQ=1): sets are told apart by k_quant_mq counts."""
import collections, csv, sys
path = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/prof_q/run_kernel_trace.csv'
labels = sys.argv[2].split(',') if len(sys.argv) > 2 else ['Q5', 'Q50', 'Q80', 'Q95']
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r['Start_Timestamp']))
seq = [r for r in rows if 'jds::' in r['Kernel_Name']]
names = ['k_quant_mq', 'k_fix_fwd', 'k_fwd32i', 'k_inv2', 'k_fwd32<', 'k_fwd_reduce']
qi = [i for i, r in enumerate(seq) if 'k_quant_mq' in r['Kernel_Name']]
per = len(qi) // len(labels)
for s, lab in enumerate(labels):
    lo = qi[s * per]
    hi = qi[(s + 1) * per] if s < len(labels) - 1 else len(seq)
    agg = collections.defaultdict(list)
    for r in seq[lo:hi]:
        for n in names:
            if n in r['Kernel_Name']:
                agg[n].append((int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1000)
    print(lab, {n: round(sum(v) / len(v), 1) for n, v in agg.items()})
