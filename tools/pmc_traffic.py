"""Write profiles/pmc_traffic.json from a tools/pmc.sh summary (gpurun_out/pmc/summary.json):
HBM bytes per launch for the bench config's forward phase and inverse kernel.

Method (MI355X_MICROARCH.md, HBM/rocprofv3 section): FETCH_SIZE and WRITE_SIZE come
from separate --pmc passes, in KB per launch.  k_fwd = k_fwd32i + k_fwd32 (border
tiles) + k_fix_fwd: its 8-byte-per-lane RGB loads are counted at face value
(calibrated: k_fwd32i FETCH = 1.00x its algorithmic RGB bytes).  k_inv = k_inv2 with
FETCH x2 (128-B requests tallied at 64 B on gfx950), WRITE at face value."""
import json, sys
src = sys.argv[1] if len(sys.argv) > 1 else 'gpurun_out/pmc/summary.json'
out = sys.argv[2] if len(sys.argv) > 2 else 'profiles/pmc_traffic.json'
tag = sys.argv[3] if len(sys.argv) > 3 else src
d = json.load(open(src))


def get(prefix):
    for k, v in d.items():
        if k.startswith(prefix):
            return v
    return None


kb = 1024
fwd = 0.0
for pre in ('void jds::k_fwd32i<2, true, false>', 'void jds::k_fwd32<2, true, false>', 'void jds::k_fix_fwd<2, true>'):
    v = get(pre)
    if v:
        fwd += (v['FETCH_SIZE'] + v['WRITE_SIZE']) * kb
inv = get('void jds::k_inv2<2, 0>')
rec = json.load(open(out)) if out and __import__('os').path.exists(out) else {}
rec['1920x1080_q50_4:2:0_pf1_b64'] = {
    'k_fwd': int(fwd), 'k_inv': int((2 * inv['FETCH_SIZE'] + inv['WRITE_SIZE']) * kb),
    'method': __doc__.split('\n\n', 1)[1].replace('\n', ' '), 'source': tag}
json.dump(rec, open(out, 'w'), indent=1)
print(json.dumps(rec, indent=1))
