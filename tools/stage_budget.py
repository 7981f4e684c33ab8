#!/usr/bin/env python3
"""ISA-derived per-stage instruction budget of the two headline kernels.

Compiles a translation unit for gfx950 with line tables only (the code object is
identical to the product's: -gline-tables-only changes no instruction), splits
the kernel's listing into basic blocks, attributes every instruction to a
pipeline stage through its `.loc` source line (inlined helpers keep their own
lines: aan8 -> IDCT, quant8 -> quantise, ...), weights each basic block by how
many times one wave executes it on the fast path, and prints per stage:
VALU fp64 / other VALU / SALU / LDS / VMEM instructions per wave and VALU
lane-operations per pixel.  The execution model (loop trip counts, which waves
of a workgroup run which branch) is stated per kernel below; the total is
checked against the PMC count (SQ_INSTS_VALU / SQ_WAVES) of the same build.

Usage: tools/stage_budget.py [inv|fwd] [--json out.json]
"""
import collections
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, 'jpeg-dsp-studio_amd', 'csrc')
HIPCC = '/opt/rocm/bin/hipcc'
# one-line helpers whose lines stand for their caller's (the multiply-add policy)
TRANSPARENT = {('jds_inv_fast.hip', next(i + 1 for i, l in enumerate(open(os.path.join(CSRC, 'jds_inv_fast.hip')))
                                         if 'struct MadDev' in l) + 1)}


def listing(src, out, extra=()):
    cmd = [HIPCC, *extra, '-std=c++17', '-O3', '--offload-arch=gfx950', '-fno-slp-vectorize', '-ffp-contract=off',
           '-gline-tables-only', f'-I{ROOT}/include', f'-I{CSRC}', '--cuda-device-only', '-S', '-o', out,
           os.path.join(CSRC, src)]
    subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)
    return open(out).read()


def func_ranges(path, names):
    """{name: (first, last)} source lines of each named function's definition
    (a line declaring `<type> name(`, brace matched from the first `{` after it)."""
    lines = open(path).read().split('\n')
    out = {}
    for name in names:
        pat = re.compile(r'(\b(void|double|float|int|uint32_t|uint4|unsigned|bool|auto)\s+|^)' + re.escape(name) + r'\s*\(')
        for i, ln in enumerate(lines):
            if not pat.search(ln) or ln.strip().startswith('//'):
                continue
            depth, started = 0, False
            for j in range(i, len(lines)):
                seg = lines[j] if started or '{' not in lines[j] else lines[j][lines[j].index('{'):]
                if not started and '{' not in lines[j] and ';' in lines[j]:
                    break  # a declaration
                depth += seg.count('{') - seg.count('}')
                started = started or '{' in seg
                if started and depth == 0:
                    out[name] = (i + 1, j + 1)
                    break
            if name in out:
                break
    return out


def classify(op):
    if op.startswith('v_'):
        return 'valu_f64' if 'f64' in op else 'valu'
    if op.startswith('s_'):
        return 'salu'
    if op.startswith('ds_'):
        return 'lds'
    if op.startswith(('global_', 'buffer_', 'flat_', 'scratch_')):
        return 'vmem'
    return 'other'


def blocks(asm, kernel_key):
    i = asm.index('\n' + kernel_key) + 1
    j = asm.index('.Lfunc_end', i)
    files = {int(m.group(1)): os.path.basename(m.group(3)) for m in
             re.finditer(r'\.file\s+(\d+)\s+"([^"]*)"\s+"([^"]*)"', asm)}
    bbs, cur, loc, loop = [], None, ('?', 0), None
    own = None  # system-header lines (fmin, shuffles, atomics) count for the repo source line that called them
    for ln in asm[i:j].split('\n'):
        s = ln.strip()
        m = re.match(r'\.loc\s+(\d+)\s+(\d+)', s)
        if m:
            f = files.get(int(m.group(1)), '?')
            if f.startswith('jds_') and int(m.group(2)) != 0 and (f, int(m.group(2))) not in TRANSPARENT:
                loc = own = (f, int(m.group(2)))
            else:
                loc = own if own else (f, int(m.group(2)))
            continue
        if re.match(r'^(\.LBB\w+:|; %bb\.\d+:)', s):
            lm = re.search(r'Header=(BB\w+) Depth=(\d)', ln) or re.search(r'(?:=>)?This (?:Inner )?Loop Header: Depth=(\d)',
                                                                          ln)
            name = s.split(':')[0].lstrip('; %').lstrip('.')
            hdr = None
            if 'Loop Header' in ln:
                hdr = name.replace('LBB', 'BB')
            elif 'in Loop: Header=' in ln:
                hdr = re.search(r'Header=(BB\w+)', ln).group(1)
            cur = {'name': name, 'loop': hdr, 'ins': []}
            bbs.append(cur)
            continue
        if not s or s.startswith(('.', ';')) or s.endswith(':'):
            continue
        if cur is None:
            cur = {'name': 'entry', 'loop': None, 'ins': []}
            bbs.append(cur)
        cur['ins'].append((s.split()[0], loc))
    return bbs


def budget(bbs, stage_of, weight_of, px_per_wave, lanes=64):
    tab = collections.defaultdict(collections.Counter)
    for bb in bbs:
        w = weight_of(bb)
        if not w:
            continue
        for op, loc in bb['ins']:
            tab[stage_of(loc, bb)][classify(op)] += w
    rows = []
    tot = collections.Counter()
    for st, c in sorted(tab.items(), key=lambda kv: -(kv[1]['valu'] + kv[1]['valu_f64'])):
        tot.update(c)
        rows.append((st, c))
    out = {'stages': {}, 'px_per_wave': px_per_wave}
    hdr = f"{'stage':34s} {'VALU f64':>9s} {'VALU other':>10s} {'SALU':>7s} {'LDS':>6s} {'VMEM':>6s} {'VALU lane-ops/px':>17s}"
    print(hdr)
    for st, c in rows + [('TOTAL', tot)]:
        v = c['valu'] + c['valu_f64']
        print(f"{st:34s} {c['valu_f64']:9.1f} {c['valu']:10.1f} {c['salu']:7.1f} {c['lds']:6.1f} {c['vmem']:6.1f} "
              f"{v * lanes / px_per_wave:17.2f}")
        out['stages'][st] = {k: round(c[k], 2) for k in ('valu_f64', 'valu', 'salu', 'lds', 'vmem')}
        out['stages'][st]['valu_lane_ops_per_px'] = round(v * lanes / px_per_wave, 2)
    return out


def inv_budget():
    """k_inv_fast<4:2:0, 0> (64 x 128 px tile, 512 threads = 8 waves): per wave,
    2 luma rounds (64 blocks each), the chroma window's 2 planes (loop of 2),
    the exact fallback (jds_inv_exact.hpp) not run on the fast path."""
    asm = listing('jds_inv_fast.hip', '/tmp/stage_inv.s', ['-DJDS_PROBE_NOFALLBACK'])
    key = [ln for ln in asm.split('\n') if ln.startswith('_ZN3jds10k_inv_fastILi2ELi0E') and ln.split(';')[0].strip().endswith(':')][0]
    bbs = blocks(asm, key.split(';')[0].strip())
    src = os.path.join(CSRC, 'jds_inv_fast.hip')
    fr = func_ranges(src, ['aan8', 'fast_col', 'fast_row', 'chroma8_fast', 'fvsum', 'fhsum', 'col_b', 'col_gt',
                           'col_r', 'col_g', 'byte_cert_y', 'pack4', 'inv_fast_tile'])
    text = open(src).read().split('\n')
    mark = {k: next(i + 1 for i, l in enumerate(text) if k in l) for k in
            ('---- 1. chroma window', '---- 2. luma rounds', '---- 3. certification')}

    def within(line, name):
        a, b = fr.get(name, (0, -1))
        return a <= line <= b

    def stage_of(loc, bb):
        f, line = loc
        if f in ('jds_inv_exact.hpp', 'jds_dct8.hpp'):
            return 'exact fallback (not on fast path)'
        if f == 'jds_inv_common.hpp':
            return 'coefficient loads (load_col)'
        if f != 'jds_inv_fast.hip':
            return 'runtime helpers (shuffles, atomics)'
        if within(line, 'aan8'):
            return 'IDCT (AAN lines)'
        if within(line, 'fast_col'):
            return 'dequantise + Dmax (fast_col)'
        if within(line, 'fast_row'):
            return 'IDCT row loads + clip (fast_row)'
        if within(line, 'chroma8_fast') or within(line, 'fvsum') or within(line, 'fhsum'):
            return 'upsample (chroma8_fast)'
        if any(within(line, n) for n in ('col_b', 'col_gt', 'col_r', 'col_g')):
            return 'colour on the magic grid'
        if within(line, 'byte_cert_y') or within(line, 'pack4'):
            return 'byte + certificate + pack'
        if within(line, 'inv_fast_tile'):
            if line < mark['---- 1. chroma window']:
                return 'tile setup (tables)'
            if line < mark['---- 2. luma rounds']:
                return 'chroma window (indexing, ring, LDS)'
            if line < mark['---- 3. certification']:
                return 'luma rounds (indexing, Yv, stores)'
            return 'tile certificate reduction'
        return 'kernel prologue / item logic'

    # the two loops of the fast path run twice per wave: the chroma plane loop
    # (its body holds fast_col) and the luma round loop (chroma8_fast); any other
    # loop (the ring column replication) is rare
    trips = collections.Counter()
    for bb in bbs:
        if bb['loop'] and any(f == 'jds_inv_fast.hip' and (within(l, 'fast_col') or within(l, 'chroma8_fast'))
                              for _, (f, l) in bb['ins']):
            trips[bb['loop']] = 2

    def weight_of(bb):
        fs = [f for _, (f, l) in bb['ins']]
        if fs and all(f in ('jds_inv_exact.hpp', 'jds_dct8.hpp') for f in fs):
            return 0.0
        return float(trips.get(bb['loop'], 1)) if bb['loop'] else 1.0

    print('k_inv_fast<4:2:0,0>: per wave (64 lanes x 2 rounds x 8 px = 1024 px of the tile)')
    return budget(bbs, stage_of, weight_of, px_per_wave=1024)


def fwd_budget():
    """k_fwd32i<4:2:0, prefilter> (32 x 64 px tile, 384 threads = 6 waves): stage 1
    (34 row segments x 8 lanes = 272 lanes) runs on waves 0-4, the luma column
    path on waves 0-3 (256 lanes), the chroma sample rows + row DCT + column path
    on waves 4-5; every wave flushes statistics.  Weights are per average wave."""
    asm = listing('jds_fast.hip', '/tmp/stage_fwd.s')
    key = [ln for ln in asm.split('\n') if ln.startswith('_ZN3jds8k_fwd32iILi2ELb1ELb0E') and ln.split(';')[0].strip().endswith(':')][0]
    bbs = blocks(asm, key.split(';')[0].strip())
    src = os.path.join(CSRC, 'jds_fast.hip')
    fr = func_ranges(src, ['fdct8_f32', 'quant8', 'pack_q', 'flag_block_list', 'stats_flush_ticket', 'byte_at',
                           'k_fwd32i'])
    text = open(src).read().split('\n')
    k0 = fr['k_fwd32i'][0]

    def at(pat, start=k0):
        return next(i + 1 for i, l in enumerate(text) if i + 1 >= start and pat in l)
    s1 = at('---- 1. row segments')
    s2 = at('---- 2./3. column passes')
    col0 = at('auto column = [&]')
    col1 = at('if constexpr (SUB) {', col0)
    luma_line = at('column(s_y + by_t * 8 * TW', col1)
    chroma0 = luma_line + 1
    chroma1 = at('column(s_cd + (blk - C::NYB) * BS32', chroma0)
    fcommon = func_ranges(os.path.join(CSRC, 'jds_fwd_common.hpp'), ['luma32m', 'cb32', 'cr32'])

    def within(line, name, ranges=fr):
        a, b = ranges.get(name, (0, -1))
        return a <= line <= b

    def stage_of(loc, bb):
        f, line = loc
        if f == 'jds_fwd_common.hpp':
            return 'colour (luma32m / cb32 / cr32)'
        if f == 'jds_device.hpp':
            return 'statistics flush (row sums)'
        if f != 'jds_fast.hip':
            return 'runtime helpers (shuffles, atomics, ballots)'
        if within(line, 'fdct8_f32'):
            return 'DCT (fdct8_f32: rows, columns, chroma rows)'
        if within(line, 'byte_at'):
            return 'byte extraction'
        if within(line, 'quant8'):
            return 'quantise + certify + statistics'
        if within(line, 'pack_q'):
            return 'int16 pack'
        if within(line, 'flag_block_list'):
            return 'fix-up list'
        if within(line, 'stats_flush_ticket'):
            return 'statistics flush'
        if s1 <= line < s2:
            return 'stage 1: loads, LDS stores, chroma taps'
        if col0 <= line < col1:
            return 'column pass: LDS reads, transpose, store'
        if chroma0 <= line <= chroma1:
            return 'chroma sample rows (vertical taps)'
        if s2 <= line:
            return 'stage 2: indexing'
        return 'prologue (tables, stats reset)'

    # hipcc tail-merges the two inlined column passes (luma and chroma lanes run
    # one copy after the branch), so only stage 1 (waves 0-4: 272 row-segment
    # lanes) and the chroma sample rows + chroma row DCT (waves 4-5) are partial;
    # the rare-bin branches of quant8 (|q| outside [-12, 19]) run in the waves
    # whose lanes hold such a value -- at Q50 the DC row of most luma blocks
    # (weight 1 for k = 0, RARE for the other 7 positions, from the frame-0
    # histogram of the bench input: see the printed note)
    RARE = 0.25
    qa, qb = fr['quant8']
    rare_lines = set(range(qa, qb + 1)) & set(i + 1 for i, l in enumerate(text) if 'atomicAdd(&s_st[2 +' in l or
                                                    'ls.hn -= 1u << (o & 28u);' in l or 'if (o >= 32u) {' in l)

    def weight_of(bb):
        lines = [l for _, (f, l) in bb['ins'] if f == 'jds_fast.hip']
        if any(s1 <= l < s2 for l in lines):
            return 5 / 6
        if lines and all(l in rare_lines for l in lines):
            return RARE
        if any(chroma0 <= l <= chroma1 for l in lines) and not any(col0 <= l < col1 for l in lines):
            return 2 / 6
        return 1.0

    print('k_fwd32i<4:2:0,pf>: per average wave (6 waves per 32 x 64 px tile: 341.3 px per wave)')
    return budget(bbs, stage_of, weight_of, px_per_wave=2048 / 6)


if __name__ == '__main__':
    which = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].startswith('--') else 'both'
    res = {}
    if which in ('inv', 'both'):
        res['k_inv_fast<2,0>'] = inv_budget()
        print()
    if which in ('fwd', 'both'):
        res['k_fwd32i<2,true>'] = fwd_budget()
    if '--json' in sys.argv:
        json.dump(res, open(sys.argv[sys.argv.index('--json') + 1], 'w'), indent=1)
