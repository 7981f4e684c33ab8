#!/usr/bin/env python3
"""Resolve compile-time A/B knobs in the HIP sources to their shipped values
(VERDICT r04 item 8): every #if / #ifdef / #ifndef / #elif / #else / #endif
whose condition names only the listed knobs is evaluated and removed, the knob
definitions disappear, and remaining uses of a knob's value in code are
replaced by the literal.  Directives naming anything else are left alone.
usage: tools/unknob.py file.hip ... (edits in place)"""
import re
import sys

# shipped values; None = undefined (flag knobs that are off)
KNOBS = {
    'JDS_FOLD_MODE': '1', 'JDS_RING_LAST': '1', 'JDS_F444_WAVE_REC': '1', 'JDS_FIX_REDUCE': '0',
    'JDS_SY_PAD': '0', 'JDS_TABLES_IDLE_WAVE': '1', 'JDS_STAGE_DPP': '1', 'JDS_QUANT8_CLASSIC': None,
    'JDS_FLUSH_BARRIER_TF': '1024', 'JDS_FLUSH_FORM': '5', 'JDS_F444_WPE': '5', 'JDS_RROWS_TILES': '64',
    'JDS_FIX_RED_TILES': '32', 'JDS_FIX_WPE': '5', 'JDS_FIX_GRID': '16384', 'JDS_FLUSH16_WAVE': '1',
    'JDS_Q16_GLOBAL': None, 'JDS_NO_CSPLIT': None, 'JDS_FIX16_WPE': '3', 'JDS_FIX16_GRID': '4096',
    'JDS_INV_QS_T': '1', 'JDS_INV_CERT_DPP': '1', 'JDS_INV_WIN_SEL': '1', 'JDS_INV_EARLY_LOADS': '1',
    'JDS_INV_QMAX_FQ': '1', 'JDS_INV_MIX_PLANES': '1', 'JDS_INV_UNROLL_C': '1', 'JDS_INV_UNROLL_Y': '1',
    'JDS_INV_ONE_BARRIER': '0', 'JDS_CW_PAD': '1', 'JDS_CW_PAD422': '4', 'JDS_COL16_INT': None,
    'JDS_INV16_TWO_WINDOWS': None,
    # retired timing probes of the forward / exact inverse (their measurements are in profiles/r03_*)
    'JDS_PROBE_NOQSTATS': None, 'JDS_PROBE_NORARE': None, 'JDS_PROBE_NOSTATS': None,
    'JDS_PROBE_FLUSH_NOTICKET': None, 'JDS_PROBE_NOLOAD': None, 'JDS_PROBE_STAGE1': None,
    'JDS_PROBE_NOSTORE': None, 'JDS_PFIX_NOSAMPLE': None, 'JDS_PFIX_NOSTAT': None, 'JDS_P16_ST1': None,
    'JDS_P16_NODCT': None, 'JDS_P16_NOQ': None, 'JDS_P16_FLAGSPREAD': None, 'JDS_P16_FIXNONE': None,
    'JDS_P16FIX_NOSAMPLE': None, 'JDS_P16FIX_NODCT': None, 'JDS_P16FIX_NODIV': None, 'JDS_P16FIX_NOSTAT': None,
    'JDS_PROBE_NOCHROMA': None, 'JDS_PROBE_NOUPS': None,
}
TOK = re.compile(r'\b(JDS_[A-Z0-9_]+|defined)\b')


def knob_only(expr):
    names = [t for t in TOK.findall(expr) if t != 'defined']
    return names and all(n in KNOBS for n in names)


def evaluate(expr):
    e = re.sub(r'defined\s*\(\s*(\w+)\s*\)', lambda m: '1' if KNOBS.get(m.group(1)) is not None else '0', expr)
    e = re.sub(r'defined\s+(\w+)', lambda m: '1' if KNOBS.get(m.group(1)) is not None else '0', e)
    e = TOK.sub(lambda m: KNOBS[m.group(1)] if KNOBS[m.group(1)] is not None else '0', e)
    e = e.replace('&&', ' and ').replace('||', ' or ').replace('!', ' not ').replace('not =', '!=')
    e = re.sub(r'//.*', '', e)
    return bool(eval(e))


def process(src):
    out = []
    stack = []  # per open directive: (resolved?, keep_current, taken_already, parent_keep)
    keep = True
    for line in src.split('\n'):
        s = line.strip()
        m = re.match(r'#\s*(ifdef|ifndef|if|elif|else|endif)\b(.*)', s)
        if not m:
            if keep:
                out.append(line)
            continue
        kind, rest = m.group(1), m.group(2).split('//')[0].strip()
        if kind in ('ifdef', 'ifndef', 'if'):
            if kind == 'ifdef':
                expr = f'defined({rest})'
            elif kind == 'ifndef':
                expr = f'!defined({rest})'
            else:
                expr = rest
            if knob_only(expr):
                v = evaluate(expr)
                stack.append(['res', keep, v])
                keep = keep and v
            else:
                stack.append(['raw', keep, None])
                if keep:
                    out.append(line)
        elif kind == 'elif':
            top = stack[-1]
            if top[0] == 'res':
                if knob_only(rest):
                    v = (not top[2]) and evaluate(rest)
                    top[2] = top[2] or v
                    keep = top[1] and v
                else:
                    raise SystemExit(f'mixed #elif: {line}')
            elif keep or top[1]:
                out.append(line)
        elif kind == 'else':
            top = stack[-1]
            if top[0] == 'res':
                keep = top[1] and not top[2]
                top[2] = True
            else:
                if top[1]:
                    out.append(line)
        else:  # endif
            top = stack.pop()
            keep = top[1]
            if top[0] == 'raw' and keep:
                out.append(line)
    assert not stack, 'unbalanced'
    text = '\n'.join(out)
    # remaining uses of knob values in code (not in // comments)
    lines = []
    for ln in text.split('\n'):
        code, sep, com = ln.partition('//')
        for k, v in KNOBS.items():
            if v is not None:
                code = re.sub(r'\b' + k + r'\b', v, code)
        lines.append(code + sep + com)
    return '\n'.join(lines)


if __name__ == '__main__':
    for f in sys.argv[1:]:
        s = open(f).read()
        t = process(s)
        if t != s:
            open(f, 'w').write(t)
            print('resolved', f)
