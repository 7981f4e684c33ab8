#!/usr/bin/env python3
"""Rigorous error bound for the certified fast inverse (csrc/jds_inv_fast.hip),
modelling the operation order the kernel SHIPS (v25).

The fast inverse computes every output value v of the reconstruction
(reference engines/pipeline.py:68-95: dequantize, idctn, +128, clip, cv2
INTER_LINEAR upsample, ycbcr_to_rgb) in fp64 in a cheaper order than the
reference.  The reference's byte is trunc(clip(v_ref, 0, 255)); the fast
kernel's byte equals it whenever no integer lies within E of v_fast, where
E >= |v_fast - v_ref|.  Both values approximate the same real number v* (the
whole chain in exact arithmetic with the exact real constants), so
E = e_fast + e_ref with e_x >= |v_x - v*|.

The kernel's chain (jds_inv_fast.hip), as modelled here:
  * dequantisation with the folded table qs[u][v] = ((Q * a_u) * a_v) * 0.125
    (a_k = c_aan[k], the doubles in the source), one product q * qs;
  * AAN 8-point IDCT along axis 0, then axis 1 (aan8, the source's doubles
    F_SQ2 / F_A2C2 / F_K10 / F_K12), NO +128, clip to [-128, 127] in both
    planes (fast_row<-128>);
  * chroma upsample (chroma8_fast) unnormalised: 4:2:0 vertical a + b * 3
    (4x the blend a * 0.25 + b * 0.75), then horizontal far + near * 3 (4x
    again): the upsampled chroma is carried at scale S = 16 (4:2:0), 4 (4:2:2)
    or 1 (4:4:4, no blend);
  * colour on the magic grid (byte_cert_y): Yv = Y' + (MAGIC + 128), then
    B = Yv + Cb * (1.772 / S), Gt = Yv + Cb * (-0.344136 / S),
    R = Yv + Cr * (1.402 / S), G = Gt + Cr * (-0.714136 / S) (the constants'
    scaling by a power of two is exact).  Each of those results lies in [2^20, 2^21) where
    the fp64 spacing is 2^-32, so each of their roundings costs <= 2^-33
    ABSOLUTE, whatever the value; G has 3 of them, R and B 2.  The kernel adds
    2^-31 (= 4 * 2^-33) to E for them; everything else (the products C * k,
    whether fused or not, the constants' representation errors, every rounding
    before the grid) is the non-grid error this tool bounds.

Model: every value carries its exact linear form over the 64 dequantised
coefficients D_uv = q_uv * Q_uv of its block (plus a constant), and an affine
error bound e = e_lin * Dmax + e_const, where Dmax >= max |D_uv| over the
coefficients the tile reads (the kernel measures max |q| * max Q).  Rounding a
result r costs u * M(r) with M(r) = Dmax * sum|L| + |const| >= |r| (u = 2^-53,
round to nearest); every fused multiply-add is modelled as two roundings (a
fused pair rounds once: fl(ab + c) errs by u|ab + c| <= u|ab| + u|fl(ab) + c|,
so whatever the compiler fuses under `fp contract(fast)` stays inside the
bound); a constant k_d standing for the real k adds |k_d - k| * M(operand),
with |k_d - k| computed exactly from the source's double (Fraction) against k
to 50 digits (Decimal).  Clip is 1-Lipschitz and bounds the magnitude; the
upsample is a convex combination.

The reference chain: pocketfft's DCT-III order (csrc/jds_dct8.hpp dct3_line,
its tabulated twiddles, three of which are 1 ulp off -- again exact
representation errors), fct 1/16 (exact) and +128 in one rounding, clip to
[0, 255], cv2's horizontal then vertical blend (float32 weights 0.25 / 0.75,
exact), NumPy's colour expressions (cr - 128, product, sum; g left to right).

Output: (e_lin, e_const) for both chains and K_LIN / K_CONST = 2 * (sums): the
factor 2 is a safety margin.  tests/test_inv_bound_cpu.py asserts the kernel's
constants are at least these and checks the chain itself against the oracle
(jds_selftest_inv_fast).
"""
import math
import os
import re
import sys
from decimal import Decimal, getcontext
from fractions import Fraction

import numpy as np

U = 2.0 ** -53
GRID_ROUNDING = 2.0 ** -33     # one rounding on the magic grid (spacing 2^-32)
GRID_ROUNDINGS_MAX = 3         # G: Yv, Gt, G
KERNEL_GRID_SLACK = 2.0 ** -31  # what jds_inv_fast.hip adds to E for them

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), 'jpeg-dsp-studio_amd', 'csrc')

# ---- exact real constants ---------------------------------------------------

getcontext().prec = 60
_PI = Decimal('3.14159265358979323846264338327950288419716939937510582097494459')


def _dcos(x: Decimal) -> Decimal:
    """cos(x) to the context precision (Taylor series; |x| <= pi)."""
    s, t, k = Decimal(1), Decimal(1), 0
    while True:
        k += 2
        t = -t * x * x / (k * (k - 1))
        if abs(t) < Decimal(10) ** -58:
            return s + t
        s += t


def cos_pi(num: int, den: int) -> Fraction:
    """cos(num * pi / den) as a Fraction accurate to ~1e-55."""
    return Fraction(_dcos(_PI * num / den))


SQRT2 = Fraction(Decimal(2).sqrt())


def rep_err(kd: float, k: Fraction) -> float:
    """|kd - k| exactly (as a float rounded up a little)."""
    return float(abs(Fraction(kd) - k)) * (1 + 1e-12)


# ---- the doubles the kernels use, read from the shipped sources --------------

def _hexconsts(path):
    out = {}
    for m in re.finditer(r'constexpr double (\w+) = (0x[0-9a-fA-F.]+p[-+]?\d+)', open(path).read()):
        out[m.group(1)] = float.fromhex(m.group(2))
    return out


def kernel_constants():
    src = open(os.path.join(CSRC, 'jds_inv_fast.hip')).read()
    c = _hexconsts(os.path.join(CSRC, 'jds_inv_fast.hip'))
    m = re.search(r'#define JDS_AAN_LIST((?:[^\n]*\\\n)*[^\n]*)\n', src)
    aan = [float.fromhex(t) if t.startswith('0x') else float(t)
           for t in (x.strip() for x in m.group(1).replace('\\\n', ' ').split(','))]
    assert len(aan) == 8, aan
    klin = re.search(r'constexpr double K_LIN = ([0-9.e+-]+) \* ([0-9.]+);', src)
    kcon = re.search(r'constexpr double K_CONST = ([0-9.e+-]+) \* ([0-9.]+);', src)
    colour = sorted(float(v) for v in re.findall(r'M::mad\(c[br], (-?\d\.\d+) \* USC<SH>, ', src))
    return {'aan': aan, 'F_SQ2': c['F_SQ2'], 'F_A2C2': c['F_A2C2'], 'F_K10': c['F_K10'], 'F_K12': c['F_K12'],
            'MAGIC': c.get('MAGIC'), 'K_LIN': float(klin.group(1)) * float(klin.group(2)),
            'K_CONST': float(kcon.group(1)) * float(kcon.group(2)), 'colour': colour}


def pocketfft_constants():
    return _hexconsts(os.path.join(CSRC, 'jds_dct8.hpp'))


# ---- values with linear forms and affine error bounds ------------------------

class V:
    """A value: exact linear form L (64 coefficient weights), constant part,
    error bound (lin, const) in units of (Dmax, 1), and an optional magnitude
    cap (after clip / for convex combinations of capped values)."""

    def __init__(self, L, c=0.0, el=0.0, ec=0.0, cap=None):
        self.L, self.c, self.el, self.ec, self.cap = L, c, el, ec, cap

    def mag(self):  # (lin, const) bound on |computed value|
        if self.cap is not None:
            return 0.0, self.cap + self.ec + 1e-6
        return float(np.abs(self.L).sum()) + self.el, abs(self.c) + self.ec

    def rnd(self):  # one rounding of this value
        ml, mc = self.mag()
        self.el += U * ml * (1 + 1e-12)
        self.ec += U * mc * (1 + 1e-12)
        return self


def add(a, b, s=1.0):
    cap = None if a.cap is None or b.cap is None else a.cap + b.cap
    return V(a.L + s * b.L, a.c + s * b.c, a.el + b.el, a.ec + b.ec, cap).rnd()


def mul(a, k: Fraction, kd: float = None, exact_product=False):
    """a * kd where kd is the double standing for the real k: propagated error
    |kd| * e(a), representation error |kd - k| * M(a), and one rounding (none
    when the product is exact, e.g. a power of two)."""
    kd = float(k) if kd is None else kd
    kf = float(k)
    ml, mc = a.mag()
    re_ = rep_err(kd, k)
    cap = None if a.cap is None else abs(kd) * a.cap
    r = V(a.L * kf, a.c * kf, abs(kd) * a.el + re_ * ml, abs(kd) * a.ec + re_ * mc, cap)
    return r if exact_product else r.rnd()


def const_add(a, k: float):  # a + k, k exactly representable
    cap = None if a.cap is None else a.cap + abs(k)
    return V(a.L.copy(), a.c + k, a.el, a.ec, cap).rnd()


def clip(a, lo, hi):
    return V(a.L, a.c, a.el, a.ec, cap=float(max(abs(lo), abs(hi))))


def fresh(cap, el, ec):
    """A value known only by magnitude and error (a clipped sample)."""
    return V(np.zeros(64), 0.0, el, ec, cap=cap)


F = Fraction
QUARTER, THREEQ = F(1, 4), F(3, 4)
UPSAMPLE_SCALE = {'4:4:4': 1, '4:2:2': 4, '4:2:0': 16}  # the fast chain's unnormalised chroma


# ---- 8-point transforms on V ---------------------------------------------------

def aan_line(v, K):
    """jds_inv_fast.hip aan8, operation for operation; FMAs as two roundings."""
    sq2 = SQRT2
    a2c2 = 2 * cos_pi(1, 8)
    k10 = 2 * (cos_pi(1, 8) - cos_pi(3, 8))
    k12 = 2 * (cos_pi(1, 8) + cos_pi(3, 8))
    t10 = add(v[0], v[4]); t11 = add(v[0], v[4], -1)
    t13 = add(v[2], v[6])
    t12 = add(mul(add(v[2], v[6], -1), sq2, K['F_SQ2']), t13, -1)
    e0 = add(t10, t13); e3 = add(t10, t13, -1); e1 = add(t11, t12); e2 = add(t11, t12, -1)
    z13 = add(v[5], v[3]); z10 = add(v[5], v[3], -1); z11 = add(v[1], v[7]); z12 = add(v[1], v[7], -1)
    o7 = add(z11, z13)
    o11 = mul(add(z11, z13, -1), sq2, K['F_SQ2'])
    z5 = mul(add(z10, z12), a2c2, K['F_A2C2'])
    o10 = add(z5, mul(z12, k10, K['F_K10']), -1)
    o12 = add(z5, mul(z10, k12, K['F_K12']), -1)
    o6 = add(o12, o7, -1); o5 = add(o11, o6, -1); o4 = add(o10, o5, -1)
    return [add(e0, o7), add(e1, o6), add(e2, o5), add(e3, o4),
            add(e3, o4, -1), add(e2, o5, -1), add(e1, o6, -1), add(e0, o7, -1)]


def pocket_dct3(c, P):
    """csrc/jds_dct8.hpp dct3_line (pocketfft's order and tabulated twiddles)."""
    tw = [cos_pi(2 * (i + 1), 32) for i in range(7)]
    twd = [P[f'TW{i}'] for i in range(7)]
    w8r, w8i = cos_pi(1, 4), cos_pi(1, 4)  # cos / sin (2 pi / 8)
    c = list(c)
    c[0] = mul(c[0], SQRT2, P['SQRT2'])
    t1 = add(c[1], c[7]); t2 = add(c[1], c[7], -1)
    c[1] = add(mul(t2, tw[0], twd[0]), mul(t1, tw[6], twd[6])); c[7] = add(mul(t1, tw[0], twd[0]), mul(t2, tw[6], twd[6]), -1)
    t1 = add(c[2], c[6]); t2 = add(c[2], c[6], -1)
    c[2] = add(mul(t2, tw[1], twd[1]), mul(t1, tw[5], twd[5])); c[6] = add(mul(t1, tw[1], twd[1]), mul(t2, tw[5], twd[5]), -1)
    t1 = add(c[3], c[5]); t2 = add(c[3], c[5], -1)
    c[3] = add(mul(t2, tw[2], twd[2]), mul(t1, tw[4], twd[4])); c[5] = add(mul(t1, tw[2], twd[2]), mul(t2, tw[4], twd[4]), -1)
    c[4] = mul(c[4], 2 * tw[3], 2 * twd[3])
    r1 = add(c[6], c[2]); g2 = add(c[6], c[2], -1)
    r2 = add(c[0], c[4]); g1 = add(c[0], c[4], -1)
    g0 = add(r2, r1); g3 = add(r2, r1, -1)
    r1 = add(c[7], c[3]); g6 = add(c[7], c[3], -1)
    r2 = add(c[1], c[5]); g5 = add(c[1], c[5], -1)
    g4 = add(r2, r1); g7 = add(r2, r1, -1)
    o0 = add(g0, g4); o7 = add(g0, g4, -1)
    o4 = mul(g7, F(-1), exact_product=True); o3 = g3
    q2 = add(mul(g5, w8r, P['W8R']), mul(g6, w8i, P['W8I']))
    qi = add(mul(g6, w8r, P['W8R']), mul(g5, w8i, P['W8I']), -1)
    o1 = add(g1, q2); o5 = add(g1, q2, -1); o2 = add(qi, g2); o6 = add(qi, g2, -1)
    return [o0, add(o1, o2, -1), add(o2, o1), add(o3, o4, -1), add(o4, o3), add(o5, o6, -1), add(o6, o5), o7]


def idct_matrix():
    """Orthonormal 8-point IDCT: x[n] = sum_k C[n][k] X[k]."""
    C = np.zeros((8, 8))
    for n in range(8):
        for k in range(8):
            C[n, k] = math.sqrt((1 if k == 0 else 2) / 8) * math.cos((2 * n + 1) * k * math.pi / 16)
    return C


def block_bound(chain, K, P):
    """Worst error over the 64 outputs of one 8x8 block IDCT for |D_uv| <= Dmax,
    before the clip; returns (el, ec) of the worst sample and checks the linear
    forms against the orthonormal IDCT (the chain computes the right function)."""
    basis = [[V(np.eye(64)[u * 8 + v].copy()) for v in range(8)] for u in range(8)]
    if chain == 'fast':
        A = [F(1)] + [SQRT2 * cos_pi(k, 16) for k in range(1, 8)]  # exact a_k
        d = [[None] * 8 for _ in range(8)]
        for u in range(8):
            for v in range(8):
                k = A[u] * A[v] / 8
                # qs = ((Q * a_u) * a_v) * 0.125: relative error of the table entry
                # (both a's representation errors, two roundings; * 0.125 exact),
                # then one rounding of q * qs
                rel = (rep_err(K['aan'][u], A[u]) / float(A[u]) + rep_err(K['aan'][v], A[v]) / float(A[v])
                       + 2 * U) * (1 + 1e-9)
                x = V(np.eye(64)[u * 8 + v] * float(k), 0.0, float(k) * rel, 0.0)
                d[u][v] = x.rnd()
        cols = [aan_line([d[u][v] for u in range(8)], K) for v in range(8)]  # axis 0
        out = [aan_line([cols[v][m] for v in range(8)], K) for m in range(8)]  # axis 1: out[row][col]
    else:
        # the reference: 16x operands (exact power-of-two scale), dct3 on axis 0
        # then axis 1, then x * (1/16) + 128 in one rounding (exact scale)
        cols = [pocket_dct3([basis[u][v] for u in range(8)], P) for v in range(8)]
        rows = [pocket_dct3([cols[v][m] for v in range(8)], P) for m in range(8)]
        out = [[const_add(mul(x, F(1, 16), exact_product=True), 128.0) for x in r] for r in rows]
    Cm = idct_matrix()
    for m in range(8):
        for n in range(8):
            want = np.kron(Cm[m], Cm[n])  # out[m][n] = sum_uv C[m][u] C[n][v] D_uv
            got = out[m][n].L
            assert np.abs(got - want).max() < 1e-12, (chain, m, n)
    worst = (0.0, 0.0)
    for r in out:
        for x in r:
            if x.el * 2048 + x.ec > worst[0] * 2048 + worst[1]:
                worst = (x.el, x.ec)
    return worst


def upsample_bound(x, chain, mode):
    """Error of one upsampled chroma value from window samples with error x."""
    if mode == '4:4:4':
        return x
    if chain == 'fast':
        # unnormalised sums (caps follow: 4x per blended axis): the colour
        # constants carry the 1 / S (UPSAMPLE_SCALE)
        v = x
        if mode == '4:2:0':  # a + b * 3 (two independent samples)
            v = add(fresh(x.cap, x.el, x.ec), mul(x, F(3)))
        w = fresh(v.cap, v.el, v.ec)
        return add(w, mul(v, F(3)))  # far + near * 3
    # cv2 HResizeLinear then VResizeLinear: S0 * a0 + S1 * a1 (products rounded, sum rounded)
    h = add(mul(x, QUARTER), mul(x, THREEQ)); h.cap = x.cap
    if mode == '4:2:0':
        h = add(mul(h, QUARTER), mul(h, THREEQ)); h.cap = x.cap
    return h


def colour_bound(ey, ec_, chain, mode):
    """Non-grid error of R, G, B (worst channel) from the clipped Y (error ey)
    and clipped chroma samples (error ec_)."""
    kr, kgb, kgr, kb = F('1.402'), F('0.344136'), F('0.714136'), F('1.772')
    if chain == 'fast':
        Y = fresh(128.0, *ey)      # Y' = clip(AAN, -128, 127); +128 rides on the grid
        C = upsample_bound(fresh(128.0, *ec_), 'fast', mode)

        sc = UPSAMPLE_SCALE[mode]

        def prod(k):  # C * (kd / S), fused into the grid add or rounded on its own (counted)
            return mul(C, k / sc, float(k) / sc)
        R = V(np.zeros(64), 0, Y.el + prod(kr).el, Y.ec + prod(kr).ec)
        B = V(np.zeros(64), 0, Y.el + prod(kb).el, Y.ec + prod(kb).ec)
        G = V(np.zeros(64), 0, Y.el + prod(kgb).el + prod(kgr).el, Y.ec + prod(kgb).ec + prod(kgr).ec)
    else:
        Y = fresh(255.0, *ey)
        C = upsample_bound(fresh(255.0, *ec_), 'ref', mode)
        cs = const_add(C, -128.0); cs.cap = 128.0
        R = add(Y, mul(cs, kr, 1.402))
        B = add(Y, mul(cs, kb, 1.772))
        G = add(add(Y, mul(cs, kgb, 0.344136), -1), mul(cs, kgr, 0.714136), -1)
    return max(((x.el, x.ec) for x in (R, G, B)), key=lambda t: t[0] * 2048 + t[1])


# ---- 16x16 blocks (BASELINE configs[4] stretch): k_inv16_fast vs k_inv16s -----

def kernel_constants16():
    """The 16-point fast chain's doubles and K_LIN16 / K_CONST16, read from
    jds_inv_fast.hip (odd-part pre- and post-scales of fidct16)."""
    src = open(os.path.join(CSRC, 'jds_inv_fast.hip')).read()

    def lst(name):
        m = re.search(r'#define ' + name + r'((?:[^\n]*\\\n)*[^\n]*)\n', src)
        return [float.fromhex(t) for t in (x.strip() for x in m.group(1).replace('\\\n', ' ').split(','))]
    klin = re.search(r'constexpr double K_LIN16 = ([0-9.e+-]+) \* ([0-9.]+);', src)
    kcon = re.search(r'constexpr double K_CONST16 = ([0-9.e+-]+) \* ([0-9.]+);', src)
    out = {'pre': lst('JDS_F16_PRE_LIST'), 'post': lst('JDS_F16_POST_LIST'),
           'K_LIN16': float(klin.group(1)) * float(klin.group(2)) if klin else None,
           'K_CONST16': float(kcon.group(1)) * float(kcon.group(2)) if kcon else None}
    assert len(out['pre']) == 7 and len(out['post']) == 8, out
    return out


def pocketfft16_constants():
    """csrc/jds_dct16.hpp's doubles: DT16[15], WR[3], WI[3], SQRT2, HSQT2."""
    src = open(os.path.join(CSRC, 'jds_dct16.hpp')).read()
    out = {}
    for m in re.finditer(r'constexpr double (\w+)\[(\d+)\] = \{([^}]*)\};', src):
        out[m.group(1)] = [float.fromhex(t.strip()) for t in m.group(3).split(',')]
        assert len(out[m.group(1)]) == int(m.group(2))
    for m in re.finditer(r'constexpr double (\w+) = (0x[0-9a-fA-F.]+p[-+]?\d+);', src):
        out[m.group(1)] = float.fromhex(m.group(2))
    return out


def fast16_line(v, K, K16):
    """jds_inv_fast.hip fidct16: the even half through aan8 (inputs pre-scaled
    a_m / 4 by the table), the odd half by Lee's identity: W_0 = Z_0,
    W_j = (Z_{j-1} + Z_j) cos(j pi / 16), aan8, then x_n = E_n + W_n p_n and
    x_{15-n} = E_n - W_n p_n with p_n = sqrt(2) / (8 cos((2n+1) pi / 32))."""
    e = aan_line([v[2 * m] for m in range(8)], K)
    w = [v[1]] + [mul(add(v[2 * j - 1], v[2 * j + 1]), cos_pi(j, 16), K16['pre'][j - 1]) for j in range(1, 8)]
    w = aan_line(w, K)
    out = [None] * 16
    for n in range(8):
        o = mul(w[n], SQRT2 / (8 * cos_pi(2 * n + 1, 32)), K16['post'][n])  # fused or not: two roundings
        out[n] = add(e[n], o)
        out[15 - n] = add(e[n], o, -1)
    return out


def _radf4(IDO, L1, cc, D):
    """jds_dct16.hpp radf4<IDO, L1> on V values (pocketfft's rfftp forward radix 4)."""
    ch = [None] * 16

    def CC(a, b, c):
        return cc[a + IDO * (b + L1 * c)]

    def CH(a, b, c, val):
        ch[a + IDO * (b + 4 * c)] = val
    hs = SQRT2 / 2
    wr = [cos_pi(j, 8) for j in (1, 2, 3)]
    wi = [cos_pi(4 - j, 8) for j in (1, 2, 3)]  # sin(j pi / 8)
    for k in range(L1):
        tr1 = add(CC(0, k, 3), CC(0, k, 1))
        CH(0, 2, k, add(CC(0, k, 3), CC(0, k, 1), -1))
        tr2 = add(CC(0, k, 0), CC(0, k, 2))
        CH(IDO - 1, 1, k, add(CC(0, k, 0), CC(0, k, 2), -1))
        CH(0, 0, k, add(tr2, tr1))
        CH(IDO - 1, 3, k, add(tr2, tr1, -1))
    if IDO == 4:
        for k in range(L1):
            ti1 = mul(add(CC(3, k, 1), CC(3, k, 3)), -hs, -D['HSQT2'])
            tr1 = mul(add(CC(3, k, 1), CC(3, k, 3), -1), hs, D['HSQT2'])
            CH(3, 0, k, add(CC(3, k, 0), tr1))
            CH(3, 2, k, add(CC(3, k, 0), tr1, -1))
            CH(0, 3, k, add(ti1, CC(3, k, 2)))
            CH(0, 1, k, add(ti1, CC(3, k, 2), -1))
        for k in range(L1):
            def rot(idx, j):  # (WR a + WI b, WR b - WI a) of (a, b) = (CC(1, k, idx), CC(2, k, idx))
                a, b = CC(1, k, idx), CC(2, k, idx)
                cr = add(mul(a, wr[j], D['WR'][j]), mul(b, wi[j], D['WI'][j]))
                ci = add(mul(b, wr[j], D['WR'][j]), mul(a, wi[j], D['WI'][j]), -1)
                return cr, ci
            cr2, ci2 = rot(1, 0)
            cr3, ci3 = rot(2, 1)
            cr4, ci4 = rot(3, 2)
            tr1 = add(cr4, cr2); tr4 = add(cr4, cr2, -1)
            ti1 = add(ci2, ci4); ti4 = add(ci2, ci4, -1)
            tr2 = add(CC(1, k, 0), cr3); tr3 = add(CC(1, k, 0), cr3, -1)
            ti2 = add(CC(2, k, 0), ci3); ti3 = add(CC(2, k, 0), ci3, -1)
            CH(1, 0, k, add(tr2, tr1)); CH(1, 3, k, add(tr2, tr1, -1))
            CH(2, 0, k, add(ti1, ti2)); CH(2, 3, k, add(ti1, ti2, -1))
            CH(1, 2, k, add(tr3, ti4)); CH(1, 1, k, add(tr3, ti4, -1))
            CH(2, 2, k, add(tr4, ti3)); CH(2, 1, k, add(tr4, ti3, -1))
    return ch


def pocket_dct3_16(c, D):
    """csrc/jds_dct16.hpp dct3_line16 (pocketfft T_dcst23 type 3, N = 16)."""
    dt = [cos_pi(i + 1, 32) for i in range(15)]
    c = list(c)
    c[0] = mul(c[0], SQRT2, D['SQRT2'])
    for k in range(1, 8):
        kc = 16 - k
        t1 = add(c[k], c[kc]); t2 = add(c[k], c[kc], -1)
        c[k] = add(mul(t2, dt[k - 1], D['DT16'][k - 1]), mul(t1, dt[kc - 1], D['DT16'][kc - 1]))
        c[kc] = add(mul(t1, dt[k - 1], D['DT16'][k - 1]), mul(t2, dt[kc - 1], D['DT16'][kc - 1]), -1)
    c[8] = mul(c[8], 2 * dt[7], 2 * D['DT16'][7])
    o = _radf4(4, 1, _radf4(1, 4, c, D), D)
    out = [o[0]] + [None] * 14 + [o[15]]
    for k in range(1, 15, 2):
        out[k] = add(o[k], o[k + 1], -1)
        out[k + 1] = add(o[k + 1], o[k])
    return out


def idct_matrix16():
    C = np.zeros((16, 16))
    for n in range(16):
        for k in range(16):
            C[n, k] = math.sqrt((1 if k == 0 else 2) / 16) * math.cos((2 * n + 1) * k * math.pi / 32)
    return C


def block_bound16(chain, K, K16, D):
    """block_bound for 16 x 16 blocks: the fast chain (((q * Q16) * s_u) * s_v,
    q * Q16 exact, s_2m = a_m / 4, s_2m+1 = 1; fidct16 on axis 0 then axis 1)
    or the exact one (q * Q, dct3_line16 twice, * 1/32 (exact) + 128 in one
    rounding)."""
    N = 256
    if chain == 'fast':
        A = [F(1)] + [SQRT2 * cos_pi(k, 16) for k in range(1, 8)]
        s = [A[k // 2] / 4 if k % 2 == 0 else F(1) for k in range(16)]
        sd = [K['aan'][k // 2] * 0.25 if k % 2 == 0 else 1.0 for k in range(16)]
        d = [[None] * 16 for _ in range(16)]
        for u in range(16):
            for v in range(16):
                k = s[u] * s[v]
                # both scales' representation errors and the rounding of the
                # first product; the second product's rounding is .rnd()
                rel = (rep_err(sd[u], s[u]) / float(s[u]) + rep_err(sd[v], s[v]) / float(s[v]) + U) * (1 + 1e-9)
                d[u][v] = V(np.eye(N)[u * 16 + v] * float(k), 0.0, float(k) * rel, 0.0).rnd()
        cols = [fast16_line([d[u][v] for u in range(16)], K, K16) for v in range(16)]
        out = [fast16_line([cols[v][m] for v in range(16)], K, K16) for m in range(16)]
    else:
        basis = [[V(np.eye(N)[u * 16 + v].copy()) for v in range(16)] for u in range(16)]
        cols = [pocket_dct3_16([basis[u][v] for u in range(16)], D) for v in range(16)]
        rows = [pocket_dct3_16([cols[v][m] for v in range(16)], D) for m in range(16)]
        out = [[const_add(mul(x, F(1, 32), exact_product=True), 128.0) for x in r] for r in rows]
    Cm = idct_matrix16()
    for m in range(16):
        for n in range(16):
            want = np.kron(Cm[m], Cm[n])
            got = out[m][n].L
            assert np.abs(got - want).max() < 1e-12, (chain, m, n, np.abs(got - want).max())
    worst = (0.0, 0.0)
    for r in out:
        for x in r:
            if x.el * 2048 + x.ec > worst[0] * 2048 + worst[1]:
                worst = (x.el, x.ec)
    return worst


def bounds16():
    K, K16, D = kernel_constants(), kernel_constants16(), pocketfft16_constants()
    res = {}
    for chain in ('fast', 'ref'):
        eb = block_bound16(chain, K, K16, D)
        res[chain] = {m: colour_bound(eb, eb, chain, m) for m in ('4:2:2', '4:2:0')}
    worst = {c: max(res[c].values(), key=lambda t: t[0] * 2048 + t[1]) for c in res}
    k_lin = 2 * (worst['fast'][0] + worst['ref'][0])
    k_const = 2 * (worst['fast'][1] + worst['ref'][1])
    return res, k_lin, k_const


def bounds():
    K, P = kernel_constants(), pocketfft_constants()
    res = {}
    for chain in ('fast', 'ref'):
        eb = block_bound(chain, K, P)
        res[chain] = {m: colour_bound(eb, eb, chain, m) for m in ('4:4:4', '4:2:2', '4:2:0')}
    worst = {c: max(res[c].values(), key=lambda t: t[0] * 2048 + t[1]) for c in res}
    k_lin = 2 * (worst['fast'][0] + worst['ref'][0])
    k_const = 2 * (worst['fast'][1] + worst['ref'][1])
    return res, k_lin, k_const


if __name__ == '__main__' and '--b16' in sys.argv:
    res, k_lin, k_const = bounds16()
    K16 = kernel_constants16()
    for chain, per in res.items():
        for m, (el, ec) in per.items():
            print(f'{chain:5s} 16x16 {m}: e <= {el:.4e} * Dmax + {ec:.4e}')
    print(f'model : K_LIN16 = {k_lin:.6e}  K_CONST16 = {k_const:.6e}  (x2 safety included)')
    print(f'kernel: K_LIN16 = {K16["K_LIN16"]}  K_CONST16 = {K16["K_CONST16"]}')
elif __name__ == '__main__':
    res, k_lin, k_const = bounds()
    K = kernel_constants()
    for chain, per in res.items():
        for m, (el, ec) in per.items():
            print(f'{chain:5s} {m}: e <= {el:.4e} * Dmax + {ec:.4e}')
    print(f'model : K_LIN = {k_lin:.6e}  K_CONST = {k_const:.6e}  (x2 safety included)')
    print(f'kernel: K_LIN = {K["K_LIN"]:.6e}  K_CONST = {K["K_CONST"]:.6e}')
    print(f'grid roundings: {GRID_ROUNDINGS_MAX} x 2^-33 = {GRID_ROUNDINGS_MAX * GRID_ROUNDING:.3e} '
          f'<= kernel slack {KERNEL_GRID_SLACK:.3e}')
    print(f'E at Dmax = 1152 (codec output): {k_lin * 1152 + k_const + KERNEL_GRID_SLACK:.3e};  '
          f'at 255*32767: {k_lin * 255 * 32767 + k_const + KERNEL_GRID_SLACK:.3e}')
