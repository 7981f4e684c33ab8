#!/usr/bin/env python3
"""Rigorous error bound for the certified fast inverse (csrc/jds_inv_fast.hip),
modelling the operation order the kernel SHIPS (v24).

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
  * chroma upsample (chroma8_fast): 4:2:0 vertical blend a * 0.25 + b * 0.75,
    then the horizontal difference form near + (far - near) * (+-0.25);
  * colour on the magic grid (byte_cert_y): Yv = Y' + (MAGIC + 128), then
    B = Yv + Cb * 1.772, Gt = Yv + Cb * -0.344136, R = Yv + Cr * 1.402,
    G = Gt + Cr * -0.714136.  Each of those results lies in [2^20, 2^21) where
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
    colour = sorted(float(v) for v in re.findall(r'M::mad\(c[br], (-?\d\.\d+), ', src))
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
        v = x
        if mode == '4:2:0':  # a * 0.25 + b * 0.75 (two independent samples)
            v = add(mul(x, QUARTER, exact_product=True), mul(x, THREEQ)); v.cap = x.cap
        w = fresh(v.cap, v.el, v.ec)
        dlt = add(v, w, -1)  # far - near
        h = add(mul(dlt, QUARTER, exact_product=True), w); h.cap = x.cap  # near + (far - near) * (+-1/4)
        return h
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

        def prod(k):  # C * kd, fused into the grid add or rounded on its own (counted)
            return mul(C, k, float(k))
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


if __name__ == '__main__':
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
