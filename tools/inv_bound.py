#!/usr/bin/env python3
"""Rigorous error bound for the certified fast inverse (csrc/jds_inv_fast.hip).

The fast inverse computes every output sample v of the reconstruction
(reference engines/pipeline.py:68-95: dequantize, idctn, +128, clip, cv2
INTER_LINEAR upsample, ycbcr_to_rgb) in fp64 with a cheaper operation order
than the reference (AAN IDCT with the scales folded into the dequantisation
table, FMAs, chroma shifted by -128 before the upsample).  The reference's byte
is trunc(clip(v_ref, 0, 255)); the fast kernel's byte equals it whenever no
integer lies within E of v_fast, where E >= |v_fast - v_ref|.  Both values
approximate the same real number v*, so E = e_fast + e_ref with e_x >= |v_x - v*|.

Model: every value carries its exact linear form over the 64 dequantised
coefficients of its block (plus a constant) and an affine error bound
e = e_lin * Dmax + e_const, where Dmax >= max |q * Q| over the coefficients the
tile reads (the kernel measures it).  Rounding of a result r costs u * M(r)
with M(r) = Dmax * sum|L| + |const| >= |r| (u = 2^-53, round to nearest);
every fused multiply-add is modelled as two roundings (conservative); a
constant c carries its representation error u*|c|.  Clip is 1-Lipschitz and
bounds the magnitude; the upsample is a convex combination.

Output: (e_lin, e_const) for the fast and the reference chains and the K_LIN /
K_CONST the kernel uses (their sums times a safety factor of 2).
"""
import math

import numpy as np

U = 2.0 ** -53


class V:
    """A value: exact linear form L (64 coefficient weights), constant part,
    error bound (lin, const) in units of (Dmax, 1), and an optional magnitude
    cap (after clip)."""

    def __init__(self, L, c=0.0, el=0.0, ec=0.0, cap=None):
        self.L, self.c, self.el, self.ec, self.cap = L, c, el, ec, cap

    def mag(self):  # (lin, const) magnitude bound
        if self.cap is not None:
            return 0.0, self.cap
        return float(np.abs(self.L).sum()), abs(self.c)

    def rnd(self):  # one rounding of this value
        ml, mc = self.mag()
        self.el += U * ml * (1 + 1e-12)
        self.ec += U * mc * (1 + 1e-12)
        return self


def add(a, b, s=1.0):
    cap = None if a.cap is None or b.cap is None else a.cap + b.cap
    return V(a.L + s * b.L, a.c + s * b.c, a.el + b.el, a.ec + b.ec, cap).rnd()


def mul(a, k):
    """a * fl(k): exact product with k, plus |k|*u representation error, one rounding."""
    ml, mc = a.mag()
    cap = None if a.cap is None else abs(k) * a.cap
    r = V(a.L * k, a.c * k, abs(k) * a.el + abs(k) * U * ml, abs(k) * a.ec + abs(k) * U * mc, cap)
    return r.rnd()


def const_add(a, k):  # a + fl(k)
    cap = None if a.cap is None else a.cap + abs(k)
    return V(a.L.copy(), a.c + k, a.el, a.ec + U * abs(k), cap).rnd()


def clip(a, lo, hi):
    return V(a.L, a.c, a.el, a.ec, cap=max(abs(lo), abs(hi)))


def fresh(val_cap, el, ec):
    """A value known only by magnitude and error (e.g. a clipped sample)."""
    return V(np.zeros(64), 0.0, el, ec, cap=val_cap)


# ---- 8-point transforms on V ------------------------------------------------

C = [math.cos(k * math.pi / 16) for k in range(8)]
SQ2 = math.sqrt(2.0)


def aan_line(v):
    """The fast IDCT line (jds_inv_fast.hip aan_idct8), FMAs as two roundings."""
    t10 = add(v[0], v[4]); t11 = add(v[0], v[4], -1)
    t13 = add(v[2], v[6]); t12 = add(mul(add(v[2], v[6], -1), SQ2), t13, -1)
    e0 = add(t10, t13); e3 = add(t10, t13, -1); e1 = add(t11, t12); e2 = add(t11, t12, -1)
    z13 = add(v[5], v[3]); z10 = add(v[5], v[3], -1); z11 = add(v[1], v[7]); z12 = add(v[1], v[7], -1)
    o7 = add(z11, z13)
    o11 = mul(add(z11, z13, -1), SQ2)
    z5 = mul(add(z10, z12), 2 * C[2])
    o10 = add(z5, mul(z12, 2 * (C[2] - C[6])), -1)
    o12 = add(z5, mul(z10, 2 * (C[2] + C[6])), -1)
    o6 = add(o12, o7, -1); o5 = add(o11, o6, -1); o4 = add(o10, o5, -1)
    return [add(e0, o7), add(e1, o6), add(e2, o5), add(e3, o4),
            add(e3, o4, -1), add(e2, o5, -1), add(e1, o6, -1), add(e0, o7, -1)]


# pocketfft's DCT-III (csrc/jds_dct8.hpp dct3_line), twiddles as exact reals
TW = [math.cos(2 * math.pi * (i + 1) / 32) for i in range(7)]
W8 = math.cos(2 * math.pi / 8)


def pocket_dct3(c):
    c = list(c)
    c[0] = mul(c[0], SQ2)
    t1 = add(c[1], c[7]); t2 = add(c[1], c[7], -1)
    c[1] = add(mul(t2, TW[0]), mul(t1, TW[6])); c[7] = add(mul(t1, TW[0]), mul(t2, TW[6]), -1)
    t1 = add(c[2], c[6]); t2 = add(c[2], c[6], -1)
    c[2] = add(mul(t2, TW[1]), mul(t1, TW[5])); c[6] = add(mul(t1, TW[1]), mul(t2, TW[5]), -1)
    t1 = add(c[3], c[5]); t2 = add(c[3], c[5], -1)
    c[3] = add(mul(t2, TW[2]), mul(t1, TW[4])); c[5] = add(mul(t1, TW[2]), mul(t2, TW[4]), -1)
    c[4] = mul(c[4], 2 * TW[3])
    r1 = add(c[6], c[2]); g2 = add(c[6], c[2], -1)
    r2 = add(c[0], c[4]); g1 = add(c[0], c[4], -1)
    g0 = add(r2, r1); g3 = add(r2, r1, -1)
    r1 = add(c[7], c[3]); g6 = add(c[7], c[3], -1)
    r2 = add(c[1], c[5]); g5 = add(c[1], c[5], -1)
    g4 = add(r2, r1); g7 = add(r2, r1, -1)
    o0 = add(g0, g4); o7 = add(g0, g4, -1)
    o4 = mul(g7, -1.0); o3 = g3
    q2 = add(mul(g5, W8), mul(g6, W8)); qi = add(mul(g6, W8), mul(g5, W8), -1)
    o1 = add(g1, q2); o5 = add(g1, q2, -1); o2 = add(qi, g2); o6 = add(qi, g2, -1)
    return [o0, add(o1, o2, -1), add(o2, o1), add(o3, o4, -1), add(o4, o3), add(o5, o6, -1), add(o6, o5), o7]


def block_bound(chain):
    """Worst error and magnitude over the 64 outputs of one 8x8 block IDCT
    (+128) for coefficients |d_uv| <= Dmax; returns (el, ec) of the worst sample."""
    basis = [[V(np.eye(64)[u * 8 + v].copy()) for v in range(8)] for u in range(8)]
    if chain == 'fast':
        aan = [1.0] + [C[k] * SQ2 for k in range(1, 8)]
        # dequantisation with the folded table: q * fl(Q * a_u * a_v / 8); the
        # table entry itself carries 4 roundings (host product)
        d = [[None] * 8 for _ in range(8)]
        for u in range(8):
            for v in range(8):
                k = aan[u] * aan[v] / 8
                x = mul(basis[u][v], k)
                x.el += 4 * U * abs(k)  # table entry error (relative 4u) times |q*Q| <= Dmax
                d[u][v] = x
        d[0][0] = const_add(d[0][0], 128.0)  # +128 folded into the DC term
        cols = [aan_line([d[u][v] for u in range(8)]) for v in range(8)]  # axis 0
        out = [aan_line([cols[v][m] for v in range(8)]) for m in range(8)]  # axis 1
    else:
        # the reference: 16x operands (exact power-of-two scale), dct3 on axis 0
        # then axis 1, then fma(x, 1/16, 128) -- one rounding (jds_inv.hip idct_row)
        cols = [pocket_dct3([basis[u][v] for u in range(8)]) for v in range(8)]
        rows = [pocket_dct3([cols[v][m] for v in range(8)]) for m in range(8)]
        out = [[const_add(mul(x, 1.0 / 16.0), 128.0) for x in r] for r in rows]
    worst = (0.0, 0.0)
    for r in out:
        for x in r:
            if x.el + x.ec * 1e-3 > worst[0] + worst[1] * 1e-3:
                worst = (x.el, x.ec)
    return worst


def colour_bound(ey, ec_, chain, mode):
    """Error of R, G, B from clipped Y (error ey) and clipped chroma (error ec_)
    through the upsample and the colour expressions (worst channel)."""
    Y = fresh(255.0, *ey)
    Cb = fresh(255.0, *ec_)
    Cr = fresh(255.0, *ec_)
    if chain == 'fast':
        # chroma shifted by -128 at the window (one rounding, |.| <= 128)
        Cb = const_add(Cb, -128.0); Cb.cap = 128.0
        Cr = const_add(Cr, -128.0); Cr.cap = 128.0
    def ups(x):
        if mode == '4:4:4':
            return x
        if chain == 'fast':
            # vertical (4:2:0): a * 0.25 + b * 0.75; horizontal in difference
            # form: near + (far - near) * (+-0.25)  (jds_inv_fast.hip chroma8_fast)
            v = x
            if mode == '4:2:0':
                v = add(mul(x, 0.25), mul(x, 0.75)); v.cap = x.cap
            w = fresh(v.cap, v.el, v.ec)
            d = add(v, w, -1)
            h = add(mul(d, 0.25), w); h.cap = x.cap
            return h
        # reference (cv2): horizontal fma pair, then vertical likewise
        h = add(mul(x, 0.25), mul(x, 0.75)); h.cap = x.cap
        if mode == '4:2:0':
            h = add(mul(h, 0.25), mul(h, 0.75)); h.cap = x.cap
        return h
    Cb, Cr = ups(Cb), ups(Cr)
    if chain == 'fast':
        R = add(Y, mul(Cr, 1.402))
        B = add(Y, mul(Cb, 1.772))
        G = add(add(Y, mul(Cb, -0.344136)), mul(Cr, -0.714136))
    else:
        cb = const_add(Cb, -128.0); cr = const_add(Cr, -128.0)
        R = add(Y, mul(cr, 1.402))
        B = add(Y, mul(cb, 1.772))
        G = add(add(Y, mul(cb, 0.344136), -1), mul(cr, 0.714136), -1)
    return max(((x.el, x.ec) for x in (R, G, B)), key=lambda t: t[0] * 2048 + t[1])


def bounds():
    res = {}
    for chain in ('fast', 'ref'):
        eb = block_bound(chain)
        res[chain] = max((colour_bound(eb, eb, chain, m) for m in ('4:4:4', '4:2:2', '4:2:0')),
                         key=lambda t: t[0] * 2048 + t[1])
    k_lin = 2 * (res['fast'][0] + res['ref'][0])
    k_const = 2 * (res['fast'][1] + res['ref'][1])
    return res, k_lin, k_const


if __name__ == '__main__':
    res, k_lin, k_const = bounds()
    for k, (el, ec) in res.items():
        print(f'{k:5s}: e <= {el:.3e} * Dmax + {ec:.3e}')
    print(f'K_LIN = {k_lin:.6e}  K_CONST = {k_const:.6e}')
    print(f'E at Dmax = 1152 (codec output): {k_lin * 1152 + k_const:.3e};  at 255*32768: {k_lin * 255 * 32768 + k_const:.3e}')
