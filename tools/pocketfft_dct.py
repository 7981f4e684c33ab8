"""Restatement of pocketfft's length-N DCT-II / DCT-III (T_dcst23, cosine,
ortho) for N in {8, 16}, operation by operation, in IEEE fp64 (Python floats /
NumPy elementwise ops: one rounding per operation, no FMA).

Purpose: derive and validate the constants and the operation order that
csrc/jds_dct8.hpp and csrc/jds_dct16.hpp hard-code.  `python tools/pocketfft_dct.py`
prints the twiddle doubles and checks the restatement bit-for-bit against
scipy.fft.dct / idct (SciPy vendors pocketfft) on random lines.

pocketfft (pocketfft_hdronly.hpp, as vendored by SciPy >= 1.4), published
algorithm restated here:
* sincos_2pibyn(n): two small tables v1 (fine) / v2 (coarse) of (cos, sin)
  computed with libm in octant-reduced form, combined by one complex product
  per entry -> some entries are 1 ulp off the correctly rounded value.
* T_dcst23 type 2: c0 *= 2, c[N-1] *= 2, MPINPLACE pairs, real backward FFT
  (rfftp, factors 4.. with a leading 2), post-twiddle with
  twiddle[i] = sincos_2pibyn(4N)[i+1].r, c[N/2] *= twiddle[N/2-1],
  c0 *= sqrt2 * 0.5 (ortho).  Type 3 is the mirror with the forward FFT.
* the norm factor fct (1/sqrt(prod 2N) = 2^-k for these sizes) is applied once
  on the first axis; it is an exact power of two and is left out here.
"""
from __future__ import annotations

import math

import numpy as np

SQRT2 = float.fromhex('0x1.6a09e667f3bcdp+0')   # T0(1.4142135623730950488L)
HSQT2 = float.fromhex('0x1.6a09e667f3bcdp-1')   # T0(0.7071067811865475244L)


def _calc(x, n, ang):
    x <<= 3
    if x < 4 * n:
        if x < 2 * n:
            if x < n:
                return (math.cos(x * ang), math.sin(x * ang))
            return (math.sin((2 * n - x) * ang), math.cos((2 * n - x) * ang))
        x -= 2 * n
        if x < n:
            return (-math.sin(x * ang), math.cos(x * ang))
        return (-math.cos((2 * n - x) * ang), math.sin((2 * n - x) * ang))
    x = 8 * n - x
    if x < 2 * n:
        if x < n:
            return (math.cos(x * ang), -math.sin(x * ang))
        return (math.sin((2 * n - x) * ang), -math.cos((2 * n - x) * ang))
    x -= 4 * n
    if x < n:
        return (-math.sin(x * ang), -math.cos(x * ang))
    return (-math.cos((2 * n - x) * ang), -math.sin((2 * n - x) * ang))


def sincos_2pibyn(n):
    """pocketfft sincos_2pibyn<double>(n) as a list of (cos, sin) for idx 0..n-1."""
    # Thigh(0.25L*pi/n): evaluated in long double, rounded to double
    ang = float(np.longdouble(0.25) * np.longdouble('3.141592653589793238462643383279502884197') / n)
    nval = (n + 2) // 2
    shift = 1
    while (1 << shift) * (1 << shift) < nval:
        shift += 1
    mask = (1 << shift) - 1
    v1 = [(1.0, 0.0)] + [_calc(i, n, ang) for i in range(1, mask + 1)]
    nv2 = (nval + mask) // (mask + 1)
    v2 = [(1.0, 0.0)] + [_calc(i * (mask + 1), n, ang) for i in range(1, nv2)]
    out = []
    for idx in range(n):
        if 2 * idx <= n:
            x1, x2 = v1[idx & mask], v2[idx >> shift]
            out.append((x1[0] * x2[0] - x1[1] * x2[1], x1[0] * x2[1] + x1[1] * x2[0]))
        else:
            j = n - idx
            x1, x2 = v1[j & mask], v2[j >> shift]
            out.append((x1[0] * x2[0] - x1[1] * x2[1], -(x1[0] * x2[1] + x1[1] * x2[0])))
    return out


def dct_twiddle(n):
    t = sincos_2pibyn(4 * n)
    return [t[i + 1][0] for i in range(n)]


def rfft_factors(n):
    f, m = [], n
    while m % 4 == 0:
        f.append(4)
        m >>= 2
    if m % 2 == 0:
        m >>= 1
        f.append(2)
        f[0], f[-1] = f[-1], f[0]
    assert m == 1, 'only powers of two are restated'
    return f


def rfft_twiddles(n):
    tw = sincos_2pibyn(n)
    out, l1 = [], 1
    fac = rfft_factors(n)
    for k, ip in enumerate(fac):
        ido = n // (l1 * ip)
        t = [0.0] * ((ip - 1) * (ido - 1))
        if k < len(fac) - 1:
            for j in range(1, ip):
                for i in range(1, (ido - 1) // 2 + 1):
                    t[(j - 1) * (ido - 1) + 2 * i - 2] = tw[j * l1 * i][0]
                    t[(j - 1) * (ido - 1) + 2 * i - 1] = tw[j * l1 * i][1]
        out.append(t)
        l1 *= ip
    return out


# ---- radix passes (arrays: each "element" is an ndarray over test lines) ----

def radb2(ido, l1, cc, ch, wa):
    CC = lambda a, b, c: cc[a + ido * (b + 2 * c)]
    def CHs(a, b, c, v): ch[a + ido * (b + l1 * c)] = v
    for k in range(l1):
        CHs(0, k, 0, CC(0, 0, k) + CC(ido - 1, 1, k))
        CHs(0, k, 1, CC(0, 0, k) - CC(ido - 1, 1, k))
    if ido % 2 == 0:
        for k in range(l1):
            CHs(ido - 1, k, 0, 2.0 * CC(ido - 1, 0, k))
            CHs(ido - 1, k, 1, -2.0 * CC(0, 1, k))
    if ido <= 2:
        return
    for k in range(l1):
        for i in range(2, ido, 2):
            ic = ido - i
            CHs(i - 1, k, 0, CC(i - 1, 0, k) + CC(ic - 1, 1, k))
            tr2 = CC(i - 1, 0, k) - CC(ic - 1, 1, k)
            ti2 = CC(i, 0, k) + CC(ic, 1, k)
            CHs(i, k, 0, CC(i, 0, k) - CC(ic, 1, k))
            wr, wi = wa[i - 2], wa[i - 1]
            CHs(i, k, 1, wr * ti2 + wi * tr2)
            CHs(i - 1, k, 1, wr * tr2 - wi * ti2)


def radb4(ido, l1, cc, ch, wa):
    CC = lambda a, b, c: cc[a + ido * (b + 4 * c)]
    def CHs(a, b, c, v): ch[a + ido * (b + l1 * c)] = v
    WA = lambda x, i: wa[i + x * (ido - 1)]
    for k in range(l1):
        tr2 = CC(0, 0, k) + CC(ido - 1, 3, k)
        tr1 = CC(0, 0, k) - CC(ido - 1, 3, k)
        tr3 = 2.0 * CC(ido - 1, 1, k)
        tr4 = 2.0 * CC(0, 2, k)
        CHs(0, k, 0, tr2 + tr3); CHs(0, k, 2, tr2 - tr3)
        CHs(0, k, 3, tr1 + tr4); CHs(0, k, 1, tr1 - tr4)
    if ido % 2 == 0:
        for k in range(l1):
            ti1 = CC(0, 3, k) + CC(0, 1, k)
            ti2 = CC(0, 3, k) - CC(0, 1, k)
            tr2 = CC(ido - 1, 0, k) + CC(ido - 1, 2, k)
            tr1 = CC(ido - 1, 0, k) - CC(ido - 1, 2, k)
            CHs(ido - 1, k, 0, tr2 + tr2)
            CHs(ido - 1, k, 1, SQRT2 * (tr1 - ti1))
            CHs(ido - 1, k, 2, ti2 + ti2)
            CHs(ido - 1, k, 3, -SQRT2 * (tr1 + ti1))
    if ido <= 2:
        return
    for k in range(l1):
        for i in range(2, ido, 2):
            ic = ido - i
            tr2 = CC(i - 1, 0, k) + CC(ic - 1, 3, k); tr1 = CC(i - 1, 0, k) - CC(ic - 1, 3, k)
            ti1 = CC(i, 0, k) + CC(ic, 3, k); ti2 = CC(i, 0, k) - CC(ic, 3, k)
            tr4 = CC(i, 2, k) + CC(ic, 1, k); ti3 = CC(i, 2, k) - CC(ic, 1, k)
            tr3 = CC(i - 1, 2, k) + CC(ic - 1, 1, k); ti4 = CC(i - 1, 2, k) - CC(ic - 1, 1, k)
            CHs(i - 1, k, 0, tr2 + tr3); cr3 = tr2 - tr3
            CHs(i, k, 0, ti2 + ti3); ci3 = ti2 - ti3
            cr4 = tr1 + tr4; cr2 = tr1 - tr4
            ci2 = ti1 + ti4; ci4 = ti1 - ti4
            for x, (cr, ci) in enumerate(((cr2, ci2), (cr3, ci3), (cr4, ci4))):
                wr, wi = WA(x, i - 2), WA(x, i - 1)
                CHs(i, k, x + 1, wr * ci + wi * cr)
                CHs(i - 1, k, x + 1, wr * cr - wi * ci)


def radf2(ido, l1, cc, ch, wa):
    CC = lambda a, b, c: cc[a + ido * (b + l1 * c)]
    def CHs(a, b, c, v): ch[a + ido * (b + 2 * c)] = v
    for k in range(l1):
        CHs(0, 0, k, CC(0, k, 0) + CC(0, k, 1))
        CHs(ido - 1, 1, k, CC(0, k, 0) - CC(0, k, 1))
    if ido % 2 == 0:
        for k in range(l1):
            CHs(0, 1, k, -CC(ido - 1, k, 1))
            CHs(ido - 1, 0, k, CC(ido - 1, k, 0))
    if ido <= 2:
        return
    for k in range(l1):
        for i in range(2, ido, 2):
            ic = ido - i
            wr, wi = wa[i - 2], wa[i - 1]
            tr2 = wr * CC(i - 1, k, 1) + wi * CC(i, k, 1)
            ti2 = wr * CC(i, k, 1) - wi * CC(i - 1, k, 1)
            CHs(i - 1, 0, k, CC(i - 1, k, 0) + tr2); CHs(ic - 1, 1, k, CC(i - 1, k, 0) - tr2)
            CHs(i, 0, k, ti2 + CC(i, k, 0)); CHs(ic, 1, k, ti2 - CC(i, k, 0))


def radf4(ido, l1, cc, ch, wa):
    CC = lambda a, b, c: cc[a + ido * (b + l1 * c)]
    def CHs(a, b, c, v): ch[a + ido * (b + 4 * c)] = v
    WA = lambda x, i: wa[i + x * (ido - 1)]
    for k in range(l1):
        tr1 = CC(0, k, 3) + CC(0, k, 1); CHs(0, 2, k, CC(0, k, 3) - CC(0, k, 1))
        tr2 = CC(0, k, 0) + CC(0, k, 2); CHs(ido - 1, 1, k, CC(0, k, 0) - CC(0, k, 2))
        CHs(0, 0, k, tr2 + tr1); CHs(ido - 1, 3, k, tr2 - tr1)
    if ido % 2 == 0:
        for k in range(l1):
            ti1 = -HSQT2 * (CC(ido - 1, k, 1) + CC(ido - 1, k, 3))
            tr1 = HSQT2 * (CC(ido - 1, k, 1) - CC(ido - 1, k, 3))
            CHs(ido - 1, 0, k, CC(ido - 1, k, 0) + tr1); CHs(ido - 1, 2, k, CC(ido - 1, k, 0) - tr1)
            CHs(0, 3, k, ti1 + CC(ido - 1, k, 2)); CHs(0, 1, k, ti1 - CC(ido - 1, k, 2))
    if ido <= 2:
        return
    for k in range(l1):
        for i in range(2, ido, 2):
            ic = ido - i
            crs, cis = [], []
            for x in range(3):
                wr, wi = WA(x, i - 2), WA(x, i - 1)
                crs.append(wr * CC(i - 1, k, x + 1) + wi * CC(i, k, x + 1))
                cis.append(wr * CC(i, k, x + 1) - wi * CC(i - 1, k, x + 1))
            cr2, cr3, cr4 = crs
            ci2, ci3, ci4 = cis
            tr1 = cr4 + cr2; tr4 = cr4 - cr2
            ti1 = ci2 + ci4; ti4 = ci2 - ci4
            tr2 = CC(i - 1, k, 0) + cr3; tr3 = CC(i - 1, k, 0) - cr3
            ti2 = CC(i, k, 0) + ci3; ti3 = CC(i, k, 0) - ci3
            CHs(i - 1, 0, k, tr2 + tr1); CHs(ic - 1, 3, k, tr2 - tr1)
            CHs(i, 0, k, ti1 + ti2); CHs(ic, 3, k, ti1 - ti2)
            CHs(i - 1, 2, k, tr3 + ti4); CHs(ic - 1, 1, k, tr3 - ti4)
            CHs(i, 2, k, tr4 + ti3); CHs(ic, 1, k, tr4 - ti3)


def rfftp(c, r2hc):
    n = len(c)
    fac, tws = rfft_factors(n), rfft_twiddles(n)
    p1, p2 = list(c), [None] * n
    if r2hc:
        l1 = n
        for k in reversed(range(len(fac))):
            ip = fac[k]
            ido = n // l1
            l1 //= ip
            (radf4 if ip == 4 else radf2)(ido, l1, p1, p2, tws[k])
            p1, p2 = p2, p1
    else:
        l1 = 1
        for k, ip in enumerate(fac):
            ido = n // (ip * l1)
            (radb4 if ip == 4 else radb2)(ido, l1, p1, p2, tws[k])
            p1, p2 = p2, p1
            l1 *= ip
    return p1


def dct2_line(c):
    """T_dcst23::exec type 2 (cosine, ortho) without fct."""
    n = len(c)
    tw = dct_twiddle(n)
    c = list(c)
    c[0] = c[0] * 2.0
    c[n - 1] = c[n - 1] * 2.0
    for k in range(1, n - 1, 2):
        a, b = c[k + 1], c[k]
        c[k + 1] = a - b
        c[k] = b + a
    c = rfftp(c, False)
    ns2 = n // 2
    for k in range(1, ns2):
        kc = n - k
        t1 = tw[k - 1] * c[kc] + tw[kc - 1] * c[k]
        t2 = tw[k - 1] * c[k] - tw[kc - 1] * c[kc]
        c[k] = 0.5 * (t1 + t2)
        c[kc] = 0.5 * (t1 - t2)
    c[ns2] = c[ns2] * tw[ns2 - 1]
    c[0] = c[0] * (SQRT2 * 0.5)
    return c


def dct3_line(c):
    """T_dcst23::exec type 3 (cosine, ortho) without fct."""
    n = len(c)
    tw = dct_twiddle(n)
    c = list(c)
    c[0] = c[0] * SQRT2
    ns2 = n // 2
    for k in range(1, ns2):
        kc = n - k
        t1 = c[k] + c[kc]
        t2 = c[k] - c[kc]
        c[k] = tw[k - 1] * t2 + tw[kc - 1] * t1
        c[kc] = tw[k - 1] * t1 - tw[kc - 1] * t2
    c[ns2] = c[ns2] * (2.0 * tw[ns2 - 1])
    c = rfftp(c, True)
    for k in range(1, n - 1, 2):
        a, b = c[k], c[k + 1]
        c[k] = a - b
        c[k + 1] = b + a
    return c


def check_against_scipy(n, blocks=2000, seed=0):
    """Mismatch counts (dctn, idctn) of the restatement applied along both axes
    of n x n blocks (axis 0 first, fct = 1/(2n) folded in) against SciPy."""
    import scipy.fft as sf
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((blocks, n, n)) * rng.choice([1.0, 100.0, 2000.0], (blocks, 1, 1))
    fct = 1.0 / (2 * n)   # exact power of two for n in {8, 16}

    def two_d(a, line):
        cols = np.stack(line([a[:, i, :] for i in range(n)]), 1) * fct
        return np.stack(line([cols[:, :, j] for j in range(n)]), 2)

    return (int(np.count_nonzero(two_d(x, dct2_line) != sf.dctn(x, type=2, norm='ortho', axes=(1, 2)))),
            int(np.count_nonzero(two_d(x, dct3_line) != sf.idctn(x, type=2, norm='ortho', axes=(1, 2)))))


if __name__ == '__main__':
    for n in (8, 16):
        print(f'N={n}  rfft factors {rfft_factors(n)}')
        print('  dct twiddle:', [t.hex() for t in dct_twiddle(n)[:n - 1]])
        print('  rfft twiddles:', [[t.hex() for t in tt] for tt in rfft_twiddles(n)])
        print('  mismatches vs scipy (dctn, idctn):', check_against_scipy(n))
