#!/usr/bin/env python3
"""Feasibility of a certified fp32 inverse, on the CPU.

Question: with a RIGOROUS per-value bound, what share of the inverse's
8-pixel output rows (one lane's unit in k_inv_fast) would an fp32 pass have
to leave to an exact fix-up list?

Model (tools/inv_bound.py's, made per coefficient): a value carries its exact
linear form L over the block's 64 dequantised coefficients D_uv, a constant,
and an error bound  e <= sum_uv el_uv |D_uv| + ec.  A rounding of a result r
costs u * (sum |L_uv| |D_uv| + |c|) >= u |r|, so the bound stays linear in
|D| per coefficient; the block's bound is then E_block = K . |D| + kc with
K_uv = max over the 64 outputs.  This replaces round 1's a-priori bound
(K_LIN * Dmax, 0.38 at |D| <= 1152 in fp32), which flags every tile.

fp32 chains (u = 2^-24, constants rounded to fp32), three IDCT orders: the
AAN order of jds_inv_fast.hip (no contraction), direct 8-term dot products,
and an even/odd butterfly (fma = one rounding); then clip, -128 for chroma,
upsample, colour.  Reference chain: pocketfft fp64 (u = 2^-53), as
tools/inv_bound.py.  Results and the cost estimate: DESIGN.md section 8, item 1.

Data: the bench's synthetic frames (uniform random RGB), the oracle's
quantised coefficients and exact pre-truncation values (oracle/cpu_ref.py).
Output: the bound's scale on these frames and the share of flagged rows.
"""
import math
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import cpu_ref as R  # noqa: E402  (tools/: checker side)

C = [math.cos(k * math.pi / 16) for k in range(8)]
SQ2 = math.sqrt(2.0)


class V:
    """Exact linear form L (64), constant c, error (el vector over |D|, ec)."""

    def __init__(self, L, c, el, ec, u, cap=None):
        self.L, self.c, self.el, self.ec, self.u, self.cap = L, c, el, ec, u, cap

    def rnd(self):
        if self.cap is not None:
            self.ec = self.ec + self.u * self.cap
        else:
            self.el = self.el + self.u * np.abs(self.L)
            self.ec = self.ec + self.u * abs(self.c)
        return self


def add(a, b, s=1.0):
    cap = None if a.cap is None or b.cap is None else a.cap + b.cap
    return V(a.L + s * b.L, a.c + s * b.c, a.el + b.el, a.ec + b.ec, a.u, cap).rnd()


def mul(a, k, k_err):
    """a * fl(k): |k| scales the error; the constant's representation error
    k_err (|fl(k) - k|) times |a|; one rounding."""
    cap = None if a.cap is None else abs(k) * a.cap
    el = abs(k) * a.el + (0.0 if a.cap is not None else k_err * np.abs(a.L))
    ec = abs(k) * a.ec + k_err * (a.cap if a.cap is not None else abs(a.c))
    return V(a.L * k, a.c * k, el, ec, a.u, cap).rnd()


def f32err(k):
    return abs(float(np.float32(k)) - k)


def f64err(k):
    return abs(k) * 2.0 ** -53


def aan_line(v, ke):
    t10 = add(v[0], v[4]); t11 = add(v[0], v[4], -1)
    t13 = add(v[2], v[6]); t12 = add(mul(add(v[2], v[6], -1), SQ2, ke(SQ2)), t13, -1)
    e0 = add(t10, t13); e3 = add(t10, t13, -1); e1 = add(t11, t12); e2 = add(t11, t12, -1)
    z13 = add(v[5], v[3]); z10 = add(v[5], v[3], -1); z11 = add(v[1], v[7]); z12 = add(v[1], v[7], -1)
    o7 = add(z11, z13)
    o11 = mul(add(z11, z13, -1), SQ2, ke(SQ2))
    k2 = 2 * C[2]; k10 = 2 * (C[2] - C[6]); k12 = 2 * (C[2] + C[6])
    z5 = mul(add(z10, z12), k2, ke(k2))
    o10 = add(z5, mul(z12, k10, ke(k10)), -1)
    o12 = add(z5, mul(z10, k12, ke(k12)), -1)
    o6 = add(o12, o7, -1); o5 = add(o11, o6, -1); o4 = add(o10, o5, -1)
    return [add(e0, o7), add(e1, o6), add(e2, o5), add(e3, o4),
            add(e3, o4, -1), add(e2, o5, -1), add(e1, o6, -1), add(e0, o7, -1)]


TW = [math.cos(2 * math.pi * (i + 1) / 32) for i in range(7)]
W8 = math.cos(2 * math.pi / 8)


def pocket_dct3(c):
    ke = f64err
    m = lambda a, k: mul(a, k, ke(k))  # noqa: E731
    c = list(c)
    c[0] = m(c[0], SQ2)
    t1 = add(c[1], c[7]); t2 = add(c[1], c[7], -1)
    c[1] = add(m(t2, TW[0]), m(t1, TW[6])); c[7] = add(m(t1, TW[0]), m(t2, TW[6]), -1)
    t1 = add(c[2], c[6]); t2 = add(c[2], c[6], -1)
    c[2] = add(m(t2, TW[1]), m(t1, TW[5])); c[6] = add(m(t1, TW[1]), m(t2, TW[5]), -1)
    t1 = add(c[3], c[5]); t2 = add(c[3], c[5], -1)
    c[3] = add(m(t2, TW[2]), m(t1, TW[4])); c[5] = add(m(t1, TW[2]), m(t2, TW[4]), -1)
    c[4] = m(c[4], 2 * TW[3])
    r1 = add(c[6], c[2]); g2 = add(c[6], c[2], -1)
    r2 = add(c[0], c[4]); g1 = add(c[0], c[4], -1)
    g0 = add(r2, r1); g3 = add(r2, r1, -1)
    r1 = add(c[7], c[3]); g6 = add(c[7], c[3], -1)
    r2 = add(c[1], c[5]); g5 = add(c[1], c[5], -1)
    g4 = add(r2, r1); g7 = add(r2, r1, -1)
    o0 = add(g0, g4); o7 = add(g0, g4, -1)
    o4 = m(g7, -1.0); o3 = g3
    q2 = add(m(g5, W8), m(g6, W8)); qi = add(m(g6, W8), m(g5, W8), -1)
    o1 = add(g1, q2); o5 = add(g1, q2, -1); o2 = add(qi, g2); o6 = add(qi, g2, -1)
    return [o0, add(o1, o2, -1), add(o2, o1), add(o3, o4, -1), add(o4, o3), add(o5, o6, -1), add(o6, o5), o7]


def block_K(chain):
    """(K[64], kc): |v_chain - v*| <= K . |D| + kc for every output of a block
    (after +128; before the clip)."""
    u = 2.0 ** -24 if chain == 'f32' else 2.0 ** -53
    ke = f32err if chain == 'f32' else f64err
    basis = [[V(np.eye(64)[i * 8 + j].copy(), 0.0, np.zeros(64), 0.0, u) for j in range(8)] for i in range(8)]
    if chain == 'f32':
        aan = [1.0] + [C[k] * SQ2 for k in range(1, 8)]
        d = [[None] * 8 for _ in range(8)]
        for i in range(8):
            for j in range(8):
                k = aan[i] * aan[j] / 8
                x = mul(basis[i][j], k, 0.0)
                x.el = x.el + 4 * u * abs(k) * np.eye(64)[i * 8 + j]  # table entry: 4 host roundings
                d[i][j] = x
        dc = d[0][0]
        d[0][0] = V(dc.L, dc.c + 128.0, dc.el, dc.ec, u).rnd()
        cols = [aan_line([d[i][j] for i in range(8)], ke) for j in range(8)]
        out = [aan_line([cols[j][m] for j in range(8)], ke) for m in range(8)]
    else:
        cols = [pocket_dct3([basis[i][j] for i in range(8)]) for j in range(8)]
        rows = [pocket_dct3([cols[j][m] for j in range(8)]) for m in range(8)]
        out = [[V(x.L / 16, x.c / 16 + 128.0, x.el / 16, x.ec / 16, u).rnd() for x in r] for r in rows]
    K = np.zeros(64)
    kc = 0.0
    for r in out:
        for x in r:
            K = np.maximum(K, x.el)
            kc = max(kc, x.ec)
    return K, kc


def colour_coeffs(mode):
    """Per channel (R, G, B): |v_f32 - v_ref| <= eY + aC eC + c0, where eY / eC
    bound |fp32 - ref| of the clipped luma / chroma samples (block bounds of
    both chains summed).  The upsample is a convex blend whatever its form
    (fp32: near + (far - near) / 4; cv2: two weighted products), so sample
    errors pass through with weight 1; each chain adds its roundings:
    fp32 (|chroma - 128| <= 128): the -128 shift u*128; 4:2:0 vertical blend
    u*(96 + 128); horizontal difference u*256/4 and sum u*128; colour products
    and sums with fp32 constants.  Reference (fp64): cv2's products and sums
    on [0, 255], the -128 shifts, colour products and sums."""
    u32, u64 = 2.0 ** -24, 2.0 ** -53
    k = np.array([1.402, 0.344136 + 0.714136, 1.772])
    kerr = np.array([f32err(1.402), f32err(0.344136) + f32err(0.714136), f32err(1.772)])
    up32 = u32 * (128 + (96 + 128 if mode == '4:2:0' else 0) + (64 + 128 if mode != '4:4:4' else 0))
    up64 = u64 * (2 * (191.25 + 255) + 128)
    # colour: |C| <= 128 (fp32 shifted chroma), products u*|k C|, sums u*|result| (<= 255 + 128 k)
    col32 = 128 * kerr + u32 * (128 * k + 2 * (255 + 128 * k))
    col64 = u64 * (128 * k + 2 * (255 + 128 * k) + 255)
    return k, (k * (up32 + up64) + col32 + col64)


def dot_line(v, W, u):
    """Direct 8-term IDCT line: out_m = sum_k fl(W[m][k]) v_k, products and
    sums each rounded once, in k order (no contraction)."""
    out = []
    for m in range(8):
        acc = None
        for kk in range(8):
            p = mul(v[kk], W[m][kk], f32err(W[m][kk]))
            acc = p if acc is None else add(acc, p)
        out.append(acc)
    return out


def block_K_direct():
    """fp32 bound of the direct form: dequantise (q * fl(Q / 8)... folded as
    q * fl(Q) then the orthonormal matrix), columns then rows."""
    u = 2.0 ** -24
    Wm = [[(math.sqrt(0.125) if kk == 0 else 0.5 * math.cos((2 * m + 1) * kk * math.pi / 16)) for kk in range(8)]
          for m in range(8)]
    basis = [[V(np.eye(64)[i * 8 + j].copy(), 0.0, np.zeros(64), 0.0, u) for j in range(8)] for i in range(8)]
    cols = [dot_line([basis[i][j] for i in range(8)], Wm, u) for j in range(8)]
    out = [dot_line([cols[j][m] for j in range(8)], Wm, u) for m in range(8)]
    K = np.zeros(64)
    kc = 0.0
    for r in out:
        for x in r:
            y = V(x.L, x.c + 128.0, x.el, x.ec, u).rnd()
            K = np.maximum(K, y.el)
            kc = max(kc, y.ec)
    return K, kc


def fma(a, k, b, s=1.0):
    """fl(a * fl(k) + s * b): one rounding (the product is exact inside the fma)."""
    cap = None if a.cap is None or b.cap is None else abs(k) * a.cap + b.cap
    el = abs(k) * a.el + (0.0 if a.cap is not None else f32err(k) * np.abs(a.L)) + b.el
    ec = abs(k) * a.ec + f32err(k) * (a.cap if a.cap is not None else abs(a.c)) + b.ec
    return V(a.L * k + s * b.L, a.c * k + s * b.c, el, ec, a.u, cap).rnd()


# even/odd partial butterfly on inputs pre-scaled by the table: X0, X4 carry
# 1/sqrt(8) (folded), the others their plain orthonormal factor 1/2 (folded)
BO = [[math.cos((2 * n + 1) * k * math.pi / 16) for k in (1, 3, 5, 7)] for n in range(4)]
BE = [[math.cos((2 * n + 1) * k * math.pi / 16) for k in (2, 6)] for n in range(2)]


def bfly_line(v):
    ee0 = add(v[0], v[4]); ee1 = add(v[0], v[4], -1)
    eo0 = fma(v[2], BE[0][0], mul(v[6], BE[0][1], f32err(BE[0][1])))
    eo1 = fma(v[2], BE[1][0], mul(v[6], BE[1][1], f32err(BE[1][1])))
    e = [add(ee0, eo0), add(ee1, eo1), add(ee1, eo1, -1), add(ee0, eo0, -1)]
    o = []
    for n in range(4):
        acc = mul(v[1], BO[n][0], f32err(BO[n][0]))
        for j, kk in enumerate((3, 5, 7)):
            acc = fma(v[kk], BO[n][j + 1], acc)
        o.append(acc)
    return [add(e[0], o[0]), add(e[1], o[1]), add(e[2], o[2]), add(e[3], o[3]),
            add(e[3], o[3], -1), add(e[2], o[2], -1), add(e[1], o[1], -1), add(e[0], o[0], -1)]


def block_K_bfly():
    """fp32 bound of the butterfly form: q * fl(Q * s_u * s_v) (s_0 = 1/sqrt(8),
    s_k = 1/2; the table entry rounded once on the host from the exact real),
    columns then rows, +128 folded into the DC entry like k_inv_fast."""
    u = 2.0 ** -24
    sc = [1 / math.sqrt(8)] + [0.5] * 7
    basis = [[V(np.eye(64)[i * 8 + j].copy(), 0.0, np.zeros(64), 0.0, u) for j in range(8)] for i in range(8)]
    d = [[None] * 8 for _ in range(8)]
    for i in range(8):
        for j in range(8):
            k = sc[i] * sc[j]
            x = mul(basis[i][j], k, 0.0)
            x.el = x.el + 2 * u * abs(k) * np.eye(64)[i * 8 + j]  # table entry: 2 roundings
            d[i][j] = x
    dc = d[0][0]
    d[0][0] = V(dc.L, dc.c + 128.0, dc.el, dc.ec, u).rnd()
    cols = [bfly_line([d[i][j] for i in range(8)]) for j in range(8)]
    out = [bfly_line([cols[j][m] for j in range(8)]) for m in range(8)]
    K = np.zeros(64)
    kc = 0.0
    for r in out:
        for x in r:
            K = np.maximum(K, x.el)
            kc = max(kc, x.ec)
    return K, kc


def main(H=1080, W=1920, seed=7, q=50, mode='4:2:0', pf=True):
    img = R.random_image(H, W, seed)
    out = R.compress_reconstruct(img, quality=q, mode=mode, prefilter=pf, metrics=False)
    qm = out['qtable']
    allq = out['coeffs']
    ny, nx = -(-H // 8), -(-W // 8)
    sy = 2 if mode == '4:2:0' else 1
    sx = 1 if mode == '4:4:4' else 2
    hc, wc = -(-H // sy), -(-W // sx)
    ncy, ncx = -(-hc // 8), -(-wc // 8)
    nyb, ncb = ny * nx, ncy * ncx
    Dy = np.abs(allq[:nyb * 64].reshape(nyb, 64).astype(np.float64) * qm.reshape(64))
    Dcb = np.abs(allq[nyb * 64:(nyb + ncb) * 64].reshape(ncb, 64).astype(np.float64) * qm.reshape(64))
    Dcr = np.abs(allq[(nyb + ncb) * 64:].reshape(ncb, 64).astype(np.float64) * qm.reshape(64))
    Kr, kcr = block_K('f64')
    aC, c0 = colour_coeffs(mode)
    res = {}
    for form in ('aan', 'direct', 'butterfly'):
        Kf, kcf = block_K('f32') if form == 'aan' else block_K_direct() if form == 'direct' else block_K_bfly()
        res[form] = flag_rate(form, Kf + Kr, kcf + kcr, aC, c0, Dy, Dcb, Dcr, out, H, W, ny, nx, ncy, ncx,
                              sy, sx, mode)
    return res


def flag_rate(form, K, kc, aC, c0, Dy, Dcb, Dcr, out, H, W, ny, nx, ncy, ncx, sy, sx, mode):
    print(f'-- fp32 {form} IDCT: K/u in [{K.min() * 2**24:.1f}, {K.max() * 2**24:.1f}] '
          f'(DC {K[0] * 2**24:.1f}), kc {kc:.3e}; colour aC {aC}, c0 {c0}')
    Ey = (Dy @ K + kc).reshape(ny, nx)
    Ec = np.maximum(Dcb @ K, Dcr @ K).reshape(ncy, ncx) + kc
    print(f'E_block (luma): median {np.median(Ey):.3e}, p99 {np.percentile(Ey, 99):.3e}, max {Ey.max():.3e}')
    print(f'E_block (chroma): median {np.median(Ec):.3e}, max {Ec.max():.3e}')
    # per-pixel bound: the pixel's luma block and the worst chroma block within one block
    Ey_px = np.repeat(np.repeat(Ey, 8, 0), 8, 1)[:H, :W]
    Ecm = Ec.copy()
    pad = np.pad(Ec, 1, mode='edge')
    for dy in (-1, 0, 1):
        for dx in (-1, 0, 1):
            Ecm = np.maximum(Ecm, pad[1 + dy:1 + dy + ncy, 1 + dx:1 + dx + ncx])
    Ec_px = np.repeat(np.repeat(Ecm, 8 * sy, 0), 8 * sx, 1)[:H, :W]
    E = Ey_px[..., None] + aC[None, None, :] * Ec_px[..., None] + c0[None, None, :]
    # exact pre-truncation values without the final clip
    y = out['y_rec']
    cb, cr = out['cb_rec'], out['cr_rec']
    if mode != '4:4:4':
        cb, cr = R.upsample_chroma(cb, cr, (H, W))
    v = np.stack([y + 1.402 * (cr - 128.0), y - 0.344136 * (cb - 128.0) - 0.714136 * (cr - 128.0),
                  y + 1.772 * (cb - 128.0)], axis=-1)
    k = np.clip(np.rint(v), 1, 255)
    unc = np.abs(v - k) <= E
    wu = W // 8 * 8
    rows = unc[:, :wu].reshape(H, wu // 8, 8 * 3).any(axis=-1)
    print(f'E per value: median {np.median(E):.3e}, max {E.max():.3e}')
    print(f'uncertain values: {unc.mean() * 100:.3f} %;  flagged 8-pixel rows: {rows.mean() * 100:.3f} % '
          f'({rows.sum()} of {rows.size} per {H}x{W} frame)')
    tiles = rows.reshape(H // 8 if H % 8 == 0 else -1, 8, -1) if H % 8 == 0 else None
    if tiles is not None:
        print(f'8x8 blocks with a flagged row: {tiles.any(axis=1).mean() * 100:.2f} %')
    return rows.mean()


if __name__ == '__main__':
    main()
