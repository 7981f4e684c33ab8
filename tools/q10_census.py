#!/usr/bin/env python3
"""Why the certified inverse fails at coarse tables: on a
random frame at a coarse quality, list the output values the certificate cannot
decide (|v_fast - round(v_fast)| <= E, E as the kernel takes it per 64 x 128
tile) and classify them by the reference's pre-truncation value v_ref and the
blocks behind the pixel:
  exact_int       v_ref is an exact integer
  luma_zero       the pixel's luma block has no nonzero coefficient
  luma_dc_only    ... only its DC
  luma_clipped    the reference's luma sample was clipped (0 or 255)
  chroma_zero     every chroma block its bilinear taps reach is all-zero (C - 128 == 0 exactly)
Runs the kernel's own arithmetic on the host (jds_selftest_inv_fast) and the
oracle; prints one JSON line.  Env: H W Q MODE PF SEED."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'jpeg-dsp-studio_amd'), ROOT, os.path.join(ROOT, 'tools')]
from scipy.ndimage import maximum_filter  # noqa: E402

import inv_bound  # noqa: E402
from jds import _abi  # noqa: E402
from oracle import cpu_ref  # noqa: E402


def planes(mode, H, W):
    sy = 2 if mode == '4:2:0' else 1
    sx = 1 if mode == '4:4:4' else 2
    return [(H, W), (H // sy, W // sx), (H // sy, W // sx)], sy, sx


def main():
    H, W = int(os.environ.get('H', 512)), int(os.environ.get('W', 768))
    q = int(os.environ.get('Q', 10))
    mode = os.environ.get('MODE', '4:2:0')
    pf = os.environ.get('PF', '0') == '1'
    img = cpu_ref.random_image(H, W, int(os.environ.get('SEED', 0)))
    ref = cpu_ref.compress_reconstruct(img, q, 8, mode, pf, metrics=False)
    Q = np.asarray(ref['qtable'], np.float64)
    cf = np.ascontiguousarray(ref['coeffs'], dtype=np.int16)
    pl, sy, sx = planes(mode, H, W)
    rec, off, qmax_b, nz_b, acnz_b, clip = [], 0, [], [], [], []
    for ph, pw in pl:
        nby, nbx = -(-ph // 8), -(-pw // 8)
        qb = cf[off:off + nby * nbx * 64].reshape(-1, 8, 8)
        off += nby * nbx * 64
        raw = cpu_ref.decode_blocks(cpu_ref.dequantize(qb, Q))  # (clipped per block)
        r = cpu_ref.merge_blocks(raw, (nby * 8, nbx * 8))[:ph, :pw]
        rec.append(r)
        clip.append((r == 0.0) | (r == 255.0))
        a = np.abs(qb.astype(np.int64)).reshape(nby, nbx, 64)
        qmax_b.append(a.max(axis=2))
        nz_b.append(a.any(axis=2))
        acnz_b.append(a[..., 1:].any(axis=2))
    y, cb, cr = rec
    if mode != '4:4:4':
        cb_u, cr_u = cpu_ref.upsample_chroma(cb, cr, (H, W))
    else:
        cb_u, cr_u = cb, cr
    v_ref = np.stack([y + 1.402 * (cr_u - 128.0), y - 0.344136 * (cb_u - 128.0) - 0.714136 * (cr_u - 128.0),
                      y + 1.772 * (cb_u - 128.0)], axis=-1)
    yy, xx = np.mgrid[0:H, 0:W]
    yb, xb = yy // 8, xx // 8
    cyb, cxb = (yy // sy) // 8, (xx // sx) // 8
    # the kernel's Dmax: max |q| over the 64 x 128 tile's blocks (and chroma ring) x max Q
    th, tw = (64, 128) if mode == '4:2:0' else ((32, 128) if mode == '4:2:2' else (32, 64))
    qm = qmax_b[0][yb, xb]
    for p in (1, 2):
        qm = np.maximum(qm, maximum_filter(qmax_b[p], size=3, mode='nearest')[cyb, cxb])
    tmax = np.zeros_like(qm)
    for t0 in range(0, H, th):
        for t1 in range(0, W, tw):
            tmax[t0:t0 + th, t1:t1 + tw] = qm[t0:t0 + th, t1:t1 + tw].max()
    K = inv_bound.kernel_constants()
    E = (K['K_LIN'] * tmax * Q.max() + K['K_CONST'] + 2.0 ** -31)[..., None]
    v = np.empty((H, W, 3), np.float64)
    by = np.empty((H, W, 3), np.uint8)
    Qc = np.ascontiguousarray(Q)
    assert _abi.lib().jds_selftest_inv_fast(_abi.MODE_CODES[mode], cf.ctypes.data, Qc.ctypes.data, H, W, 1,
                                            v.ctypes.data, by.ctypes.data) == 0
    unc = np.abs(v - np.rint(v)) <= E
    czero = np.ones((H, W), bool)
    for p in (1, 2):
        dil = maximum_filter(nz_b[p].astype(np.uint8), size=3, mode='nearest')
        czero &= dil[cyb, cxb] == 0
    ex = v_ref == np.rint(v_ref)
    cls = {'exact_int': ex, 'luma_zero': ~nz_b[0][yb, xb][..., None],
           'luma_dc_only': (nz_b[0] & ~acnz_b[0])[yb, xb][..., None], 'luma_clipped': clip[0][..., None],
           'chroma_zero': czero[..., None]}
    tiles = unc.any(axis=2)
    nt = sum(1 for t0 in range(0, H, th) for t1 in range(0, W, tw))
    hit = sum(bool(tiles[t0:t0 + th, t1:t1 + tw].any()) for t0 in range(0, H, th) for t1 in range(0, W, tw))
    out = {'H': H, 'W': W, 'Q': q, 'mode': mode, 'prefilter': pf, 'values': int(unc.size),
           'uncertain': int(unc.sum()), 'tiles': nt, 'tiles_uncertain': hit,
           'median_E': float(np.median(E))}
    for k, m in cls.items():
        out[k] = int((unc & m).sum())
    out['exact_int_and_chroma_zero'] = int((unc & ex & czero[..., None]).sum())
    out['exact_int_luma_clipped_chroma_zero'] = int((unc & ex & czero[..., None] & clip[0][..., None]).sum())
    out['exact_int_luma_dc_only_chroma_zero'] = int(
        (unc & ex & czero[..., None] & (nz_b[0] & ~acnz_b[0])[yb, xb][..., None]).sum())
    out['not_exact'] = int((unc & ~ex).sum())
    # the exact-value rule round 5 tried (k_inv_fast<.., EX>, retired): luma exactly known (all-zero block, or the
    # fast value beyond the clip range by more than E) and every chroma tap of the channel's
    # plane(s) from an all-zero block -- per pixel (PER_LANE=1: the lane's 8 pixels together)
    if mode != '4:4:4':
        hc, wc = pl[1]
        m = yy // sy
        if sy == 2:
            rq = np.clip(np.where(yy & 1, m + 1, m - 1), 0, hc - 1)
        else:
            rq = np.clip(m, 0, hc - 1)
        rt = np.clip(m, 0, hc - 1)
        j = xx // 2
        c_a = np.clip(np.where(xx & 1, j, j - 1), 0, wc - 1)
        c_b = np.clip(np.where(xx & 1, j + 1, j), 0, wc - 1)
        zpl = []
        for p in (1, 2):
            zb = ~nz_b[p]
            z = np.ones((H, W), bool)
            for r_ in (rq, rt):
                for c_ in (c_a, c_b):
                    z &= zb[r_ // 8, c_ // 8]
            if os.environ.get('PER_LANE') == '1':
                z = z.reshape(H, W // 8, 8).all(axis=2).repeat(8, axis=1)
            zpl.append(z)
        ny_, nx_ = -(-H // 8), -(-W // 8)
        # fast luma before clip: approximated by the reference's unclipped luma (within E of it)
        from scipy import fft as sfft
        qb = cf[:ny_ * nx_ * 64].reshape(-1, 8, 8)
        raw = cpu_ref.merge_blocks(sfft.idctn(cpu_ref.dequantize(qb, Q), type=2, norm='ortho', axes=(-2, -1)),
                                   (ny_ * 8, nx_ * 8))[:H, :W]
        margin = np.maximum(-128.0 - raw, raw - 127.0)
        yex = (~nz_b[0])[yb, xb] | (margin > E[..., 0])
        if os.environ.get('DC_ONLY') == '1':  # luma DC-only blocks replayed exactly
            yex |= (~acnz_b[0])[yb, xb]
        exv = np.stack([yex & zpl[1], yex & zpl[0] & zpl[1], yex & zpl[0]], axis=-1)
        left = unc & ~exv
        out['ex_rule_covers'] = int((unc & exv).sum())
        out['ex_rule_left'] = int(left.sum())
        tl = left.any(axis=2)
        out['ex_rule_tiles_left'] = sum(bool(tl[t0:t0 + th, t1:t1 + tw].any())
                                        for t0 in range(0, H, th) for t1 in range(0, W, tw))
    print(json.dumps(out))


if __name__ == '__main__':
    main()
