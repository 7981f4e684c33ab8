#!/usr/bin/env python3
"""Would a certified fp32 inverse pay?  A census on the bench's own input.

The certified fp64 inverse (csrc/jds_inv_fast.hip) is bit-exact because it
recomputes every 64 x 128 tile in which an output value lands within its
rigorous error bound E of an integer (the truncation edge of
trunc(clip(v)), engines/pipeline.py:95).  With fp64, E ~ 1e-9 and ~1e-3 of the
tiles are recomputed.  This tool measures what the same scheme would face in
fp32: the whole pixel chain of the 4:2:0 inverse (dequantise, 8 x 8 IDCT, clip,
exact-2x bilinear upsample, colour) evaluated in float32 on a uniform-random
1080p frame (the bench's input distribution, Q50, prefilter on), compared with
the reference's fp64 values (oracle/cpu_ref.py, engines/pipeline.py:68-95).

No certificate can be smaller than the largest error actually observed, so the
census uses THAT as an (unattainably optimistic) uniform bound and counts the
output values, 512-pixel waves and 64 x 128-pixel tiles with a value within it
of an integer: the fraction of work the exact fallback would redo even then.
It repeats the count with the fp64 chain's rigorous bound (the shipped
kernel's K_LIN, K_CONST) for comparison.  Tool, not product; the oracle is the
checker here.  Usage: tools/fp32_inverse_census.py [--json out.json]
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import cpu_ref  # noqa: E402

K_LIN, K_CONST = 1.103043e-12 * 1.01, 1.081459e-12 * 1.01  # csrc/jds_inv_fast.hip


def idct_matrix(dtype):
    k = np.arange(8)
    c = np.where(k == 0, np.sqrt(1 / 8), np.sqrt(2 / 8))
    return (c[:, None] * np.cos((2 * k[None, :] + 1) * k[:, None] * np.pi / 16)).astype(dtype)  # [u, x]


def plane_idct(q, Q, nby, nbx, dtype):
    """(q * Q) blocks -> IDCT (axis 0 then axis 1) -> clip, as one plane."""
    M = idct_matrix(dtype)
    d = (q.reshape(nby, nbx, 8, 8).astype(np.int64) * Q.astype(np.int64)).astype(dtype)
    s = np.einsum('ux,abuv->abxv', M, d, dtype=dtype)
    s = np.einsum('vy,abxv->abxy', M, s, dtype=dtype)
    s = np.clip(s + dtype(128), dtype(0), dtype(255))
    return s.transpose(0, 2, 1, 3).reshape(nby * 8, nbx * 8)


def up2(c, H, W, dtype):
    """cv2 INTER_LINEAR at an exact 2x scale (weights 1/4, 3/4, clamped taps)."""
    def axis(a, n_out, ax):
        m = np.arange(n_out) // 2
        odd = (np.arange(n_out) & 1) == 1
        nb = np.clip(np.where(odd, m + 1, m - 1), 0, a.shape[ax] - 1)
        near = np.take(a, m, axis=ax)
        far = np.take(a, nb, axis=ax)
        return near * dtype(0.75) + far * dtype(0.25)
    return axis(axis(c, H, 0), W, 1)


def chain(coeffs, Q, H, W, dtype):
    nby, nbx = (H + 7) // 8, (W + 7) // 8
    hc, wc = (H + 1) // 2, (W + 1) // 2
    ncy, ncx = (hc + 7) // 8, (wc + 7) // 8
    ny, nc = nby * nbx * 64, ncy * ncx * 64
    Y = plane_idct(coeffs[:ny], Q, nby, nbx, dtype)[:H, :W]
    Cb = plane_idct(coeffs[ny:ny + nc], Q, ncy, ncx, dtype)[:hc, :wc]
    Cr = plane_idct(coeffs[ny + nc:], Q, ncy, ncx, dtype)[:hc, :wc]
    Cb, Cr = up2(Cb, H, W, dtype) - dtype(128), up2(Cr, H, W, dtype) - dtype(128)
    R = Y + dtype(1.402) * Cr
    G = Y - dtype(0.344136) * Cb - dtype(0.714136) * Cr
    B = Y + dtype(1.772) * Cb
    return np.stack([R, G, B], axis=-1), max(int(np.abs(coeffs.astype(np.int64)).max()), 1) * float(Q.max())


def census(v, E, H, W):
    """Fractions of values / 512-px waves (8 rows x 64 px) / 64 x 128 tiles
    holding a value within E of an integer inside [0, 255]."""
    # trunc(clip(v, 0, 255)) changes value only at the integers 1 .. 255
    n = np.clip(np.rint(v), 1, 255)
    unc = np.abs(v - n) <= E
    px = unc.any(axis=-1)

    def frac_groups(th, tw):
        hh, ww = (H + th - 1) // th * th, (W + tw - 1) // tw * tw
        p = np.zeros((hh, ww), bool)
        p[:H, :W] = px
        return float(p.reshape(hh // th, th, ww // tw, tw).any(axis=(1, 3)).mean())
    return {'values': float(unc.mean()), 'waves_512px': frac_groups(8, 64), 'tiles_64x128': frac_groups(64, 128)}


def main():
    H, W = 1080, 1920
    img = cpu_ref.random_image(H, W, 1234)
    r = cpu_ref.compress_reconstruct(img, 50, 8, '4:2:0', True, metrics=False)
    ref = r['rgb_rec_f']  # the reference's fp64 values (ycbcr_to_rgb clips to [0, 255])
    coeffs = r['coeffs']
    Qb = r['qtable'].reshape(8, 8)
    v32, dmax = chain(coeffs, Qb, H, W, np.float32)
    v64, _ = chain(coeffs, Qb, H, W, np.float64)
    # the chains' values are unclipped; the reference's are clipped
    err64 = float(np.abs(np.clip(v64, 0, 255) - ref).max())
    err32 = float(np.abs(v32.astype(np.float64) - v64).max())
    e64_bound = K_LIN * dmax + K_CONST + 2 ** -31
    out = {
        'frame': f'{H}x{W} uniform random (cpu_ref.random_image seed 1234), Q50 4:2:0 prefilter on',
        'dmax_qQ': dmax,
        'fp32': {'max_abs_error_observed_vs_fp64_chain': err32, 'uncertain_with_that_as_bound': census(v32.astype(np.float64), err32, H, W)},
        'fp64_matrix_chain': {'max_abs_error_vs_reference': err64},
        'fp64_shipped_bound': {'E': e64_bound, 'uncertain': census(v64, e64_bound, H, W)},
    }
    s = json.dumps(out, indent=1)
    print(s)
    if '--json' in sys.argv:
        open(sys.argv[sys.argv.index('--json') + 1], 'w').write(s + '\n')


if __name__ == '__main__':
    main()
