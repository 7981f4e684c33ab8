"""Adversarial check of the certified fp32 forward's error bound (CPU, no GPU).

The forward kernels (csrc/jds_fast.hip) compute colour, prefilter, area average
and the 8x8 DCT in fp32 and trust a coefficient's rounding only when its fp32
quotient is farther than E_uv / Q (+ slack) from a half-integer, with E_uv a
host-derived bound on |c_fp32 - c_exact| (fast_fwd_bounds).  Here the kernels'
fp32 chain, restated on the host (jds_selftest_fwd32), runs on structured
worst cases -- saturated colours, all-0 / all-255, checkerboards at several
phases, one-pixel spikes, hard colour edges under the prefilter -- and the
exact reference coefficients come from the oracle (the reference's fp64 chain,
engines/color_space.py + engines/dct_engine.py).  The same for the 16x16
forward (csrc/jds_fast16.hip, jds_selftest_fwd16; table kron(Q8, ones(2,2))).
Asserted: the measured error
stays below the bound (ratio < 1) for both pass orders, and every coefficient
the certificate accepts at Q in {1, 50, 95, 100} rounds exactly like the
reference's np.round(c / Q) (engines/quantizer.py:22-24)."""
import ctypes as C

import numpy as np
import pytest

from oracle import cpu_ref


@pytest.fixture(scope='module')
def L():
    from jds import _abi
    return _abi.lib()


def _images():
    rng = np.random.default_rng(123)
    H, W = 32, 64  # every plane a multiple of 16 (the 16x16 variant) at every subsampling
    imgs = {}
    imgs['black'] = np.zeros((H, W, 3), np.uint8)
    imgs['white'] = np.full((H, W, 3), 255, np.uint8)
    imgs['extremes'] = (rng.integers(0, 2, (H, W, 3)) * 255).astype(np.uint8)
    yy, xx = np.mgrid[0:H, 0:W]
    for p in (1, 2, 3, 4):
        for ph in (0, 1):
            m = (((yy + ph) // p + xx // p) % 2).astype(bool)
            img = np.zeros((H, W, 3), np.uint8)
            img[m] = (255, 0, 255)
            img[~m] = (0, 255, 0)
            imgs[f'checker{p}_{ph}'] = img
    prim = np.zeros((H, W, 3), np.uint8)
    cols = [(255, 0, 0), (0, 255, 0), (0, 0, 255), (255, 255, 0), (0, 255, 255), (255, 0, 255), (255, 255, 255),
            (0, 0, 0)]
    for i in range(4):
        for j in range(6):
            prim[8 * i:8 * i + 8, 8 * j:8 * j + 8] = cols[(i * 6 + j) % 8]
    imgs['primaries'] = prim
    edge = np.zeros((H, W, 3), np.uint8)
    edge[:, : W // 2 + 1] = (255, 0, 0)
    edge[:, W // 2 + 1:] = (0, 0, 255)
    imgs['red_blue_edge'] = edge
    spikes = np.zeros((H, W, 3), np.uint8)
    spikes[::7, ::5] = 255
    imgs['spikes'] = spikes
    imgs['random'] = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    imgs['ramp'] = np.broadcast_to((np.arange(W) * 255 // (W - 1)).astype(np.uint8)[None, :, None], (H, W, 3)).copy()
    return imgs


IMAGES = _images()
BLOCKS = {8: 'jds_selftest_fwd32', 16: 'jds_selftest_fwd16'}


def _exact_planes(img, mode, pf):
    ycc = cpu_ref.rgb_to_ycbcr(img.astype(np.float64))
    cb, cr = cpu_ref.subsample_chroma(ycc[..., 1], ycc[..., 2], mode, pf)
    return [ycc[..., 0], cb, cr]


def _thr(E, Q):
    """fast_fwd_thresholds' certification limit (0.5 - E/Q - slack, rounded down to fp32)."""
    t = E / Q * (1 + 1e-5) + 1e-7
    lim = 0.5 - t * (1 + 2.0 ** -20) - 2.0 ** -23
    f = lim.astype(np.float32)
    f = np.where(f.astype(np.float64) > lim, np.nextafter(f, np.float32(0)), f)
    return f


@pytest.mark.parametrize('bs', [8, 16])
@pytest.mark.parametrize('mode,pf', [('4:2:0', True), ('4:2:0', False), ('4:2:2', True), ('4:2:2', False),
                                     ('4:4:4', False)])
def test_fp32_forward_error_within_certified_bound(L, mode, pf, bs):
    gk = cpu_ref.gaussian_kernel3(0.75)
    code = {'4:4:4': 0, '4:2:2': 1, '4:2:0': 2}[mode]
    worst = 0.0
    accepted = wrong = 0
    for name, img in IMAGES.items():
        img = np.ascontiguousarray(img)
        planes = _exact_planes(img, mode, pf)
        for plane in range(3):
            exact = cpu_ref.encode_blocks(cpu_ref.split_blocks(planes[plane], bs)).reshape(-1, bs * bs)
            # bit 0: pass order, bit 1: the combined-tap chroma chain (every certified
            # forward kernel uses it; the bounds cover it alone)
            for rows_first in (3, 2):
                c32 = np.empty(exact.shape, np.float32)
                bound = np.empty(bs * bs, np.float64)
                rc = getattr(L, BLOCKS[bs])(code, int(pf), gk.ctypes.data, img.ctypes.data, img.shape[0],
                                          img.shape[1], plane, rows_first, c32.ctypes.data, bound.ctypes.data)
                assert rc == 0
                ratio = np.abs(c32.astype(np.float64) - exact) / bound
                worst = max(worst, float(ratio.max()))
                assert ratio.max() < 1.0, (name, plane, rows_first, float(ratio.max()))
                # the certificate at several qualities: accepted roundings are the reference's
                for q in (1, 50, 95, 100):
                    Q = cpu_ref.scale_quant_matrix(cpu_ref.JPEG_LUMA_Q50, q)
                    Q = (np.kron(Q, np.ones((2, 2))) if bs == 16 else Q).reshape(-1)  # include/jds.h: Q16
                    rq = (1.0 / Q).astype(np.float32)
                    t = c32 * rq
                    r = np.rint(t)
                    lim = _thr(bound, Q)
                    ok = np.abs(t - r) < (lim - np.abs(t) * np.float32(2.0 ** -22))
                    ref_q = np.round(exact / Q)
                    accepted += int(ok.sum())
                    wrong += int(np.sum(ok & (r != ref_q)))
    print(f'{bs}x{bs} {mode} pf={pf}: worst |c32 - c_exact| / E = {worst:.4f}; {accepted} certified roundings, {wrong} wrong')
    assert wrong == 0
    assert accepted > 0
