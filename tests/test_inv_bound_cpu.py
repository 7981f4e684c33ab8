"""The certified fast inverse's error bound, pinned on the CPU (no GPU).

k_inv_fast (csrc/jds_inv_fast.hip) computes the reconstruction (reference
engines/pipeline.py:68-95: dequantize, idctn, +128, clip, cv2 INTER_LINEAR
upsample, ycbcr_to_rgb) in fp64 in a cheaper order than the reference and
trusts a byte only when no integer lies within E = K_LIN * Dmax + K_CONST +
2^-31 of its value (Dmax >= max |q * Q| of the tile).  Here:

* tools/inv_bound.py models the chain as it stands in the kernel source (it
  reads the kernel's constants from the file) and the kernel's K_LIN / K_CONST
  must be at least the model's;
* the kernel's own arithmetic helpers run on the host (jds_selftest_inv_fast,
  unfused and fully fused multiply-adds) on adversarial inputs -- saturated,
  flat, checker, spike, edge, ramp and random images through the oracle's
  forward at Q in {1, 10, 50, 95, 100}, and arbitrary int16 coefficients with
  |q| up to 32767 -- in every mode; the reference's pre-truncation values come
  from the oracle (engines/dct_engine.py:23-27 via scipy, the cv2 INTER_LINEAR
  restatement, engines/color_space.py:17-24 without the final clip).

Asserted: |v_fast - v_ref| < E everywhere (with Dmax taken over the blocks each
pixel reads, tighter than the kernel's tile-wide Dmax), also against the
model's bound without its x2 safety factor, and every value the certificate
accepts truncates to the reference's byte."""
import os
import sys

import numpy as np
import pytest
from scipy.ndimage import maximum_filter

from oracle import cpu_ref

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'tools'))
import inv_bound  # noqa: E402

GRID = 2.0 ** -31  # the kernel's slack for the <= 3 roundings on the magic grid
MODES = {'4:4:4': 0, '4:2:2': 1, '4:2:0': 2}


@pytest.fixture(scope='module')
def L():
    from jds import _abi
    return _abi.lib()


@pytest.fixture(scope='module')
def model():
    res, k_lin, k_const = inv_bound.bounds()
    return k_lin, k_const


def test_kernel_constants_cover_the_model(model):
    k_lin, k_const = model
    K = inv_bound.kernel_constants()
    assert K['K_LIN'] >= k_lin and K['K_CONST'] >= k_const, (K['K_LIN'], k_lin, K['K_CONST'], k_const)
    # the colour terms the model prices are the kernel's
    assert K['colour'] == sorted([1.772, -0.344136, 1.402, -0.714136])
    assert K['MAGIC'] == 1.5 * 2 ** 20
    assert inv_bound.GRID_ROUNDINGS_MAX * inv_bound.GRID_ROUNDING <= inv_bound.KERNEL_GRID_SLACK == GRID
    # the kernel adds exactly that slack
    src = open(os.path.join(inv_bound.CSRC, 'jds_inv_fast.hip')).read()
    assert 'const double E = K_LIN * (q * s_qmax) + K_CONST + 0x1p-31;' in src


def _images(H, W):
    rng = np.random.default_rng(7)
    imgs = {'black': np.zeros((H, W, 3), np.uint8), 'white': np.full((H, W, 3), 255, np.uint8),
            'gray128': np.full((H, W, 3), 128, np.uint8),
            'extremes': (rng.integers(0, 2, (H, W, 3)) * 255).astype(np.uint8),
            'random': rng.integers(0, 256, (H, W, 3), dtype=np.uint8)}
    yy, xx = np.mgrid[0:H, 0:W]
    for p in (1, 3):
        m = ((yy // p + xx // p) % 2).astype(bool)
        img = np.zeros((H, W, 3), np.uint8)
        img[m] = (255, 0, 255)
        img[~m] = (0, 255, 0)
        imgs[f'checker{p}'] = img
    edge = np.zeros((H, W, 3), np.uint8)
    edge[:, : W // 2 + 1] = (255, 0, 0)
    edge[:, W // 2 + 1:] = (0, 0, 255)
    imgs['red_blue_edge'] = edge
    spikes = np.zeros((H, W, 3), np.uint8)
    spikes[::7, ::5] = 255
    imgs['spikes'] = spikes
    imgs['ramp'] = np.broadcast_to((np.arange(W) * 255 // (W - 1)).astype(np.uint8)[None, :, None], (H, W, 3)).copy()
    return imgs


def _planes(mode, H, W):
    sy = 2 if mode == '4:2:0' else 1
    sx = 1 if mode == '4:4:4' else 2
    return [(H, W), (H // sy, W // sx), (H // sy, W // sx)]


def _reference_values(q, Q, mode, H, W):
    """The reference's pre-truncation values (unclipped RGB, fp64) from the
    coefficients, through the oracle."""
    rec, off, bmax = [], 0, []
    for ph, pw in _planes(mode, H, W):
        nby, nbx = -(-ph // 8), -(-pw // 8)
        qb = q[off:off + nby * nbx * 64].reshape(-1, 8, 8)
        off += nby * nbx * 64
        r = cpu_ref.decode_blocks(cpu_ref.dequantize(qb, Q))
        rec.append(cpu_ref.merge_blocks(r, (nby * 8, nbx * 8))[:ph, :pw])
        bmax.append(np.abs(qb.astype(np.int64)).reshape(nby, nbx, 64).max(axis=2) * float(Q.max()))
    y, cb, cr = rec
    if mode != '4:4:4':
        cb, cr = cpu_ref.upsample_chroma(cb, cr, (H, W))
    r = y + 1.402 * (cr - 128.0)
    g = y - 0.344136 * (cb - 128.0) - 0.714136 * (cr - 128.0)
    b = y + 1.772 * (cb - 128.0)
    # Dmax per pixel: its luma block and the chroma blocks its taps can reach
    sy, sx = H // _planes(mode, H, W)[1][0], W // _planes(mode, H, W)[1][1]
    yy, xx = np.mgrid[0:H, 0:W]
    dmax = bmax[0][yy // 8, xx // 8]
    for p in (1, 2):
        dil = maximum_filter(bmax[p], size=3, mode='nearest')
        dmax = np.maximum(dmax, dil[(yy // sy) // 8, (xx // sx) // 8])
    return np.stack([r, g, b], axis=-1), dmax


def _check(L, q, Q, mode, H, W, k_model, stats):
    v_ref, dmax = _reference_values(q, Q, mode, H, W)
    k_lin, k_const = k_model
    K = inv_bound.kernel_constants()
    E = (K['K_LIN'] * dmax + K['K_CONST'] + GRID)[..., None]
    E_model = (k_lin / 2 * dmax + k_const / 2 + 3 * 2.0 ** -33)[..., None]  # no safety factor
    ref_bytes = np.clip(v_ref, 0, 255).astype(np.uint8)
    q = np.ascontiguousarray(q, dtype=np.int16)
    Qc = np.ascontiguousarray(Q, dtype=np.float64)
    for fuse in (0, 1):
        v = np.empty((H, W, 3), np.float64)
        by = np.empty((H, W, 3), np.uint8)
        assert L.jds_selftest_inv_fast(MODES[mode], q.ctypes.data, Qc.ctypes.data, H, W, fuse, v.ctypes.data,
                                       by.ctypes.data) == 0
        err = np.abs(v - v_ref)
        stats['worst'] = max(stats['worst'], float((err / E).max()))
        stats['worst_model'] = max(stats['worst_model'], float((err / E_model).max()))
        assert (err < E).all(), float((err / E).max())
        assert (err <= E_model).all(), float((err / E_model).max())
        # the kernel's byte is clamp(floor(v'), 0, 255) (byte_cert_y)
        assert np.array_equal(by, np.clip(np.floor(v), 0, 255).astype(np.uint8))
        dist = np.abs(v - np.rint(v))
        cert = dist > E
        stats['values'] += cert.size
        stats['certified'] += int(cert.sum())
        bad = cert & (by != ref_bytes)
        assert not bad.any(), (mode, fuse, np.argwhere(bad)[:5])
    return ref_bytes


@pytest.mark.parametrize('mode', list(MODES))
def test_inv_fast_chain_within_bound_codec_outputs(L, model, mode):
    H, W = 40, 72  # not a multiple of 16: padded blocks and a half MCU row at 4:2:0
    stats = {'worst': 0.0, 'worst_model': 0.0, 'values': 0, 'certified': 0}
    for name, img in _images(H, W).items():
        for quality in (1, 10, 50, 95, 100):
            for pf in ((False, True) if mode != '4:4:4' else (False,)):
                out = cpu_ref.compress_reconstruct(img, quality, 8, mode, pf, metrics=False)
                Q = cpu_ref.scale_quant_matrix(cpu_ref.JPEG_LUMA_Q50, quality)
                ref_bytes = _check(L, out['coeffs'], Q, mode, H, W, model, stats)
                # the oracle chain above reproduces the oracle's own reconstruction
                assert np.array_equal(ref_bytes, out['reconstructed']), (name, quality, pf)
    print(f"{mode}: worst |v_fast - v_ref| / E = {stats['worst']:.3e} (model w/o x2: {stats['worst_model']:.3e}); "
          f"{stats['certified']} / {stats['values']} values certified")
    assert stats['certified'] > 0.5 * stats['values']


@pytest.mark.parametrize('mode', list(MODES))
def test_inv_fast_chain_within_bound_arbitrary_coefficients(L, model, mode):
    """int16 coefficients the codec never produces: |q| up to 32767 (the bound
    scales with the tile's max |q|), sparse giants, dense noise, DC-only."""
    H, W = 32, 48
    rng = np.random.default_rng(11)
    n = sum(-(-ph // 8) * -(-pw // 8) * 64 for ph, pw in _planes(mode, H, W))
    cases = {
        'full_range': rng.integers(-32768, 32768, n),
        'small': rng.integers(-3, 4, n),
        'dc_only': np.where(np.arange(n) % 64 == 0, rng.integers(-2000, 2000, n), 0),
        'sparse_giants': np.where(rng.random(n) < 0.02, rng.choice([-32767, 32767], n), rng.integers(-2, 3, n)),
        'ac_max': np.where(np.arange(n) % 64 == 63, 32767, 0),
    }
    stats = {'worst': 0.0, 'worst_model': 0.0, 'values': 0, 'certified': 0}
    for name, q in cases.items():
        for quality in (1, 50, 100):
            Q = cpu_ref.scale_quant_matrix(cpu_ref.JPEG_LUMA_Q50, quality)
            _check(L, q.astype(np.int16), Q, mode, H, W, model, stats)
    print(f"{mode}: worst |v_fast - v_ref| / E = {stats['worst']:.3e} (model w/o x2: {stats['worst_model']:.3e}); "
          f"{stats['certified']} / {stats['values']} values certified")


# ---- 16x16 blocks (k_inv16_fast, BASELINE configs[4] stretch) -------------------
MODES16 = {'4:2:2': 1, '4:2:0': 2}


@pytest.fixture(scope='module')
def model16():
    res, k_lin, k_const = inv_bound.bounds16()
    return k_lin, k_const


def test_kernel_constants16_cover_the_model(model16):
    k_lin, k_const = model16
    K16 = inv_bound.kernel_constants16()
    assert K16['K_LIN16'] >= k_lin and K16['K_CONST16'] >= k_const, (K16, k_lin, k_const)
    src = open(os.path.join(inv_bound.CSRC, 'jds_inv_fast.hip')).read()
    assert 'const double E = K_LIN16 * (q * s_qmax) + K_CONST16 + 0x1p-31;' in src


def _planes16(mode, H, W):
    sy = 2 if mode == '4:2:0' else 1
    return [(H, W), (H // sy, W // 2), (H // sy, W // 2)]


def _reference_values16(q, Q8, mode, H, W):
    """Pre-truncation values of the 16x16 path through the oracle (scipy's
    16-point idctn, the kron(Q8, ones(2, 2)) table, cv2's bilinear restatement)."""
    Q = cpu_ref.quant_table16(Q8)
    rec, off, bmax = [], 0, []
    for ph, pw in _planes16(mode, H, W):
        nby, nbx = -(-ph // 16), -(-pw // 16)
        qb = q[off:off + nby * nbx * 256].reshape(-1, 16, 16)
        off += nby * nbx * 256
        r = cpu_ref.decode_blocks(cpu_ref.dequantize(qb, Q))
        rec.append(cpu_ref.merge_blocks(r, (nby * 16, nbx * 16))[:ph, :pw])
        bmax.append(np.abs(qb.astype(np.int64)).reshape(nby, nbx, 256).max(axis=2) * float(Q.max()))
    y, cb, cr = rec
    cb, cr = cpu_ref.upsample_chroma(cb, cr, (H, W))
    r = y + 1.402 * (cr - 128.0)
    g = y - 0.344136 * (cb - 128.0) - 0.714136 * (cr - 128.0)
    b = y + 1.772 * (cb - 128.0)
    sy, sx = H // _planes16(mode, H, W)[1][0], 2
    yy, xx = np.mgrid[0:H, 0:W]
    dmax = bmax[0][yy // 16, xx // 16]
    for p in (1, 2):
        dil = maximum_filter(bmax[p], size=3, mode='nearest')
        dmax = np.maximum(dmax, dil[(yy // sy) // 16, (xx // sx) // 16])
    return np.stack([r, g, b], axis=-1), dmax


def _check16(L, q, Q8, mode, H, W, k_model, stats):
    v_ref, dmax = _reference_values16(q, Q8, mode, H, W)
    k_lin, k_const = k_model
    K16 = inv_bound.kernel_constants16()
    E = (K16['K_LIN16'] * dmax + K16['K_CONST16'] + GRID)[..., None]
    E_model = (k_lin / 2 * dmax + k_const / 2 + 3 * 2.0 ** -33)[..., None]
    ref_bytes = np.clip(v_ref, 0, 255).astype(np.uint8)
    q = np.ascontiguousarray(q, dtype=np.int16)
    Qc = np.ascontiguousarray(Q8, dtype=np.float64)
    for fuse in (0, 1):
        v = np.empty((H, W, 3), np.float64)
        by = np.empty((H, W, 3), np.uint8)
        assert L.jds_selftest_inv_fast16(MODES16[mode], q.ctypes.data, Qc.ctypes.data, H, W, fuse, v.ctypes.data,
                                         by.ctypes.data) == 0
        err = np.abs(v - v_ref)
        stats['worst'] = max(stats['worst'], float((err / E).max()))
        stats['worst_model'] = max(stats['worst_model'], float((err / E_model).max()))
        assert (err < E).all(), float((err / E).max())
        assert (err <= E_model).all(), float((err / E_model).max())
        assert np.array_equal(by, np.clip(np.floor(v), 0, 255).astype(np.uint8))
        cert = np.abs(v - np.rint(v)) > E
        stats['values'] += cert.size
        stats['certified'] += int(cert.sum())
        bad = cert & (by != ref_bytes)
        assert not bad.any(), (mode, fuse, np.argwhere(bad)[:5])
    return ref_bytes


@pytest.mark.parametrize('mode', list(MODES16))
def test_inv_fast16_chain_within_bound_codec_outputs(L, model16, mode):
    H, W = 48, 80  # not multiples of 32: padded blocks and a half MCU row at 4:2:0
    stats = {'worst': 0.0, 'worst_model': 0.0, 'values': 0, 'certified': 0}
    for name, img in _images(H, W).items():
        for quality in (1, 10, 50, 100):
            pf = name in ('random', 'checker1', 'red_blue_edge')
            out = cpu_ref.compress_reconstruct(img, quality, 16, mode, pf, metrics=False, stretch=True)
            Q8 = cpu_ref.scale_quant_matrix(cpu_ref.JPEG_LUMA_Q50, quality)
            ref_bytes = _check16(L, out['coeffs'], Q8, mode, H, W, model16, stats)
            assert np.array_equal(ref_bytes, out['reconstructed']), (name, quality)
    print(f"16x16 {mode}: worst |v_fast - v_ref| / E = {stats['worst']:.3e} "
          f"(model w/o x2: {stats['worst_model']:.3e}); {stats['certified']} / {stats['values']} values certified")
    assert stats['certified'] > 0.5 * stats['values']


@pytest.mark.parametrize('mode', list(MODES16))
def test_inv_fast16_chain_within_bound_arbitrary_coefficients(L, model16, mode):
    H, W = 32, 64
    rng = np.random.default_rng(13)
    n = sum(-(-ph // 16) * -(-pw // 16) * 256 for ph, pw in _planes16(mode, H, W))
    cases = {
        'full_range': rng.integers(-32768, 32768, n),
        'small': rng.integers(-3, 4, n),
        'dc_only': np.where(np.arange(n) % 256 == 0, rng.integers(-4000, 4000, n), 0),
        'sparse_giants': np.where(rng.random(n) < 0.02, rng.choice([-32767, 32767], n), rng.integers(-2, 3, n)),
        'ac_max': np.where(np.arange(n) % 256 == 255, 32767, 0),
        'odd_only': np.where((np.arange(n) % 256) % 2 == 1, rng.integers(-300, 300, n), 0),
    }
    stats = {'worst': 0.0, 'worst_model': 0.0, 'values': 0, 'certified': 0}
    for name, q in cases.items():
        for quality in (1, 50, 100):
            Q8 = cpu_ref.scale_quant_matrix(cpu_ref.JPEG_LUMA_Q50, quality)
            _check16(L, q.astype(np.int16), Q8, mode, H, W, model16, stats)
    print(f"16x16 {mode}: worst |v_fast - v_ref| / E = {stats['worst']:.3e} "
          f"(model w/o x2: {stats['worst_model']:.3e}); {stats['certified']} / {stats['values']} values certified")
