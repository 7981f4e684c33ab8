"""Pin the CPU oracle (oracle/cpu_ref.py) against the reference's golden vectors.

The fixtures were produced by running the reference itself
(tests/golden/make_golden.py).  Bit-exact: reconstruction bytes, int16
coefficients, error maps, histogram, nonzero count, selected-block arrays.
Metrics: PSNR exact; SSIM vs skimage 0.18.3 within 1e-12.
"""
import numpy as np
import pytest
import scipy.fft as sfft

from oracle import cpu_ref
from golden_util import golden, arrays, sha, case_input, case_params

SMALL = [k for k, v in golden().items() if v['shape'][0] * v['shape'][1] <= 512 * 512]
BIG = [k for k, v in golden().items() if k not in SMALL]


def _check(name, out, metrics=True):
    g = golden()[name]
    assert sha(out['reconstructed']) == g['sha_recon']
    assert sha(out['coeffs']) == g['sha_coeffs']
    assert sha(out['error_map_y']) == g['sha_error_map_y']
    assert sha(out['error_map_rgb']) == g['sha_error_map_rgb']
    assert [int(v) for v in out['hist']] == g['hist']
    br = out['bitrate']
    assert br['nonzero_count'] == g['nonzero_coeffs']
    assert br['total_coeffs'] == g['total_coeffs']
    bpp_key = 'np2_bpp' if np.lib.NumpyVersion(np.__version__) >= '2.0.0' else 'np1_bpp'
    assert br['bpp'] == g[bpp_key]
    if metrics:
        m = out['metrics']
        # log10 differs by <=1 ulp between NumPy 1.26 (golden run) and 2.x
        assert m['psnr_rgb'] == pytest.approx(g['psnr_rgb'], rel=4e-16, abs=0)
        assert m['psnr_y'] == pytest.approx(g['psnr_y'], rel=1e-13, abs=0)
        assert abs(m['ssim_rgb'] - g['ssim_rgb']) < 1e-12
        assert abs(m['ssim_y'] - g['ssim_y']) < 1e-12
    a = arrays()
    if out['selected'] is not None and f'{name}/sel_dct' in a:
        for k, v in out['selected'].items():
            assert np.array_equal(v, a[f'{name}/sel_{k}']), k


@pytest.mark.parametrize('name', SMALL)
def test_oracle_matches_reference_golden(name):
    out = cpu_ref.compress_reconstruct(case_input(name), **case_params(name))
    _check(name, out)
    a = arrays()
    if f'{name}/recon' in a:
        assert np.array_equal(out['reconstructed'], a[f'{name}/recon'])
        assert np.array_equal(out['coeffs'], a[f'{name}/coeffs'])


@pytest.mark.parametrize('name', BIG)
def test_oracle_matches_reference_golden_fullsize(name):
    out = cpu_ref.compress_reconstruct(case_input(name), **case_params(name), metrics=False)
    _check(name, out, metrics=False)


def test_batched_dctn_equals_per_block_calls():
    """The oracle batches scipy.fft.dctn over (n,8,8); the reference calls it
    per block (engines/dct_engine.py:7-14).  Pin that they are bit-identical."""
    rng = np.random.default_rng(0)
    b = rng.random((2000, 8, 8)) * 255 - 128
    batched = sfft.dctn(b, type=2, norm='ortho', axes=(-2, -1))
    single = np.stack([sfft.dctn(x, type=2, norm='ortho') for x in b])
    assert np.array_equal(batched, single)
    ib = sfft.idctn(batched, type=2, norm='ortho', axes=(-2, -1))
    isg = np.stack([sfft.idctn(x, type=2, norm='ortho') for x in batched])
    assert np.array_equal(ib, isg)


def test_quant_tables_at_sweep_qualities():
    """min..max, clipped-to-255 and ==1 counts."""
    exp = {5: (100, 255, 45, 0), 10: (50, 255, 38, 0), 20: (25, 255, 9, 0),
           50: (10, 121, 0, 0), 80: (4, 48, 0, 0), 95: (1, 12, 0, 8)}
    for q, (lo, hi, n255, n1) in exp.items():
        t = cpu_ref.scale_quant_matrix(cpu_ref.JPEG_LUMA_Q50, q)
        assert (t.min(), t.max(), int((t == 255).sum()), int((t == 1).sum())) == (lo, hi, n255, n1)
    assert np.all(cpu_ref.scale_quant_matrix(cpu_ref.JPEG_LUMA_Q50, 100) == 1)


@pytest.mark.parametrize('mode,pf', [('4:2:0', True), ('4:2:2', False), ('4:4:4', False)])
def test_faithful_per_block_loop_equals_vectorised(mode, pf):
    """bench.py's 'faithful' CPU baseline (per-block scipy calls, the
    reference's loop structure) computes the same outputs as the batched oracle."""
    img = cpu_ref.random_image(72, 104, 11)
    a = cpu_ref.compress_reconstruct_faithful(img, 40, mode, pf)
    b = cpu_ref.compress_reconstruct(img, 40, 8, mode, pf, metrics=False)
    assert np.array_equal(a['coeffs'], b['coeffs'])
    assert np.array_equal(a['reconstructed'], b['reconstructed'])


def test_resize_nearest_restatement_properties():
    """cv2 INTER_NEAREST (resizeNN) as restated for upsample_chroma(method=
    'nearest') (reference engines/color_space.py:63).  cv2 is not importable
    here, so the restatement is parity-unpinned; what is pinned: at an exact 2x
    scale every output is the input sample (y // 2, x // 2) (OpenCV's
    documented nearest mapping), outputs are always input values, and at odd
    sizes the source index is floor(d * (1 / (dst / src))) clamped."""
    rng = np.random.default_rng(3)
    c = rng.standard_normal((7, 9))
    up = cpu_ref.resize_nearest(c, 14, 18)
    yy, xx = np.mgrid[0:14, 0:18]
    assert np.array_equal(up, c[yy // 2, xx // 2])
    odd = cpu_ref.resize_nearest(c, 13, 17)
    assert np.isin(odd, c).all()
    sx = [min(int(np.floor(x * (1.0 / (17 / 9)))), 8) for x in range(17)]
    sy = [min(int(np.floor(y * (1.0 / (13 / 7)))), 6) for y in range(13)]
    assert np.array_equal(odd, c[np.ix_(sy, sx)])
    cb, cr = cpu_ref.upsample_chroma(c, -c, (14, 18), method='nearest')
    assert np.array_equal(cb, up) and np.array_equal(cr, -up)
