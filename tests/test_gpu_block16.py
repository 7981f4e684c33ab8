"""GPU parity of the 16x16 block path (BASELINE configs[4] stretch: "16x16
block path + 4:2:2 at 4K, int-coeff bit-exact check").

The reference has no runnable 16x16 path (its quantizer raises,
engines/quantizer.py:24), so there are no reference vectors: parity is the HIP
path against the CPU oracle run with block_size=16 and the documented table
Q16 = np.kron(Q8, ones((2, 2))) (oracle/cpu_ref.py::quant_table16) -- "parity
unpinned" against the reference itself.  The oracle's 16-point transforms are
SciPy's (pocketfft), the same library the reference calls.  Bar: bit-exact
coefficients, bytes, error maps, histogram and counts."""
import numpy as np
import pytest
import scipy.fft as sfft

from oracle import cpu_ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module', autouse=True)
def gpu():
    from jds import build, _abi
    build.build()
    assert _abi.device_count() >= 1, 'no HIP device: the MI355X path has no CPU fallback'


def run16(img, quality, mode, prefilter, sel=(0, 0)):
    from engines.pipeline import compress_reconstruct_stretch
    from models import CompressionParams
    return compress_reconstruct_stretch(img, CompressionParams(block_size=16, quality=quality, subsampling_mode=mode,
                                                               use_prefilter=prefilter), sel)


@pytest.mark.parametrize('h,w,mode,pf,q', [
    (64, 64, '4:2:0', True, 50), (100, 150, '4:2:0', False, 23), (48, 40, '4:2:2', True, 77),
    (33, 47, '4:4:4', False, 5), (256, 320, '4:2:2', False, 95), (264, 200, '4:2:0', True, 1),
    (130, 98, '4:2:2', True, 50), (7, 9, '4:4:4', False, 100), (1090, 1000, '4:2:0', True, 60),
    (1080, 1920, '4:2:0', True, 50),
])
def test_block16_matches_oracle(h, w, mode, pf, q):
    img = cpu_ref.random_image(h, w, h * 7 + w)
    ref = cpu_ref.compress_reconstruct(img, q, 16, mode, pf, metrics=True, stretch=True)
    res, inter = run16(img, q, mode, pf)
    assert np.array_equal(inter.all_quantized_coeffs, ref['coeffs'])
    assert np.array_equal(res.reconstructed_image, ref['reconstructed'])
    assert np.array_equal(inter.error_map_y, ref['error_map_y'])
    assert np.array_equal(inter.error_map_rgb, ref['error_map_rgb'])
    assert np.array_equal(inter.quantized_histogram, ref['hist'])
    b = ref['bitrate']
    assert (res.nonzero_coeffs, res.total_coeffs) == (b['nonzero_count'], b['total_coeffs'])
    assert (res.bpp, res.compression_ratio) == (b['bpp'], b['compression_ratio'])
    m = ref['metrics']
    assert (res.psnr_y, res.psnr_rgb, res.ssim_y, res.ssim_rgb) == (m['psnr_y'], m['psnr_rgb'], m['ssim_y'], m['ssim_rgb'])
    assert inter.selected_block_dct is None  # 8x8-only IntermediateData field (include/jds.h)


def test_block16_tiny_images_through_raw_api():
    from jds.codec import compress_reconstruct_raw
    for (h, w, mode) in [(2, 2, '4:2:0'), (1, 5, '4:4:4'), (6, 4, '4:2:2')]:
        img = cpu_ref.random_image(h, w, h + w)
        ref = cpu_ref.compress_reconstruct(img, 50, 16, mode, True, metrics=False, stretch=True)
        raw = compress_reconstruct_raw(img, 50, ref['qtable'][::2, ::2], mode, True, block_size=16)
        assert np.array_equal(raw['coeffs'], ref['coeffs'])
        assert np.array_equal(raw['reconstructed'], ref['reconstructed'])


def test_block16_4k_422_full_size():
    """configs[4] at full size: 3840x2160, 4:2:2, 16x16 blocks, bit-exact coefficients and bytes."""
    img = cpu_ref.random_image(2160, 3840, 45)
    res, inter = run16(img, 50, '4:2:2', True)
    ref = cpu_ref.compress_reconstruct(img, 50, 16, '4:2:2', True, metrics=False, stretch=True)
    assert inter.all_quantized_coeffs.size == 16588800
    assert np.array_equal(inter.all_quantized_coeffs, ref['coeffs'])
    assert np.array_equal(res.reconstructed_image, ref['reconstructed'])


def test_block16_batched_plan():
    import torch
    from jds import _abi, codec
    qs = [5, 50, 95]
    H, W = 360, 648
    frames = np.stack([cpu_ref.random_image(H, W, 100 + s) for s in range(len(qs))])
    params = [_abi.make_params(q, cpu_ref.scale_quant_matrix(cpu_ref.JPEG_LUMA_Q50, q), '4:2:2', True,
                               codec.gaussian_kernel3(), block_size=16) for q in qs]
    plan = _abi.Plan(_abi.context(0), params, H, W)
    cpf = plan.geometry.coeffs_per_frame
    dev = torch.device('cuda:0')
    rgb = torch.from_numpy(frames).to(dev)
    out = torch.empty_like(rgb)
    cf = torch.empty((len(qs), cpf), dtype=torch.int16, device=dev)
    st = torch.zeros((len(qs), _abi.STATS_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    plan.run(rgb.data_ptr(), out.data_ptr(), cf.data_ptr(), st.data_ptr(), _abi.RUN_SSE,
             torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    stats = st.cpu().numpy().view(_abi.STATS_DTYPE).reshape(-1)
    out, cf = out.cpu().numpy(), cf.cpu().numpy()
    for i, q in enumerate(qs):
        ref = cpu_ref.compress_reconstruct(frames[i], q, 16, '4:2:2', True, metrics=False, stretch=True)
        assert np.array_equal(cf[i], ref['coeffs']), q
        assert np.array_equal(out[i], ref['reconstructed']), q
        assert stats[i]['nonzero'] == ref['bitrate']['nonzero_count']
        assert stats[i]['total_coeffs'] == ref['bitrate']['total_coeffs']
        assert np.array_equal(stats[i]['hist'], ref['hist'])
        assert stats[i]['sse_rgb'] == int(((frames[i].astype(np.int64) - ref['reconstructed']) ** 2).sum())
    plan.close()


def test_block16_stage_api():
    """engines.dct2 / idct2 / encode_block / decode_block on 16x16 blocks, quantize with a 16x16
    table: the reference's functions accept these shapes (dct_engine.py:7-27, quantizer.py:22-29)."""
    import engines as E
    rng = np.random.default_rng(16)
    blocks = rng.random((200, 16, 16)) * 255
    d = cpu_ref.encode_blocks(blocks)
    assert np.array_equal(E.encode_block(blocks), d)
    assert np.array_equal(E.dct2(blocks - 128.0), sfft.dctn(blocks - 128.0, type=2, norm='ortho', axes=(1, 2)))
    assert np.array_equal(E.idct2(d), sfft.idctn(d, type=2, norm='ortho', axes=(1, 2)))
    assert np.array_equal(E.decode_block(d), cpu_ref.decode_blocks(d))
    q16 = cpu_ref.quant_table16(cpu_ref.scale_quant_matrix(cpu_ref.JPEG_LUMA_Q50, 30))
    qq = E.quantize(d, q16)
    assert qq.dtype == np.int16 and np.array_equal(qq, cpu_ref.quantize(d, q16))
    assert np.array_equal(E.dequantize(qq, q16), cpu_ref.dequantize(qq, q16))
    with pytest.raises(ValueError, match=r'operands could not be broadcast together with shapes \(200,16,16\) \(8,8\)'):
        E.quantize(d, q16[::2, ::2])
