"""GPU parity for odd image sizes with chroma subsampling (jds_gen.hip).

The reference resizes chroma with cv2.resize(..., INTER_AREA) for any size
(engines/color_space.py:42-49); an odd H (4:2:0) or odd W (4:2:x) takes
OpenCV's fractional-area path, and the INTER_LINEAR upsample back to H x W
(color_space.py:63-65) has non-2x weights.  The golden fixtures of such sizes
(odd*, checker257, gradient131; tests/golden/make_golden.py) run through
test_gpu_parity.py; here: random sizes vs the oracle through the drop-in, the
raw ABI (images under skimage's 7x7 SSIM window), device plans (incl. quality
sweeps) and the per-stage API.  Bar: bit-exact coefficients, bytes, maps,
statistics."""
import numpy as np
import pytest

from oracle import cpu_ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module', autouse=True)
def gpu():
    from jds import build, _abi
    build.build()
    assert _abi.device_count() >= 1, 'no HIP device: the MI355X path has no CPU fallback'


def _drop_in(img, q, mode, pf, sel=(0, 0)):
    from engines import compress_reconstruct
    from models import CompressionParams
    return compress_reconstruct(img, CompressionParams(quality=q, subsampling_mode=mode, use_prefilter=pf), sel)


@pytest.mark.parametrize('h,w,mode,pf,q', [
    (71, 97, '4:2:0', True, 50), (71, 97, '4:2:2', False, 50), (100, 151, '4:2:0', False, 23),
    (49, 40, '4:2:0', True, 77), (48, 41, '4:2:2', True, 95), (257, 8, '4:2:0', True, 10),
    (9, 255, '4:2:2', True, 100), (7, 7, '4:2:0', True, 50), (15, 17, '4:2:0', False, 1),
    (513, 511, '4:2:0', True, 60),
])
def test_odd_sizes_drop_in_vs_oracle(h, w, mode, pf, q):
    img = cpu_ref.random_image(h, w, 31 * h + w)
    ref = cpu_ref.compress_reconstruct(img, q, 8, mode, pf, selected_block_idx=(0, 1))
    res, inter = _drop_in(img, q, mode, pf, (0, 1))
    assert np.array_equal(inter.all_quantized_coeffs, ref['coeffs'])
    assert np.array_equal(res.reconstructed_image, ref['reconstructed'])
    assert np.array_equal(inter.error_map_y, ref['error_map_y'])
    assert np.array_equal(inter.error_map_rgb, ref['error_map_rgb'])
    assert np.array_equal(inter.quantized_histogram, ref['hist'])
    assert res.nonzero_coeffs == ref['bitrate']['nonzero_count']
    m = ref['metrics']
    assert (res.psnr_y, res.psnr_rgb, res.ssim_y, res.ssim_rgb) == (m['psnr_y'], m['psnr_rgb'], m['ssim_y'],
                                                                    m['ssim_rgb'])
    if ref['selected'] is not None:
        for k, v in ref['selected'].items():
            assert np.array_equal(getattr(inter, f'selected_block_{k}'), v), k


@pytest.mark.parametrize('h,w,mode', [(3, 3, '4:2:0'), (2, 3, '4:2:2'), (5, 2, '4:2:0'), (3, 6, '4:2:0'),
                                      (1, 5, '4:2:2')])
def test_odd_tiny_raw_path(h, w, mode):
    # below skimage's 7x7 window the drop-in raises like the reference; the raw ABI still runs
    from jds.codec import compress_reconstruct_raw
    img = cpu_ref.random_image(h, w, h * 7 + w)
    for pf in (False, True):
        ref = cpu_ref.compress_reconstruct(img, 50, 8, mode, pf, metrics=False)
        raw = compress_reconstruct_raw(img, 50, ref['qtable'], mode, pf)
        assert np.array_equal(raw['coeffs'], ref['coeffs'])
        assert np.array_equal(raw['reconstructed'], ref['reconstructed'])
        assert np.array_equal(raw['error_map_y'], ref['error_map_y'])


def test_empty_chroma_plane_raises_like_cv2():
    img = cpu_ref.random_image(1, 9, 3)
    with pytest.raises(ValueError, match='dsize.empty'):
        from jds.codec import compress_reconstruct_raw
        compress_reconstruct_raw(img, 50, cpu_ref.scale_quant_matrix(cpu_ref.JPEG_LUMA_Q50, 50), '4:2:0', False)


def _plan_run(frames, params, H, W, nq=1, flags=0):
    import torch
    from jds import _abi
    plan = _abi.Plan(_abi.context(0), params, H, W, nq=nq)
    cpf = plan.geometry.coeffs_per_frame
    dev = torch.device('cuda:0')
    rgb = torch.from_numpy(frames).to(dev)
    n = len(params)
    out = torch.empty((n, H, W, 3), dtype=torch.uint8, device=dev)
    cf = torch.empty((n, cpf), dtype=torch.int16, device=dev)
    st = torch.zeros((n, _abi.STATS_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    for _ in range(2):  # a second run must not see state of the first
        plan.run(rgb.data_ptr(), out.data_ptr(), cf.data_ptr(), st.data_ptr(), flags,
                 torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    stats = st.cpu().numpy().view(_abi.STATS_DTYPE).reshape(-1)
    plan.close()
    return out.cpu().numpy(), cf.cpu().numpy(), stats


@pytest.mark.parametrize('H,W,mode,pf', [(1081, 1919, '4:2:0', True), (135, 241, '4:2:2', False)])
def test_odd_size_plan_vs_oracle(H, W, mode, pf):
    from jds import _abi, codec
    qs = [10, 50, 90]
    frames = np.stack([cpu_ref.random_image(H, W, 100 + s) for s in range(len(qs))])
    params = [_abi.make_params(q, cpu_ref.scale_quant_matrix(cpu_ref.JPEG_LUMA_Q50, q), mode, pf,
                               codec.gaussian_kernel3()) for q in qs]
    out, cf, stats = _plan_run(frames, params, H, W, flags=_abi.RUN_SSE)
    for i, q in enumerate(qs):
        ref = cpu_ref.compress_reconstruct(frames[i], q, 8, mode, pf, metrics=False)
        assert np.array_equal(cf[i], ref['coeffs']), q
        assert np.array_equal(out[i], ref['reconstructed']), q
        assert stats[i]['nonzero'] == ref['bitrate']['nonzero_count']
        assert np.array_equal(stats[i]['hist'], ref['hist'])
        assert stats[i]['total_coeffs'] == ref['coeffs'].size
        assert stats[i]['sse_rgb'] == int(((frames[i].astype(np.int64) - ref['reconstructed']) ** 2).sum())


def test_odd_size_sweep_plan_vs_oracle():
    from jds import _abi, codec
    H, W, qs = 99, 131, [5, 50, 95]
    frames = np.stack([cpu_ref.random_image(H, W, 200 + s) for s in range(2)])
    params = [_abi.make_params(q, cpu_ref.scale_quant_matrix(cpu_ref.JPEG_LUMA_Q50, q), '4:2:0', True,
                               codec.gaussian_kernel3()) for _ in range(2) for q in qs]
    out, cf, stats = _plan_run(frames, params, H, W, nq=len(qs), flags=_abi.RUN_SSE)
    for f in range(2):
        for j, q in enumerate(qs):
            it = f * len(qs) + j
            ref = cpu_ref.compress_reconstruct(frames[f], q, 8, '4:2:0', True, metrics=False)
            assert np.array_equal(cf[it], ref['coeffs']), (f, q)
            assert np.array_equal(out[it], ref['reconstructed']), (f, q)
            assert stats[it]['sse_rgb'] == int(((frames[f].astype(np.int64) - ref['reconstructed']) ** 2).sum())


@pytest.mark.parametrize('h,w,mode,pf', [(37, 53, '4:2:0', True), (40, 37, '4:2:2', False), (3, 3, '4:2:0', True),
                                         (64, 33, '4:2:0', False)])
def test_stage_subsample_odd(h, w, mode, pf):
    from engines.color_space import subsample_chroma, upsample_chroma
    rng = np.random.default_rng(h * w)
    cb = rng.uniform(0, 255, (h, w))
    cr = rng.uniform(0, 255, (h, w))
    got = subsample_chroma(cb, cr, mode, pf)
    want = cpu_ref.subsample_chroma(cb, cr, mode, pf)
    assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])
    up = upsample_chroma(got[0], got[1], (h, w))
    up_ref = cpu_ref.upsample_chroma(want[0], want[1], (h, w))
    assert np.array_equal(up[0], up_ref[0]) and np.array_equal(up[1], up_ref[1])
