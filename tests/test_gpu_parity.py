"""GPU parity: the HIP path (through the C-ABI) against the reference's golden
vectors and against the CPU oracle.  Bar: bit-exact int16 coefficients,
reconstruction bytes, histogram, counts, IntermediateData arrays; PSNR/SSIM
equal to the reference's skimage values up to NumPy's log10 ulp."""
import numpy as np
import pytest

from golden_util import golden, arrays, sha, case_input, case_params
from oracle import cpu_ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module', autouse=True)
def gpu():
    from jds import build, _abi
    build.build()
    n = _abi.device_count()
    assert n >= 1, 'no HIP device: the MI355X path has no CPU fallback'
    return n


def run(img, quality, mode, prefilter, sel=(0, 0)):
    from engines import compress_reconstruct
    from models import CompressionParams
    return compress_reconstruct(img, CompressionParams(quality=quality, subsampling_mode=mode,
                                                       use_prefilter=prefilter), sel)


@pytest.mark.parametrize('name', sorted(golden()))
def test_gpu_matches_reference_golden(name):
    g = golden()[name]
    p = case_params(name)
    res, inter = run(case_input(name), p['quality'], p['mode'], p['prefilter'], p['selected_block_idx'])
    assert sha(inter.all_quantized_coeffs) == g['sha_coeffs']
    assert sha(res.reconstructed_image) == g['sha_recon']
    assert sha(inter.error_map_y) == g['sha_error_map_y']
    assert sha(inter.error_map_rgb) == g['sha_error_map_rgb']
    assert [int(v) for v in inter.quantized_histogram] == g['hist']
    assert res.nonzero_coeffs == g['nonzero_coeffs'] and res.total_coeffs == g['total_coeffs']
    bpp_key = 'np2_bpp' if np.lib.NumpyVersion(np.__version__) >= '2.0.0' else 'np1_bpp'
    ratio_key = bpp_key.replace('bpp', 'compression_ratio')
    assert res.bpp == g[bpp_key] and res.compression_ratio == g[ratio_key]
    # log10 may differ by one ulp between the golden run's NumPy 1.26 and NumPy 2.x
    assert res.psnr_rgb == pytest.approx(g['psnr_rgb'], rel=4e-16, abs=0)
    assert res.psnr_y == pytest.approx(g['psnr_y'], rel=4e-16, abs=0)
    assert res.ssim_y == g['ssim_y']
    assert res.ssim_rgb == pytest.approx(g['ssim_rgb'], rel=2e-16, abs=0)
    a = arrays()
    if f'{name}/sel_dct' in a:
        for k in ('original', 'shifted', 'dct', 'quantized', 'dequantized', 'reconstructed'):
            assert np.array_equal(getattr(inter, f'selected_block_{k}'), a[f'{name}/sel_{k}']), k
    if f'{name}/recon' in a:
        assert np.array_equal(res.reconstructed_image, a[f'{name}/recon'])
        assert np.array_equal(inter.all_quantized_coeffs, a[f'{name}/coeffs'])


@pytest.mark.parametrize('h,w,mode,pf,q', [
    (72, 96, '4:2:0', True, 50), (100, 150, '4:2:0', False, 23), (48, 40, '4:2:2', True, 77),
    (33, 47, '4:4:4', False, 5), (256, 320, '4:2:2', False, 95), (2, 2, '4:2:0', True, 50),
    (14, 6, '4:2:0', True, 50), (7, 7, '4:4:4', False, 100), (264, 200, '4:2:0', True, 1),
])
def test_gpu_matches_oracle_random(h, w, mode, pf, q):
    img = cpu_ref.random_image(h, w, h * 1000 + w)
    ref = cpu_ref.compress_reconstruct(img, q, 8, mode, pf, metrics=h >= 7 and w >= 7)
    if h < 7 or w < 7:
        with pytest.raises(ValueError, match='win_size exceeds image extent'):
            run(img, q, mode, pf)
        from jds.codec import compress_reconstruct_raw
        raw = compress_reconstruct_raw(img, q, ref['qtable'], mode, pf)
        assert np.array_equal(raw['coeffs'], ref['coeffs'])
        assert np.array_equal(raw['reconstructed'], ref['reconstructed'])
        return
    res, inter = run(img, q, mode, pf)
    assert np.array_equal(inter.all_quantized_coeffs, ref['coeffs'])
    assert np.array_equal(res.reconstructed_image, ref['reconstructed'])
    assert np.array_equal(inter.error_map_y, ref['error_map_y'])
    assert np.array_equal(inter.error_map_rgb, ref['error_map_rgb'])
    assert np.array_equal(inter.quantized_histogram, ref['hist'])
    m = ref['metrics']
    assert (res.psnr_y, res.psnr_rgb, res.ssim_y, res.ssim_rgb) == (m['psnr_y'], m['psnr_rgb'], m['ssim_y'], m['ssim_rgb'])


def test_psnr_ssim_standalone_bit_exact():
    from utils.metrics import compute_psnr_ssim
    for (h, w, s) in [(64, 64, 1), (57, 203, 2), (1080, 1920, 3)]:
        a = cpu_ref.random_image(h, w, s)
        b = np.clip(a.astype(np.int16) + cpu_ref.random_image(h, w, s + 7).astype(np.int16) // 16 - 8, 0, 255).astype(np.uint8)
        assert compute_psnr_ssim(a, b) == cpu_ref.compute_psnr_ssim(a, b)


def test_batched_plan_quality_sweep_1080p():
    """Device-resident batch path (bench / cfg4): 6 frames, Q in {5,10,20,50,80,95}."""
    import torch
    from jds import _abi, codec
    qs = [5, 10, 20, 50, 80, 95]
    H, W = 1080, 1920
    frames = np.stack([cpu_ref.random_image(H, W, s) for s in range(len(qs))])
    params = [_abi.make_params(q, cpu_ref.scale_quant_matrix(cpu_ref.JPEG_LUMA_Q50, q), '4:2:0', True,
                               codec.gaussian_kernel3()) for q in qs]
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
        ref = cpu_ref.compress_reconstruct(frames[i], q, 8, '4:2:0', True, metrics=False)
        assert np.array_equal(cf[i], ref['coeffs']), q
        assert np.array_equal(out[i], ref['reconstructed']), q
        assert stats[i]['nonzero'] == ref['bitrate']['nonzero_count']
        assert np.array_equal(stats[i]['hist'], ref['hist'])
        assert stats[i]['sse_rgb'] == int(((frames[i].astype(np.int64) - ref['reconstructed']) ** 2).sum())
    plan.close()


def test_per_stage_api_matches_oracle():
    import engines as E
    rng = np.random.default_rng(5)
    img = rng.integers(0, 256, (40, 56, 3)).astype(np.float64)
    ycc = E.rgb_to_ycbcr(img)
    assert np.array_equal(ycc, cpu_ref.rgb_to_ycbcr(img))
    z = ycc + np.random.default_rng(9).random(ycc.shape) * 30 - 15
    assert np.array_equal(E.ycbcr_to_rgb(z), cpu_ref.ycbcr_to_rgb(z))
    cb, cr = ycc[..., 1], ycc[..., 2]
    for mode in ('4:2:2', '4:2:0'):
        for pf in (False, True):
            got = E.subsample_chroma(cb, cr, mode, pf)
            exp = cpu_ref.subsample_chroma(cb, cr, mode, pf)
            assert np.array_equal(got[0], exp[0]) and np.array_equal(got[1], exp[1]), (mode, pf)
            up = E.upsample_chroma(got[0], got[1], (40, 56))
            upe = cpu_ref.upsample_chroma(exp[0], exp[1], (40, 56))
            assert np.array_equal(up[0], upe[0]) and np.array_equal(up[1], upe[1])
    blocks = rng.random((300, 8, 8)) * 255
    assert np.array_equal(E.encode_block(blocks), cpu_ref.encode_blocks(blocks))
    d = cpu_ref.encode_blocks(blocks)
    assert np.array_equal(E.dct2(blocks - 128.0), d)
    assert np.array_equal(E.decode_block(d), cpu_ref.decode_blocks(d))
    qm = E.scale_quant_matrix(E.JPEG_LUMA_Q50, 37)
    assert np.array_equal(qm, cpu_ref.scale_quant_matrix(cpu_ref.JPEG_LUMA_Q50, 37))
    qq = E.quantize(d, qm)
    assert qq.dtype == np.int16 and np.array_equal(qq, cpu_ref.quantize(d, qm))
    assert np.array_equal(E.dequantize(qq, qm), cpu_ref.dequantize(qq, qm))
    import scipy.fft as sfft
    assert np.array_equal(E.idct2(d), sfft.idctn(d, type=2, norm='ortho', axes=(1, 2)))


@pytest.mark.parametrize('h,w,H,W', [(20, 28, 40, 56), (540, 960, 1080, 1920), (19, 27, 37, 53), (7, 9, 13, 17),
                                      (32, 48, 32, 96)])
def test_upsample_chroma_nearest_matches_oracle(h, w, H, W):
    """upsample_chroma(..., method='nearest') (reference engines/color_space.py:63,
    cv2.INTER_NEAREST) through the per-stage kernel vs the oracle's resizeNN
    restatement: a gather, so equality is exact."""
    import engines as E
    rng = np.random.default_rng(h * 1000 + w)
    cb, cr = rng.uniform(0, 255, (h, w)), rng.uniform(0, 255, (h, w))
    got = E.upsample_chroma(cb, cr, (H, W), method='nearest')
    want = cpu_ref.upsample_chroma(cb, cr, (H, W), method='nearest')
    assert got[0].shape == (H, W)
    assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])


def test_4k_420_full_size_bit_exact():
    img = cpu_ref.random_image(2160, 3840, 21)
    res, inter = run(img, 50, '4:2:0', False)
    ref = cpu_ref.compress_reconstruct(img, 50, 8, '4:2:0', False, metrics=False)
    assert np.array_equal(inter.all_quantized_coeffs, ref['coeffs'])
    assert np.array_equal(res.reconstructed_image, ref['reconstructed'])


def _plan_run(frames, qs, mode, pf, flags):
    import torch
    from jds import _abi, codec
    H, W = frames.shape[1:3]
    params = [_abi.make_params(q, cpu_ref.scale_quant_matrix(cpu_ref.JPEG_LUMA_Q50, q), mode, pf,
                               codec.gaussian_kernel3()) for q in qs]
    plan = _abi.Plan(_abi.context(0), params, H, W)
    dev = torch.device('cuda:0')
    rgb = torch.from_numpy(np.ascontiguousarray(frames)).to(dev)
    out = torch.empty_like(rgb)
    cf = torch.empty((len(qs), plan.geometry.coeffs_per_frame), dtype=torch.int16, device=dev)
    st = torch.zeros((len(qs), _abi.STATS_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    plan.run(rgb.data_ptr(), out.data_ptr(), cf.data_ptr(), st.data_ptr(), flags, 0)
    torch.cuda.synchronize()
    fix = plan.fix_counts()
    plan.close()
    return out.cpu().numpy(), cf.cpu().numpy(), st.cpu().numpy().view(_abi.STATS_DTYPE).reshape(-1), fix


@pytest.mark.parametrize('h,w,mode,pf', [(1080, 1920, '4:2:0', True), (720, 1280, '4:2:2', True),
                                          (256, 384, '4:4:4', False), (130, 98, '4:2:0', False),
                                          (64, 48, '4:2:2', False), (360, 648, '4:2:0', False),
                                          (200, 328, '4:2:2', True), (184, 260, '4:4:4', False),
                                          (226, 516, '4:2:0', True), (98, 196, '4:2:2', False),
                                          # first/last tile rows with MCU rows outside the planes
                                          # folded into the interior launch (fold_rows in jds_fast.hip)
                                          (72, 128, '4:4:4', False), (104, 192, '4:2:0', True),
                                          (88, 128, '4:2:0', True), (72, 256, '4:2:2', True)])
def test_fast_path_equals_exact_path_and_oracle(h, w, mode, pf):
    """Certified fp32 + fp64 fix-up (default) == all-fp64 kernels == oracle, bit for bit."""
    from jds import _abi
    qs = [5, 50, 95, 100]
    frames = np.stack([cpu_ref.random_image(h, w, 300 + i) for i in range(len(qs))])
    o_fast, c_fast, s_fast, fix = _plan_run(frames, qs, mode, pf, _abi.RUN_SSE)
    o_ex, c_ex, s_ex, _ = _plan_run(frames, qs, mode, pf, _abi.RUN_SSE | _abi.RUN_EXACT)
    assert np.array_equal(c_fast, c_ex)
    assert np.array_equal(o_fast, o_ex)
    for f in ('nonzero', 'magnitude_bits', 'hist', 'sse_rgb', 'total_coeffs'):
        assert np.array_equal(s_fast[f], s_ex[f]), f
    ref = cpu_ref.compress_reconstruct(frames[1], 50, 8, mode, pf, metrics=False)
    assert np.array_equal(c_fast[1], ref['coeffs'])
    assert fix[0] < 0.10 * len(qs) * c_fast.shape[1] / 64  # fix-up stays rare on random data (Q=100 is the worst)


def test_fast_path_resolves_exact_ties_through_fixup():
    """Flat planes put DC/Q exactly on k + 1/2 (pocketfft's rounding decides): every
    such block must go through the fp64 fix-up and match the reference."""
    from jds import _abi
    frames = np.stack([np.full((32, 48, 3), v, np.uint8) for v in (127, 129, 131, 133)])
    qs = [50] * 4
    o, c, s, fix = _plan_run(frames, qs, '4:2:0', True, 0)
    assert fix[0] > 0
    for i, v in enumerate((127, 129, 131, 133)):
        g = golden()[f'flat{v}_q50_420_pf']
        assert sha(c[i]) == g['sha_coeffs'] and sha(o[i]) == g['sha_recon']


def test_sweep_device_matches_oracle():
    """cfg4-style sweep: (frame, Q) items through one device-resident plan."""
    from jds.sweep import sweep_device
    frames = np.stack([cpu_ref.random_image(96, 160, s) for s in (1, 2)])
    qs = [10, 50, 95]
    items = sweep_device(frames, qs, '4:2:0', True)
    assert [(it['frame'], it['quality']) for it in items] == [(f, q) for f in range(2) for q in qs]
    for it in items:
        f = frames[it['frame']]
        ref = cpu_ref.compress_reconstruct(f, it['quality'], 8, '4:2:0', True, metrics=False)
        assert it['nonzero'] == ref['bitrate']['nonzero_count']
        assert np.array_equal(it['hist'], ref['hist'])
        assert it['sse_rgb'] == int(((f.astype(np.int64) - ref['reconstructed']) ** 2).sum())


def test_quality_sweep_matches_per_call_reference():
    """BatchSweepWorker.run (gui/worker.py:55-74) semantics."""
    from jds.sweep import quality_sweep
    from models.compression_params import CompressionParams
    img = cpu_ref.random_image(64, 96, 4)
    res = quality_sweep(img, CompressionParams(quality=50, subsampling_mode='4:2:2', use_prefilter=True), 20, 80, 30)
    assert [q for q, _ in res] == [20, 50, 80]
    for q, r in res:
        ref = cpu_ref.compress_reconstruct(img, q, 8, '4:2:2', True, metrics=True)
        assert np.array_equal(r.reconstructed_image, ref['reconstructed'])
        assert (r.psnr_rgb, r.ssim_y) == (ref['metrics']['psnr_rgb'], ref['metrics']['ssim_y'])


@pytest.mark.gpu
def test_plan_rejects_non_integer_quant_table():
    """scale_quant_matrix always yields integers (engines/quantizer.py:16-18); the
    C-ABI rejects anything else with EINVAL (the kernels dequantise in integers)."""
    from jds import _abi, codec
    q = np.full((8, 8), 16.0)
    q[3, 4] = 16.5
    with pytest.raises(ValueError, match='not an integer'):
        _abi.Plan(_abi.context(0), [_abi.make_params(50, q, '4:2:0', True, codec.gaussian_kernel3())], 16, 16)


@pytest.mark.gpu
def test_plan_rejects_misaligned_buffers():
    """Batch buffers must be 16-byte aligned (the kernels' wide loads and stores)."""
    import torch
    from jds import _abi, codec
    params = [_abi.make_params(50, cpu_ref.scale_quant_matrix(cpu_ref.JPEG_LUMA_Q50, 50), '4:2:0', True,
                               codec.gaussian_kernel3())]
    plan = _abi.Plan(_abi.context(0), params, 32, 32)
    dev = torch.device('cuda:0')
    raw = torch.zeros(32 * 32 * 3 + 16, dtype=torch.uint8, device=dev)
    out = torch.empty(32 * 32 * 3, dtype=torch.uint8, device=dev)
    cf = torch.empty(plan.geometry.coeffs_per_frame, dtype=torch.int16, device=dev)
    st = torch.zeros(_abi.STATS_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    try:
        with pytest.raises(ValueError, match='16-byte aligned'):
            plan.run(raw.data_ptr() + 1, out.data_ptr(), cf.data_ptr(), st.data_ptr(), 0, 0)
        plan.run(raw.data_ptr() + 16, out.data_ptr(), cf.data_ptr(), st.data_ptr(), 0, 0)
        torch.cuda.synchronize()
    finally:
        plan.close()


@pytest.mark.parametrize('nq', [1, 3])
def test_repeated_runs_any_phase_order_give_identical_results(nq):
    """The plan keeps no per-run state that leaks into the next run: the
    statistics reset, the per-item fix-up counters and bitmaps are re-armed by
    the kernels themselves (no memsets).  Any sequence of combined, forward-only,
    inverse-only and exact runs reproduces the first run's coefficients, bytes,
    statistics and fix-up count."""
    import torch
    from jds import _abi, codec
    h, w = 200, 328
    qs = [50, 95, 100][:nq]
    frames = np.stack([cpu_ref.random_image(h, w, 900 + i) for i in range(2)])
    params = [_abi.make_params(q, cpu_ref.scale_quant_matrix(cpu_ref.JPEG_LUMA_Q50, q), '4:2:0', True,
                               codec.gaussian_kernel3()) for _ in range(2) for q in qs]
    plan = _abi.Plan(_abi.context(0), params, h, w, nq=nq)
    dev = torch.device('cuda:0')
    rgb = torch.from_numpy(frames).to(dev)
    n = len(params)
    out = torch.empty((n, h, w, 3), dtype=torch.uint8, device=dev)
    cf = torch.empty((n, plan.geometry.coeffs_per_frame), dtype=torch.int16, device=dev)
    st = torch.zeros((n, _abi.STATS_DTYPE.itemsize), dtype=torch.uint8, device=dev)

    def snap():
        torch.cuda.synchronize()
        s = st.cpu().numpy().view(_abi.STATS_DTYPE).reshape(-1)
        return (out.cpu().numpy().copy(), cf.cpu().numpy().copy(),
                {f: s[f].copy() for f in ('nonzero', 'magnitude_bits', 'hist', 'sse_rgb', 'total_coeffs')},
                int(plan.fix_counts()[0]))

    def run(flags):
        out.zero_()
        cf.zero_()
        plan.run(rgb.data_ptr(), out.data_ptr(), cf.data_ptr(), st.data_ptr(), flags, 0)

    try:
        run(_abi.RUN_SSE)
        ref = snap()
        assert ref[3] > 0  # Q >= 50 on random frames always needs some fix-up
        seqs = [[_abi.RUN_SSE], [_abi.RUN_FWD, _abi.RUN_INV | _abi.RUN_SSE], [_abi.RUN_FWD, _abi.RUN_FWD],
                [_abi.RUN_SSE | _abi.RUN_EXACT], [_abi.RUN_SSE]]
        for seq in seqs:
            for fl in seq:
                if fl == _abi.RUN_INV | _abi.RUN_SSE:
                    plan.run(rgb.data_ptr(), out.data_ptr(), cf.data_ptr(), st.data_ptr(), fl, 0)
                else:
                    run(fl)
            if seq == [_abi.RUN_FWD, _abi.RUN_FWD]:
                plan.run(rgb.data_ptr(), out.data_ptr(), cf.data_ptr(), st.data_ptr(), _abi.RUN_INV | _abi.RUN_SSE, 0)
            got = snap()
            assert np.array_equal(got[0], ref[0]) and np.array_equal(got[1], ref[1]), seq
            for f in ref[2]:
                assert np.array_equal(got[2][f], ref[2][f]), (seq, f)
            if not (seq[0] & _abi.RUN_EXACT):
                assert got[3] == ref[3], seq
    finally:
        plan.close()
