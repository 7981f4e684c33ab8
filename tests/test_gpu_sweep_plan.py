"""GPU parity of quality-sweep plans (jds_plan_create_q, BASELINE configs[3]):
the quality-independent front end runs once per frame (k_fwd32i / k_fwd32 in
MQ mode -> fp32 coefficients), k_quant_mq certifies and quantises them for
every table, k_fix_fwd recomputes uncertain blocks per item.  Every item must
equal an independent per-item run (plain plan, exact fp64 kernels) and the
oracle, bit for bit, statistics included."""
import numpy as np
import pytest

from golden_util import golden, sha
from oracle import cpu_ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module', autouse=True)
def gpu():
    from jds import build, _abi
    build.build()
    assert _abi.device_count() >= 1, 'no HIP device: the MI355X path has no CPU fallback'


def run_plan(frames, qs, mode, pf, flags, nq):
    """frames: [F, H, W, 3]; nq > 1: one sweep plan over F frames x qs; nq == 1: a plain
    plan over the replicated items.  Returns (rgb_out, coeffs, stats, fix counts) per item."""
    import torch
    from jds import _abi, codec
    F, H, W = frames.shape[:3]
    params = [_abi.make_params(q, cpu_ref.scale_quant_matrix(cpu_ref.JPEG_LUMA_Q50, q), mode, pf,
                               codec.gaussian_kernel3()) for _ in range(F) for q in qs]
    plan = _abi.Plan(_abi.context(0), params, H, W, nq=nq)
    dev = torch.device('cuda:0')
    src = frames if nq > 1 else np.repeat(frames, len(qs), axis=0)
    rgb = torch.from_numpy(np.ascontiguousarray(src)).to(dev)
    out = torch.empty((len(params), H, W, 3), dtype=torch.uint8, device=dev)
    cf = torch.empty((len(params), plan.geometry.coeffs_per_frame), dtype=torch.int16, device=dev)
    st = torch.zeros((len(params), _abi.STATS_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    plan.run(rgb.data_ptr(), out.data_ptr(), cf.data_ptr(), st.data_ptr(), flags,
             torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    fix = plan.fix_counts()
    plan.close()
    return out.cpu().numpy(), cf.cpu().numpy(), st.cpu().numpy().view(_abi.STATS_DTYPE).reshape(-1), fix


@pytest.mark.parametrize('h,w,mode,pf', [(360, 648, '4:2:0', True), (200, 328, '4:2:2', True),
                                          (184, 260, '4:4:4', False), (130, 98, '4:2:0', False),
                                          (98, 196, '4:2:2', False), (1080, 1920, '4:2:0', True)])
def test_sweep_plan_equals_per_item_runs(h, w, mode, pf):
    from jds import _abi
    qs = [5, 10, 20, 50, 80, 95] if h < 1000 else [10, 50, 95]
    frames = np.stack([cpu_ref.random_image(h, w, 700 + i) for i in range(2)])
    o_s, c_s, s_s, fix = run_plan(frames, qs, mode, pf, _abi.RUN_SSE, len(qs))
    o_p, c_p, s_p, _ = run_plan(frames, qs, mode, pf, _abi.RUN_SSE | _abi.RUN_EXACT, 1)
    assert np.array_equal(c_s, c_p)
    assert np.array_equal(o_s, o_p)
    for fld in ('nonzero', 'magnitude_bits', 'hist', 'sse_rgb', 'total_coeffs', 'block_overhead_bits', 'pixels'):
        assert np.array_equal(s_s[fld], s_p[fld]), fld
    ref = cpu_ref.compress_reconstruct(frames[1], qs[1], 8, mode, pf, metrics=False)
    assert np.array_equal(c_s[len(qs) + 1], ref['coeffs'])
    assert np.array_equal(o_s[len(qs) + 1], ref['reconstructed'])


def test_sweep_plan_exact_mode():
    """RUN_EXACT on a sweep plan: the all-fp64 kernels read frame item // nq."""
    from jds import _abi
    qs = [20, 80, 100]
    frames = np.stack([cpu_ref.random_image(72, 96, 40 + i) for i in range(3)])
    o_e, c_e, s_e, _ = run_plan(frames, qs, '4:2:0', True, _abi.RUN_SSE | _abi.RUN_EXACT, len(qs))
    o_f, c_f, s_f, _ = run_plan(frames, qs, '4:2:0', True, _abi.RUN_SSE, len(qs))
    assert np.array_equal(c_e, c_f) and np.array_equal(o_e, o_f)
    assert np.array_equal(s_e['sse_rgb'], s_f['sse_rgb'])


def test_sweep_plan_resolves_exact_ties():
    """Flat frames put DC/Q on k + 1/2: every tie goes through the per-item fix-up."""
    from jds import _abi
    vals = (127, 129, 131, 133)
    frames = np.stack([np.full((32, 48, 3), v, np.uint8) for v in vals])
    o, c, s, fix = run_plan(frames, [50, 50], '4:2:0', True, 0, 2)
    assert fix[0] > 0
    for i, v in enumerate(vals):
        g = golden()[f'flat{v}_q50_420_pf']
        for q in range(2):
            assert sha(c[2 * i + q]) == g['sha_coeffs'] and sha(o[2 * i + q]) == g['sha_recon']


def test_sweep_device_chunks_more_than_eight_qualities():
    from jds.sweep import sweep_device
    frames = np.stack([cpu_ref.random_image(64, 96, s) for s in (5, 6)])
    qs = list(range(5, 100, 9))  # 11 qualities: plans of 8 + 3
    items = sweep_device(frames, qs, '4:2:2', False)
    assert [(it['frame'], it['quality']) for it in items] == [(f, q) for f in range(2) for q in qs]
    for it in items[::4]:
        ref = cpu_ref.compress_reconstruct(frames[it['frame']], it['quality'], 8, '4:2:2', False, metrics=True)
        assert it['nonzero'] == ref['bitrate']['nonzero_count']
        assert np.array_equal(it['hist'], ref['hist'])
        f = frames[it['frame']]
        assert it['sse_rgb'] == int(((f.astype(np.int64) - ref['reconstructed']) ** 2).sum())
        # the CompressionResult metrics a BatchSweepWorker item carries (gui/worker.py:62-68):
        # PSNR from the exact integer SSE (same float64 value as skimage's), luma PSNR from
        # the fp64 luma SSE summed in tile order (NumPy sums pairwise: a few ulps apart)
        assert it['psnr_rgb'] == pytest.approx(ref['metrics']['psnr_rgb'], rel=1e-12)
        assert it['psnr_y'] == pytest.approx(ref['metrics']['psnr_y'], rel=1e-12)
        # bpp / ratio from NumPy's float32 magnitude-bits sum, as the reference computes them
        assert it['bpp'] == ref['bitrate']['bpp'] and it['compression_ratio'] == ref['bitrate']['compression_ratio']


def test_sweep_device_ssim_fields():
    """ssim=True: the reference CompressionResult's SSIM fields per item, from the
    device-resident reconstructions (jds_psnr_ssim_dev), against the oracle's
    skimage restatement and the host-copy entry point."""
    from jds import codec
    from jds.sweep import sweep_device
    frames = np.stack([cpu_ref.random_image(40, 56, s) for s in (11, 12)])
    qs = [10, 50, 90]
    items = sweep_device(frames, qs, '4:2:0', True, ssim=True)
    for it in items:
        ref = cpu_ref.compress_reconstruct(frames[it['frame']], it['quality'], 8, '4:2:0', True, metrics=True)
        # bitwise: the batched device SSIM is skimage's double, and ssim_rgb the
        # same NumPy mean of the three channel values
        assert it['ssim_rgb'] == ref['metrics']['ssim_rgb']
        assert it['ssim_y'] == ref['metrics']['ssim_y']
        host = codec.psnr_ssim_raw(frames[it['frame']], ref['reconstructed'])
        assert it['ssim_y'] == host[3]
        # with ssim, mse_y is the bit-exact NumPy mean, so psnr_y is the reference's double
        assert it['mse_y'] == host[4] and it['psnr_y'] == ref['metrics']['psnr_y']
        assert it['bpp'] == ref['bitrate']['bpp']


def test_magnitude_bits_f32_dev_matches_numpy_float32_sum():
    """jds_magnitude_bits_f32_dev on device coefficients == NumPy's float32
    np.sum of the reference's magnitude bits (utils/metrics.py:77-78), also past
    2^24 where float32 no longer holds the exact integer sum."""
    import torch
    from jds import codec
    rng = np.random.default_rng(4)
    for n_blocks in (1, 1000, 300000):
        q = rng.integers(-2047, 2048, n_blocks * 64).astype(np.int16)
        q[rng.random(q.size) < 0.3] = 0
        nz = q[q != 0]
        want = float(np.sum(np.ceil(np.log2(np.abs(nz).astype(np.float32) + 1)) + 1, dtype=np.float32))
        d = torch.from_numpy(q).to('cuda:0')
        torch.cuda.synchronize()
        got = codec.magnitude_bits_f32_dev(d.data_ptr(), q.size, 0, None)
        assert got == want, (n_blocks, got, want)


def test_sweep_plan_rejects_bad_shapes():
    from jds import _abi, codec
    q = cpu_ref.scale_quant_matrix(cpu_ref.JPEG_LUMA_Q50, 50)
    p = _abi.make_params(50, q, '4:2:0', True, codec.gaussian_kernel3())
    with pytest.raises(ValueError):
        _abi.Plan(_abi.context(0), [p] * 18, 64, 64, nq=9)  # more than 8 tables per frame
    with pytest.raises(ValueError):
        _abi.Plan(_abi.context(0), [p] * 5, 64, 64, nq=2)   # not a whole number of frames


def exact_sse_y(orig, rec):
    """sum over pixels of (Y(orig) - Y(rec))^2 with Y = .299R + .587G + .114B,
    as the library states it: the integer sum of (299dR + 587dG + 114dB)^2 / 1e6"""
    d = orig.astype(np.int64) - rec.astype(np.int64)
    D = 299 * d[..., 0] + 587 * d[..., 1] + 114 * d[..., 2]
    return int((D * D).sum()) / 1e6


@pytest.mark.parametrize('h,w,mode', [(200, 328, '4:2:0'), (136, 264, '4:2:2'), (1080, 1920, '4:2:0')])
def test_sweep_plan_sse_through_fast_inverse(h, w, mode):
    """RUN_SSE | RUN_INV_FAST on a sweep plan: the certified inverse with the SSE
    terms (k_inv_fast<MODE, 1>) where the library routes them there, coarse
    items through its per-item exact mode from the second run on.  Two runs of
    one plan, both bit-identical to the exact kernels, SSE fields included."""
    import torch
    from jds import _abi, codec
    qs = [5, 10, 20, 50, 80, 95] if h < 1000 else [10, 50]
    F = 2
    frames = np.stack([cpu_ref.random_image(h, w, 810 + i) for i in range(F)])
    o_x, c_x, s_x, _ = run_plan(frames, qs, mode, True, _abi.RUN_SSE | _abi.RUN_EXACT, len(qs))
    # sse_y is an exact integer sum of (299dR + 587dG + 114dB)^2 scaled by 1e-6
    # (the same two roundings as Python's int / float): the same bits from every inverse route, and from NumPy
    _, _, s_2, _ = run_plan(frames, qs, mode, True, _abi.RUN_SSE, len(qs))
    want = np.array([exact_sse_y(frames[i // len(qs)], o_x[i]) for i in range(F * len(qs))])
    assert np.array_equal(s_x['sse_y'].view(np.uint64), want.view(np.uint64))
    assert np.array_equal(s_2['sse_y'].view(np.uint64), want.view(np.uint64))
    params = [_abi.make_params(q, cpu_ref.scale_quant_matrix(cpu_ref.JPEG_LUMA_Q50, q), mode, True,
                               codec.gaussian_kernel3()) for _ in range(F) for q in qs]
    plan = _abi.Plan(_abi.context(0), params, h, w, nq=len(qs))
    dev = torch.device('cuda:0')
    rgb = torch.from_numpy(np.ascontiguousarray(frames)).to(dev)
    out = torch.empty((len(params), h, w, 3), dtype=torch.uint8, device=dev)
    cf = torch.empty((len(params), plan.geometry.coeffs_per_frame), dtype=torch.int16, device=dev)
    st = torch.zeros((len(params), _abi.STATS_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    try:
        for run in range(2):
            out.zero_()
            plan.run(rgb.data_ptr(), out.data_ptr(), cf.data_ptr(), st.data_ptr(),
                     _abi.RUN_SSE | _abi.RUN_INV_FAST, torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            s_f = st.cpu().numpy().view(_abi.STATS_DTYPE).reshape(-1)
            assert np.array_equal(cf.cpu().numpy(), c_x), run
            assert np.array_equal(out.cpu().numpy(), o_x), run
            for fld in ('sse_rgb', 'nonzero', 'magnitude_bits', 'hist', 'pixels'):
                assert np.array_equal(s_f[fld], s_x[fld]), (run, fld)
            assert np.array_equal(s_f['sse_y'].view(np.uint64), s_2['sse_y'].view(np.uint64)), run
    finally:
        plan.close()
