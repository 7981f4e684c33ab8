"""The certified fast inverse (csrc/jds_inv_fast.hip) against the replayed-order
exact inverse (k_inv2) and the oracle.

The fast kernel reaches the reference's bytes (engines/pipeline.py:68-95)
through a different fp64 operation order and certifies every truncation with
a rigorous bound (tools/inv_bound.py); tiles with an uncertain sample go
through the exact kernel (k_inv2_list).  Bar: bit-identical bytes, SSE and
luma SSE with the default (fast), JDS_RUN_EXACT_INV (exact) and
JDS_RUN_INV_FIXALL (fast, then every tile recomputed by the exact tile code).
Plans take the wave-local k_inv_fast444 at 4:4:4 and, for 4:2:x plans with a
coarse table, the exact k_inv2 (most tiles of such frames would fall back);
JDS_RUN_INV_FAST asks for the certified kernel there.  Both are checked
against the exact kernel."""
import numpy as np
import pytest

from oracle import cpu_ref
from golden_util import golden, sha

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module', autouse=True)
def gpu():
    from jds import _abi
    assert _abi.device_count() >= 1, 'no HIP device: the MI355X path has no CPU fallback'


def _plan(frames, qs, mode, pf, flags_list, coeffs=None):
    """Run one plan once per flags value on the same frames; optionally replace
    the coefficients before an inverse-only run.  Returns [(out, cf, stats, fix)]."""
    import torch
    from jds import _abi, codec
    H, W = frames.shape[1:3]
    params = [_abi.make_params(q, cpu_ref.scale_quant_matrix(cpu_ref.JPEG_LUMA_Q50, q), mode, pf,
                               codec.gaussian_kernel3()) for q in qs]
    plan = _abi.Plan(_abi.context(0), params, H, W)
    dev = torch.device('cuda:0')
    rgb = torch.from_numpy(np.ascontiguousarray(frames)).to(dev)
    res = []
    for flags in flags_list:
        out = torch.zeros_like(rgb)
        cf = torch.empty((len(qs), plan.geometry.coeffs_per_frame), dtype=torch.int16, device=dev)
        st = torch.zeros((len(qs), _abi.STATS_DTYPE.itemsize), dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        if coeffs is not None:
            plan.run(rgb.data_ptr(), out.data_ptr(), cf.data_ptr(), st.data_ptr(), _abi.RUN_FWD, 0)
            cf.copy_(torch.from_numpy(coeffs).to(dev))
            flags |= _abi.RUN_INV
        plan.run(rgb.data_ptr(), out.data_ptr(), cf.data_ptr(), st.data_ptr(), flags, 0)
        torch.cuda.synchronize()
        res.append((out.cpu().numpy(), cf.cpu().numpy(), st.cpu().numpy().view(_abi.STATS_DTYPE).reshape(-1),
                    plan.fix_counts()))
    plan.close()
    return res


def _same(a, b, sse=False):
    assert np.array_equal(a[0], b[0]), int(np.sum(a[0] != b[0]))
    assert np.array_equal(a[1], b[1])
    if sse:
        assert np.array_equal(a[2]['sse_rgb'], b[2]['sse_rgb'])
        assert np.array_equal(a[2]['sse_y'], b[2]['sse_y'])


@pytest.mark.parametrize('h,w,mode,pf', [(1080, 1920, '4:2:0', True), (720, 1280, '4:2:2', True),
                                          (256, 384, '4:4:4', False), (130, 98, '4:2:0', False),
                                          (64, 48, '4:2:2', False), (226, 516, '4:2:0', True),
                                          (184, 260, '4:4:4', False), (98, 196, '4:2:2', False),
                                          (8, 16, '4:2:0', False), (2, 2, '4:2:0', True)])
def test_fast_inverse_equals_exact_inverse_random(h, w, mode, pf):
    from jds import _abi
    qs = [1, 10, 50, 95, 100]
    frames = np.stack([cpu_ref.random_image(h, w, 700 + i) for i in range(len(qs))])
    F = _abi.RUN_INV_FAST  # the plan would pick k_inv2 for some of these 4:2:x qualities
    fast, exact, fixall = _plan(frames, qs, mode, pf, [F, _abi.RUN_EXACT_INV, F | _abi.RUN_INV_FIXALL])
    _same(fast, exact)
    _same(fixall, exact)
    assert fixall[3][1] > 0  # every tile was listed
    ref = cpu_ref.compress_reconstruct(frames[2], 50, 8, mode, pf, metrics=False)
    assert np.array_equal(fast[0][2], ref['reconstructed'])
    fs, es = _plan(frames, qs, mode, pf, [_abi.RUN_SSE | F, _abi.RUN_SSE | _abi.RUN_EXACT_INV])
    _same(fs, es, sse=True)


def test_fast_inverse_lists_few_tiles_on_random_1080p():
    frames = np.stack([cpu_ref.random_image(1080, 1920, 800 + i) for i in range(4)])
    (out, cf, st, fix), = _plan(frames, [50] * 4, '4:2:0', True, [0])
    tiles = 4 * 17 * 15  # 64 x 128 tiles of a 1080p 4:2:0 frame
    assert fix[1] <= 0.01 * tiles
    ref = cpu_ref.compress_reconstruct(frames[3], 50, 8, '4:2:0', True, metrics=False)
    assert np.array_equal(out[3], ref['reconstructed'])


STRUCTURED = {
    'checker': lambda: cpu_ref.generate_colored_checkerboard(256),
    'gray': lambda: np.full((96, 160, 3), 128, np.uint8),
    'black_white': lambda: np.concatenate([np.zeros((64, 128, 3), np.uint8), np.full((64, 128, 3), 255, np.uint8)]),
    'stripes': lambda: cpu_ref.generate_thin_stripes(128, 2),
    'flat127': lambda: np.full((64, 96, 3), 127, np.uint8),
    'ramp': lambda: np.broadcast_to((np.arange(256, dtype=np.uint8)[None, :, None]), (64, 256, 3)).copy(),
}


@pytest.mark.parametrize('name', sorted(STRUCTURED))
@pytest.mark.parametrize('mode', ['4:2:0', '4:2:2', '4:4:4'])
def test_fast_inverse_structured_images(name, mode):
    """Exact ties (reference values an integer up to pocketfft noise) must be
    listed and recomputed: bytes equal the exact kernel's and the oracle's."""
    from jds import _abi
    img = STRUCTURED[name]()
    frames = np.stack([img, img])
    fast, exact = _plan(frames, [50, 90], mode, mode != '4:4:4', [_abi.RUN_INV_FAST, _abi.RUN_EXACT_INV])
    _same(fast, exact)
    ref = cpu_ref.compress_reconstruct(img, 90, 8, mode, mode != '4:4:4', metrics=False)
    assert np.array_equal(fast[0][1], ref['reconstructed'])


def test_fast_inverse_checkerboard_golden_needs_fixups():
    """cfg1: every sample of value 30 decodes to 29.999... in the reference
    (SURVEY §8(a)(13)); the fast kernel must hand those tiles to the exact one."""
    from jds import _abi
    img = cpu_ref.generate_colored_checkerboard(512)
    (out, cf, st, fix), = _plan(img[None], [50], '4:4:4', False, [_abi.RUN_INV_FAST])
    assert fix[1] > 0
    g = golden()['cfg1_checker512_q50_444']
    assert sha(out[0]) == g['sha_recon']


@pytest.mark.parametrize('scale', [1, 40, 32767])
def test_fast_inverse_arbitrary_int16_coefficients(scale):
    """Inverse-only runs on coefficients the codec never produces (|q| up to
    32767): the bound scales with the tile's max |q| * Q, so the bytes still
    match the exact kernel."""
    from jds import _abi
    h, w = 128, 256
    frames = np.stack([cpu_ref.random_image(h, w, 900 + i) for i in range(3)])
    rng = np.random.default_rng(scale)
    geo_cpf = None
    for mode in ('4:2:0', '4:4:4'):
        from jds import codec
        geo_cpf = _abi.geometry(_abi.make_params(50, cpu_ref.scale_quant_matrix(cpu_ref.JPEG_LUMA_Q50, 50), mode,
                                                 False, codec.gaussian_kernel3()), h, w).coeffs_per_frame
        cf = np.clip(rng.normal(0, scale, (3, geo_cpf)), -32768, 32767).astype(np.int16)
        fast, exact = _plan(frames, [5, 50, 100], mode, False, [_abi.RUN_INV_FAST, _abi.RUN_EXACT_INV], coeffs=cf)
        _same(fast, exact)


@pytest.mark.parametrize('mode,q,fast', [('4:2:0', 50, True), ('4:2:2', 20, True), ('4:2:0', 10, False),
                                         ('4:4:4', 50, True), ('4:4:4', 10, True)])
def test_default_inverse_route(mode, q, fast):
    """The plan's own choice (the certified fast inverse, the wave-local
    k_inv_fast444 at 4:4:4, k_inv2 for coarse 4:2:x tables) gives the exact
    kernel's bytes; the fix-up counter shows which
    kernel ran (k_inv2 reports none, the fast kernels list the checkerboard's
    ties)."""
    from jds import _abi
    frames = np.stack([cpu_ref.generate_colored_checkerboard(256)] * 2)  # ties: the fast kernel lists tiles
    dflt, exact = _plan(frames, [q, q], mode, mode != '4:4:4', [0, _abi.RUN_EXACT_INV])
    _same(dflt, exact)
    if not fast:
        assert dflt[3][1] == 0
    else:
        assert dflt[3][1] > 0


def _coarse_frames(h, w, seed):
    """Random frames plus saturated structure: pure primaries, black and white
    blocks (clipped luma beside all-zero chroma blocks at coarse tables)."""
    rnd = cpu_ref.random_image(h, w, seed)
    prim = np.zeros((h, w, 3), np.uint8)
    cols = np.array([[255, 0, 0], [0, 255, 0], [0, 0, 255], [255, 255, 255], [0, 0, 0], [255, 255, 0]], np.uint8)
    yy, xx = np.mgrid[0:h, 0:w]
    prim[:] = cols[((yy // 24) * 7 + xx // 40) % len(cols)]
    half = rnd.copy()
    half[:, : w // 2] = 255
    half[h // 2:, :, 1:] = 0
    return [rnd, prim, half]


@pytest.mark.parametrize('mode', ['4:2:0', '4:2:2'])
@pytest.mark.parametrize('h,w', [(256, 384), (136, 200), (1080, 1920)])
def test_coarse_tables(mode, h, w):
    """Coarse tables: the default route (k_inv2) == the certified kernel
    (RUN_INV_FAST) == k_inv2 asked for == the certified kernel with every tile
    recomputed == the oracle, on random and saturated frames at Q 1 .. 13; on
    random Q10 frames the certified kernel hands tiles to its fallback and the
    default route reports none."""
    from jds import _abi
    qs = [1, 5, 10, 13, 10, 5] if h * w < 1e6 else [10, 5]
    fr = _coarse_frames(h, w, 40)
    frames = np.stack([fr[i % 3] for i in range(len(qs))])
    ex, = _plan(frames, qs, mode, False, [0])
    plain, = _plan(frames, qs, mode, False, [_abi.RUN_INV_FAST])
    exact, fixall = _plan(frames, qs, mode, False, [_abi.RUN_EXACT_INV, _abi.RUN_INV_FIXALL])
    _same(ex, exact)
    _same(plain, exact)
    _same(fixall, exact)
    for i in (0, 1, 2) if len(qs) > 2 else (0, 1):
        ref = cpu_ref.compress_reconstruct(frames[i], qs[i], 8, mode, False, metrics=False)
        assert np.array_equal(ex[0][i], ref['reconstructed']), (i, qs[i])
    # random frames at Q10: the plain certificate hands most tiles to the exact code
    rnd = np.stack([cpu_ref.random_image(h, w, 50 + i) for i in range(2)])
    ex2, = _plan(rnd, [10, 10], mode, False, [0])
    plain2, = _plan(rnd, [10, 10], mode, False, [_abi.RUN_INV_FAST])
    _same(ex2, plain2)
    assert ex2[3][1] == 0, ex2[3]
    assert plain2[3][1] > 0 or h * w < 1e5, plain2[3]  # (a small frame may certify every tile)
