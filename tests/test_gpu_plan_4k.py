"""The BENCHMARKED plan kernels at the 3840x2160 geometry (BASELINE configs[2],
configs[4] 8x8 and the north-star point) against the reference.

The drop-in compress_reconstruct runs the all-fp64 exact kernels; bench.py runs
device-resident plans whose default kernels differ: the certified fp32
forward k_fwd32i with the first tile row's MCU row folded in (fold_rows: at
2160 rows the tiles are bottom-aligned, so the first 4:2:0 tile row holds an MCU
row above the image), the fp64 fix-up k_fix_fwd, and the certified fast inverse
k_inv_fast (or k_inv2 at coarse tables such as Q10).  Here those kernels run at
full 4K size and must reproduce the reference-run golden digests
(tests/golden, made by running /root/reference: cfg3 = Q10 4:2:0 no prefilter,
cfg5 = Q50 4:2:2 no prefilter), the all-fp64 kernels (RUN_EXACT), the fast
inverse with every tile recomputed (RUN_INV_FIXALL) and the oracle (north-star
point: Q50 4:2:0 with prefilter; reference engines/pipeline.py:17-167)."""
import numpy as np
import pytest

from golden_util import golden, sha, case_input, case_params
from oracle import cpu_ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module', autouse=True)
def gpu():
    from jds import build, _abi
    build.build()
    assert _abi.device_count() >= 1, 'no HIP device: the MI355X path has no CPU fallback'


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


def _golden_check(name, flags_list):
    from jds import _abi  # noqa: F401
    g = golden()[name]
    p = case_params(name)
    img = case_input(name)
    for flags in flags_list:
        o, c, s, fix = _plan_run(img[None], [p['quality']], p['mode'], p['prefilter'], flags)
        assert sha(c[0]) == g['sha_coeffs'], (name, flags)
        assert sha(o[0]) == g['sha_recon'], (name, flags)
        assert [int(v) for v in s[0]['hist']] == g['hist'], (name, flags)
        assert int(s[0]['nonzero']) == g['nonzero_coeffs'] and int(s[0]['total_coeffs']) == g['total_coeffs']


def test_cfg3_4k_q10_420_plan_matches_reference_golden():
    """configs[2]: the plan's default kernels (at this coarse table the exact
    inverse k_inv2), the certified fast inverse (RUN_INV_FAST) with and without
    FIXALL, the exact inverse asked for and the all-fp64 kernels."""
    from jds import _abi
    _golden_check('cfg3_rand4k_s0_q10_420_nopf', [0, _abi.RUN_INV_FAST, _abi.RUN_INV_FAST | _abi.RUN_INV_FIXALL,
                                                  _abi.RUN_EXACT_INV, _abi.RUN_EXACT])


def test_cfg5_4k_q50_422_plan_matches_reference_golden():
    """configs[4], 8x8 blocks: 4:2:2 tiles (8-wave forward workgroups, row-record
    statistics) and k_inv_fast<4:2:2>."""
    from jds import _abi
    _golden_check('cfg5_rand4k_s0_q50_422_nopf', [0, _abi.RUN_INV_FIXALL, _abi.RUN_EXACT])


def test_cfg2_1080p_plan_default_route_matches_reference_golden():
    """configs[1], the headline: the plan's default route (flags = 0: k_fwd32i +
    k_fwd_reduce_rows + k_fix_fwd, then the certified k_inv_fast with its
    in-launch exact tile fallback -- exactly what bench.py times) against the
    reference-run cfg2 digest; then the fallback forced on every tile and the
    exact kernels (the cfg2 golden had only been checked
    through the drop-in's exact kernels and the SSE route)."""
    from jds import _abi
    _golden_check('cfg2_rand1080p_s0_q50_420_pf', [0, _abi.RUN_INV_FIXALL, _abi.RUN_EXACT])


def test_north_star_4k_q50_420_prefilter_plan_equals_exact_and_oracle():
    """The north-star point (BASELINE.json north_star: 4K / Q50 / 4:2:0, prefilter
    on): default == RUN_EXACT == RUN_INV_FIXALL, bit for bit (coefficients,
    bytes, statistics), and == the oracle on every frame."""
    from jds import _abi
    frames = np.stack([cpu_ref.random_image(2160, 3840, 900 + i) for i in range(2)])
    qs = [50, 50]
    o, c, s, fix = _plan_run(frames, qs, '4:2:0', True, 0)
    o_ex, c_ex, s_ex, _ = _plan_run(frames, qs, '4:2:0', True, _abi.RUN_EXACT)
    o_fa, c_fa, s_fa, fix_fa = _plan_run(frames, qs, '4:2:0', True, _abi.RUN_INV_FIXALL)
    assert np.array_equal(c, c_ex) and np.array_equal(c, c_fa)
    assert np.array_equal(o, o_ex) and np.array_equal(o, o_fa)
    for f in ('nonzero', 'magnitude_bits', 'hist', 'total_coeffs'):
        assert np.array_equal(s[f], s_ex[f]) and np.array_equal(s[f], s_fa[f]), f
    assert fix[1] < fix_fa[1]  # the fast inverse certified most tiles; FIXALL recomputed all
    for i in range(len(frames)):
        ref = cpu_ref.compress_reconstruct(frames[i], 50, 8, '4:2:0', True, metrics=False)
        assert np.array_equal(c[i], ref['coeffs']), i
        assert np.array_equal(o[i], ref['reconstructed']), i
        assert [int(v) for v in s[i]['hist']] == [int(v) for v in ref['hist']]


def test_north_star_4k_structured_frames_plan_equals_oracle():
    """Saturated / flat / checker content at 4K: exact ties in the forward and
    exact-integer reconstructions in the inverse, so the fix-up and the
    in-place exact tile fallback both run at the 4K geometry."""
    H, W = 2160, 3840
    yy, xx = np.mgrid[0:H, 0:W]
    checker = np.where(((yy // 3 + xx // 3) % 2)[..., None] == 1, np.uint8(255), np.uint8(0)).repeat(3, axis=2)
    half = np.zeros((H, W, 3), np.uint8)
    half[:, W // 2:] = 255
    half[H // 3:, :, 1] = 128
    frames = np.stack([checker, half])
    o, c, s, fix = _plan_run(frames, [50, 50], '4:2:0', True, 0)
    assert fix[0] > 0 and fix[1] > 0
    for i in range(len(frames)):
        ref = cpu_ref.compress_reconstruct(frames[i], 50, 8, '4:2:0', True, metrics=False)
        assert np.array_equal(c[i], ref['coeffs']), i
        assert np.array_equal(o[i], ref['reconstructed']), i
