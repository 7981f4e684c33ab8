"""GPU parity of the certified fp32 16x16 forward (csrc/jds_fast16.hip).

k_fwd16f computes colour, prefilter, area average and the 16x16 DCT in fp32.
It keeps a coefficient's rounding only when the host bound (fast_fwd16_bounds,
pinned on the CPU by tests/test_cert_bound_cpu.py) certifies it. Blocks with
an uncertain coefficient go to k_fix_fwd16, the exact fp64 chain of k_fwd16.
Bar: the plan's default (certified) run gives bit-identical coefficients,
reconstruction and statistics to
  * the exact fp64 run (JDS_RUN_EXACT),
  * a run that recomputes every block (JDS_RUN_FWD_FIXALL), and
  * the CPU oracle with Q16 = kron(Q8, ones(2, 2)), at oracle-sized inputs.
Inputs: random images, structured worst cases (flat grays, saturated
primaries, checkerboards, hard edges), ragged sizes, mixed-quality batches, and
BASELINE configs[4] at full size (3840x2160, 4:2:2, 16x16)."""
import numpy as np
import pytest

from oracle import cpu_ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module', autouse=True)
def gpu():
    from jds import build, _abi
    build.build()
    assert _abi.device_count() >= 1, 'no HIP device: the MI355X path has no CPU fallback'


def _structured(h, w, kind, seed=0):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    if kind == 'gray':
        return np.full((h, w, 3), 128, np.uint8)
    if kind == 'primaries':
        cols = np.array([(255, 0, 0), (0, 255, 0), (0, 0, 255), (255, 255, 0), (0, 255, 255), (255, 0, 255),
                         (255, 255, 255), (0, 0, 0)], np.uint8)
        return cols[((yy // 16) * 5 + xx // 16) % 8]
    if kind == 'checker':
        m = ((yy + xx) % 2).astype(bool)
        img = np.zeros((h, w, 3), np.uint8)
        img[m] = (255, 0, 255)
        img[~m] = (0, 255, 0)
        return img
    if kind == 'edges':
        img = np.zeros((h, w, 3), np.uint8)
        img[:, : w // 3] = (255, 0, 0)
        img[:, 2 * w // 3:] = (0, 0, 255)
        img[h // 2:] ^= 255
        return img
    if kind == 'noise_low':  # small integer noise on a flat field: many near-tie roundings
        return np.clip(128 + rng.integers(-2, 3, (h, w, 3)), 0, 255).astype(np.uint8)
    return cpu_ref.random_image(h, w, seed)


def _run(frames, qs, mode, pf, flags):
    import torch
    from jds import _abi, codec
    n, H, W = frames.shape[:3]
    params = [_abi.make_params(q, cpu_ref.scale_quant_matrix(cpu_ref.JPEG_LUMA_Q50, q), mode, pf,
                               codec.gaussian_kernel3(), block_size=16) for q in qs]
    plan = _abi.Plan(_abi.context(0), params, H, W)
    try:
        cpf = plan.geometry.coeffs_per_frame
        dev = torch.device('cuda:0')
        rgb = torch.from_numpy(np.ascontiguousarray(frames)).to(dev)
        out = torch.empty_like(rgb)
        cf = torch.empty((n, cpf), dtype=torch.int16, device=dev)
        st = torch.zeros((n, _abi.STATS_DTYPE.itemsize), dtype=torch.uint8, device=dev)
        # twice: the second run checks that k_fix_fwd16 re-armed its counters
        for _ in range(2):
            plan.run(rgb.data_ptr(), out.data_ptr(), cf.data_ptr(), st.data_ptr(), _abi.RUN_SSE | flags,
                     torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        fixed = int(plan.fix_counts()[0])
        stats = st.cpu().numpy().view(_abi.STATS_DTYPE).reshape(-1).copy()
        return cf.cpu().numpy(), out.cpu().numpy(), stats, fixed, cpf // 256
    finally:
        plan.close()


def _same(a, b):
    for x, y in zip(a[:3], b[:3]):
        assert np.array_equal(x, y)


CASES = [
    ((64, 64), '4:2:0', True, [50]), ((100, 150), '4:2:0', False, [23]), ((48, 40), '4:2:2', True, [77]),
    ((33, 47), '4:4:4', False, [5]), ((256, 320), '4:2:2', False, [95]), ((264, 200), '4:2:0', True, [1]),
    ((130, 98), '4:2:2', True, [50, 10, 100]), ((7, 9), '4:4:4', False, [100]), ((2, 2), '4:2:0', True, [50]),
    ((360, 648), '4:2:2', True, [5, 50, 95]),
]


@pytest.mark.parametrize('shape,mode,pf,qs', CASES)
def test_fast16_matches_exact_fixall_and_oracle(shape, mode, pf, qs):
    h, w = shape
    frames = np.stack([cpu_ref.random_image(h, w, h * 7 + w + i) for i in range(len(qs))])
    fast = _run(frames, qs, mode, pf, 0)
    exact = _run(frames, qs, mode, pf, 8)
    allfix = _run(frames, qs, mode, pf, 64)
    _same(fast, exact)
    _same(allfix, exact)
    assert allfix[3] == len(qs) * allfix[4]  # every block listed and recomputed
    assert fast[3] <= len(qs) * fast[4]
    cf, out, stats = fast[:3]
    for i, q in enumerate(qs):
        ref = cpu_ref.compress_reconstruct(frames[i], q, 16, mode, pf, metrics=False, stretch=True)
        assert np.array_equal(cf[i], ref['coeffs']), q
        assert np.array_equal(out[i], ref['reconstructed']), q
        assert stats[i]['nonzero'] == ref['bitrate']['nonzero_count']
        assert np.array_equal(stats[i]['hist'], ref['hist'])


@pytest.mark.parametrize('kind', ['gray', 'primaries', 'checker', 'edges', 'noise_low'])
@pytest.mark.parametrize('mode,pf', [('4:2:0', True), ('4:2:2', False), ('4:4:4', False)])
def test_fast16_structured_inputs(kind, mode, pf):
    qs = [1, 10, 50, 90, 100]
    frames = np.stack([_structured(96, 160, kind, seed=i) for i in range(len(qs))])
    fast = _run(frames, qs, mode, pf, 0)
    exact = _run(frames, qs, mode, pf, 8)
    _same(fast, exact)
    for i, q in enumerate(qs):
        ref = cpu_ref.compress_reconstruct(frames[i], q, 16, mode, pf, metrics=False, stretch=True)
        assert np.array_equal(fast[0][i], ref['coeffs']), (kind, q)


def test_fast16_configs4_full_size():
    """BASELINE configs[4]: 3840x2160, 4:2:2, 16x16, Q50 -- certified run == exact run == oracle."""
    img = cpu_ref.random_image(2160, 3840, 45)[None]
    fast = _run(img, [50], '4:2:2', True, 0)
    exact = _run(img, [50], '4:2:2', True, 8)
    _same(fast, exact)
    ref = cpu_ref.compress_reconstruct(img[0], 50, 16, '4:2:2', True, metrics=False, stretch=True)
    assert np.array_equal(fast[0][0], ref['coeffs'])
    assert np.array_equal(fast[1][0], ref['reconstructed'])
    rate = fast[3] / fast[4]
    print(f'configs[4]: {fast[3]} of {fast[4]} blocks recomputed ({100 * rate:.2f} %)')
    assert rate < 0.25
