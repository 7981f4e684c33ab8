"""GPU parity of the certified fast 16x16 inverse (k_inv16_fast,
csrc/jds_inv_fast.hip; BASELINE configs[4] stretch).

k_inv16_fast reconstructs 4:2:x frames of 16x16 blocks with fidct16 lines, the
difference-form upsample and the colour terms on the magic grid, and certifies
every truncation against E = K_LIN16 * Dmax + K_CONST16 + 2^-31
(tools/inv_bound.py --b16, pinned on the CPU by tests/test_inv_bound_cpu.py);
a tile with an uncertain value is recomputed by k_inv16s's exact body.  Plans
run it by default for 4:2:x without SSE terms (it measured 511 vs 522 us
against k_inv16s at configs[4]); JDS_RUN_EXACT_INV keeps the exact kernel.
Bar: the fast inverse gives
bit-identical bytes to the exact k_inv16s, to JDS_RUN_INV_FIXALL (every
tile recomputed) and to the CPU oracle with Q16 = kron(Q8, ones(2, 2)):
random and structured frames, ragged sizes, arbitrary int16 coefficients, and
configs[4] at full size.  Runs with SSE terms and 4:4:4 keep the exact
kernels."""
import numpy as np
import pytest

from oracle import cpu_ref
from test_gpu_fast16 import _structured

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module', autouse=True)
def gpu():
    from jds import _abi
    assert _abi.device_count() >= 1, 'no HIP device: the MI355X path has no CPU fallback'


def _run(frames, qs, mode, pf, flags_list, coeffs=None):
    """One plan; per flags value a run on the same frames (forward + inverse,
    or forward then an inverse-only run on `coeffs`).  Returns
    [(rgb_out, coeffs, inverse tiles recomputed)]."""
    import torch
    from jds import _abi, codec
    n, H, W = frames.shape[:3]
    params = [_abi.make_params(q, cpu_ref.scale_quant_matrix(cpu_ref.JPEG_LUMA_Q50, q), mode, pf,
                               codec.gaussian_kernel3(), block_size=16) for q in qs]
    plan = _abi.Plan(_abi.context(0), params, H, W)
    try:
        dev = torch.device('cuda:0')
        rgb = torch.from_numpy(np.ascontiguousarray(frames)).to(dev)
        res = []
        for flags in flags_list:
            out = torch.zeros_like(rgb)
            cf = torch.empty((n, plan.geometry.coeffs_per_frame), dtype=torch.int16, device=dev)
            st = torch.zeros((n, _abi.STATS_DTYPE.itemsize), dtype=torch.uint8, device=dev)
            torch.cuda.synchronize()
            if coeffs is not None:
                plan.run(rgb.data_ptr(), out.data_ptr(), cf.data_ptr(), st.data_ptr(), _abi.RUN_FWD, 0)
                cf.copy_(torch.from_numpy(coeffs).to(dev))
                flags |= _abi.RUN_INV
            plan.run(rgb.data_ptr(), out.data_ptr(), cf.data_ptr(), st.data_ptr(), flags, 0)
            torch.cuda.synchronize()
            res.append((out.cpu().numpy(), cf.cpu().numpy(), int(plan.fix_counts()[1])))
        return res
    finally:
        plan.close()


def _tiles(mode, h, w):
    th, tw = (64, 64) if mode == '4:2:0' else (32, 128)
    return -(-h // th) * -(-w // tw)


CASES = [((64, 64), '4:2:0', True, [50]), ((100, 150), '4:2:0', False, [23, 90]), ((48, 40), '4:2:2', True, [77]),
         ((256, 320), '4:2:2', False, [95, 5]), ((264, 200), '4:2:0', True, [1, 50]),
         ((130, 98), '4:2:2', True, [50, 10, 100]), ((2, 2), '4:2:0', True, [50]), ((360, 648), '4:2:2', True, [50])]


@pytest.mark.parametrize('shape,mode,pf,qs', CASES)
def test_inv16_fast_matches_exact_fixall_and_oracle(shape, mode, pf, qs):
    from jds import _abi
    h, w = shape
    frames = np.stack([cpu_ref.random_image(h, w, 3 * h + w + i) for i in range(len(qs))])
    F = _abi.RUN_INV_FAST
    fast, exact, fixall, default = _run(frames, qs, mode, pf, [F, _abi.RUN_EXACT_INV, F | _abi.RUN_INV_FIXALL, 0])
    assert np.array_equal(fast[1], exact[1])
    assert np.array_equal(fast[0], exact[0]), int(np.sum(fast[0] != exact[0]))
    assert np.array_equal(fixall[0], exact[0])
    assert fixall[2] == len(qs) * _tiles(mode, h, w)  # every tile recomputed
    assert exact[2] == 0 and fast[2] <= fixall[2]
    assert np.array_equal(default[0], fast[0]) and default[2] == fast[2]  # the plan's default is the fast kernel
    for i, q in enumerate(qs):
        ref = cpu_ref.compress_reconstruct(frames[i], q, 16, mode, pf, metrics=False, stretch=True)
        assert np.array_equal(fast[0][i], ref['reconstructed']), q


@pytest.mark.parametrize('kind', ['gray', 'primaries', 'checker', 'edges', 'noise_low'])
@pytest.mark.parametrize('mode,pf', [('4:2:0', True), ('4:2:2', False)])
def test_inv16_fast_structured_inputs(kind, mode, pf):
    """Exact ties (flat and saturated reconstructions) must be listed and
    recomputed: bytes equal the exact kernel's and the oracle's."""
    from jds import _abi
    qs = [1, 10, 50, 90, 100]
    frames = np.stack([_structured(96, 160, kind, seed=i) for i in range(len(qs))])
    fast, exact = _run(frames, qs, mode, pf, [_abi.RUN_INV_FAST, _abi.RUN_EXACT_INV])
    assert np.array_equal(fast[0], exact[0]), (kind, int(np.sum(fast[0] != exact[0])))
    for i, q in enumerate(qs):
        ref = cpu_ref.compress_reconstruct(frames[i], q, 16, mode, pf, metrics=False, stretch=True)
        assert np.array_equal(fast[0][i], ref['reconstructed']), (kind, q)


@pytest.mark.parametrize('scale', [1, 40, 32767])
@pytest.mark.parametrize('mode', ['4:2:2', '4:2:0'])
def test_inv16_fast_arbitrary_int16_coefficients(scale, mode):
    """Inverse-only runs on coefficients the codec never produces (|q| up to
    32767): the bound scales with the tile's max |q| * Q."""
    from jds import _abi, codec
    h, w = 96, 256
    frames = np.stack([cpu_ref.random_image(h, w, 900 + i) for i in range(3)])
    cpf = _abi.geometry(_abi.make_params(50, cpu_ref.scale_quant_matrix(cpu_ref.JPEG_LUMA_Q50, 50), mode, False,
                                         codec.gaussian_kernel3(), block_size=16), h, w).coeffs_per_frame
    rng = np.random.default_rng(scale)
    cf = np.clip(rng.normal(0, scale, (3, cpf)), -32768, 32767).astype(np.int16)
    fast, exact = _run(frames, [5, 50, 100], mode, False, [_abi.RUN_INV_FAST, _abi.RUN_EXACT_INV], coeffs=cf)
    assert np.array_equal(fast[0], exact[0]), int(np.sum(fast[0] != exact[0]))


def test_inv16_fast_configs4_full_size():
    """BASELINE configs[4] (3840x2160, 4:2:2, 16x16, Q50, prefilter): the fast
    inverse == the default exact inverse == oracle, and few tiles fall back."""
    from jds import _abi
    img = cpu_ref.random_image(2160, 3840, 46)[None]
    fast, exact = _run(img, [50], '4:2:2', True, [_abi.RUN_INV_FAST, _abi.RUN_EXACT_INV])
    assert np.array_equal(fast[0], exact[0])
    ref = cpu_ref.compress_reconstruct(img[0], 50, 16, '4:2:2', True, metrics=False, stretch=True)
    assert np.array_equal(fast[0][0], ref['reconstructed'])
    tiles = _tiles('4:2:2', 2160, 3840)
    print(f'configs[4]: {fast[2]} of {tiles} inverse tiles recomputed')
    assert fast[2] <= 0.05 * tiles


@pytest.mark.parametrize('mode,flags', [('4:2:2', 16), ('4:4:4', 0), ('4:4:4', 128)])
def test_inv16_exact_and_444_keep_exact_kernels(mode, flags):
    """JDS_RUN_EXACT_INV (16) keeps k_inv16s, and 4:4:4 16x16 plans keep
    k_chroma16 + k_inv16 even when the fast inverse is requested (no fix-up
    count)."""
    img = cpu_ref.random_image(64, 96, 5)[None]
    (out, cf, fixed), = _run(img, [50], mode, False, [flags])
    assert fixed == 0
    ref = cpu_ref.compress_reconstruct(img[0], 50, 16, mode, False, metrics=False, stretch=True)
    assert np.array_equal(out[0], ref['reconstructed'])
