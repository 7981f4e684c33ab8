"""Host-side utilities of the drop-in surface, pinned without a GPU.

* utils.metrics.estimate_bitrate_no_entropy follows the reference's NumPy
  dtype rules (reference utils/metrics.py:72-92): float32 pairwise summation of
  the magnitude bits for int16 input (visible once the sum passes 2**24),
  float64 for int32/int64 input.
* utils.test_images.generate_* reproduce the reference's generators byte for
  byte: their outputs are the inputs of golden cases whose sha256 was taken
  from the reference's own generator (tests/golden/make_golden.py:114-169).
"""
import numpy as np
import pytest

from golden_util import golden, sha


def _reference_expression(q, shape, b):
    """The reference's arithmetic, restated independently (utils/metrics.py:62-92):
    per-element float of ceil(log2(|c|+1)) + 1 in the dtype NumPy picks for
    np.log2 of the input, summed by np.sum."""
    h, w = shape
    nz = q[q != 0]
    nb = (-(-h // b)) * (-(-w // b))
    ftype = np.log2(np.ones(1, dtype=q.dtype)).dtype
    terms = np.ceil(np.log2((np.abs(nz) + 1).astype(nz.dtype))).astype(ftype) + ftype.type(1)
    bits = nb * 2 + (6 * nz.size + terms.sum()) if nz.size else nb * 2
    return int(bits), float(bits / (h * w))


@pytest.mark.parametrize('dtype', [np.int16, np.int32, np.int64])
def test_bitrate_estimate_dtype_rules_above_2_pow_24(dtype):
    from utils.metrics import estimate_bitrate_no_entropy
    rng = np.random.default_rng(7)
    # 4K 4:2:0-sized coefficient array of large magnitudes: the magnitude sum is
    # ~1.9e8 > 2**24, where float32 accumulation loses integers
    q = rng.integers(-1023, 1024, 12_441_600).astype(dtype)
    r = estimate_bitrate_no_entropy(q, (2160, 3840), 8)
    bits, bpp = _reference_expression(q, (2160, 3840), 8)
    assert r['estimated_bits'] == bits
    assert r['bpp'] == bpp
    exact = 129600 * 2 + int(np.sum(7 + np.frexp(np.abs(q[q != 0]).astype(np.float64))[1]))
    if dtype == np.int16:
        assert r['estimated_bits'] != exact  # the reference's float32 drift is reproduced
    else:
        assert r['estimated_bits'] == exact  # float64 accumulation is exact here
    assert r['nonzero_count'] == int(np.count_nonzero(q)) and r['total_coeffs'] == q.size


def test_bitrate_estimate_matches_oracle_and_small_cases():
    from oracle import cpu_ref
    from utils.metrics import estimate_bitrate_no_entropy
    for q, shape in ((np.zeros(192, np.int16), (8, 8)), (np.array([0, 1, -1, 5, -100, 1023], np.int16), (3, 2)),
                     (np.arange(-300, 300, dtype=np.int16), (20, 10))):
        assert estimate_bitrate_no_entropy(q, shape) == cpu_ref.estimate_bitrate_no_entropy(q, shape)


@pytest.mark.parametrize('case,gen,args', [
    ('cfg1_checker512_q50_444', 'generate_colored_checkerboard', (512,)),
    ('checker257_q50_420_pf', 'generate_colored_checkerboard', (257,)),
    ('stripes256w2_q50_422_nopf', 'generate_thin_stripes', (256, 2)),
    ('gradient256_q50_420_pf', 'generate_gradient', (256,)),
    ('gradient131_q60_422_pf', 'generate_gradient', (131,)),
    ('text256_q75_420_nopf', 'generate_text_edges', (256,)),
    ('chroma256_q30_422_pf', 'generate_chroma_stripes', (256,)),
    ('photo256_q50_420_pf', 'generate_photo', (256,)),
])
def test_test_image_generators_match_reference_digests(case, gen, args):
    from utils import test_images
    img = getattr(test_images, gen)(*args)
    assert img.dtype == np.uint8 and img.flags.c_contiguous
    assert sha(img) == golden()[case]['sha_input']
