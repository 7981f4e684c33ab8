"""K4 v2 (csrc/jds_ssim_band.hip): the batched, band-swept SSIM pipeline against
the oracle's NumPy / scipy restatement of utils/metrics.py:9-28
(oracle/cpu_ref.py psnr_ssim_raw), bit for bit on all six values, over sizes
that exercise every edge of the sweep (7-px images, partial bands, partial
column chunks, partial NumPy buffers, odd map sizes).  (Rounds 1-4 compared
with the round-1..3 kernels instead; those left the product library in round 5.)"""
import numpy as np
import pytest

from oracle import cpu_ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module', autouse=True)
def gpu():
    from jds import build, _abi
    build.build()
    assert _abi.device_count() >= 1, 'no HIP device: the MI355X path has no CPU fallback'


def _pair(h, w, seed, kind):
    a = cpu_ref.random_image(h, w, seed)
    if kind == 'noise':    # a reconstruction-like neighbour of a
        d = cpu_ref.random_image(h, w, seed + 101).astype(np.int16) // 16 - 8
        b = np.clip(a.astype(np.int16) + d, 0, 255).astype(np.uint8)
    elif kind == 'flat':   # constant images: zero variances, exact-integer corner cases
        a = np.full((h, w, 3), 30, np.uint8)
        b = np.full((h, w, 3), 29, np.uint8)
    elif kind == 'smooth':  # gradients: large sums, small differences
        yy, xx = np.mgrid[0:h, 0:w]
        a = np.stack([(xx * 255 // max(w - 1, 1)), (yy * 255 // max(h - 1, 1)), (xx + yy) % 256], -1).astype(np.uint8)
        b = np.clip(a.astype(np.int16) + (xx % 3 - 1)[..., None], 0, 255).astype(np.uint8)
    else:                  # independent images
        b = cpu_ref.random_image(h, w, seed + 202)
    return np.ascontiguousarray(a), np.ascontiguousarray(b)


SIZES = [(7, 7), (7, 40), (40, 7), (8, 9), (13, 8), (14, 14), (15, 39), (23, 70), (31, 37), (64, 64),
         (100, 37), (129, 131), (135, 131), (255, 257), (518, 931), (1080, 1920)]  # 135x131: odd NB, W, items


@pytest.mark.parametrize('h,w', SIZES)
def test_batched_pipeline_equals_oracle_bitwise(h, w):
    import torch
    from jds import codec
    kinds = ['noise', 'indep', 'flat', 'smooth'] if h * w <= 300000 else ['noise']
    pairs = [_pair(h, w, 17 + i, k) for i, k in enumerate(kinds)]
    dev = torch.device('cuda', 0)
    ta = [torch.from_numpy(a).to(dev) for a, _ in pairs]
    tb = [torch.from_numpy(b).to(dev) for _, b in pairs]
    torch.cuda.synchronize()
    batch = codec.psnr_ssim_batch_dev([t.data_ptr() for t in ta], [t.data_ptr() for t in tb], h, w, 0, None)
    for k, (a, b) in enumerate(pairs):
        ref = cpu_ref.psnr_ssim_raw(a, b)
        one = codec.psnr_ssim_dev(ta[k].data_ptr(), tb[k].data_ptr(), h, w, 0)
        assert np.array_equal(batch[k].view(np.uint64), ref.view(np.uint64)), (kinds[k], batch[k], ref)
        assert np.array_equal(one.view(np.uint64), ref.view(np.uint64)), (kinds[k], one, ref)


@pytest.mark.parametrize('h,w', [(7, 7), (31, 37), (100, 37), (257, 130)])
def test_metrics_api_equals_oracle(h, w):
    """utils.metrics.compute_psnr_ssim (host arrays) against the restatement (the
    golden fixtures pin that one to skimage)."""
    from utils.metrics import compute_psnr_ssim
    for i, k in enumerate(['noise', 'indep', 'smooth']):
        a, b = _pair(h, w, 5 + i, k)
        assert compute_psnr_ssim(a, b) == cpu_ref.compute_psnr_ssim(a, b)


def test_batch_of_37_small_pairs():
    """37 small pairs: R, G, B by the rows kernel (>= 32 pairs), the luma in one
    launch (the 16 GB scratch budget holds them all; the multi-group case is
    test_scratch_budget_groups_equal_oracle)."""
    import torch
    from jds import codec
    h, w = 21, 29
    pairs = [_pair(h, w, 300 + i, 'noise' if i % 2 else 'indep') for i in range(37)]
    dev = torch.device('cuda', 0)
    ta = [torch.from_numpy(a).to(dev) for a, _ in pairs]
    tb = [torch.from_numpy(b).to(dev) for _, b in pairs]
    torch.cuda.synchronize()
    r = codec.psnr_ssim_batch_dev([t.data_ptr() for t in ta], [t.data_ptr() for t in tb], h, w, 0, None)
    for k, (a, b) in enumerate(pairs):
        ref = codec.psnr_ssim_raw(a, b)
        assert np.array_equal(r[k], ref)


ROWS_SIZES = [(7, 7), (8, 9), (15, 39), (23, 70), (100, 37), (129, 131), (135, 131), (255, 257), (518, 931)]


@pytest.mark.parametrize('h,w', ROWS_SIZES)
def test_rows_path_equals_oracle_bitwise(h, w):
    """Batches of 32 pairs or more take the R, G, B rows kernel (k_ss_rows: leaf
    sums in-lane, row-crossing leaves and the partial buffer raw, k_ss_rgbsum):
    every item bit-exact against the oracle, over narrow maps (a leaf per slot),
    wide ones (a slot per row boundary), partial buffers and images whose byte
    count is not a multiple of 4 (the staging's patched last dword)."""
    import torch
    from jds import codec
    kinds = ['noise', 'indep', 'flat', 'smooth']
    pairs = [_pair(h, w, 41 + i, k) for i, k in enumerate(kinds)]
    refs = [cpu_ref.psnr_ssim_raw(a, b) for a, b in pairs]
    dev = torch.device('cuda', 0)
    ta = [torch.from_numpy(a).to(dev) for a, _ in pairs]
    tb = [torch.from_numpy(b).to(dev) for _, b in pairs]
    torch.cuda.synchronize()
    order = [(7 * i + 3) % 4 for i in range(34)]  # 34 items, every pair several times, mixed order
    r = codec.psnr_ssim_batch_dev([ta[k].data_ptr() for k in order], [tb[k].data_ptr() for k in order], h, w, 0, None)
    for i, k in enumerate(order):
        assert np.array_equal(r[i].view(np.uint64), refs[k].view(np.uint64)), (h, w, i, kinds[k], r[i], refs[k])


@pytest.mark.parametrize('h,w', [(7, 7), (8, 9), (15, 39), (135, 131), (255, 257)])
def test_column_chain_path_equals_oracle_bitwise(h, w):
    """Launches of 8 pairs or more run the luma chains a lane per column (all
    five quantities, SSE from the bytes) and form the luma from the bytes in
    the band kernel and the luma MSE, with no fp64 planes; 12 pairs keep the R,
    G, B band kernel (under 32): every item bit-exact against the oracle."""
    import torch
    from jds import codec
    kinds = ['noise', 'indep', 'flat', 'smooth']
    pairs = [_pair(h, w, 71 + i, k) for i, k in enumerate(kinds)]
    refs = [cpu_ref.psnr_ssim_raw(a, b) for a, b in pairs]
    dev = torch.device('cuda', 0)
    ta = [torch.from_numpy(a).to(dev) for a, _ in pairs]
    tb = [torch.from_numpy(b).to(dev) for _, b in pairs]
    torch.cuda.synchronize()
    order = [(5 * i + 1) % 4 for i in range(12)]
    r = codec.psnr_ssim_batch_dev([ta[k].data_ptr() for k in order], [tb[k].data_ptr() for k in order], h, w, 0, None)
    for i, k in enumerate(order):
        assert np.array_equal(r[i].view(np.uint64), refs[k].view(np.uint64)), (h, w, i, kinds[k], r[i], refs[k])


def test_batch_rejects_small_images():
    import torch
    from jds import codec
    t = torch.zeros((6, 9, 3), dtype=torch.uint8, device='cuda')
    torch.cuda.synchronize()
    with pytest.raises(ValueError, match='win_size exceeds image extent'):
        codec.psnr_ssim_batch_dev([t.data_ptr()], [t.data_ptr()], 6, 9, 0, None)


@pytest.mark.parametrize('n', [12, 32])
def test_full_hd_batch_routes_equal_oracle_bitwise(n):
    """The batched routes the 384-item sweep runs, at the sweep's own size
    (1080p: a map row spans 1,914 columns, a leaf/row-crossing layout the
    smaller ROWS_SIZES do not reach): 12 pairs take the overlapped R, G, B band
    kernel and the byte-formed luma; 32 pairs the rows kernel (k_ss_rows +
    k_ss_rgbsum).  Items first, middle and last checked bit for bit against
    the oracle."""
    import torch
    from jds import codec
    h, w = 1080, 1920
    kinds = ['noise', 'indep', 'smooth']
    pairs = [_pair(h, w, 900 + i, k) for i, k in enumerate(kinds)]
    dev = torch.device('cuda', 0)
    ta = [torch.from_numpy(a).to(dev) for a, _ in pairs]
    tb = [torch.from_numpy(b).to(dev) for _, b in pairs]
    torch.cuda.synchronize()
    # item i uses pair order[i]; the checked items 0, n // 2, n - 1 hold three distinct pairs
    order = [(i * 7 + 1) % 3 for i in range(n)]
    checks = [0, n // 2, n - 1]
    order[checks[0]], order[checks[1]], order[checks[2]] = 0, 1, 2
    r = codec.psnr_ssim_batch_dev([ta[k].data_ptr() for k in order], [tb[k].data_ptr() for k in order], h, w, 0, None)
    for i in checks:
        a, b = pairs[order[i]]
        ref = cpu_ref.psnr_ssim_raw(a, b)
        assert np.array_equal(r[i].view(np.uint64), ref.view(np.uint64)), (n, i, kinds[order[i]], r[i], ref)
    # every other item equals the checked item of its pair (same inputs, same launch)
    for i in range(n):
        assert np.array_equal(r[i].view(np.uint64), r[checks[order[i]]].view(np.uint64)), (n, i)


@pytest.mark.parametrize('n', [12, 34])
def test_scratch_budget_groups_equal_oracle(n):
    """A small SSIM scratch budget (jds_ctx_set_ssim_scratch) splits the luma into
    several launch groups, each laid out by its own size: groups under 8 pairs
    keep fp64 planes and need more scratch per item than the others; the scratch
    is sized for the groups that run, full ones and the remainder (ADVICE r05:
    sized by the batch's layout, a planes group wrote past the buffer).  Every
    budget gives the oracle's values bit for bit."""
    import torch
    from jds import _abi, codec
    h, w = 135, 131
    kinds = ['noise', 'indep', 'flat', 'smooth']
    pairs = [_pair(h, w, 500 + i, k) for i, k in enumerate(kinds)]
    refs = [cpu_ref.psnr_ssim_raw(a, b) for a, b in pairs]
    dev = torch.device('cuda', 0)
    ta = [torch.from_numpy(a).to(dev) for a, _ in pairs]
    tb = [torch.from_numpy(b).to(dev) for _, b in pairs]
    torch.cuda.synchronize()
    order = [(3 * i + 2) % 4 for i in range(n)]
    ctx = _abi.Context(0)
    try:
        # ~0.6 MB per item without planes, ~0.9 MB with them at 135 x 131: budgets for
        # groups of 1 (planes), 2 (planes), 10 (+ a planes remainder) and the default
        for budget in (1, 2_500_000, 6_000_000, 0):
            ctx.set_ssim_scratch(budget)
            r = codec.psnr_ssim_batch_dev([ta[k].data_ptr() for k in order], [tb[k].data_ptr() for k in order],
                                          h, w, 0, None, ctx=ctx)
            for i, k in enumerate(order):
                assert np.array_equal(r[i].view(np.uint64), refs[k].view(np.uint64)), (budget, i, kinds[k])
    finally:
        ctx.close()
