"""GPU parity of the JPEG entropy coder (csrc/jds_entropy.hip) against the CPU
oracle (oracle/jpeg_entropy.py): identical JFIF bytes and scan bit counts, on
coefficients from the codec path and on synthetic extreme coefficients; the
GPU file decodes with libjpeg (Pillow)."""
import io

import numpy as np
import pytest

from oracle import cpu_ref
from oracle import jpeg_entropy as je

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module', autouse=True)
def gpu():
    from jds import build, _abi
    build.build()
    assert _abi.device_count() >= 1, 'no HIP device: the MI355X path has no CPU fallback'


def counts(h, w, mode):
    ny = ((h + 7) // 8) * ((w + 7) // 8)
    sy, sx = (2, 2) if mode == '4:2:0' else ((1, 2) if mode == '4:2:2' else (1, 1))
    nc = ((h // sy + 7) // 8) * ((w // sx + 7) // 8)
    return ny, nc


@pytest.mark.parametrize('h,w,mode,q,pf', [
    (64, 96, '4:2:0', 50, True), (48, 40, '4:2:2', 90, False), (33, 47, '4:4:4', 10, False),
    (120, 160, '4:2:0', 100, True), (16, 16, '4:2:0', 1, False), (2, 2, '4:2:0', 50, False),
    (1, 9, '4:4:4', 75, False), (264, 200, '4:2:2', 95, True), (1080, 1920, '4:2:0', 50, True),
])
def test_gpu_jfif_matches_oracle(h, w, mode, q, pf):
    from jds import entropy
    from jds.codec import compress_reconstruct_raw
    img = cpu_ref.random_image(h, w, 31 * h + w + q)
    qt = cpu_ref.scale_quant_matrix(cpu_ref.JPEG_LUMA_Q50, q)
    raw = compress_reconstruct_raw(img, q, qt, mode, pf, maps=False)
    ny, nc = counts(h, w, mode)
    ref, ref_bits = je.encode_jfif(raw['coeffs'], h, w, mode, qt, ny, nc)
    got, bits = entropy.encode_jfif(raw['coeffs'], h, w, mode, qt)
    assert bits == ref_bits
    assert got == ref
    if h >= 8:
        from PIL import Image
        im = np.asarray(Image.open(io.BytesIO(got)).convert('RGB')).astype(np.int64)
        assert np.abs(im - raw['reconstructed']).max() <= 4


def test_gpu_jfif_extreme_coefficients():
    """Synthetic coefficients at the baseline limits: category-11 DC differences,
    +-1023 AC, long zero runs (ZRL), coefficient 63 set (no EOB), dense blocks."""
    from jds import entropy
    h, w, mode = 96, 128, '4:4:4'
    ny, nc = counts(h, w, mode)
    rng = np.random.default_rng(11)
    blk = np.zeros((ny + 2 * nc, 64), np.int64)
    blk[:, 0] = rng.choice([1023, -1024, 0, 5], len(blk))
    zz = je.ZIGZAG
    kind = rng.integers(0, 5, len(blk))
    for i in np.flatnonzero(kind == 1):
        blk[i, zz[63]] = rng.choice([1023, -1023, 1])
    for i in np.flatnonzero(kind == 2):
        blk[i, zz[1:]] = rng.integers(-1023, 1024, 63)
    for i in np.flatnonzero(kind == 3):
        pos = rng.choice(np.arange(1, 64), 3, replace=False)
        blk[i, zz[pos]] = rng.integers(-1023, 1024, 3)
    cf = blk.astype(np.int16).reshape(-1)
    qt = np.ones((8, 8))
    ref, ref_bits = je.encode_jfif(cf, h, w, mode, qt, ny, nc)
    got, bits = entropy.encode_jfif(cf, h, w, mode, qt)
    assert bits == ref_bits and got == ref
    assert np.array_equal(je.decode_jfif(got)['coeffs'], cf)


def test_gpu_plan_entropy_batch():
    """Device-resident path: a plan's coefficients -> one file per frame (different Q per frame)."""
    import torch
    from jds import _abi, codec, entropy
    qs = [5, 50, 95]
    H, W, mode = 360, 648, '4:2:0'
    frames = np.stack([cpu_ref.random_image(H, W, 200 + s) for s in range(len(qs))])
    params = [_abi.make_params(q, cpu_ref.scale_quant_matrix(cpu_ref.JPEG_LUMA_Q50, q), mode, True,
                               codec.gaussian_kernel3()) for q in qs]
    plan = _abi.Plan(_abi.context(0), params, H, W)
    ent = entropy.PlanEntropy(plan)
    dev = torch.device('cuda:0')
    rgb = torch.from_numpy(frames).to(dev)
    out = torch.empty_like(rgb)
    cf = torch.empty((len(qs), plan.geometry.coeffs_per_frame), dtype=torch.int16, device=dev)
    st = torch.zeros((len(qs), _abi.STATS_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    files = torch.empty((len(qs), ent.capacity), dtype=torch.uint8, device=dev)
    lengths = torch.zeros(len(qs), dtype=torch.int64, device=dev)
    sbits = torch.zeros((len(qs), 3), dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    plan.run(rgb.data_ptr(), out.data_ptr(), cf.data_ptr(), st.data_ptr(), 0, s)
    ent.run(cf.data_ptr(), files.data_ptr(), ent.capacity, lengths.data_ptr(), sbits.data_ptr(), s)
    torch.cuda.synchronize()
    ny, nc = counts(H, W, mode)
    for i, q in enumerate(qs):
        ref = cpu_ref.compress_reconstruct(frames[i], q, 8, mode, True, metrics=False)
        data, bits = je.encode_jfif(ref['coeffs'], H, W, mode, ref['qtable'], ny, nc)
        n = int(lengths[i])
        assert files[i, :n].cpu().numpy().tobytes() == data, q
        assert sbits[i].cpu().tolist() == bits
    plan.close()


def test_gpu_plan_entropy_64_frame_1080p_batch_matches_oracle():
    """The bench's entropy leg exactly: PlanEntropy over a 64-frame 1080p Q50 4:2:0
    batch (507 luma segments per scan, every frame in one launch) against the
    oracle encoder on the same coefficients, frame by frame."""
    import multiprocessing as mp
    import os
    import torch
    from jds import _abi, codec, entropy
    H, W, mode, q, B = 1080, 1920, '4:2:0', 50, 64
    qt = cpu_ref.scale_quant_matrix(cpu_ref.JPEG_LUMA_Q50, q)
    params = [_abi.make_params(q, qt, mode, True, codec.gaussian_kernel3())] * B
    plan = _abi.Plan(_abi.context(0), params, H, W)
    ent = entropy.PlanEntropy(plan)
    dev = torch.device('cuda:0')
    gen = torch.Generator(device=dev)
    gen.manual_seed(77)
    rgb = torch.randint(0, 256, (B, H, W, 3), dtype=torch.uint8, device=dev, generator=gen)
    out = torch.empty_like(rgb)
    cf = torch.empty((B, plan.geometry.coeffs_per_frame), dtype=torch.int16, device=dev)
    st = torch.zeros((B, _abi.STATS_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    files = torch.empty((B, ent.capacity), dtype=torch.uint8, device=dev)
    lengths = torch.zeros(B, dtype=torch.int64, device=dev)
    sbits = torch.zeros((B, 3), dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    plan.run(rgb.data_ptr(), out.data_ptr(), cf.data_ptr(), st.data_ptr(), 0, s)
    ent.run(cf.data_ptr(), files.data_ptr(), ent.capacity, lengths.data_ptr(), sbits.data_ptr(), s)
    torch.cuda.synchronize()
    ny, nc = counts(H, W, mode)
    cfh, n_h, bits_h = cf.cpu().numpy(), lengths.cpu().numpy(), sbits.cpu().numpy()
    files_h = files.cpu().numpy()
    plan.close()
    workers = max(1, min(16, len(os.sched_getaffinity(0))))
    with mp.get_context('spawn').Pool(workers) as pool:
        # (oracle worker processes: no GPU; ~5 s of Python per 1080p frame)
        refs = pool.starmap(je.encode_jfif, [(cfh[i], H, W, mode, qt, ny, nc) for i in range(B)])
    for i, (data, bits) in enumerate(refs):
        assert int(n_h[i]) == len(data), i
        assert files_h[i, :len(data)].tobytes() == data, i
        assert bits_h[i].tolist() == bits, i


def test_gpu_plan_entropy_4k_long_scans_match_oracle():
    """Scans of more than 512 segments (4K 4:2:0 luma: 129,600 blocks = 2,025
    segments of 64) take k_entropy's long-scan placement: a k_ent_fscan<false>
    prefix launch, then pre = segoff[g] - segoff[g - q.seg] in k_ent_place
    (ADVICE r05); the 1080p tests stay on the self-summing branch.  Two frames
    at different qualities, bytes and scan bits against the oracle encoder."""
    import multiprocessing as mp
    import torch
    from jds import _abi, codec, entropy
    H, W, mode, qs = 2160, 3840, '4:2:0', [50, 90]
    tabs = [cpu_ref.scale_quant_matrix(cpu_ref.JPEG_LUMA_Q50, q) for q in qs]
    params = [_abi.make_params(q, t, mode, True, codec.gaussian_kernel3()) for q, t in zip(qs, tabs)]
    plan = _abi.Plan(_abi.context(0), params, H, W)
    ent = entropy.PlanEntropy(plan)
    dev = torch.device('cuda:0')
    gen = torch.Generator(device=dev)
    gen.manual_seed(4242)
    rgb = torch.randint(0, 256, (len(qs), H, W, 3), dtype=torch.uint8, device=dev, generator=gen)
    out = torch.empty_like(rgb)
    cf = torch.empty((len(qs), plan.geometry.coeffs_per_frame), dtype=torch.int16, device=dev)
    st = torch.zeros((len(qs), _abi.STATS_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    files = torch.empty((len(qs), ent.capacity), dtype=torch.uint8, device=dev)
    lengths = torch.zeros(len(qs), dtype=torch.int64, device=dev)
    sbits = torch.zeros((len(qs), 3), dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    plan.run(rgb.data_ptr(), out.data_ptr(), cf.data_ptr(), st.data_ptr(), 0, s)
    ent.run(cf.data_ptr(), files.data_ptr(), ent.capacity, lengths.data_ptr(), sbits.data_ptr(), s)
    torch.cuda.synchronize()
    ny, nc = counts(H, W, mode)
    assert ny // 64 > 512  # the long-scan branch is the one under test
    cfh, n_h, bits_h, files_h = cf.cpu().numpy(), lengths.cpu().numpy(), sbits.cpu().numpy(), files.cpu().numpy()
    plan.close()
    with mp.get_context('spawn').Pool(len(qs)) as pool:  # (no GPU in the workers; ~20 s of Python per frame)
        refs = pool.starmap(je.encode_jfif, [(cfh[i], H, W, mode, tabs[i], ny, nc) for i in range(len(qs))])
    for i, (data, bits) in enumerate(refs):
        assert int(n_h[i]) == len(data), i
        assert files_h[i, :len(data)].tobytes() == data, i
        assert bits_h[i].tolist() == bits, i


@pytest.mark.parametrize('nblk,rows,seed', [(65, 1, 1), (129, 1, 2), (65, 2, 3), (66, 1, 6), (193, 1, 5)])
def test_gpu_jfif_short_last_segment(nblk, rows, seed):
    """Scans whose last segment (nblk mod 64 blocks) is short and mostly zero
    blocks, with a few nonzero DC values so the segment boundary is not word
    aligned: the last segment fits inside the previous segment's final word
    (k_ent_place's fused-pad path and the skipped head word)."""
    from jds import entropy
    h, w, mode = 8 * rows, 8 * nblk, '4:4:4'
    ny, nc = counts(h, w, mode)
    rng = np.random.default_rng(seed)
    blk = np.zeros((ny + 2 * nc, 64), np.int64)
    pick = rng.choice(len(blk), max(1, len(blk) // 9), replace=False)
    blk[pick, 0] = rng.integers(-40, 41, len(pick))
    cf = blk.astype(np.int16).reshape(-1)
    qt = np.ones((8, 8))
    ref, ref_bits = je.encode_jfif(cf, h, w, mode, qt, ny, nc)
    got, bits = entropy.encode_jfif(cf, h, w, mode, qt)
    assert bits == ref_bits and got == ref
    # the case is the one asked for: some scan's last segment starts off a word
    # boundary and ends inside the same 32-bit word
    n = ny
    inside = []
    for c in range(3):
        bb = je.block_bits(blk[c * n:(c + 1) * n], c > 0)
        cum = np.concatenate([[0], np.cumsum(bb)])
        s0, e0 = int(cum[64 * ((n - 1) // 64)]), int(cum[n])
        inside.append(s0 % 32 != 0 and s0 // 32 == (e0 - 1) // 32)
    assert any(inside)
    assert np.array_equal(je.decode_jfif(got)['coeffs'], cf)


def test_gpu_jfif_rejects_non_baseline_coefficients():
    from jds import entropy
    h, w, mode = 16, 16, '4:4:4'
    ny, nc = counts(h, w, mode)
    cf = np.zeros((ny + 2 * nc) * 64, np.int16)
    cf[64 * 2 + 5] = 2000  # AC category 11
    with pytest.raises(ValueError, match='baseline'):
        entropy.encode_jfif(cf, h, w, mode, np.ones((8, 8)))
    cf[64 * 2 + 5] = 0
    cf[64 * 3] = 3000  # DC difference category 12
    with pytest.raises(ValueError, match='baseline'):
        entropy.encode_jfif(cf, h, w, mode, np.ones((8, 8)))
