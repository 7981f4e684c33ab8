"""Quality sweeps: the GUI's BatchSweepWorker (reference gui/worker.py:39-74) and
the frame-sharded multi-GPU sweep of BASELINE cfg4 (64 frames x Q in
{5,10,20,50,80,95}).

* ``quality_sweep`` mirrors BatchSweepWorker.run: one ``compress_reconstruct``
  per quality in ``range(start, end + 1, step)``, returning ``[(q, result)]``.
* ``sweep_device`` runs (frame, Q) items as device-resident quality-sweep
  plans on one GPU (the quality-independent front end once per frame) and
  returns per-item statistics: nonzero count, exact magnitude bits, histogram,
  integer SSE.
* ``distributed_sweep`` shards frames across the ranks of an initialised
  ``torch.distributed`` group (one process per GPU, no data-path collective):
  rank 0 builds the quant tables and one ``broadcast`` (RCCL over xGMI with
  the nccl backend) hands every rank the same float64 tables; the per-item
  statistics come back to every rank with one ``all_gather_object``.
"""
from __future__ import annotations

from typing import Callable, Iterable, List, Optional, Sequence, Tuple

import numpy as np


def quality_sweep(image: np.ndarray, base_params, quality_start: int = 10, quality_end: int = 90,
                  quality_step: int = 10, progress: Optional[Callable[[int, int], None]] = None):
    """BatchSweepWorker.run (gui/worker.py:55-74) without Qt: [(quality, CompressionResult)]."""
    from engines.pipeline import compress_reconstruct
    from models.compression_params import CompressionParams
    qualities = list(range(quality_start, quality_end + 1, quality_step))
    results = []
    for i, quality in enumerate(qualities):
        params = CompressionParams(block_size=base_params.block_size, quality=quality,
                                   subsampling_mode=base_params.subsampling_mode,
                                   use_prefilter=base_params.use_prefilter)
        result, _ = compress_reconstruct(image, params)
        results.append((quality, result))
        if progress is not None:
            progress(i + 1, len(qualities))
    return results


def shard(n: int, rank: int, world: int) -> range:
    """Contiguous, balanced share of n items for `rank` of `world` (first n % world ranks get one more)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f'bad rank {rank} of world {world}')
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return range(lo, lo + base + (1 if rank < extra else 0))


def sweep_device(frames, qualities: Sequence[int], mode: str = '4:2:0', prefilter: bool = True,
                 device: int = 0, tables: Optional[np.ndarray] = None, ssim: bool = False) -> List[dict]:
    """All (frame, quality) items of `frames` (uint8 [F, H, W, 3], NumPy or a torch
    tensor on the device) through quality-sweep plans (jds_plan_create_q: the
    colour / prefilter / subsample / DCT front end runs once per frame and is
    quantised for up to 8 tables at a time).  Items are ordered frame-major.
    Returns one dict per item; bpp / compression_ratio come from NumPy's float32
    magnitude-bits sum (jds_magnitude_bits_f32_dev), as the reference computes
    them (utils/metrics.py:77-78).  ssim=True adds the SSIM fields of the
    reference's per-item CompressionResult (ssim_rgb, ssim_y; gui/worker.py:62-68
    -> utils/metrics.py:9-28) from the device-resident reconstructions
    (jds_psnr_ssim_batch_dev: bit-identical to skimage, every item of a chunk
    in one batched launch sequence) and takes mse_y / psnr_y from the same bit-exact reduction."""
    import torch
    from jds import _abi, codec
    from engines.quantizer import scale_quant_matrix
    from utils.constants import JPEG_LUMA_Q50
    from utils.metrics import bitrate_from_counts, psnr_from_mse

    dev = torch.device('cuda', device)
    fr = frames if isinstance(frames, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(frames))
    fr = fr.to(dev).contiguous()
    F, H, W = int(fr.shape[0]), int(fr.shape[1]), int(fr.shape[2])
    qs = [int(q) for q in qualities]
    gk = codec.gaussian_kernel3()
    stats = np.zeros((F, len(qs)), dtype=_abi.STATS_DTYPE)
    ssims = np.full((F, len(qs), 3), np.nan)  # ssim_rgb, ssim_y, mse_y (bit-exact, jds_psnr_ssim_dev)
    magf = np.zeros((F, len(qs)))  # NumPy float32 magnitude_bits per item (bpp, compression_ratio)
    for c0 in range(0, len(qs), 8):
        qc = qs[c0:c0 + 8]
        qt = [scale_quant_matrix(JPEG_LUMA_Q50, q) if tables is None else tables[c0 + i] for i, q in enumerate(qc)]
        params = [_abi.make_params(q, qt[i], mode, prefilter, gk) for _ in range(F) for i, q in enumerate(qc)]
        plan = _abi.Plan(_abi.context(device), params, H, W, nq=len(qc))
        try:
            out = torch.empty((F * len(qc), H, W, 3), dtype=torch.uint8, device=dev)
            cf = torch.empty((len(params), plan.geometry.coeffs_per_frame), dtype=torch.int16, device=dev)
            st = torch.zeros((len(params), _abi.STATS_DTYPE.itemsize), dtype=torch.uint8, device=dev)
            torch.cuda.synchronize(dev)
            plan.run(fr.data_ptr(), out.data_ptr(), cf.data_ptr(), st.data_ptr(), _abi.RUN_SSE, 0)
            torch.cuda.synchronize(dev)
            stats[:, c0:c0 + len(qc)] = st.cpu().numpy().view(_abi.STATS_DTYPE).reshape(F, len(qc))
            cpf = plan.geometry.coeffs_per_frame
            nit = F * len(qc)
            # the images and coefficients are complete (synchronised above): one
            # batched call each for every item of the chunk
            magf[:, c0:c0 + len(qc)] = codec.magnitude_bits_f32_batch_dev(
                cf.data_ptr(), nit, cpf, cpf, device, None).reshape(F, len(qc))
            if ssim:
                a = [fr[f].data_ptr() for f in range(F) for _ in qc]
                b = [out[k].data_ptr() for k in range(nit)]
                r = codec.psnr_ssim_batch_dev(a, b, H, W, device, None)
                for f in range(F):
                    for i in range(len(qc)):
                        rk = r[f * len(qc) + i]
                        ssims[f, c0 + i] = (float(np.mean(rk[:3])), rk[3], rk[4])  # channel_axis=2: mean of R, G, B
        finally:
            plan.close()
    items = []
    for f in range(F):
        for qi, q in enumerate(qs):
            s = stats[f, qi]
            # bpp from NumPy's float32 sum (the reference's np.sum, exact below 2^24)
            br = bitrate_from_counts(int(s['nonzero']), float(magf[f, qi]), int(s['total_coeffs']), (H, W), 8)
            mse = float(s['sse_rgb']) / (H * W * 3)
            # mse_y: with ssim, the bit-exact NumPy mean (jds_psnr_ssim_dev); otherwise the
            # luma SSE (an exact integer sum / 1e6) over H W -- NumPy's pairwise mean to ~1e-15 relative
            mse_y = float(ssims[f, qi, 2]) if ssim else float(s['sse_y']) / (H * W)
            items.append({'frame': f, 'quality': q, 'nonzero': int(s['nonzero']),
                          'magnitude_bits': int(s['magnitude_bits']), 'magnitude_bits_f32': float(magf[f, qi]),
                          'total_coeffs': int(s['total_coeffs']),
                          'hist': s['hist'].astype(np.int64), 'sse_rgb': int(s['sse_rgb']),
                          'psnr_rgb': float('inf') if mse == 0 else float(10 * np.log10(255.0 ** 2 / mse)),
                          'mse_y': mse_y, 'psnr_y': psnr_from_mse(mse_y),
                          'bpp': br['bpp'], 'compression_ratio': br['compression_ratio']})
            if ssim:
                items[-1].update(ssim_rgb=float(ssims[f, qi, 0]), ssim_y=float(ssims[f, qi, 1]))
    return items


def quant_tables(qualities: Sequence[int]) -> np.ndarray:
    """[nq, 8, 8] float64: scale_quant_matrix(JPEG_LUMA_Q50, q) per quality
    (engines/quantizer.py:7-19 applied to utils/constants.py:6-15)."""
    from engines.quantizer import scale_quant_matrix
    from utils.constants import JPEG_LUMA_Q50
    return np.stack([scale_quant_matrix(JPEG_LUMA_Q50, int(q)) for q in qualities]).astype(np.float64)


def broadcast_tables(qualities: Sequence[int], group=None) -> np.ndarray:
    """Rank 0's quant tables on every rank: one broadcast of nq x 64 float64
    (3 KB for the six sweep qualities) -- through RCCL over xGMI when the group's
    backend is nccl (device tensor), gloo otherwise.  Every rank then quantises
    with bit-identical tables, whatever its own host computed."""
    import torch
    import torch.distributed as dist
    tables = quant_tables(qualities)
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return tables
    dev = torch.device('cuda', torch.cuda.current_device()) if dist.get_backend(group) == 'nccl' else torch.device('cpu')
    t = torch.from_numpy(tables.reshape(len(qualities), 64)).to(dev)
    if dist.get_rank(group) != 0:
        t.zero_()
    src = dist.get_global_rank(group, 0) if group is not None else 0
    dist.broadcast(t, src=src, group=group)
    return t.cpu().numpy().reshape(-1, 8, 8)


def distributed_sweep(n_frames: int, qualities: Sequence[int],
                      compute: Callable[[range, Sequence[int], np.ndarray], List[dict]],
                      group=None) -> List[dict]:
    """Frame-shard a sweep over the ranks of the initialised torch.distributed
    group: rank 0's quant tables are broadcast to all ranks, rank r computes
    `compute(frames_of_r, qualities, tables)` (its items in frame-major order,
    each dict carrying a global 'frame'), then one all_gather_object gives
    every rank the whole list in global item order."""
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    mine = shard(n_frames, rank, world)
    tables = broadcast_tables(qualities, group)
    local = compute(mine, list(qualities), tables)
    if world == 1:
        return local
    parts: List[Optional[List[dict]]] = [None] * world
    dist.all_gather_object(parts, local, group=group)
    items = [it for p in parts for it in p]
    items.sort(key=lambda it: (it['frame'], list(qualities).index(it['quality'])))
    return items
