"""The multi-rank sweep with the real per-rank compute (the
CPU gloo tests use a stand-in): two ranks on the box's one GPU (gloo carries
the table broadcast and the all_gather; RCCL refuses two ranks on one device,
the driver's 8-GPU runs use nccl), each running sweep_device -- quality-sweep
plans, batched SSIM and float32 magnitude bits -- over its shard of the
frames.  Every rank ends up holding the whole sweep, item for item equal to a
one-process sweep_device over all frames and to the oracle on frame 0."""
import json
import os
import socket

import numpy as np
import pytest

from oracle import cpu_ref

pytestmark = pytest.mark.gpu

QS = [10, 50, 90]
H, W, NF = 48, 64, 3


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _frames():
    return np.stack([cpu_ref.random_image(H, W, 40 + f) for f in range(NF)])


def _summary(it):
    return [it['frame'], it['quality'], it['nonzero'], it['magnitude_bits'], it['sse_rgb'], it['bpp'],
            it['ssim_rgb'], it['ssim_y'], it['mse_y'], [int(x) for x in it['hist']]]


def _worker(rank, world, port, out_dir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        from jds.sweep import distributed_sweep, sweep_device
        frames = _frames()

        def compute(mine, qualities, tables):
            items = sweep_device(frames[list(mine)], qualities, '4:2:0', True, tables=tables, ssim=True)
            for it in items:
                it['frame'] = mine[it['frame']]  # local -> global frame index
            return items

        items = distributed_sweep(NF, QS, compute)
        with open(os.path.join(out_dir, f'rank{rank}.json'), 'w') as fh:
            json.dump([_summary(it) for it in items], fh)
    finally:
        dist.destroy_process_group()


def test_two_ranks_real_compute_equal_one_process(tmp_path):
    import torch.multiprocessing as mp
    from jds import build
    from jds.sweep import sweep_device
    build.build()
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    one = [_summary(it) for it in sweep_device(_frames(), QS, '4:2:0', True, ssim=True)]
    for r in range(2):
        got = json.load(open(tmp_path / f'rank{r}.json'))
        assert got == one
    # frame 0 against the oracle (coefficient statistics and SSIM)
    f0 = _frames()[0]
    for qi, q in enumerate(QS):
        ref = cpu_ref.compress_reconstruct(f0, q, 8, '4:2:0', True, metrics=True)
        it = one[qi]
        assert it[2] == ref['bitrate']['nonzero_count']
        assert it[6] == ref['metrics']['ssim_rgb'] and it[7] == ref['metrics']['ssim_y']  # bitwise
