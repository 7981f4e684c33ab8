"""Multi-rank sweep logic on CPU (gloo, world_size 2) and the shard arithmetic.

The GPU half (sweep_device through the HIP plan) is in test_gpu_parity.py; here
the per-rank compute is a deterministic stand-in so the sharding and the one
all_gather_object of the path run without a GPU."""
import json
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from jds.sweep import distributed_sweep, shard

QS = [5, 10, 20, 50, 80, 95]


def fake_compute(frames, qualities, tables):
    # the broadcast tables ride along: their DC entry per quality
    return [{'frame': f, 'quality': q, 'nonzero': 1000 * f + q, 'q00': float(tables[i][0, 0])}
            for f in frames for i, q in enumerate(qualities)]


def test_shard_covers_exactly_once():
    for n in (0, 1, 5, 63, 64, 65, 384):
        for world in (1, 2, 3, 8):
            parts = [shard(n, r, world) for r in range(world)]
            flat = [i for p in parts for i in p]
            assert flat == list(range(n))
            sizes = [len(p) for p in parts]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard(10, 2, 2)


def test_single_process_sweep_is_frame_major():
    items = distributed_sweep(3, QS, fake_compute)
    assert [(it['frame'], it['quality']) for it in items] == [(f, q) for f in range(3) for q in QS]


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n_frames, out_dir):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        seen = []

        def compute(frames, qualities, tables):
            seen.extend(frames)
            return fake_compute(frames, qualities, tables)

        items = distributed_sweep(n_frames, QS, compute)
        with open(os.path.join(out_dir, f'rank{rank}.txt'), 'w') as fh:
            json.dump([[[it['frame'], it['quality'], it['nonzero'], it['q00']] for it in items], list(seen)], fh)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('n_frames', [64, 7])
def test_gloo_two_ranks_gather_whole_sweep(tmp_path, n_frames):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), n_frames, str(tmp_path)), nprocs=world, join=True)
    from jds.sweep import quant_tables
    q00 = {q: float(t[0, 0]) for q, t in zip(QS, quant_tables(QS))}
    expect = [[f, q, 1000 * f + q, q00[q]] for f in range(n_frames) for q in QS]
    shards = []
    for r in range(world):
        items, seen = json.load(open(tmp_path / f'rank{r}.txt'))
        assert items == expect  # every rank holds the whole sweep in item order
        shards.append(seen)
    assert shards[0] == list(shard(n_frames, 0, world)) and shards[1] == list(shard(n_frames, 1, world))


def _bcast_worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        import numpy as np
        from jds import sweep
        # a rank whose own table builder disagrees still quantises with rank 0's tables
        if rank == 1:
            sweep.quant_tables = lambda qs: np.full((len(qs), 8, 8), -1.0)
        t = sweep.broadcast_tables(QS)
        np.save(os.path.join(out_dir, f'tables{rank}.npy'), t)
    finally:
        dist.destroy_process_group()


def test_gloo_two_ranks_broadcast_quant_tables(tmp_path):
    """Rank 0's scale_quant_matrix tables reach every rank (the broadcast is RCCL
    with the nccl backend; gloo here)."""
    import numpy as np
    from jds.sweep import quant_tables
    mp.spawn(_bcast_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    ref = quant_tables(QS)
    for r in range(2):
        t = np.load(tmp_path / f'tables{r}.npy')
        assert t.dtype == np.float64 and np.array_equal(t, ref)
