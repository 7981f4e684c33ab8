#!/usr/bin/env python3
"""bench.py — Mpixels/s of the forward+inverse block-DCT pipeline @ Q=50 4:2:0 (+PSNR vs reference).

Workload (BASELINE.json configs[1]): 1920x1080 uniform-random RGB frames, Q=50,
4:2:0, prefilter ON, through the fused HIP kernels (forward phase: k_fwd32i +
k_fwd_reduce_rows + k_fix_fwd, RGB -> int16 coefficients + statistics; inverse
phase: the certified k_inv_fast, coefficients -> RGB, with its in-launch exact
tile fix-up).  One step = one pass over a batch of
`--frames` device-resident 1080p frames per GPU (default 64, the size of the
reference's cfg4 batch sweep); inputs are generated on the device before the
timed region.  A step is one jds_plan_run (forward then inverse) on one stream;
`--pipeline 1` instead overlaps the forward of batch k+1 with the inverse of
batch k on a second stream (two buffer sets).  Multi-GPU: one process per GPU (torchrun), frames shard across
ranks with no data-path collective (weak scaling); RCCL carries the quant-table
broadcast from rank 0, the barrier, the max-over-ranks time and the per-rank
frame-0 parity gather (`parity_ranks`).

Prints ONE JSON line (rank 0).  The roofline object describes the dominant
kernel -- the single longest launch of a step -- with ALGORITHMIC bytes: a
forward front end (k_fwd32i) reads 3 B/px RGB and writes 2*S B/px int16
coefficients, an inverse (k_inv_fast) the reverse (S = coefficients per pixel,
1.5037 at 1080p 4:2:0).  Launch durations (`kernels_ms`) come from the plan
itself: K more steps exactly as timed, right after the timed region, with
jds_plan_profile's event marks after every launch on the launch stream; the
intervals tile the profiled span, so they sum to the step time.  `traffic`
(HBM bytes/launch of that kernel from rocprofv3 FETCH_SIZE / WRITE_SIZE PMC)
is read from profiles/pmc_traffic.json when it matches this configuration.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, 'jpeg-dsp-studio_amd')
for _p in (PKG, ROOT):
    if _p not in sys.path:
        sys.path.insert(0, _p)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)
HBM_COPY_GBS = 6290.0  # measured float4 device copy (MI355X_MICROARCH.md: 6.29 TB/s, 79 % of spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--frames', type=int, default=64, help='1080p frames per GPU per step')
    ap.add_argument('--height', type=int, default=1080)
    ap.add_argument('--width', type=int, default=1920)
    ap.add_argument('--quality', type=int, default=50)
    ap.add_argument('--mode', default='4:2:0')
    ap.add_argument('--prefilter', type=int, default=1)
    ap.add_argument('--block', type=int, default=8, choices=(8, 16),
                    help='16 = the configs[4] 16x16 stretch path (jds_fast16.hip certified fp32 forward, '
                         'jds_b16.hip fp64 inverse)')
    ap.add_argument('--inv-fast', action='store_true',
                    help='A/B: coarse tables (DC quantiser > 60): the certified fast inverse '
                         '(JDS_RUN_INV_FAST) instead of the exact k_inv2 the plan picks')
    ap.add_argument('--exact-inv', action='store_true',
                    help='A/B: force the exact replayed-order inverse (JDS_RUN_EXACT_INV: k_inv2 / k_inv16s)')
    ap.add_argument('--exact', action='store_true',
                    help='all-fp64 kernels (JDS_RUN_EXACT) instead of the certified fast ones (A/B)')
    ap.add_argument('--cpu-baseline-seconds', type=float, default=20.0,
                    help='CPU budget over the 4 legs (faithful / vectorised x 1 core / pool)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-parity', action='store_true')
    ap.add_argument('--no-north-star', action='store_true',
                    help='skip the north-star leg (16 x 3840x2160, Q=50, 4:2:0, prefilter) that the default run '
                         'measures after the headline configs[1] line')
    ap.add_argument('--no-host-path', action='store_true',
                    help='skip the PCIe-inclusive engines.compress_reconstruct measurement (1080p, host arrays)')
    ap.add_argument('--sweep', action='store_true',
                    help='BASELINE configs[3]: --frames frames per GPU x Q in {5,10,20,50,80,95} per step '
                         '(quality-sweep plan: shared front end), SSE on; value = Mpixels/s over all items')
    ap.add_argument('--sweep-replicate', action='store_true',
                    help='with --sweep: a plain plan over frames replicated per Q (no shared front end)')
    ap.add_argument('--no-entropy', action='store_true',
                    help='skip the JPEG entropy-coding measurement (8x8 only, outside the timed region)')
    ap.add_argument('--pipeline', type=int, default=0, choices=(0, 1),
                    help='1: image-stream pipelining, two buffer sets; the forward of batch k+1 runs beside the '
                         'inverse of batch k on a second stream (measured no faster: the launches share CUs at '
                         'workgroup granularity).  0 (default): one jds_plan_run (forward then inverse) per step')
    ap.add_argument('--dry-run', action='store_true',
                    help='launcher check without a GPU: each rank joins the process group (gloo), one all-reduce, '
                         'rank 0 prints the world it saw (tests/test_bench_launch_cpu.py)')
    return ap.parse_args()


def launch_decision(gpus, env, visible_gpus, dry_run=False):
    """How `bench.py --gpus N` runs (--gpus must never be
    ignored).  Returns (action, detail):
      * ('run', None): this process is the whole job (N = 1) or one rank of a
        torchrun job whose WORLD_SIZE equals N;
      * ('spawn', backend): N > 1 without torchrun -- start N ranks as child
        processes (torch.distributed.run) before any GPU call: 'nccl' with one
        rank per GPU when N GPUs are visible, 'gloo' sharing the visible GPU(s)
        when JDS_BENCH_REHEARSE=1 asks for the rehearsal (or for --dry-run);
      * ('error', message): a mismatch -- exit non-zero, print nothing as JSON."""
    if gpus < 1:
        return 'error', f'--gpus must be >= 1, got {gpus}'
    ws = env.get('WORLD_SIZE')
    if ws is not None:
        if int(ws) != gpus:
            return 'error', (f'--gpus {gpus} but WORLD_SIZE={ws}: launch with torchrun --nproc-per-node {gpus} '
                             f'(or without torchrun and let bench.py start the ranks)')
        return 'run', None
    if gpus == 1:
        return 'run', None
    if dry_run:
        return 'spawn', 'gloo'
    if visible_gpus >= gpus:
        return 'spawn', 'nccl'
    if env.get('JDS_BENCH_REHEARSE') == '1':
        return 'spawn', 'gloo'
    return 'error', (f'--gpus {gpus} but only {visible_gpus} GPU(s) visible; set JDS_BENCH_REHEARSE=1 to rehearse '
                     f'{gpus} ranks sharing them over gloo (the line is then marked as a rehearsal)')


def _free_port():
    import socket
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(gpus, backend, argv):
    """Start `gpus` ranks of this script under torch.distributed.run as a child
    process (never exec: the parent has touched no GPU, and a child keeps the
    launcher's exit status) and return its exit code."""
    import subprocess
    env = dict(os.environ)
    env.setdefault('HSA_ENABLE_IPC_MODE_LEGACY', '0')
    if backend == 'gloo':
        env['JDS_BENCH_BACKEND'] = 'gloo'
        env['JDS_BENCH_SHARE_GPU'] = '1'
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={gpus}',
           '--master-addr=127.0.0.1', f'--master-port={_free_port()}', os.path.abspath(__file__)] + list(argv)
    return subprocess.call(cmd, env=env)


def dry_run_main(args):
    """One all-reduce over the ranks (gloo, no GPU); rank 0 prints what it saw."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    if world > 1:
        dist.init_process_group('gloo')
    t = torch.tensor([rank + 1.0])
    if world > 1:
        dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({'dry_run': True, 'gpus_flag': args.gpus, 'world_size': world,
                          'rank_sum': float(t.item()), 'backend': os.environ.get('JDS_BENCH_BACKEND', 'nccl')}),
              flush=True)
    if world > 1:
        dist.destroy_process_group()


PREWARM_S = 0.3
PROFILE_CHUNK = 500  # profiled steps per jds_plan_profile_read (event pool: 8192 marks)


def init_dist(world, local):
    """One process per GPU over RCCL (backend nccl).  JDS_BENCH_BACKEND=gloo with
    JDS_BENCH_SHARE_GPU=1 rehearses the N > 1 path with several ranks on one GPU
    (a one-GPU box; RCCL refuses two ranks on one device): ranks map onto the
    visible devices round-robin and the timing reductions go through host
    tensors.  Returns (device index, backend)."""
    import torch
    import torch.distributed as dist
    backend = os.environ.get('JDS_BENCH_BACKEND', 'nccl')
    if os.environ.get('JDS_BENCH_SHARE_GPU') == '1':
        local = local % max(1, torch.cuda.device_count())
    if world > 1:
        torch.cuda.set_device(local)
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
        else:
            dist.init_process_group(backend)
    return local, backend


def max_over_ranks(x, dev, backend):
    """The slowest rank's value (one all-reduce)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([x], dtype=torch.float64, device=dev if backend == 'nccl' else 'cpu')
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def prewarm(run_step, warmup, dev):
    """The W untimed warmup steps, continued until PREWARM_S seconds of sustained
    load have passed.  The MI355X raises its clocks over the first ~40 ms of
    load: in a rocprofv3 trace of 3 warmup + 20 steps, k_inv2 took 549 us at
    the start of the timed region and 404 us after 40 launches (k_fwd32i 420 ->
    321 us), so a 3-step warmup times the ramp, not the steady state of an
    image stream.  Returns the number of warmup steps run."""
    import torch
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    k = 0
    while k < warmup or (time.perf_counter() - t0 < PREWARM_S and k < 2000):
        run_step(k)
        k += 1
        if k % 4 == 0:
            torch.cuda.synchronize(dev)
    torch.cuda.synchronize(dev)
    return k


def _cpu_model():
    try:
        for line in open('/proc/cpuinfo'):
            if line.startswith('model name'):
                return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return 'unknown'


def _cpu_workers():
    """Host cores this process may use: the affinity set, capped at the
    OMP_NUM_THREADS share the GPU box gives one GPU (16 there)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, 'sched_getaffinity') else (os.cpu_count() or 1)
    cap = int(os.environ.get('OMP_NUM_THREADS', '0') or 0)
    return max(1, min(n, cap) if cap > 0 else n)


def _cpu_frame(args):
    """One frame through the oracle in a worker process (1 thread)."""
    img, quality, mode, pf, block, faithful = args
    from oracle import cpu_ref
    if faithful:
        cpu_ref.compress_reconstruct_faithful(img, quality, mode, pf)
    else:
        cpu_ref.compress_reconstruct(img, quality, block, mode, pf, metrics=False, stretch=block == 16)
    return 0


def cpu_baseline(frames_host, quality, mode, pf, budget_s, block=8):
    """The CPU pipeline timed on this box's host cores beside the GPU line
    (SURVEY.md §8(d)), on a bounded sample of the same frames, in two modes:
      * faithful: the reference's structure, a Python loop of per-block
        scipy dctn/idctn calls (engines/pipeline.py:47-82) -- like for like;
      * vectorised: the oracle's batched restatement -- a stronger CPU bound;
    each on 1 core and on a process pool over frames (one process per core,
    spawned: the parent holds a HIP context).  Without SSIM or maps on every
    leg.  The headline `value` is the strongest leg."""
    import multiprocessing as mp
    from oracle import cpu_ref
    h, w = frames_host.shape[1:3]
    legs = {}
    leg_s = budget_s / 4.0
    faith_ok = block == 8
    for name, faithful in (('vectorised', False), ('faithful', True)):
        if faithful and not faith_ok:
            continue
        t0 = time.perf_counter()
        n = 0
        while n < len(frames_host):
            _cpu_frame((frames_host[n], quality, mode, pf, block, faithful))
            n += 1
            if time.perf_counter() - t0 >= leg_s:
                break
        dt = time.perf_counter() - t0
        legs[f'{name}_1core'] = {'value': round(n * h * w / dt / 1e6, 4), 'cores': 1, 'frames': n,
                                 'seconds': round(dt, 2)}
    P = _cpu_workers()
    if P > 1:
        ctx = mp.get_context('spawn')
        with ctx.Pool(P) as pool:
            pool.map(_cpu_frame, [(frames_host[0][:16, :16].copy(), quality, mode, pf, block, False)] * P)  # imports
            for name, faithful in (('vectorised', False), ('faithful', True)):
                if faithful and not faith_ok:
                    continue
                one = legs[f'{name}_1core']
                per = max(1, int(round(leg_s / (one['seconds'] / one['frames']))))
                jobs = [(frames_host[i % len(frames_host)], quality, mode, pf, block, faithful) for i in range(P * per)]
                t0 = time.perf_counter()
                pool.map(_cpu_frame, jobs, chunksize=1)
                dt = time.perf_counter() - t0
                legs[f'{name}_{P}cores'] = {'value': round(len(jobs) * h * w / dt / 1e6, 4), 'cores': P,
                                            'frames': len(jobs), 'seconds': round(dt, 2)}
    best_k = max(legs, key=lambda k: legs[k]['value'])
    best = legs[best_k]
    return {'value': best['value'], 'unit': 'Mpixels/s', 'cores': best['cores'], 'kind': 'port',
            'sample': f'{best["frames"]} x {w}x{h} frames (Q{quality} {mode} prefilter={bool(pf)} {block}x{block}) '
                      f'through oracle/cpu_ref.py ({best_k}), {best["seconds"]} s, no SSIM/maps',
            'legs': legs, 'cpu_model': _cpu_model(), 'host_cores_visible': os.cpu_count(),
            'reference_per_block_loop_note': 'faithful = engines/pipeline.py:47-82 loop structure (one scipy '
                                             'call per 8x8 block); vectorised = batched dctn over (n, 8, 8)',
            'reconciliation': 'BASELINE.md section 2 measured the reference itself at 0.87-0.97 Mpix/s (1080p cfg2, '
                              '1 core, no SSIM) on the survey container\'s Xeon; the faithful leg on that same '
                              'container type runs 0.76-0.81 Mpix/s (2.55-2.74 s per 1080p frame, DESIGN.md section 4), '
                              'so the legs here differ from it by the host CPU (this box: ' + _cpu_model() + '), '
                              'not by the work timed'}


def host_path(quality, mode, pf, H=1080, W=1920, reps=5):
    """Mpixels/s of the drop-in engines.compress_reconstruct on one host frame:
    what the GUI's worker gets (gui/worker.py:29) -- H2D upload, both phases,
    IntermediateData maps and selected block, PSNR/SSIM, D2H of every output
    (PCIe-inclusive; never the headline value)."""
    import numpy as np
    from engines import compress_reconstruct
    from models import CompressionParams
    img = np.random.default_rng(5).integers(0, 256, (H, W, 3), dtype=np.uint8)
    prm = CompressionParams(quality=quality, subsampling_mode=mode, use_prefilter=bool(pf))
    compress_reconstruct(img, prm)  # warm: context, scratch, code objects
    t0 = time.perf_counter()
    for _ in range(reps):
        compress_reconstruct(img, prm)
    dt = (time.perf_counter() - t0) / reps
    return {'value': round(H * W / dt / 1e6, 2), 'unit': 'Mpixels/s', 'ms_per_frame': round(dt * 1e3, 3),
            'frame': f'{W}x{H} Q{quality} {mode} prefilter={bool(pf)}', 'reps': reps,
            'includes': 'H2D + forward + inverse + error maps + selected block + PSNR/SSIM (GPU) + D2H, '
                        'engines.compress_reconstruct from NumPy'}


def workload_label(H, W, q, mode, pf, block):
    """Which BASELINE.json config a bench line measures (configs[0] is the CPU-only case)."""
    if block == 16:
        return 'BASELINE configs[4] stretch (16x16 blocks)' if (H, W, mode) == (2160, 3840, '4:2:2') else \
            '16x16 stretch path (custom size)'
    if (H, W, q, mode, bool(pf)) == (1080, 1920, 50, '4:2:0', True):
        return 'BASELINE configs[1]'
    if (H, W, q, mode) == (2160, 3840, 10, '4:2:0'):
        return 'BASELINE configs[2]'
    if (H, W, q, mode) == (2160, 3840, 50, '4:2:0'):
        return 'north_star measurement point (4K / Q=50 / 4:2:0)'
    if (H, W, mode) == (2160, 3840, '4:2:2'):
        return 'BASELINE configs[4] at 8x8 blocks'
    if (H, W, q, mode, bool(pf)) == (512, 512, 50, '4:4:4', False):
        return 'BASELINE configs[0] geometry (512x512 4:4:4) on the GPU'
    return 'custom configuration'


def metric_name(q, mode):
    """BASELINE.json's metric, with the quality / mode actually measured."""
    return f'Mpixels/s forward+inverse pipeline @ Q={q} {mode}; PSNR vs ref'


def dist_info(world, backend):
    import torch.distributed as dist
    if world > 1 and dist.is_initialized():
        d = {'world_size': dist.get_world_size(), 'backend': dist.get_backend()}
        if os.environ.get('JDS_BENCH_SHARE_GPU') == '1':
            # ranks share the visible GPU(s): a rehearsal of the N > 1 path, not an N-GPU measurement
            import torch
            d['rehearsal_shared_gpus'] = torch.cuda.device_count()
        return d
    return {'world_size': 1, 'backend': None}


def gather_parity(local, world, backend):
    """Every rank's own frame-0 parity record on rank 0 (one all_gather_object
    outside the timed region), so the line shows every rank's shard checked."""
    import torch.distributed as dist
    rec = dict(local)
    if world > 1 and dist.is_initialized():
        rec['rank'] = dist.get_rank()
        parts = [None] * dist.get_world_size()
        dist.all_gather_object(parts, rec)
    else:
        rec['rank'] = 0
        parts = [rec]
    return {'world_size': len(parts), 'backend': backend if world > 1 else None, 'ranks': parts,
            'all_exact': all(p.get('mismatches', 0) == 0 and p.get('coeff_mismatch', 0) == 0 and
                             p.get('recon_mismatch_bytes', 0) == 0 for p in parts)}


SWEEP_QS = [5, 10, 20, 50, 80, 95]  # BASELINE configs[3]


def sweep_main(args):
    """configs[3]: every frame at every sweep quality, frames sharded across ranks."""
    import numpy as np
    import torch
    import torch.distributed as dist
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    local, backend = init_dist(world, local)
    dev = torch.device('cuda', local)
    torch.cuda.set_device(dev)
    from jds import _abi, codec
    from jds.sweep import broadcast_tables
    F, H, W, nq = args.frames, args.height, args.width, len(SWEEP_QS)
    # rank 0's quant tables reach every rank in one broadcast (RCCL over xGMI at N > 1)
    tables = broadcast_tables(SWEEP_QS)
    params = [_abi.make_params(q, tables[i], args.mode, bool(args.prefilter), codec.gaussian_kernel3())
              for _ in range(F) for i, q in enumerate(SWEEP_QS)]
    rep = args.sweep_replicate
    plan = _abi.Plan(_abi.context(local), params, H, W, nq=1 if rep else nq)
    gen = torch.Generator(device=dev)
    gen.manual_seed(2000 + rank)
    rgb = torch.randint(0, 256, (F, H, W, 3), dtype=torch.uint8, device=dev, generator=gen)
    if rep:
        rgb = rgb.repeat_interleave(nq, dim=0).contiguous()
    out = torch.empty((F * nq, H, W, 3), dtype=torch.uint8, device=dev)
    cf = torch.empty((F * nq, plan.geometry.coeffs_per_frame), dtype=torch.int16, device=dev)
    st = torch.zeros((F * nq, _abi.STATS_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    s = torch.cuda.Stream(dev)
    torch.cuda.synchronize(dev)

    def step():
        plan.run(rgb.data_ptr(), out.data_ptr(), cf.data_ptr(), st.data_ptr(),
                 _abi.RUN_SSE | (_abi.RUN_INV_FAST if args.inv_fast else 0), s.cuda_stream)

    nwarm = prewarm(lambda k: step(), args.warmup, dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        elapsed = max_over_ranks(elapsed, dev, backend)
    items = F * nq * world
    value = items * H * W * args.steps / elapsed / 1e6
    result = {'metric': 'Mpixels/s quality sweep (configs[3]); items = frames x Q', 'value': round(value, 2),
              'unit': 'Mpixels/s', 'n_gpus': world, 'steps': args.steps, 'warmup': args.warmup,
              'warmup_steps_run': nwarm, 'ms_per_step': round(elapsed / args.steps * 1e3, 4), 'higher_is_better': True, 'scaling': 'weak',
              'vs_baseline': None, 'dtype': 'f32+f64', 'data': 'synthetic (uniform random RGB generated on device)',
              'config': {'workload': f'{F} x {W}x{H} frames per GPU x Q{SWEEP_QS}, {args.mode}, '
                                     f'prefilter={"on" if args.prefilter else "off"} (BASELINE configs[3])',
                         'items_per_step': items, 'items_per_s': round(items * args.steps / elapsed, 1),
                         'front_end': 'replicated per item' if rep else 'shared per frame (jds_plan_create_q)',
                         'parallelism': f'frame-shard x{world}', **dist_info(world, backend)}}
    # the per-item statistics of every rank reach every rank (distributed_sweep's
    # all_gather_object, gui/worker.py:55-74's result list), once, outside the
    # timed region: the record shows the gather ran and what it carried
    from jds.sweep import distributed_sweep
    st_np = st.cpu().numpy().view(_abi.STATS_DTYPE).reshape(F, nq)

    def mine_items(frames, qs, tabs):
        assert len(frames) == F and np.array_equal(tabs, tables)
        return [{'frame': frames[f], 'quality': q, 'nonzero': int(st_np[f, i]['nonzero']),
                 'magnitude_bits': int(st_np[f, i]['magnitude_bits']), 'sse_rgb': int(st_np[f, i]['sse_rgb'])}
                for f in range(F) for i, q in enumerate(qs)]
    tg = time.perf_counter()
    gathered = distributed_sweep(F * world, SWEEP_QS, mine_items)
    result['gather'] = {'collective': 'broadcast (tables) + all_gather_object (per-item stats)' if world > 1
                        else 'none (one rank)', 'items_gathered': len(gathered), 'items_expected': F * nq * world,
                        'frames_covered': sorted({it['frame'] for it in gathered}) == list(range(F * world)),
                        'seconds': round(time.perf_counter() - tg, 4), **dist_info(world, backend)}
    # the per-item SSIM of the reference's CompressionResult (gui/worker.py:62-68 ->
    # utils/metrics.py:9-28) for every item of the step, batched on the device
    # (jds_psnr_ssim_batch_dev), timed on its own after the headline region
    if not rep:
        from jds import codec as _codec
        pa = [rgb[f].data_ptr() for f in range(F) for _ in SWEEP_QS]
        pb = [out[k].data_ptr() for k in range(F * nq)]
        torch.cuda.synchronize(dev)
        _codec.psnr_ssim_batch_dev(pa, pb, H, W, local, None)  # warm: scratch, code objects
        reps = 3
        t0s = time.perf_counter()
        for _ in range(reps):
            ss = _codec.psnr_ssim_batch_dev(pa, pb, H, W, local, None)
        dt = (time.perf_counter() - t0s) / reps
        result['ssim'] = {'entry': 'jds_psnr_ssim_batch_dev (csrc/jds_ssim_band.hip)', 'items': F * nq,
                          'ms_per_item': round(dt * 1e3 / (F * nq), 4), 'ms_per_step': round(dt * 1e3, 3),
                          'items_per_s': round(F * nq / dt, 1), 'includes': 'SSIM R/G/B/Y + luma MSE + RGB SSE '
                          'per item, host wall time of the call (launches + one copy back)',
                          'ssim_rgb_item0': float(np.mean(ss[0][:3])), 'ssim_y_item0': float(ss[0][3])}
    if not args.no_parity:
        # every rank checks its own frame 0 at every quality against the oracle
        from oracle import cpu_ref
        stats = st.cpu().numpy().view(_abi.STATS_DTYPE).reshape(-1)
        f0 = rgb[0].cpu().numpy()
        bad = 0
        ssim_bad = None
        for qi, q in enumerate(SWEEP_QS):
            ref = cpu_ref.compress_reconstruct(f0, q, 8, args.mode, bool(args.prefilter), metrics=False)
            bad += int(np.sum(cf[qi].cpu().numpy() != ref['coeffs']))
            bad += int(stats[qi]['sse_rgb'] != int(((f0.astype(np.int64) - ref['reconstructed']) ** 2).sum()))
            if qi == 3 and 'ssim' in result:  # Q50: the batched SSIM of item (0, Q50) vs the oracle's skimage restatement
                m = cpu_ref.compute_psnr_ssim(f0, out[qi].cpu().numpy())
                ssim_bad = int(m['ssim_y'] != ss[qi][3]) + int(m['ssim_rgb'] != float(np.mean(ss[qi][:3])))
        rec = {'frame': 0, 'qualities': SWEEP_QS, 'mismatches': bad}
        if ssim_bad is not None:
            rec['ssim_mismatches_q50'] = ssim_bad
        pr = gather_parity(rec, world, backend)
        if rank == 0:
            result['parity'] = rec
            result['parity_ranks'] = pr
    plan.close()
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def run_point(args, dev, world, backend, rank, B, H, W, quality, mode, pf, block=8, qtable=None, seed=1000):
    """One measured configuration: B device-resident frames per GPU, W untimed
    warmup steps (continued to PREWARM_S of load), then exactly K timed steps
    bracketed by barrier + synchronize, max over ranks; then a serial
    calibration pass timing each phase with HIP events on its launch stream.
    Returns (result dict, state) -- state keeps the plans and buffers for the
    legs that follow (entropy, parity); the caller closes the plans."""
    import torch
    import torch.distributed as dist
    from jds import _abi, codec
    from engines.quantizer import scale_quant_matrix
    from utils.constants import JPEG_LUMA_Q50

    qt = scale_quant_matrix(JPEG_LUMA_Q50, quality) if qtable is None else qtable
    prm = _abi.make_params(quality, qt, mode, bool(pf), codec.gaussian_kernel3(), block)
    # image stream: NS buffer sets (plan + frames + outputs); with pipelining the
    # forward of batch k+1 (set (k+1) % 2) runs beside the inverse of batch k on
    # a second stream, and batch k+2 reuses set k % 2 once batch k's inverse is done
    NS = 2 if args.pipeline else 1
    plans = [_abi.Plan(_abi.context(dev.index), [prm] * B, H, W) for _ in range(NS)]
    geo = plans[0].geometry
    cpf = geo.coeffs_per_frame

    # device-resident synthetic frames (uniform random RGB), distinct per rank and set
    gen = torch.Generator(device=dev)
    gen.manual_seed(seed + rank)
    rgbs = [torch.randint(0, 256, (B, H, W, 3), dtype=torch.uint8, device=dev, generator=gen) for _ in range(NS)]
    outs = [torch.empty_like(r) for r in rgbs]
    coefs = [torch.empty((B, cpf), dtype=torch.int16, device=dev) for _ in range(NS)]
    stats_l = [torch.zeros((B, _abi.STATS_DTYPE.itemsize), dtype=torch.uint8, device=dev) for _ in range(NS)]
    s_f = torch.cuda.Stream(dev)  # forward launches (and their events)
    s_i = torch.cuda.Stream(dev) if NS > 1 else s_f  # inverse launches
    torch.cuda.synchronize(dev)  # inputs were produced on the default stream
    torch.cuda.set_stream(s_f)
    done_inv = [torch.cuda.Event() for _ in range(NS)]  # set b's last inverse finished (its buffers are free)
    fwd_done = [torch.cuda.Event() for _ in range(NS)]
    used = [False] * NS

    xflags = ((_abi.RUN_EXACT if args.exact else 0) | (_abi.RUN_INV_FAST if args.inv_fast else 0) |
              (_abi.RUN_EXACT_INV if args.exact_inv else 0))

    def ptrs(b):
        return (rgbs[b].data_ptr(), outs[b].data_ptr(), coefs[b].data_ptr(), stats_l[b].data_ptr())

    def step(k, ev=None, si=None):
        si = si or s_i
        b = k % NS
        if used[b]:
            s_f.wait_event(done_inv[b])
        used[b] = True
        if ev is not None:
            ev[0].record(s_f)
        plans[b].run(*ptrs(b), _abi.RUN_FWD | xflags, s_f.cuda_stream)
        if ev is not None:
            ev[1].record(s_f)
        fwd_done[b].record(s_f)
        si.wait_event(fwd_done[b])
        if ev is not None:
            ev[2].record(si)
        plans[b].run(*ptrs(b), _abi.RUN_INV | xflags, si.cuda_stream)
        if ev is not None:
            ev[3].record(si)
        done_inv[b].record(si)

    def run_step(k):
        if NS > 1:
            step(k)
        else:  # both phases in one call on one stream: no events inside the timed region
            plans[0].run(*ptrs(0), xflags, s_f.cuda_stream)

    nwarm = prewarm(run_step, args.warmup, dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        run_step(nwarm + k)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    # Per-kernel launch durations of the same runs (outside the timed region):
    # K more steps exactly as timed, with the plan marking its stream after
    # every launch (jds_plan_profile); the intervals between marks tile the
    # span, so they sum to the profiled step time.  With pipelining (two
    # streams) the phases overlap: then a serial pass with events per phase.
    kernels, kprof = {}, None
    if NS == 1:
        plans[0].profile(True)
        torch.cuda.synchronize(dev)
        # the plan's event pool holds 8192 marks (~7 per step): read every
        # PROFILE_CHUNK steps and sum (a read past the pool fails loudly)
        kt, span = {}, 0.0
        for k in range(args.steps):
            run_step(nwarm + args.steps + k)
            if (k + 1) % PROFILE_CHUNK == 0 or k + 1 == args.steps:
                part, sp = plans[0].profile_read()
                span += sp
                for name, (tot, cnt) in part.items():
                    t0_, c0_ = kt.get(name, (0.0, 0))
                    kt[name] = (t0_ + tot, c0_ + cnt)
        plans[0].profile(False)
        kernels = {name: {'ms_per_step': tot / args.steps, 'launches_per_step': cnt / args.steps,
                          'avg_launch_ms': tot / cnt} for name, (tot, cnt) in kt.items()}
        kprof = {'profiled_step_ms': span / args.steps,
                 'sum_ms': sum(v['ms_per_step'] for v in kernels.values()),
                 'timing': 'jds_plan_profile: an event after every launch of the plan\'s runs, K steps after the '
                           'timed region on the same stream; "(between runs)" = host gaps between runs'}
        fwd_keys = [k for k in kernels if k.startswith(FWD_PREFIXES)]
        inv_keys = [k for k in kernels if k.startswith(INV_PREFIXES)]
        t_fwd = sum(kernels[k]['ms_per_step'] for k in fwd_keys)
        t_inv = sum(kernels[k]['ms_per_step'] for k in inv_keys)
    else:
        evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(args.steps)]
        torch.cuda.synchronize(dev)
        for k in range(args.steps):
            step(k * NS, evs[k], si=s_f)
        torch.cuda.synchronize(dev)
        t_fwd = sum(e[0].elapsed_time(e[1]) for e in evs) / args.steps
        t_inv = sum(e[2].elapsed_time(e[3]) for e in evs) / args.steps
        kernels = {'forward phase': {'ms_per_step': t_fwd, 'launches_per_step': 1, 'avg_launch_ms': t_fwd},
                   'inverse phase': {'ms_per_step': t_inv, 'launches_per_step': 1, 'avg_launch_ms': t_inv}}
    if world > 1:
        elapsed = max_over_ranks(elapsed, dev, backend)

    px_per_step = B * H * W
    value = world * px_per_step * args.steps / elapsed / 1e6
    S = cpf / (H * W)
    bytes_fwd = int(px_per_step * 3 + px_per_step * S * 2)  # one launch processes one batch
    bytes_inv = int(px_per_step * S * 2 + px_per_step * 3)
    # the dominant kernel: the single longest launch of the step, with its own
    # algorithmic bytes (front-end kernels: RGB in + coefficients out; inverse
    # kernels: coefficients in + RGB out; both per launch over the whole batch)
    cand = {k: v for k, v in kernels.items() if not k.startswith('(')}
    kname = max(cand, key=lambda k: cand[k]['avg_launch_ms'])
    t_dom = cand[kname]['avg_launch_ms']
    dom = 'k_inv' if kname.startswith(INV_PREFIXES) or kname == 'inverse phase' else 'k_fwd'
    dom_bytes = bytes_inv if dom == 'k_inv' else bytes_fwd
    achieved = dom_bytes / (t_dom * 1e-3) / 1e9
    # PMC records of the same configuration (profiles/pmc_valu.json,
    # profiles/pmc_traffic.json: tools/r6_pmc.sh + tools/r6_valu.py), per kernel;
    # recorded for some frames-per-launch count B0, scaled to this B
    base = f'{W}x{H}_q{quality}_{mode}_pf{int(bool(pf))}' + ('_B16' if block == 16 else '') + '_b'

    def pmc_entry(fname):
        f = os.path.join(ROOT, 'profiles', fname)
        if not os.path.exists(f):
            return None, None, None
        try:
            rec = json.load(open(f))
        except ValueError:
            return None, None, None
        want = kname.split('<')[0]
        for kk, vv in rec.items():
            if not kk.startswith(base) or not isinstance(vv, dict) or 'kernels' not in vv:
                continue
            cands = {k: v for k, v in vv['kernels'].items() if k.replace('jds::', '').split('<')[0] == want}
            if cands:
                pick = max(cands, key=lambda k: cands[k]['valu_insts'] if isinstance(cands[k], dict) else cands[k])
                return cands[pick], int(kk[len(base):]), f'profiles/{fname}[{kk}] ({vv.get("source", "")})'
        return None, None, None

    traffic, traffic_src = None, None
    tb, tb0, tsrc = pmc_entry('pmc_traffic.json')
    if tb is not None:
        traffic, traffic_src = int(tb * B / tb0), tsrc

    # VALU issue of the dominant kernel from its own PMC counts: every class at
    # its minimum (peak-rate) issue cost over the SIMD-cycles of the profiled
    # launches -- a lower bound on VALU-busy, <= 1 by construction
    # (tools/r6_valu.py); frac_upper prices int32 / unclassified at the slow class
    valu = None
    vr, _, vsrc = pmc_entry('pmc_valu.json')
    if vr is not None and not (args.exact or args.exact_inv or args.inv_fast):
        valu = {'frac': round(vr['valu_frac'], 4), 'frac_upper': round(vr['valu_frac_upper'], 4),
                'valu_insts_per_wave': round(vr['valu_per_wave'], 1),
                'wave_split': {k: round(v, 3) for k, v in vr['wave_split'].items()},
                'lds_conflict_share': round(vr['lds_conflict_share'], 3),
                'peak': 'SIMD-cycles of the profiled launches (1024 x GRBM_GUI_ACTIVE / 8); each VALU class at its '
                        'minimum wave64 issue cost (fp64 4, fp32 / int32 / moves 2, cvt 4, transcendental 8 cycles)',
                'source': vsrc}
    bound = 'valu' if valu and valu['frac'] > achieved / HBM_PEAK_GBS else 'hbm'

    result = {
        'metric': metric_name(quality, mode),
        'value': round(value, 2),
        'unit': 'Mpixels/s',
        'n_gpus': world,
        'steps': args.steps,
        'warmup': args.warmup,
        'warmup_steps_run': nwarm,
        'ms_per_step': round(elapsed / args.steps * 1e3, 4),
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': None,
        'dtype': 'f32+f64',  # forward: fp32 certified + fp64 fix-up; inverse: fp64 (u8 in/out, int16 coefficients)
        'data': 'synthetic (uniform random RGB generated on device)',
        'config': {'workload': f'{W}x{H} RGB, Q={quality}, {mode}, prefilter={"on" if pf else "off"}, '
                               f'{block}x{block} blocks (' + workload_label(H, W, quality, mode, pf, block) + ')',
                   'frames_per_gpu_per_step': B, 'global_batch_frames': B * world,
                   'pipeline': ('image stream: forward of batch k+1 beside the inverse of batch k (two streams, '
                                'two buffer sets)' if NS > 1 else 'serial forward then inverse per step'),
                   'parallelism': f'frame-shard x{world}', **dist_info(world, backend)},
        'roofline': {'bound': bound, 'kernel': kname, 'achieved': round(achieved, 2), 'peak': HBM_PEAK_GBS,
                     'unit': 'GB/s', 'frac': round(achieved / HBM_PEAK_GBS, 4), 'traffic': traffic,
                     'traffic_source': traffic_src,
                     'frac_vs_measured_copy_bw': round(achieved / HBM_COPY_GBS, 4),
                     'algorithmic_bytes_per_launch': dom_bytes,
                     'algorithmic_bytes_note': (f'{B} frames x {H}x{W} px x ' +
                                                (f'(2 x {S:.4f} B coefficients in + 3 B RGB out)' if dom == 'k_inv'
                                                 else f'(3 B RGB in + 2 x {S:.4f} B coefficients out)')),
                     'avg_launch_ms': round(t_dom, 4),
                     'timing': ('jds_plan_profile marks (kernels_ms)' if kprof else
                                'HIP events per phase, serial calibration pass after the timed region'),
                     'valu': valu,
                     'note': ('kernel: the longest single launch of the step; achieved / peak / frac: the HBM '
                              'roofline by its algorithmic bytes; bound: the resource with the larger fraction '
                              '(valu.frac: a lower bound on the VALU-busy fraction from the kernel\'s own PMC counts, '
                              'DESIGN.md section 4); traffic: HBM bytes per launch from calibrated FETCH / WRITE '
                              'counters')},
        'kernels_ms': {k: round(v['ms_per_step'], 4) for k, v in kernels.items()},
        'kernels_profile': kprof and {**{k: round(v, 4) if isinstance(v, float) else v for k, v in kprof.items()},
                                      'avg_launch_ms': {k: round(v['avg_launch_ms'], 4) for k, v in kernels.items()},
                                      'phases_ms': {'forward': round(t_fwd, 4), 'inverse': round(t_inv, 4)}},
        'fixups_last_step': {'fwd_blocks': int(plans[0].fix_counts()[0]), 'inv_tiles': int(plans[0].fix_counts()[1])},
        'pipeline_roofline_frac': round(value / world * 1e6 * (6 + 2 * S) / (HBM_PEAK_GBS * 1e9), 4),
    }
    state = {'plans': plans, 'rgb': rgbs[0], 'out': outs[0], 'coeffs': coefs[0], 'stats': stats_l[0], 's_f': s_f,
             'cpf': cpf, 'qt': qt}
    return result, state


# launch-mark names (jds_plan_profile) by phase: the forward front ends,
# reductions and fix-ups; the inverse kernels and their per-frame tail
FWD_PREFIXES = ('k_fwd', 'k_fix_fwd', 'k_quant_mq')
INV_PREFIXES = ('k_inv', 'k_chroma16', 'k_finalize', 'k_sel_')


def frame0_parity(state, quality, mode, pf, block):
    """Frame 0 against the oracle (outside the timed region): coefficient and
    byte mismatches, PSNR and its difference from the reference's."""
    import numpy as np
    from oracle import cpu_ref
    f0 = state['rgb'][0].cpu().numpy()
    ref = cpu_ref.compress_reconstruct(f0, quality, block, mode, bool(pf), metrics=False, stretch=block == 16)
    rec0, cf0 = state['out'][0].cpu().numpy(), state['coeffs'][0].cpu().numpy()
    mse = np.mean((f0.astype(np.float64) - rec0) ** 2)
    mse_ref = np.mean((f0.astype(np.float64) - ref['reconstructed']) ** 2)
    return {'frame': 0, 'coeff_mismatch': int(np.sum(cf0 != ref['coeffs'])),
            'recon_mismatch_bytes': int(np.sum(rec0 != ref['reconstructed'])),
            'psnr_rgb': float(10 * np.log10(255 ** 2 / mse)),
            'dpsnr_rgb_vs_ref': float(10 * np.log10(255 ** 2 / mse) - 10 * np.log10(255 ** 2 / mse_ref))}


NORTH_STAR = dict(B=16, H=2160, W=3840, quality=50, mode='4:2:0', pf=1)  # BASELINE.json north_star point


def main():
    args = parse()
    visible = 0
    if args.gpus > 1 and 'WORLD_SIZE' not in os.environ and not args.dry_run:
        import torch  # (counting devices does not initialise the GPU on this image)
        visible = torch.cuda.device_count()
    action, detail = launch_decision(args.gpus, os.environ, visible, args.dry_run)
    if action == 'error':
        print(f'bench.py: {detail}', file=sys.stderr, flush=True)
        sys.exit(2)
    if action == 'spawn':
        sys.exit(spawn_ranks(args.gpus, detail, sys.argv[1:]))
    if args.dry_run:
        return dry_run_main(args)
    if args.sweep:
        return sweep_main(args)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    local, backend = init_dist(world, local)
    dev = torch.device('cuda', local)
    torch.cuda.set_device(dev)

    from jds import _abi
    from jds.sweep import broadcast_tables

    B, H, W = args.frames, args.height, args.width
    # rank 0's quant table reaches every rank in one broadcast (RCCL over xGMI
    # at N > 1, the north star's exchange; outside the timed region)
    qt = broadcast_tables([args.quality])[0]
    result, state = run_point(args, dev, world, backend, rank, B, H, W, args.quality, args.mode, args.prefilter,
                              args.block, qt)
    result['config']['quant_table'] = ('rank 0 -> all ranks, one broadcast of 64 float64 '
                                       f'({"RCCL over xGMI" if backend == "nccl" else backend})' if world > 1
                                       else 'local (one rank)')
    plans, rgb, coeffs, stats, s_f, cpf = (state[k] for k in ('plans', 'rgb', 'coeffs', 'stats', 's_f', 'cpf'))
    px_per_step = B * H * W

    if not args.no_entropy and args.block == 8:
        # JPEG entropy coding of the step's coefficients (jds_entropy.hip), timed on
        # its own after the headline region: files per frame, real bits per pixel
        from jds import entropy
        ent = entropy.PlanEntropy(plans[0])
        files = torch.empty((B, ent.capacity), dtype=torch.uint8, device=dev)
        lengths = torch.zeros(B, dtype=torch.int64, device=dev)
        for _ in range(5):
            ent.run(coeffs.data_ptr(), files.data_ptr(), ent.capacity, lengths.data_ptr(), 0, s_f.cuda_stream)
        reps = 50  # (~12 ms: steady clocks; 10 repetitions read ~2 % high)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s_f)
        for _ in range(reps):
            ent.run(coeffs.data_ptr(), files.data_ptr(), ent.capacity, lengths.data_ptr(), 0, s_f.cuda_stream)
        e1.record(s_f)
        torch.cuda.synchronize(dev)
        t_ent = e0.elapsed_time(e1) / reps
        nbytes = int(lengths.sum().item())
        moved = B * cpf * 2 + nbytes  # algorithmic: coefficients in, files out
        result['entropy'] = {
            'kernels': 'k_ent_walk, k_ent_place (segment offsets, shared words completed), k_ent_fscan (0xFF counts, output offsets, markers), k_ent_emit3', 'ms_per_step': round(t_ent, 4),
            'Mpixels_per_s': round(px_per_step / (t_ent * 1e-3) / 1e6 * world, 2),
            'file_bytes_per_frame': round(nbytes / B, 1), 'bpp': round(8 * nbytes / px_per_step, 4),
            'bpp_estimate_no_entropy': None,
            'achieved_GBps': round(moved / (t_ent * 1e-3) / 1e9, 2),
            'frac': round(moved / (t_ent * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
        st0 = stats[0].cpu().numpy().view(_abi.STATS_DTYPE)[0]
        from utils.metrics import bitrate_from_counts
        result['entropy']['bpp_estimate_no_entropy'] = round(bitrate_from_counts(
            int(st0['nonzero']), float(st0['magnitude_bits']), int(st0['total_coeffs']), (H, W), 8)['bpp'], 4)
        del files

    if not args.no_parity:
        # PSNR / bytes vs the reference restatement on frame 0 (outside the timed
        # region) -- on every rank, its own frames; rank 0 reports all of them
        par = frame0_parity(state, args.quality, args.mode, args.prefilter, args.block)
        pr = gather_parity(par, world, backend)
        if rank == 0:
            result['parity'] = par
            result['parity_ranks'] = pr
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        n = max(1, min(B, 64))
        host = rgb[:n].cpu().numpy()
        result['cpu_baseline'] = cpu_baseline(host, args.quality, args.mode, bool(args.prefilter),
                                              args.cpu_baseline_seconds, args.block)
    else:
        result['cpu_baseline'] = None
    for p_ in plans:
        p_.close()
    del state, rgb, coeffs, stats

    default_point = (H, W, args.quality, args.mode, bool(args.prefilter), args.block) == (1080, 1920, 50, '4:2:0',
                                                                                          True, 8)
    if default_point and not args.no_north_star:
        # the north-star point (BASELINE.json north_star: 4K / Q=50 / 4:2:0), same
        # timing method, same ranks: the driver's default run carries it
        ns = NORTH_STAR
        nqt = broadcast_tables([ns['quality']])[0]
        r_ns, st_ns = run_point(args, dev, world, backend, rank, ns['B'], ns['H'], ns['W'], ns['quality'],
                                ns['mode'], ns['pf'], 8, nqt, seed=3000)
        keep = ('metric', 'value', 'unit', 'ms_per_step', 'warmup_steps_run', 'roofline', 'kernels_ms', 'kernels_profile',
                'fixups_last_step', 'pipeline_roofline_frac')
        result['north_star'] = {k: r_ns[k] for k in keep}
        result['north_star']['config'] = {'workload': r_ns['config']['workload'],
                                          'frames_per_gpu_per_step': ns['B'], 'steps': args.steps}
        result['north_star']['target_pipeline_roofline_frac'] = 0.60
        if not args.no_parity:
            par = frame0_parity(st_ns, ns['quality'], ns['mode'], ns['pf'], 8)
            pr = gather_parity(par, world, backend)
            if rank == 0:
                result['north_star']['parity'] = par
                result['north_star']['parity_ranks'] = {k: pr[k] for k in ('world_size', 'backend', 'all_exact')}
        for p_ in st_ns['plans']:
            p_.close()
        del st_ns
    if rank == 0 and not args.no_host_path and args.block == 8:
        result['host_path'] = host_path(args.quality, args.mode, args.prefilter)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
