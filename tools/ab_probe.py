"""A/B timing of plan variants under steady clocks (not product code).

The MI355X ramps its clocks over the first ~40 ms of sustained load (k_inv2
549 -> 404 us across the first 40 launches of a bench run), so single-shot
comparisons of variants run one after the other are biased toward the later
one.  This probe prewarms for 0.5 s, then interleaves blocks of steps of each
variant and reports the median block time per variant.

Variants (argv, comma separated): serial (one jds_plan_run per step),
side (same, plan created with JDS_SIDE_STREAM=1), piped (forward of batch k+1
beside inverse of batch k on a second stream).
"""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'jpeg-dsp-studio_amd'), ROOT]
import torch  # noqa: E402
from jds import _abi, codec  # noqa: E402
from engines.quantizer import scale_quant_matrix  # noqa: E402
from utils.constants import JPEG_LUMA_Q50  # noqa: E402

variants = (sys.argv[1] if len(sys.argv) > 1 else 'serial,side,piped').split(',')
B, H, W, Q = 64, 1080, 1920, int(os.environ.get('Q', '50'))
dev = torch.device('cuda:0')
prm = _abi.make_params(Q, scale_quant_matrix(JPEG_LUMA_Q50, Q), '4:2:0', True, codec.gaussian_kernel3())
ctx = _abi.context(0)
gen = torch.Generator(device=dev)
gen.manual_seed(1)
sets = []
for i in range(2):
    rgb = torch.randint(0, 256, (B, H, W, 3), dtype=torch.uint8, device=dev, generator=gen)
    sets.append(dict(rgb=rgb, out=torch.empty_like(rgb)))
plans = {}
for v in variants:
    os.environ['JDS_SIDE_STREAM'] = '1' if v == 'side' else '0'
    plans[v] = [_abi.Plan(ctx, [prm] * B, H, W) for _ in range(2)]
os.environ.pop('JDS_SIDE_STREAM')
cpf = plans[variants[0]][0].geometry.coeffs_per_frame
for s in sets:
    s['cf'] = torch.empty((B, cpf), dtype=torch.int16, device=dev)
    s['st'] = torch.zeros((B, _abi.STATS_DTYPE.itemsize), dtype=torch.uint8, device=dev)
s_f, s_i = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
ev_f = [torch.cuda.Event(), torch.cuda.Event()]
ev_i = [torch.cuda.Event(), torch.cuda.Event()]
used = [False, False]


def ptr(b):
    s = sets[b]
    return s['rgb'].data_ptr(), s['out'].data_ptr(), s['cf'].data_ptr(), s['st'].data_ptr()


def run(v, k):
    if v == 'piped':
        b = k & 1
        if used[b]:
            s_f.wait_event(ev_i[b])
        used[b] = True
        plans[v][b].run(*ptr(b), _abi.RUN_FWD, s_f.cuda_stream)
        ev_f[b].record(s_f)
        s_i.wait_event(ev_f[b])
        plans[v][b].run(*ptr(b), _abi.RUN_INV, s_i.cuda_stream)
        ev_i[b].record(s_i)
    else:
        plans[v][0].run(*ptr(0), 0, s_f.cuda_stream)


torch.cuda.synchronize()
t0 = time.perf_counter()
k = 0
while time.perf_counter() - t0 < 0.5:
    run(variants[0], k)
    k += 1
    if k % 8 == 0:
        torch.cuda.synchronize()
torch.cuda.synchronize()
res = {v: [] for v in variants}
for rep in range(6):
    for v in variants:
        torch.cuda.synchronize()
        t = time.perf_counter()
        for k in range(10):
            run(v, k)
        torch.cuda.synchronize()
        res[v].append((time.perf_counter() - t) / 10 * 1e3)
for v in variants:
    m = statistics.median(res[v])
    print(f'{v:8s} median {m:.4f} ms/batch  {B * H * W / m / 1e3:10.0f} Mpix/s   blocks: ' +
          ' '.join(f'{x:.3f}' for x in res[v]), flush=True)
