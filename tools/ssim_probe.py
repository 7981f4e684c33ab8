"""Time K4 (SSIM / PSNR) per 1080p frame: the batched band pipeline
(jds_psnr_ssim_batch_dev) at batch 1, 8 and 32 (BATCH env).  Prints
one JSON line.  Run on the GPU box (optionally under rocprofv3 --kernel-trace
--stats for per-kernel times)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'jpeg-dsp-studio_amd'), ROOT]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from jds import codec  # noqa: E402


def main():
    H, W = (int(x) for x in (sys.argv[1:3] if len(sys.argv) > 2 else (1080, 1920)))
    reps = int(os.environ.get('REPS', '10'))
    dev = torch.device('cuda', 0)
    g = torch.Generator(device=dev).manual_seed(0)
    n = int(os.environ.get('BATCH', '8'))
    a = torch.randint(0, 256, (n, H, W, 3), dtype=torch.uint8, device=dev, generator=g)
    noise = torch.randint(-8, 8, (n, H, W, 3), dtype=torch.int16, device=dev, generator=g)
    b = (a.to(torch.int16) + noise).clamp(0, 255).to(torch.uint8)
    torch.cuda.synchronize()
    pa = [a[i].data_ptr() for i in range(n)]
    pb = [b[i].data_ptr() for i in range(n)]
    res = {'H': H, 'W': W}

    def timeit(fn, k):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(k):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / k * 1e3

    r1 = None

    def one():
        nonlocal r1
        r1 = codec.psnr_ssim_batch_dev(pa[:1], pb[:1], H, W, 0, None)
    res['batch1_ms'] = timeit(one, reps)
    r8 = None

    def eight():
        nonlocal r8
        r8 = codec.psnr_ssim_batch_dev(pa, pb, H, W, 0, None)
    res[f'batch{n}_ms_per_item'] = timeit(eight, max(2, reps // 4)) / n
    res['bitwise_equal_batch'] = bool(np.array_equal(r8[0].view(np.uint64), r1[0].view(np.uint64)))
    res['values'] = [float(x) for x in r1[0]]
    print(json.dumps(res))


if __name__ == '__main__':
    main()
