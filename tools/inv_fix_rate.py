#!/usr/bin/env python3
"""Tiles the certified fast inverse recomputes exactly, per quality (random 1080p
4:2:0 frames), and the fast vs exact inverse kernel time of each (not product code)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'jpeg-dsp-studio_amd'), ROOT]
import torch  # noqa: E402
from jds import _abi, codec  # noqa: E402
from engines.quantizer import scale_quant_matrix  # noqa: E402
from utils.constants import JPEG_LUMA_Q50  # noqa: E402

B, H, W = 16, 1080, 1920
dev = torch.device('cuda:0')
rgb = torch.randint(0, 256, (B, H, W, 3), dtype=torch.uint8, device=dev)
out = torch.empty_like(rgb)
for q in [int(x) for x in os.environ.get('QS', '5,10,20,50,80,95,100').split(',')]:
    prm = _abi.make_params(q, scale_quant_matrix(JPEG_LUMA_Q50, q), '4:2:0', True, codec.gaussian_kernel3())
    plan = _abi.Plan(_abi.context(0), [prm] * B, H, W)
    cf = torch.empty((B, plan.geometry.coeffs_per_frame), dtype=torch.int16, device=dev)
    st = torch.zeros((B, _abi.STATS_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    res = {}
    for name, fl in (('fast', 0), ('exact', _abi.RUN_EXACT_INV), ('fast_sse', _abi.RUN_SSE),
                     ('exact_sse', _abi.RUN_SSE | _abi.RUN_EXACT_INV)):
        plan.run(rgb.data_ptr(), out.data_ptr(), cf.data_ptr(), st.data_ptr(), fl, 0)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(5):
            plan.run(rgb.data_ptr(), out.data_ptr(), cf.data_ptr(), st.data_ptr(), fl | _abi.RUN_INV, 0)
        e1.record()
        torch.cuda.synchronize()
        res[name] = (round(e0.elapsed_time(e1) / 5, 4), plan.fix_counts()[1])
    print(q, res, flush=True)
    plan.close()
