"""Fix-up counts of the certified fp32 forward per quality (not product code)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, 'jpeg-dsp-studio_amd'), ROOT]
import torch
from jds import _abi, codec
from engines.quantizer import scale_quant_matrix
from utils.constants import JPEG_LUMA_Q50

F, H, W = 16, 1080, 1920
dev = torch.device('cuda:0')
rgb = torch.randint(0, 256, (F, H, W, 3), dtype=torch.uint8, device=dev)
for q in (5, 10, 20, 50, 80, 90, 95, 100):
    params = [_abi.make_params(q, scale_quant_matrix(JPEG_LUMA_Q50, q), '4:2:0', True, codec.gaussian_kernel3())] * F
    plan = _abi.Plan(_abi.context(0), params, H, W)
    out = torch.empty_like(rgb)
    cf = torch.empty((F, plan.geometry.coeffs_per_frame), dtype=torch.int16, device=dev)
    st = torch.zeros((F, _abi.STATS_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    for _ in range(2):
        plan.run(rgb.data_ptr(), out.data_ptr(), cf.data_ptr(), st.data_ptr(), _abi.RUN_FWD, 0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        plan.run(rgb.data_ptr(), out.data_ptr(), cf.data_ptr(), st.data_ptr(), _abi.RUN_FWD, 0)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / 5 * 1e3
    fix = int(plan.fix_counts()[0])
    nb = F * plan.geometry.coeffs_per_frame // 64
    print(f'Q={q:3d} fwd {ms:7.3f} ms / {F} frames   flagged {fix:8d} blocks = {100 * fix / nb:6.2f} %', flush=True)
    plan.close()
