"""Baseline JPEG entropy coding on the GPU (include/jds.h: jds_encode_jfif,
jds_plan_entropy): the reference's quantised coefficients -> a standard JFIF
file (the reference itself only estimates the size,
utils/metrics.py:51-92).  Byte-for-byte definition: oracle/jpeg_entropy.py."""
from __future__ import annotations

import ctypes as C
from typing import List, Tuple

import numpy as np

from . import _abi
from ._abi import check, lib, make_params


def encode_jfif(coeffs: np.ndarray, H: int, W: int, mode: str, qtable: np.ndarray,
                device: int = 0) -> Tuple[bytes, List[int]]:
    """One frame: all_quantized_coeffs (int16, Y/Cb/Cr blocks) -> (file bytes,
    entropy-coded bits of the Y, Cb, Cr scans)."""
    p = make_params(50, qtable, mode, False, np.zeros(3))
    geo = _abi.geometry(p, H, W)
    cf = np.ascontiguousarray(coeffs, dtype=np.int16).reshape(-1)
    if cf.size != geo.coeffs_per_frame:
        raise ValueError(f'expected {geo.coeffs_per_frame} coefficients for {H}x{W} {mode}, got {cf.size}')
    n = C.c_int64(0)
    bits = (C.c_uint64 * 3)()
    # a random frame at high quality stays far below this; the C side reports the exact need
    cap = max(1 << 16, 8 * cf.size)
    while True:
        out = np.empty(cap, np.uint8)
        with _abi.lease(device) as ctx:
            rc = lib().jds_encode_jfif(ctx.handle, C.byref(p), H, W, cf.ctypes.data, out.ctypes.data,
                                       cap, C.byref(n), bits)
        if rc == _abi.JDS_EINVAL and n.value > cap:
            cap = n.value
            continue
        check(rc)
        return out[:n.value].tobytes(), [int(b) for b in bits]


def bitrate_from_jfif(nbytes: int, shape) -> dict:
    """bpp / compression ratio of a real file, in estimate_bitrate_no_entropy's
    terms (utils/metrics.py:62-92: 24-bit originals)."""
    h, w = shape
    bits = 8 * int(nbytes)
    return {'estimated_bits': bits, 'bpp': float(bits / (h * w)),
            'compression_ratio': float(h * w * 3 * 8 / max(bits, 1)), 'label': 'Baseline JPEG (Huffman, JFIF)'}


class PlanEntropy:
    """Device-resident entropy coding for a jds_plan: out[i] holds frame i's file."""

    def __init__(self, plan: _abi.Plan):
        self.plan = plan
        cap = C.c_int64(0)
        check(lib().jds_plan_entropy_capacity(plan.handle, C.byref(cap)))
        self.capacity = int(cap.value)

    def run(self, coeffs_dev: int, out_dev: int, out_stride: int, lengths_dev: int, scan_bits_dev: int = 0,
            stream: int | None = None):
        if stream is None:
            stream = lib().jds_ctx_stream(self.plan.ctx.handle)
        check(lib().jds_plan_entropy(self.plan.handle, coeffs_dev, out_dev, out_stride, lengths_dev,
                                     scan_bits_dev or None, stream))
