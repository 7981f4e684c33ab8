"""Host-side calls into libjds.so for the drop-in engines.* / utils.metrics API.

Everything here marshals NumPy arrays across the C-ABI; all per-sample
arithmetic happens in the HIP kernels.  Only parameter setup is done on the
host: the quantisation table (engines/quantizer.py:7-19, computed by the caller
with the reference's NumPy expression) and the 3 prefilter taps below.
"""
from __future__ import annotations

import ctypes as C
import math
from typing import Dict, Tuple

import numpy as np

from . import _abi
from ._abi import check, lease, lib, make_params


def gaussian_kernel3(sigma: float = 0.75) -> np.ndarray:
    """Taps of cv2.GaussianBlur(ksize=(3,3), sigmaX=sigma) for CV_64F
    (engines/color_space.py:39-40): OpenCV's getGaussianKernelBitExact for n=3:
    t = exp(4 * (-0.125 / sigma^2)), k = [t, 1, t] / (2t + 1) computed as t * (1/sum)."""
    scale2x = -0.125 / (float(sigma) * float(sigma))
    t = math.exp(4.0 * scale2x)
    mul1 = 1.0 / ((t * 2.0) + 1.0)
    e = t * mul1
    return np.array([e, mul1, e], dtype=np.float64)


def _u8_image(image: np.ndarray) -> np.ndarray:
    a = np.asarray(image)
    if a.ndim != 3 or a.shape[2] != 3:
        raise ValueError('Input images must have the same dimensions.' if a.ndim == 3 else
                         f'compress_reconstruct expects an HxWx3 RGB image, got shape {a.shape}')
    if a.dtype != np.uint8:
        if not np.issubdtype(a.dtype, np.integer) or a.min(initial=0) < 0 or a.max(initial=0) > 255:
            raise ValueError(f'the MI355X path takes uint8 RGB images (got {a.dtype})')
        a = a.astype(np.uint8)
    return np.ascontiguousarray(a)


def compress_reconstruct_raw(image: np.ndarray, quality: int, qtable: np.ndarray, mode: str, prefilter: bool,
                             block_size: int = 8, selected_block_idx: Tuple[int, int] = (0, 0),
                             maps: bool = True, device: int = 0) -> Dict[str, object]:
    """One jds_compress_reconstruct call (include/jds.h): returns the raw outputs."""
    img = _u8_image(image)
    H, W = img.shape[:2]
    p = make_params(quality, qtable, mode, prefilter, gaussian_kernel3(0.75), block_size)
    geo = _abi.geometry(p, H, W)
    out = np.empty_like(img)
    coeffs = np.empty(geo.coeffs_per_frame, dtype=np.int16)
    st = _abi.FrameStats()
    ey = np.empty((H, W), np.float64) if maps else None
    er = np.empty((H, W), np.float64) if maps else None
    sel = _abi.SelectedBlock()
    sel_ok = C.c_int32(0)
    with lease(device) as ctx:
        check(lib().jds_compress_reconstruct(
            ctx.handle, C.byref(p), img.ctypes.data, H, W, out.ctypes.data, coeffs.ctypes.data, C.byref(st),
            ey.ctypes.data if maps else None, er.ctypes.data if maps else None,
            int(selected_block_idx[0]), int(selected_block_idx[1]), C.byref(sel), C.byref(sel_ok)))
    res: Dict[str, object] = {'reconstructed': out, 'coeffs': coeffs, 'stats': st, 'geometry': geo,
                              'error_map_y': ey, 'error_map_rgb': er, 'selected': None}
    if sel_ok.value:
        def arr(field, dt=np.float64):
            return np.ctypeslib.as_array(getattr(sel, field)).astype(dt).reshape(8, 8)
        res['selected'] = {'original': arr('original'), 'shifted': arr('shifted'), 'dct': arr('dct'),
                           'quantized': arr('quantized', np.int16), 'dequantized': arr('dequantized'),
                           'reconstructed': arr('reconstructed')}
    return res


def psnr_ssim_raw(a: np.ndarray, b: np.ndarray, device: int = 0) -> np.ndarray:
    """jds_psnr_ssim: [ssim_R, ssim_G, ssim_B, ssim_Y, mse_Y, mse_RGB] for two HxWx3 uint8 images."""
    a = _u8_image(a)
    b = _u8_image(b)
    if a.shape != b.shape:
        raise ValueError('Input images must have the same dimensions.')
    out = np.empty(6, np.float64)
    with lease(device) as ctx:
        check(lib().jds_psnr_ssim(ctx.handle, a.ctypes.data, b.ctypes.data, a.shape[0], a.shape[1], out.ctypes.data))
    return out


def _after(after):
    """`after` of the *_dev calls: None = the caller has synchronised (JDS_AFTER_NONE);
    otherwise a hipStream_t handle, passed unchanged (0 = the HIP null stream, waited for)."""
    return _abi.AFTER_NONE if after is None else C.c_void_p(int(after))


def psnr_ssim_dev(a_ptr: int, b_ptr: int, H: int, W: int, device: int = 0, after=-1) -> np.ndarray:
    """jds_psnr_ssim_dev: psnr_ssim_raw's six values for two HxWx3 uint8 images
    already in device memory (raw device pointers, e.g. torch tensors' data_ptr()).
    after: -1 = wait for the whole device (jds_psnr_ssim_dev); None = the caller
    has synchronised the images; a stream handle = wait only for that stream's
    queued work (jds_psnr_ssim_dev_after)."""
    out = np.empty(6, np.float64)
    with lease(device) as ctx:
        if after == -1:
            check(lib().jds_psnr_ssim_dev(ctx.handle, int(a_ptr), int(b_ptr), int(H), int(W), out.ctypes.data))
        else:
            check(lib().jds_psnr_ssim_dev_after(ctx.handle, int(a_ptr), int(b_ptr), int(H), int(W), out.ctypes.data,
                                                _after(after)))
    return out


def psnr_ssim_batch_dev(a_ptrs, b_ptrs, H: int, W: int, device: int = 0, after=None, ctx=None) -> np.ndarray:
    """jds_psnr_ssim_batch_dev: [n, 6] (psnr_ssim_raw's six values) for n
    device-resident image pairs (a_ptrs[i], b_ptrs[i]) of one size, run together
    on the GPU (the batch sweep's per-item SSIM).  after as in psnr_ssim_dev
    (None: the caller has synchronised).  ctx: a caller-owned Context of that
    device (e.g. with its own SSIM scratch budget) instead of a pooled one."""
    n = len(a_ptrs)
    if len(b_ptrs) != n:
        raise ValueError('a_ptrs and b_ptrs differ in length')
    out = np.empty((n, 6), np.float64)
    if n == 0:
        return out
    pa = (C.c_void_p * n)(*[int(p) for p in a_ptrs])
    pb = (C.c_void_p * n)(*[int(p) for p in b_ptrs])
    if ctx is not None:
        check(lib().jds_psnr_ssim_batch_dev(ctx.handle, n, pa, pb, int(H), int(W), out.ctypes.data, _after(after)))
        return out
    with lease(device) as c:
        check(lib().jds_psnr_ssim_batch_dev(c.handle, n, pa, pb, int(H), int(W), out.ctypes.data, _after(after)))
    return out


def magnitude_bits_f32_dev(coeffs_ptr: int, n_coeffs: int, device: int = 0, after=None) -> float:
    """jds_magnitude_bits_f32_dev: NumPy's float32 np.sum of magnitude_bits
    (utils/metrics.py:77-78) over n_coeffs device-resident int16 coefficients."""
    out = C.c_double()
    with lease(device) as ctx:
        check(lib().jds_magnitude_bits_f32_dev(ctx.handle, int(coeffs_ptr), int(n_coeffs), C.byref(out),
                                               _after(after)))
    return float(out.value)


def magnitude_bits_f32_batch_dev(coeffs_ptr: int, n_items: int, n_coeffs: int, item_stride: int,
                                 device: int = 0, after=None) -> np.ndarray:
    """jds_magnitude_bits_f32_batch_dev: magnitude_bits_f32_dev for n_items
    coefficient arrays at coeffs_ptr + 2 * i * item_stride bytes, one host wait."""
    out = np.empty(n_items, np.float64)
    if n_items == 0:
        return out
    with lease(device) as ctx:
        check(lib().jds_magnitude_bits_f32_batch_dev(ctx.handle, int(coeffs_ptr), int(n_items), int(n_coeffs),
                                                     int(item_stride), out.ctypes.data, _after(after)))
    return out


# ----------------------------------------------------------- per-stage ops

def _f64(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float64)


def stage_rgb_ycbcr(x: np.ndarray, inverse: bool) -> np.ndarray:
    x = _f64(x)
    if x.shape[-1] != 3:
        raise IndexError('index 2 is out of bounds for axis 2')
    out = np.empty_like(x)
    fn = lib().jds_stage_ycbcr_to_rgb if inverse else lib().jds_stage_rgb_to_ycbcr
    with lease() as ctx:
        check(fn(ctx.handle, x.ctypes.data, out.ctypes.data, x.size // 3))
    return out


def stage_subsample(cb: np.ndarray, cr: np.ndarray, mode: str, prefilter: bool):
    cb, cr = _f64(cb), _f64(cr)
    H, W = cb.shape
    oh = H // 2 if mode == '4:2:0' else H
    ocb = np.empty((oh, W // 2), np.float64)
    ocr = np.empty((oh, W // 2), np.float64)
    g = gaussian_kernel3(0.75)
    with lease() as ctx:
        check(lib().jds_stage_subsample(ctx.handle, cb.ctypes.data, cr.ctypes.data, H, W,
                                        _abi.MODE_CODES[mode], 1 if prefilter else 0, g.ctypes.data,
                                        ocb.ctypes.data, ocr.ctypes.data))
    return ocb, ocr


def stage_resize(x: np.ndarray, H: int, W: int, nearest: bool) -> np.ndarray:
    x = _f64(x)
    out = np.empty((H, W), np.float64)
    with lease() as ctx:
        check(lib().jds_stage_upsample(ctx.handle, x.ctypes.data, x.shape[0], x.shape[1], H, W,
                                       1 if nearest else 0, out.ctypes.data))
    return out


def stage_block(x: np.ndarray, op: int) -> np.ndarray:
    """op: 0 dct2, 1 idct2, 2 encode_block, 3 decode_block on (..., 8, 8) or (..., 16, 16)."""
    x = _f64(x)
    if x.ndim < 2 or x.shape[-2:] not in ((8, 8), (16, 16)):
        raise ValueError(f'the MI355X block transforms are 8x8 and 16x16 (got {x.shape})')
    b = x.shape[-1]
    out = np.empty_like(x)
    with lease() as ctx:
        check(lib().jds_stage_block_dct_n(ctx.handle, x.ctypes.data, out.ctypes.data, x.size // (b * b), b, op))
    return out


def stage_quant(x: np.ndarray, q: np.ndarray, dequant: bool) -> np.ndarray:
    q = _f64(q)
    if q.shape not in ((8, 8), (16, 16)) or x.shape[-2:] != q.shape:
        # NumPy's broadcast error for c / Q (engines/quantizer.py:24)
        fmt = lambda s: '(' + ','.join(str(d) for d in s) + (',)' if len(s) == 1 else ')')
        raise ValueError(f'operands could not be broadcast together with shapes {fmt(x.shape)} {fmt(q.shape)} ')
    if dequant:
        x = np.ascontiguousarray(x, dtype=np.int16)
        out = np.empty(x.shape, np.float64)
    else:
        x = _f64(x)
        out = np.empty(x.shape, np.int16)
    with lease() as ctx:
        check(lib().jds_stage_quantize_n(ctx.handle, x.ctypes.data, q.ctypes.data, q.size, out.ctypes.data,
                                         x.size, 1 if dequant else 0))
    return out
