"""ctypes binding of the C-ABI in include/jds.h (libjds.so, hand-written HIP for gfx950).

The HIP runtime: PyTorch-ROCm ships its own libamdhip64.so (SONAME
libamdhip64.so.7, same as /opt/rocm's).  To keep ONE runtime per process, the
torch copy is preloaded (RTLD_GLOBAL) before libjds.so when torch is installed,
so libjds.so, torch tensors and torch streams share it.

There is no CPU fallback: if libjds.so is missing or no HIP device is present,
the calls raise.
"""
from __future__ import annotations

import ctypes as C
import importlib.util
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# JDS_LIB_PATH: load another build of the same ABI (A/B timing of kernel variants, tools/ab_lib.sh)
LIB_PATH = os.environ.get('JDS_LIB_PATH') or os.path.join(_HERE, 'libjds.so')

JDS_OK, JDS_EINVAL, JDS_ENOTSUP, JDS_EHIP, JDS_ENOMEM = 0, -1, -2, -3, -4
SS_444, SS_422, SS_420 = 0, 1, 2
MODE_CODES = {'4:4:4': SS_444, '4:2:2': SS_422, '4:2:0': SS_420}
RUN_SSE, RUN_FWD, RUN_INV, RUN_EXACT, RUN_EXACT_INV, RUN_INV_FIXALL, RUN_FWD_FIXALL, RUN_INV_FAST = 1, 2, 4, 8, 16, 32, 64, 128


class Params(C.Structure):
    _fields_ = [('block_size', C.c_int32), ('quality', C.c_int32), ('subsampling', C.c_int32),
                ('prefilter', C.c_int32), ('qtable', C.c_double * 64), ('gauss', C.c_double * 3)]


class FrameStats(C.Structure):
    _fields_ = [('nonzero', C.c_uint64), ('total_coeffs', C.c_uint64), ('magnitude_bits', C.c_uint64),
                ('block_overhead_bits', C.c_uint64), ('hist', C.c_uint64 * 50), ('sse_rgb', C.c_uint64),
                ('sse_y', C.c_double), ('pixels', C.c_uint64), ('fwd_ms', C.c_double),
                ('inv_ms', C.c_double), ('ssim', C.c_double * 4), ('mse_y', C.c_double),
                ('magnitude_bits_f32', C.c_double), ('reserved', C.c_uint64 * 1)]


# the same record as a NumPy dtype, for stats arrays that live in device memory
STATS_DTYPE = np.dtype([('nonzero', '<u8'), ('total_coeffs', '<u8'), ('magnitude_bits', '<u8'),
                        ('block_overhead_bits', '<u8'), ('hist', '<u8', (50,)), ('sse_rgb', '<u8'),
                        ('sse_y', '<f8'), ('pixels', '<u8'), ('fwd_ms', '<f8'), ('inv_ms', '<f8'),
                        ('ssim', '<f8', (4,)), ('mse_y', '<f8'), ('magnitude_bits_f32', '<f8'),
                        ('reserved', '<u8', (1,))])
assert STATS_DTYPE.itemsize == C.sizeof(FrameStats)


class Geometry(C.Structure):
    _fields_ = [('H', C.c_int64), ('W', C.c_int64), ('chroma_h', C.c_int64), ('chroma_w', C.c_int64),
                ('y_blocks_y', C.c_int64), ('y_blocks_x', C.c_int64), ('c_blocks_y', C.c_int64),
                ('c_blocks_x', C.c_int64), ('coeffs_per_frame', C.c_int64), ('cb_offset', C.c_int64),
                ('cr_offset', C.c_int64), ('tiles', C.c_int32), ('threads_fwd', C.c_int32),
                ('threads_inv', C.c_int32), ('reserved', C.c_int32)]


class SelectedBlock(C.Structure):
    _fields_ = [('original', C.c_double * 64), ('shifted', C.c_double * 64), ('dct', C.c_double * 64),
                ('quantized', C.c_int16 * 64), ('dequantized', C.c_double * 64),
                ('reconstructed', C.c_double * 64)]


class KernelTime(C.Structure):
    _fields_ = [('name', C.c_char * 64), ('total_ms', C.c_double), ('launches', C.c_int64)]


class JDSError(RuntimeError):
    pass


_P = C.c_void_p
ABI_VERSION = 3
# `after` of the *_dev calls: no wait (the caller has synchronised); include/jds.h JDS_AFTER_NONE
AFTER_NONE = C.c_void_p(-1 & ((1 << (8 * C.sizeof(C.c_void_p))) - 1))
_SIGS = {
    'jds_abi_version': (C.c_int, []),
    'jds_last_error': (C.c_char_p, []),
    'jds_device_count': (C.c_int, [C.POINTER(C.c_int)]),
    'jds_geometry_of': (C.c_int, [C.POINTER(Params), C.c_int64, C.c_int64, C.POINTER(Geometry)]),
    'jds_ctx_create': (C.c_int, [C.c_int, C.POINTER(_P)]),
    'jds_ctx_destroy': (None, [_P]),
    'jds_ctx_stream': (_P, [_P]),
    'jds_ctx_set_ssim_scratch': (C.c_int, [_P, C.c_int64]),
    'jds_plan_create': (C.c_int, [_P, C.POINTER(Params), C.c_int, C.c_int64, C.c_int64, C.POINTER(_P)]),
    'jds_plan_create_q': (C.c_int, [_P, C.POINTER(Params), C.c_int, C.c_int, C.c_int64, C.c_int64, C.POINTER(_P)]),
    'jds_plan_run': (C.c_int, [_P, _P, _P, _P, _P, C.c_uint32, _P]),
    'jds_plan_geometry': (C.c_int, [_P, C.POINTER(Geometry)]),
    'jds_plan_fix_counts': (C.c_int, [_P, _P]),
    'jds_plan_destroy': (None, [_P]),
    'jds_plan_profile': (C.c_int, [_P, C.c_int]),
    'jds_plan_profile_read': (C.c_int, [_P, C.POINTER(KernelTime), C.c_int, C.POINTER(C.c_int),
                                        C.POINTER(C.c_double)]),
    'jds_compress_reconstruct': (C.c_int, [_P, C.POINTER(Params), _P, C.c_int64, C.c_int64, _P, _P,
                                           C.POINTER(FrameStats), _P, _P, C.c_int32, C.c_int32,
                                           C.POINTER(SelectedBlock), C.POINTER(C.c_int32)]),
    'jds_psnr_ssim': (C.c_int, [_P, _P, _P, C.c_int64, C.c_int64, _P]),
    'jds_psnr_ssim_dev': (C.c_int, [_P, _P, _P, C.c_int64, C.c_int64, _P]),
    'jds_psnr_ssim_dev_after': (C.c_int, [_P, _P, _P, C.c_int64, C.c_int64, _P, _P]),
    'jds_magnitude_bits_f32_dev': (C.c_int, [_P, _P, C.c_int64, _P, _P]),
    'jds_magnitude_bits_f32_batch_dev': (C.c_int, [_P, _P, C.c_int32, C.c_int64, C.c_int64, _P, _P]),
    'jds_psnr_ssim_batch_dev': (C.c_int, [_P, C.c_int32, _P, _P, C.c_int64, C.c_int64, _P, _P]),
    'jds_stage_rgb_to_ycbcr': (C.c_int, [_P, _P, _P, C.c_int64]),
    'jds_stage_ycbcr_to_rgb': (C.c_int, [_P, _P, _P, C.c_int64]),
    'jds_stage_subsample': (C.c_int, [_P, _P, _P, C.c_int64, C.c_int64, C.c_int32, C.c_int32, _P, _P, _P]),
    'jds_stage_upsample': (C.c_int, [_P, _P, C.c_int64, C.c_int64, C.c_int64, C.c_int64, C.c_int32, _P]),
    'jds_stage_block_dct': (C.c_int, [_P, _P, _P, C.c_int64, C.c_int32]),
    'jds_stage_quantize': (C.c_int, [_P, _P, _P, _P, C.c_int64, C.c_int32]),
    'jds_stage_block_dct_n': (C.c_int, [_P, _P, _P, C.c_int64, C.c_int32, C.c_int32]),
    'jds_stage_quantize_n': (C.c_int, [_P, _P, _P, C.c_int32, _P, C.c_int64, C.c_int32]),
    'jds_plan_entropy_capacity': (C.c_int, [_P, C.POINTER(C.c_int64)]),
    'jds_plan_entropy': (C.c_int, [_P, _P, _P, C.c_int64, _P, _P, _P]),
    'jds_encode_jfif': (C.c_int, [_P, C.POINTER(Params), C.c_int64, C.c_int64, _P, _P, C.c_int64,
                                  C.POINTER(C.c_int64), _P]),
    'jds_selftest_dct8x8': (C.c_int, [_P, _P, C.c_int64, C.c_int32]),
    'jds_selftest_dct16x16': (C.c_int, [_P, _P, C.c_int64, C.c_int32]),
    'jds_selftest_area_tab': (C.c_int, [C.c_int32, C.c_int32, _P, _P, _P]),
    'jds_selftest_inv_fast': (C.c_int, [C.c_int32, _P, _P, C.c_int64, C.c_int64, C.c_int32, _P, _P]),
    'jds_selftest_inv_fast16': (C.c_int, [C.c_int32, _P, _P, C.c_int64, C.c_int64, C.c_int32, _P, _P]),
    'jds_selftest_fwd32': (C.c_int, [C.c_int32, C.c_int32, _P, _P, C.c_int64, C.c_int64, C.c_int32, C.c_int32, _P,
                                     _P]),
    'jds_selftest_fwd16': (C.c_int, [C.c_int32, C.c_int32, _P, _P, C.c_int64, C.c_int64, C.c_int32, C.c_int32, _P,
                                     _P]),
}
_OPTIONAL_SIGS: dict = {}

_lib = None
_lock = threading.Lock()


def _preload_torch_hip():
    spec = importlib.util.find_spec('torch')
    if spec is None or not spec.submodule_search_locations:
        return None
    cand = os.path.join(list(spec.submodule_search_locations)[0], 'lib', 'libamdhip64.so')
    if os.path.exists(cand):
        return C.CDLL(cand, mode=C.RTLD_GLOBAL)
    return None


def lib():
    """Load libjds.so (raises if it has not been built — there is no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(f'{LIB_PATH} is missing: build it with `python -c "import __graft_entry__ as g; '
                              f'g.build()"` (hipcc --offload-arch=gfx950)')
        _preload_torch_hip()
        h = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        for name, (res, args) in _SIGS.items():
            f = getattr(h, name)
            f.restype, f.argtypes = res, args
        for name, (res, args) in _OPTIONAL_SIGS.items():
            f = getattr(h, name, None)
            if f is not None:
                f.restype, f.argtypes = res, args
        if h.jds_abi_version() != ABI_VERSION:
            raise ImportError('libjds.so ABI version mismatch')
        _lib = h
        return h


def check(rc: int):
    if rc == JDS_OK:
        return
    msg = lib().jds_last_error().decode(errors='replace')
    if rc in (JDS_EINVAL, JDS_ENOTSUP):
        raise ValueError(msg)
    raise JDSError(f'libjds error {rc}: {msg}')


def ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def device_count() -> int:
    n = C.c_int(0)
    rc = lib().jds_device_count(C.byref(n))
    return n.value if rc == JDS_OK else 0


class Context:
    """A jds_ctx: one HIP stream + device scratch, bound to one device."""

    def __init__(self, device: int = 0):
        h = C.c_void_p()
        check(lib().jds_ctx_create(device, C.byref(h)))
        self.handle = h
        self.device = device

    def set_ssim_scratch(self, nbytes: int = 0):
        """SSIM luma scratch budget per launch group (jds_ctx_set_ssim_scratch; 0 = default)."""
        check(lib().jds_ctx_set_ssim_scratch(self.handle, int(nbytes)))

    def close(self):
        if self.handle:
            lib().jds_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_tls = threading.local()


def context(device: int = 0) -> Context:
    """Per-thread, per-device context for long-lived owners (plans, benches):
    the ABI is re-entrant per ctx."""
    ctxs = getattr(_tls, 'ctxs', None)
    if ctxs is None:
        ctxs = _tls.ctxs = {}
    c = ctxs.get(device)
    if c is None:
        c = ctxs[device] = Context(device)
    return c


# Contexts for single calls (engines.compress_reconstruct and the per-stage
# API).  The reference's callers run the pipeline from short-lived worker
# threads -- one QThread per run (gui/worker.py:10-36), concurrently from
# dialogs (gui/dialogs/aliasing_demo_dialog.py:158, report_exporter.py:107) --
# so a context per thread would create a HIP stream and grow device scratch on
# every run.  A call leases an idle context of its device for its duration
# instead: concurrent calls get distinct contexts (streams, scratch), and the
# next thread reuses the warm one.
_POOL_MAX = 8
_pool: dict = {}
_pool_lock = threading.Lock()


class lease:
    """`with lease(device) as ctx:` -- exclusive use of a pooled Context."""

    def __init__(self, device: int = 0):
        self.device = device
        self.ctx = None

    def __enter__(self) -> Context:
        with _pool_lock:
            free = _pool.setdefault(self.device, [])
            self.ctx = free.pop() if free else None
        if self.ctx is None:
            self.ctx = Context(self.device)
        return self.ctx

    def __exit__(self, *exc):
        c, self.ctx = self.ctx, None
        with _pool_lock:
            free = _pool.setdefault(self.device, [])
            if len(free) < _POOL_MAX:
                free.append(c)
                c = None
        if c is not None:
            c.close()
        return False


def pool_size(device: int = 0) -> int:
    with _pool_lock:
        return len(_pool.get(device, []))


def make_params(quality: int, qtable: np.ndarray, mode: str, prefilter: bool, gauss: np.ndarray,
                block_size: int = 8) -> Params:
    p = Params()
    p.block_size = int(block_size)
    p.quality = int(quality)
    p.subsampling = MODE_CODES[mode]
    p.prefilter = 1 if prefilter else 0
    qt = np.ascontiguousarray(qtable, dtype=np.float64).reshape(-1)
    if qt.size != 64:
        raise ValueError(f'operands could not be broadcast together with shapes '
                         f'({block_size},{block_size}) (8,8) ')
    C.memmove(p.qtable, qt.ctypes.data, 64 * 8)
    g = np.ascontiguousarray(gauss, dtype=np.float64)
    C.memmove(p.gauss, g.ctypes.data, 3 * 8)
    return p


def geometry(p: Params, H: int, W: int) -> Geometry:
    g = Geometry()
    check(lib().jds_geometry_of(C.byref(p), H, W, C.byref(g)))
    return g


class Plan:
    """A jds_plan: fixed geometry + per-frame tables for the device-resident batch path."""

    def __init__(self, ctx: Context, params, H: int, W: int, nq: int = 1):
        """params: one per item; nq > 1 makes a quality-sweep plan (jds_plan_create_q):
        len(params) // nq frames, item = frame * nq + q, shared front end."""
        if nq < 1 or len(params) % nq:
            raise ValueError(f'{len(params)} tables do not split into frames of {nq}')
        arr = (Params * len(params))(*params)
        h = C.c_void_p()
        check(lib().jds_plan_create_q(ctx.handle, arr, len(params) // nq, nq, H, W, C.byref(h)))
        self.handle, self.ctx, self.n, self.H, self.W = h, ctx, len(params), H, W
        self.nq, self.frames = nq, len(params) // nq
        self.geometry = Geometry()
        check(lib().jds_plan_geometry(h, C.byref(self.geometry)))

    def run(self, rgb_dev: int, out_dev: int, coeffs_dev: int, stats_dev: int, flags: int = 0,
            stream: int | None = None):
        """stream: a hipStream_t handle (0 = the null stream); None = the context's stream."""
        if stream is None:
            stream = lib().jds_ctx_stream(self.ctx.handle)
        check(lib().jds_plan_run(self.handle, rgb_dev, out_dev, coeffs_dev, stats_dev, flags, stream))

    def fix_counts(self):
        """[forward blocks, inverse tiles] sent to the exact fp64 fix-up by the last run."""
        c = np.zeros(2, np.uint32)
        check(lib().jds_plan_fix_counts(self.handle, c.ctypes.data))
        return c

    def profile(self, enable: bool = True):
        """Launch marks on every following run of this plan (jds_plan_profile)."""
        check(lib().jds_plan_profile(self.handle, 1 if enable else 0))

    def profile_read(self):
        """(per-kernel {name: (total_ms, launches)} in first-seen order, span_ms) of the
        runs since the last read; the intervals sum to span_ms."""
        arr = (KernelTime * 64)()
        n, span = C.c_int(0), C.c_double(0.0)
        check(lib().jds_plan_profile_read(self.handle, arr, 64, C.byref(n), C.byref(span)))
        return {arr[i].name.decode(): (arr[i].total_ms, int(arr[i].launches)) for i in range(n.value)}, span.value

    def close(self):
        if self.handle:
            lib().jds_plan_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
