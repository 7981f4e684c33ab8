"""Re-entrancy of the drop-in boundary.

The reference's callers run compress_reconstruct from Qt worker threads, and
dialogs can run concurrently with the main tab (gui/worker.py:10-36,
gui/dialogs/aliasing_demo_dialog.py:158, gui/dialogs/report_exporter.py:107).
Here two Python threads call the drop-in at the same time (ctypes releases the
GIL, so the two C-ABI calls overlap on the device) on different sizes and
modes, and every result must be bit-exact with the oracle.  Short-lived
threads must reuse pooled contexts (jds._abi.lease) rather than create a HIP
stream and scratch per run."""
import threading

import numpy as np
import pytest

from oracle import cpu_ref

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module', autouse=True)
def gpu():
    from jds import _abi
    assert _abi.device_count() >= 1, 'no HIP device: the MI355X path has no CPU fallback'


JOBS = [
    [(cpu_ref.random_image(270, 480, 41), 50, '4:2:0', True), (cpu_ref.random_image(37, 53, 42), 30, '4:2:0', False),
     (cpu_ref.random_image(128, 96, 43), 90, '4:4:4', False)],
    [(cpu_ref.random_image(200, 333, 44), 75, '4:2:2', True), (cpu_ref.random_image(64, 64, 45), 10, '4:2:0', True),
     (cpu_ref.random_image(81, 160, 46), 50, '4:2:2', False)],
]


def _run(img, q, mode, pf):
    from engines import compress_reconstruct
    from models import CompressionParams
    res, inter = compress_reconstruct(img, CompressionParams(quality=q, subsampling_mode=mode, use_prefilter=pf))
    return res.reconstructed_image, inter.all_quantized_coeffs, res.psnr_y, inter.error_map_rgb


def test_two_threads_concurrent_drop_in_bit_exact():
    refs = [[cpu_ref.compress_reconstruct(img, q, 8, mode, pf) for img, q, mode, pf in jobs] for jobs in JOBS]
    reps = 3
    results = [[None] * (len(JOBS[0]) * reps) for _ in JOBS]
    errors = []
    start = threading.Barrier(len(JOBS))

    def worker(t):
        try:
            start.wait()
            for r in range(reps):
                for j, job in enumerate(JOBS[t]):
                    results[t][r * len(JOBS[t]) + j] = _run(*job)
        except Exception as e:  # surfaced in the main thread
            errors.append(e)

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(len(JOBS))]
    for th in ths:
        th.start()
    for th in ths:
        th.join(timeout=120)
    assert not any(th.is_alive() for th in ths), 'a worker thread hung'
    assert not errors, errors
    for t, jobs in enumerate(JOBS):
        for k, (rec, cf, psnr_y, emap) in enumerate(results[t]):
            ref = refs[t][k % len(jobs)]
            assert np.array_equal(cf, ref['coeffs']), (t, k)
            assert np.array_equal(rec, ref['reconstructed']), (t, k)
            assert np.array_equal(emap, ref['error_map_rgb']), (t, k)
            assert psnr_y == ref['metrics']['psnr_y'], (t, k)


def test_short_lived_threads_reuse_pooled_contexts():
    from jds import _abi
    created = []
    orig = _abi.Context.__init__

    def counting_init(self, device=0):
        created.append(device)
        orig(self, device)

    img = cpu_ref.random_image(40, 56, 47)
    _run(img, 50, '4:2:0', True)  # the pool holds at least one warm context now
    _abi.Context.__init__ = counting_init
    try:
        for _ in range(6):  # one QThread per run, as gui/worker.py does
            th = threading.Thread(target=_run, args=(img, 50, '4:2:0', True))
            th.start()
            th.join(timeout=60)
    finally:
        _abi.Context.__init__ = orig
    assert created == [], 'each run created a new context (HIP stream + scratch)'
    assert 1 <= _abi.pool_size(0) <= _abi._POOL_MAX
