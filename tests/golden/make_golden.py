"""Generate golden fixtures by RUNNING THE REFERENCE in this container.

The reference (Xneonz0/JPEG-DSP-Studio at /root/reference, read-only, pure
Python) is imported as-is.  Two things it needs are absent here and are
provided by shims created at run time (none of its source is copied):

* ``cv2`` (opencv-python) is not installed anywhere: a stand-in module backed
  by ``oracle/cpu_ref.py``'s restatement of cv2.GaussianBlur / cv2.resize.
  Outputs of 4:2:2 / 4:2:0 cases therefore pin everything EXCEPT the cv2
  stages (parity unpinned there).  4:4:4 cases touch no cv2.
* ``skimage`` exists only under /opt/conda/bin/python3.9 (0.18.3).  That run
  is the primary one (real SSIM/PSNR); 0.18 spells ``channel_axis=2`` as
  ``multichannel=True``, so that keyword is translated.  Under python3.10
  (NumPy 2) skimage is replaced by the oracle's restatement and the run only
  contributes the NumPy-2 ``bpp``/``compression_ratio`` (utils/metrics.py:77-88
  promotes to float32 under NEP 50) and a cross-stack digest check.

Usage (from the repo root):
    /opt/conda/bin/python3.9 tests/golden/make_golden.py          # writes golden.json + arrays.npz
    python3 tests/golden/make_golden.py --np2                      # adds the NumPy-2 fields
"""
from __future__ import annotations

import __future__ as _future
import hashlib
import json
import os
import sys
import types

import numpy as np

REF = '/root/reference'
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.dont_write_bytecode = True
sys.path.insert(0, REPO)
from oracle import cpu_ref  # noqa: E402  (the restated cv2 stages back the stand-in)


def _install_cv2_standin():
    cv2 = types.ModuleType('cv2')
    cv2.INTER_NEAREST, cv2.INTER_LINEAR, cv2.INTER_AREA = 0, 1, 3

    def GaussianBlur(src, ksize, sigmaX, sigmaY=0):
        assert tuple(ksize) == (3, 3) and sigmaY == 0
        return cpu_ref.gaussian_blur3(np.asarray(src, np.float64), cpu_ref.gaussian_kernel3(sigmaX))

    def resize(src, dsize, interpolation=1):
        w, h = dsize
        if interpolation == 3:  # fast integer path or fractional area path, as cv::hal::resize picks
            return cpu_ref.resize_area(src, h, w)
        if interpolation == 1:
            return cpu_ref.resize_linear(src, h, w)
        raise NotImplementedError(interpolation)

    cv2.GaussianBlur, cv2.resize = GaussianBlur, resize
    cv2.imread = cv2.imwrite = cv2.cvtColor = None
    sys.modules['cv2'] = cv2


def _install_skimage():
    try:
        import skimage.metrics as skm  # real one (python3.9 / skimage 0.18.3)
        orig = skm.structural_similarity

        def ssim(im1, im2, *a, channel_axis=None, **kw):
            if channel_axis is not None:
                kw['multichannel'] = True
            return orig(im1, im2, *a, **kw)
        skm.structural_similarity = ssim
        return 'skimage-' + __import__('skimage').__version__
    except ImportError:
        sk = types.ModuleType('skimage')
        skm = types.ModuleType('skimage.metrics')

        def ssim(im1, im2, channel_axis=None, data_range=255):
            if channel_axis is None:
                return cpu_ref._ssim2d(im1, im2, data_range)
            return float(np.mean([cpu_ref._ssim2d(im1[..., c], im2[..., c], data_range)
                                  for c in range(im1.shape[-1])]))
        skm.structural_similarity = ssim
        skm.peak_signal_noise_ratio = lambda a, b, data_range=255: cpu_ref._psnr(a, b, data_range)
        sk.metrics = skm
        sys.modules['skimage'] = sk
        sys.modules['skimage.metrics'] = skm
        return 'oracle-standin'


def _import_reference():
    _install_cv2_standin()
    sk = _install_skimage()
    sys.path.insert(0, REF)
    # utils/test_images.py:165 uses a PEP 604 annotation; compile it with
    # postponed annotations so python3.9 can load it unchanged.
    path = os.path.join(REF, 'utils', 'test_images.py')
    src = open(path).read()
    mod = types.ModuleType('utils.test_images')
    mod.__file__ = path
    exec(compile(src, path, 'exec', flags=_future.annotations.compiler_flag, dont_inherit=True),
         mod.__dict__)
    sys.modules['utils.test_images'] = mod   # found by utils/__init__.py's relative import
    import utils  # noqa: F401
    from engines.pipeline import compress_reconstruct
    from models.compression_params import CompressionParams
    import utils.test_images as ti
    return compress_reconstruct, CompressionParams, ti, sk


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def cases(ti):
    """(name, image, quality, mode, prefilter, selected_block, store_full_arrays)."""
    rnd = cpu_ref.random_image
    out = [
        ('cfg1_checker512_q50_444', ti.generate_colored_checkerboard(512), 50, '4:4:4', False, (3, 5), False),
        ('rand256_s1_q10_444', rnd(256, 256, 1), 10, '4:4:4', False, (0, 0), True),
        ('checker256_q50_420_nopf', ti.generate_colored_checkerboard(256), 50, '4:2:0', False, (1, 2), True),
        ('checker256_q50_420_pf', ti.generate_colored_checkerboard(256), 50, '4:2:0', True, (1, 2), True),
        ('stripes256w2_q50_422_nopf', ti.generate_thin_stripes(256, 2), 50, '4:2:2', False, (0, 0), True),
        ('stripes256w2_q50_422_pf', ti.generate_thin_stripes(256, 2), 50, '4:2:2', True, (0, 0), True),
        ('gradient256_q50_420_pf', ti.generate_gradient(256), 50, '4:2:0', True, (10, 10), True),
        ('text256_q75_420_nopf', ti.generate_text_edges(256), 75, '4:2:0', False, (20, 3), True),
        ('chroma256_q30_422_pf', ti.generate_chroma_stripes(256), 30, '4:2:2', True, (2, 2), True),
        ('photo256_q90_444', ti.generate_photo(256), 90, '4:4:4', False, (31, 31), True),
        ('photo256_q50_420_pf', ti.generate_photo(256), 50, '4:2:0', True, (5, 7), True),
    ]
    for mode in ('4:4:4', '4:2:2', '4:2:0'):
        for pf in ((False,) if mode == '4:4:4' else (False, True)):
            for q in (1, 10, 50, 95, 100):
                out.append((f'rand64_s2_q{q}_{mode.replace(":", "")}_{"pf" if pf else "nopf"}',
                            rnd(64, 64, 2), q, mode, pf, (7, 7), True))
    for q in (5, 10, 20, 50, 80, 95):
        out.append((f'sweep128_s3_q{q}_420_pf', rnd(128, 128, 3), q, '4:2:0', True, (4, 4), True))
    # ragged / padded geometries (reflect padding reaching into the previous block)
    out += [
        ('ragged37x53_s4_q50_444', rnd(37, 53, 4), 50, '4:4:4', False, (4, 6), True),
        ('ragged52x70_s5_q75_420_pf', rnd(52, 70, 5), 75, '4:2:0', True, (6, 8), True),
        ('ragged34x66_s6_q40_420_nopf', rnd(34, 66, 6), 40, '4:2:0', False, (4, 8), True),
        ('ragged40x36_s7_q30_422_pf', rnd(40, 36, 7), 30, '4:2:2', True, (0, 4), True),
        ('ragged18x22_s8_q60_420_pf', rnd(18, 22, 8), 60, '4:2:0', True, (2, 2), True),
        ('ragged8x8_s9_q50_444', rnd(8, 8, 9), 50, '4:4:4', False, (0, 0), True),
        ('ragged16x16_s10_q50_420_pf', rnd(16, 16, 10), 50, '4:2:0', True, (1, 1), True),
        ('ragged9x17_s11_q50_444', rnd(9, 17, 11), 50, '4:4:4', False, (1, 2), True),
        ('ragged130x98_s12_q65_420_pf', rnd(130, 98, 12), 65, '4:2:0', True, (3, 3), True),
    ]
    # exact-tie edge cases: flat planes whose DC/Q lands on k + 0.5
    for v in (127, 129, 131, 133):
        img = np.full((32, 48, 3), v, np.uint8)
        out.append((f'flat{v}_q50_444', img, 50, '4:4:4', False, (0, 0), True))
        out.append((f'flat{v}_q50_420_pf', img, 50, '4:2:0', True, (0, 0), True))
    # odd sizes with chroma subsampling: cv2's fractional INTER_AREA and non-2x INTER_LINEAR
    out += [
        ('odd37x53_s14_q50_420_pf', rnd(37, 53, 14), 50, '4:2:0', True, (4, 6), True),
        ('odd37x53_s14_q50_420_nopf', rnd(37, 53, 14), 50, '4:2:0', False, (1, 1), True),
        ('odd40x37_s15_q50_422_pf', rnd(40, 37, 15), 50, '4:2:2', True, (2, 3), True),
        ('odd40x37_s15_q50_422_nopf', rnd(40, 37, 15), 50, '4:2:2', False, (0, 0), True),
        ('odd33x64_s16_q75_420_pf', rnd(33, 64, 16), 75, '4:2:0', True, (4, 7), True),
        ('odd64x33_s17_q30_420_nopf', rnd(64, 33, 17), 30, '4:2:0', False, (7, 4), True),
        ('odd64x33_s17_q30_422_pf', rnd(64, 33, 17), 30, '4:2:2', True, (3, 2), True),
        ('odd7x9_s18_q50_420_pf', rnd(7, 9, 18), 50, '4:2:0', True, (0, 1), True),
        ('odd9x7_s19_q95_422_pf', rnd(9, 7, 19), 95, '4:2:2', True, (1, 0), True),
        ('odd17x17_s20_q90_420_pf', rnd(17, 17, 20), 90, '4:2:0', True, (2, 2), True),
        ('odd17x17_s20_q5_420_nopf', rnd(17, 17, 20), 5, '4:2:0', False, (0, 0), True),
        ('odd255x257_s21_q10_420_pf', rnd(255, 257, 21), 10, '4:2:0', True, (31, 32), True),
        ('checker257_q50_420_pf', ti.generate_colored_checkerboard(257), 50, '4:2:0', True, (5, 5), True),
        ('gradient131_q60_422_pf', ti.generate_gradient(131), 60, '4:2:2', True, (3, 9), True),
        ('odd1081x1919_s13_q50_420_pf', rnd(1081, 1919, 13), 50, '4:2:0', True, (67, 119), False),
    ]
    out += [
        ('cfg2_rand1080p_s0_q50_420_pf', rnd(1080, 1920, 0), 50, '4:2:0', True, (67, 119), False),
        ('cfg3_rand4k_s0_q10_420_nopf', rnd(2160, 3840, 0), 10, '4:2:0', False, (0, 0), False),
        ('cfg5_rand4k_s0_q50_422_nopf', rnd(2160, 3840, 0), 50, '4:2:2', False, (0, 0), False),
    ]
    return out


def main():
    np2 = '--np2' in sys.argv
    only = [a for a in sys.argv[1:] if not a.startswith('--')]
    cr, Params, ti, sk = _import_reference()
    gpath = os.path.join(HERE, 'golden.json')
    golden = json.load(open(gpath)) if os.path.exists(gpath) else {'cases': {}}
    arrays = {}
    apath = os.path.join(HERE, 'arrays.npz')
    if os.path.exists(apath) and not np2:
        arrays = dict(np.load(apath, allow_pickle=False))
    for name, img, q, mode, pf, sel, full in cases(ti):
        if only and name not in only:
            continue
        res, inter = cr(img, Params(quality=q, block_size=8, subsampling_mode=mode, use_prefilter=pf), sel)
        rec, coeffs = res.reconstructed_image, inter.all_quantized_coeffs
        if np2:
            g = golden['cases'][name]
            assert g['sha_recon'] == sha(rec), name
            assert g['sha_coeffs'] == sha(coeffs), name
            g['np2_bpp'] = res.bpp
            g['np2_compression_ratio'] = res.compression_ratio
            print('np2', name, res.bpp)
            continue
        g = {
            'shape': list(img.shape), 'quality': q, 'mode': mode, 'prefilter': pf,
            'selected_block_idx': list(sel), 'full': full,
            'sha_input': sha(img), 'sha_recon': sha(rec), 'sha_coeffs': sha(coeffs),
            'sha_error_map_y': sha(inter.error_map_y), 'sha_error_map_rgb': sha(inter.error_map_rgb),
            'psnr_y': res.psnr_y, 'ssim_y': res.ssim_y, 'psnr_rgb': res.psnr_rgb, 'ssim_rgb': res.ssim_rgb,
            'np1_bpp': res.bpp, 'np1_compression_ratio': res.compression_ratio,
            'nonzero_coeffs': res.nonzero_coeffs, 'total_coeffs': res.total_coeffs,
            'hist': [int(v) for v in inter.quantized_histogram],
            'coeff_min': int(coeffs.min()), 'coeff_max': int(coeffs.max()),
            'stack': {'python': sys.version.split()[0], 'numpy': np.__version__,
                      'scipy': __import__('scipy').__version__, 'metrics': sk},
        }
        if inter.selected_block_original is not None:
            for k in ('original', 'shifted', 'dct', 'quantized', 'dequantized', 'reconstructed'):
                arrays[f'{name}/sel_{k}'] = getattr(inter, f'selected_block_{k}')
        if full:
            if not name.startswith(('rand', 'odd')):
                arrays[f'{name}/input'] = img
            arrays[f'{name}/recon'] = rec
            arrays[f'{name}/coeffs'] = coeffs
            if img.shape[0] * img.shape[1] <= 64 * 64:
                arrays[f'{name}/error_map_y'] = inter.error_map_y
                arrays[f'{name}/error_map_rgb'] = inter.error_map_rgb
        golden['cases'][name] = g
        print(name, 'psnr_y %.6f ssim_rgb %.6f nnz %d' % (res.psnr_y, res.ssim_rgb, res.nonzero_coeffs),
              flush=True)
    golden['generator'] = 'tests/golden/make_golden.py (runs /root/reference with a cv2 stand-in)'
    json.dump(golden, open(gpath, 'w'), indent=1, sort_keys=True)
    if not np2:
        np.savez_compressed(apath, **arrays)


if __name__ == '__main__':
    main()
