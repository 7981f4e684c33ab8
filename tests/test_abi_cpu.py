"""CPU-side checks of the C-ABI library (no GPU needed): it builds for gfx950,
loads, exports every symbol include/jds.h declares, computes the reference's
geometry, and its DCT expressions (evaluated on the host through the test-only
jds_selftest_dct8x8) are bit-identical to scipy.fft.dctn / idctn."""
import ctypes as C
import os
import re
import subprocess

import numpy as np
import pytest
import scipy.fft as sfft

from conftest import ROOT
from golden_util import golden
from oracle import cpu_ref


@pytest.fixture(scope='module')
def L():
    from jds import build, _abi
    build.build()
    return _abi.lib()


def declared_symbols():
    src = open(os.path.join(ROOT, 'include', 'jds.h')).read()
    return sorted(set(re.findall(r'^\s*(?:int|void|const char\*)\s+(jds_\w+)\s*\(', src, re.M)))


def test_library_exports_every_declared_symbol(L):
    from jds import _abi
    names = declared_symbols()
    assert len(names) >= 19
    out = subprocess.run(['nm', '-D', '--defined-only', _abi.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r'\sT\s(jds_\w+)', out))
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    for n in names:
        assert hasattr(L, n)
    assert L.jds_abi_version() == _abi.ABI_VERSION == 3


def test_every_csrc_include_is_a_build_input():
    """jds/build.py's up_to_date() must see every header a source includes, or a
    non-forced build can reuse a stale libjds.so."""
    from jds import build
    csrc = build.CSRC
    inputs = {os.path.basename(f) for f in build._inputs()}
    for f in sorted(os.listdir(csrc)):
        if not f.endswith(('.hip', '.hpp')):
            continue
        for inc in re.findall(r'^\s*#\s*include\s+"([^"]+)"', open(os.path.join(csrc, f)).read(), re.M):
            assert os.path.basename(inc) in inputs, (f, inc)
    for s in build.SOURCES:
        assert s in inputs
    hips = {f for f in os.listdir(csrc) if f.endswith('.hip')}
    assert hips == set(build.SOURCES), hips ^ set(build.SOURCES)


def test_library_has_gfx950_code_object(L):
    from jds import _abi
    out = subprocess.run(['/opt/rocm/lib/llvm/bin/llvm-readelf', '-n', _abi.LIB_PATH], capture_output=True, text=True)
    blob = open(_abi.LIB_PATH, 'rb').read()
    assert b'gfx950' in blob


@pytest.mark.parametrize('inverse', [0, 1])
def test_device_dct_expressions_bit_exact_vs_scipy(L, inverse):
    rng = np.random.default_rng(11 + inverse)
    x = np.concatenate([
        rng.random((4000, 8, 8)) * 255 - 128,
        rng.integers(0, 256, (2000, 8, 8)).astype(np.float64) - 128,
        rng.integers(-1024, 1024, (2000, 8, 8)).astype(np.float64) * rng.integers(1, 256, (1, 8, 8)),
    ])
    out = np.empty_like(x)
    assert L.jds_selftest_dct8x8(x.ctypes.data, out.ctypes.data, len(x), inverse) == 0
    f = sfft.idctn if inverse else sfft.dctn
    ref = f(x, type=2, norm='ortho', axes=(1, 2))
    assert np.array_equal(out, ref)


def test_geometry_matches_reference_coefficient_counts(L):
    from jds import _abi, codec
    for name, g in golden().items():
        h, w, _ = g['shape']
        p = _abi.make_params(g['quality'], cpu_ref.scale_quant_matrix(cpu_ref.JPEG_LUMA_Q50, g['quality']),
                             g['mode'], g['prefilter'], codec.gaussian_kernel3())
        geo = _abi.geometry(p, h, w)
        assert geo.coeffs_per_frame == g['total_coeffs'], name


def test_survey_geometry_table(L):
    from jds import _abi, codec
    q = cpu_ref.scale_quant_matrix(cpu_ref.JPEG_LUMA_Q50, 50)
    cases = [((512, 512, '4:4:4'), 786432), ((1080, 1920, '4:2:0'), 3118080), ((2160, 3840, '4:2:0'), 12441600),
             ((2160, 3840, '4:2:2'), 16588800)]
    for (h, w, mode), total in cases:
        geo = _abi.geometry(_abi.make_params(50, q, mode, True, codec.gaussian_kernel3()), h, w)
        assert geo.coeffs_per_frame == total


def test_errors_map_to_reference_exceptions(L):
    from jds import _abi, codec
    q = cpu_ref.scale_quant_matrix(cpu_ref.JPEG_LUMA_Q50, 50)
    for b in (4, 32):
        with pytest.raises(ValueError, match=rf'operands could not be broadcast together with shapes \({b},{b}\) \(8,8\)'):
            _abi.geometry(_abi.make_params(50, q, '4:2:0', False, codec.gaussian_kernel3(), block_size=b), 64, 64)
    # 16x16: the configs[4] stretch geometry (B*B coefficients per block)
    g16 = _abi.geometry(_abi.make_params(50, q, '4:2:0', False, codec.gaussian_kernel3(), block_size=16), 1080, 1920)
    assert (g16.y_blocks_y, g16.y_blocks_x, g16.c_blocks_y, g16.c_blocks_x) == (68, 120, 34, 60)
    assert g16.coeffs_per_frame == 256 * (68 * 120 + 2 * 34 * 60)
    # odd sizes with subsampling: cv2's floor-sized chroma planes (engines/color_space.py:42-49)
    g = _abi.geometry(_abi.make_params(50, q, '4:2:0', False, codec.gaussian_kernel3()), 63, 65)
    assert (g.chroma_h, g.chroma_w, g.y_blocks_y, g.y_blocks_x, g.c_blocks_y, g.c_blocks_x) == (31, 32, 8, 9, 4, 4)
    g = _abi.geometry(_abi.make_params(50, q, '4:2:2', False, codec.gaussian_kernel3()), 17, 17)
    assert (g.chroma_h, g.chroma_w, g.c_blocks_y, g.c_blocks_x) == (17, 8, 3, 1)
    # an empty chroma plane is cv2.resize's !dsize.empty() assertion in the reference
    for h, w, mode in ((1, 64, '4:2:0'), (64, 1, '4:2:2')):
        with pytest.raises(ValueError, match='dsize.empty'):
            _abi.geometry(_abi.make_params(50, q, mode, False, codec.gaussian_kernel3()), h, w)
    with pytest.raises(ValueError, match='16x16 blocks with an odd'):
        _abi.geometry(_abi.make_params(50, q, '4:2:0', False, codec.gaussian_kernel3(), block_size=16), 63, 64)
    # 4:4:4 takes any size
    assert _abi.geometry(_abi.make_params(50, q, '4:4:4', False, codec.gaussian_kernel3()), 63, 65).tiles > 0


def test_drop_in_rejects_block16_like_the_reference():
    # the reference validates block_size 16 but its quantizer raises (engines/quantizer.py:24);
    # the check happens on the host, before any device work
    from engines.pipeline import compress_reconstruct
    from models.compression_params import CompressionParams
    img = np.zeros((32, 32, 3), np.uint8)
    for b in (4, 16, 32):
        with pytest.raises(ValueError, match=rf'operands could not be broadcast together with shapes \({b},{b}\) \(8,8\)'):
            compress_reconstruct(img, CompressionParams(block_size=b))


@pytest.mark.parametrize('inverse', [0, 1])
def test_dct16_expressions_match_scipy(L, inverse):
    rng = np.random.default_rng(7 + inverse)
    x = np.concatenate([
        rng.standard_normal((1500, 16, 16)) * rng.choice([1.0, 100.0, 3000.0], (1500, 1, 1)),
        rng.integers(-1024, 1024, (1500, 16, 16)).astype(np.float64) * rng.integers(1, 256, (1, 16, 16)),
    ])
    out = np.empty_like(x)
    assert L.jds_selftest_dct16x16(x.ctypes.data, out.ctypes.data, len(x), inverse) == 0
    f = sfft.idctn if inverse else sfft.dctn
    assert np.array_equal(out, f(x, type=2, norm='ortho', axes=(1, 2)))


def test_gaussian_taps_match_oracle():
    from jds import codec
    assert np.array_equal(codec.gaussian_kernel3(0.75), cpu_ref.gaussian_kernel3(0.75))


def test_struct_layouts_match_the_c_header(tmp_path):
    """ctypes mirrors == the C compiler's view of include/jds.h (sizes and offsets)."""
    from jds import _abi
    structs = {'jds_params': _abi.Params, 'jds_frame_stats': _abi.FrameStats, 'jds_geometry': _abi.Geometry,
               'jds_selected_block': _abi.SelectedBlock, 'jds_kernel_time': _abi.KernelTime}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "jds.h"', 'int main(void) {']
    for cname, py in structs.items():
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for fname, _ in py._fields_:
            lines.append(f'printf("{cname}.{fname} %zu\\n", offsetof({cname}, {fname}));')
    lines.append('return 0; }')
    src = tmp_path / 'layout.c'
    src.write_text('\n'.join(lines))
    exe = tmp_path / 'layout'
    subprocess.run(['gcc', '-I', os.path.join(ROOT, 'include'), str(src), '-o', str(exe)], check=True)
    got = dict(l.rsplit(' ', 1) for l in subprocess.run([str(exe)], capture_output=True, text=True).stdout.split('\n') if l)
    for cname, py in structs.items():
        assert int(got[cname]) == C.sizeof(py), cname
        for fname, _ in py._fields_:
            assert int(got[f'{cname}.{fname}']) == getattr(py, fname).offset, (cname, fname)
    assert _abi.STATS_DTYPE.itemsize == C.sizeof(_abi.FrameStats)


@pytest.mark.parametrize('src', [3, 5, 7, 9, 17, 37, 53, 255, 257, 1081, 1919, 2161, 4095, 40, 1080])
def test_area_table_matches_oracle(L, src):
    """The host-built cv2 INTER_AREA table (jds_gen.hip area_tab_build, OpenCV
    computeResizeAreaTab) equals the oracle's restatement tap for tap."""
    for dst in sorted({src // 2, src}):
        n = np.zeros(dst, np.int32)
        si = np.zeros(4 * dst, np.int32)
        a = np.zeros(4 * dst, np.float64)
        assert L.jds_selftest_area_tab(src, dst, n.ctypes.data, si.ctypes.data, a.ctypes.data) == 0
        di_r, si_r, a_r = cpu_ref.area_tab(src, dst)
        k = 0
        for d in range(dst):
            for t in range(n[d]):
                assert di_r[k] == d and si_r[k] == si[4 * d + t] and a_r[k] == a[4 * d + t], (src, dst, d, t)
                k += 1
        assert k == len(di_r)
        # weights sum to 1 up to the partial cells OpenCV drops (< 1e-3 of a source sample)
        sums = np.bincount(di_r, weights=a_r, minlength=dst)
        assert np.allclose(sums, 1.0, atol=1e-3)
