"""Host-side check of the kernels' tiling invariants (no GPU): for every
geometry, each sample a workgroup reads through np.pad-'reflect' padding and
the chroma prefilter ring lies inside its LDS window, and the inverse's chroma
window covers every bilinear tap.  Mirrors csrc/jds_internal.hpp (Cfg) and
jds_abi.hip (make_geo) index arithmetic."""
import numpy as np
import pytest

from golden_util import golden

CFG = {  # mode: (SY, SX, TH, TW)
    '4:2:0': (2, 2, 32, 64), '4:2:2': (1, 2, 32, 64), '4:4:4': (1, 1, 16, 64),
}


def reflect_pad(i, n):
    if i < n:
        return i
    if n == 1:
        return 0
    p = 2 * (n - 1)
    i %= p
    return p - i if i >= n else i


def geo(H, W, mode):
    SY, SX, TH, TW = CFG[mode]
    MH, MW = 8 * SY, 8 * SX
    MY, MX = TH // MH, TW // MW
    hc, wc = H // SY, W // SX
    nby, nbx, ncy, ncx = -(-H // 8), -(-W // 8), -(-hc // 8), -(-wc // 8)
    nmy, nmx = (nby, nbx) if mode == '4:4:4' else (ncy, ncx)
    ty, tx = -(-nmy // MY), -(-nmx // MX)
    return dict(SY=SY, SX=SX, TH=TH, TW=TW, MH=MH, MW=MW, MY=MY, MX=MX, hc=hc, wc=wc, nby=nby, nbx=nbx,
                ncy=ncy, ncx=ncx, tiles_y=ty, tiles_x=tx, ty_off=ty * MY - nmy, tx_off=tx * MX - nmx)


def check_geometry(H, W, mode):
    g = geo(H, W, mode)
    WR, WC = g['TH'] + 2, g['TW'] + 2
    YBR, YBC = g['TH'] // 8, g['TW'] // 8
    CBR, CBC = g['TH'] // g['MH'], g['TW'] // g['MW']
    covered = np.zeros((g['nby'], g['nbx']), int)
    for ty in range(g['tiles_y']):
        for tx in range(g['tiles_x']):
            m0y, m0x = ty * g['MY'] - g['ty_off'], tx * g['MX'] - g['tx_off']
            y0, x0 = m0y * g['MH'], m0x * g['MW']
            for br in range(YBR):
                for bc in range(YBC):
                    gy, gx = m0y * g['SY'] + br, m0x * g['SX'] + bc
                    if not (0 <= gy < g['nby'] and 0 <= gx < g['nbx']):
                        continue
                    covered[gy, gx] += 1
                    for i in range(8):
                        sy = reflect_pad(gy * 8 + i, H) - y0 + 1
                        sx = reflect_pad(gx * 8 + i, W) - x0 + 1
                        assert 0 <= sy < WR and 0 <= sx < WC, (H, W, mode, gy, gx)
            if mode == '4:4:4':
                continue
            for br in range(CBR):
                for bc in range(CBC):
                    gy, gx = m0y + br, m0x + bc
                    if not (0 <= gy < g['ncy'] and 0 <= gx < g['ncx']):
                        continue
                    for i in range(8):
                        sr = reflect_pad(gy * 8 + i, g['hc'])
                        sc = reflect_pad(gx * 8 + i, g['wc'])
                        wr0, wc0 = g['SY'] * sr - y0 + 1, g['SX'] * sc - x0 + 1
                        # blur taps: rows wr0-1 .. wr0+SY, cols wc0 .. wc0+1
                        assert 1 <= wr0 and wr0 + g['SY'] < WR, (H, W, mode, 'rows', gy, i)
                        assert 1 <= wc0 and wc0 + 1 < WC - 1, (H, W, mode, 'cols', gx, i)
            # inverse: chroma window [8*m0y - RY, +CWR) x [8*m0x - RX, +CWC)
            RY, RX = (1 if g['SY'] == 2 else 0), 1
            cwy0, cwx0 = 8 * m0y - RY, 8 * m0x - RX
            CWR, CWC = 8 * CBR + 2 * RY, 8 * CBC + 2 * RX
            up_sy, up_sx = 1.0 / (H / g['hc']), 1.0 / (W / g['wc'])
            for y in range(max(y0, 0), min(y0 + g['TH'], H)):
                fy = np.float32((y + 0.5) * up_sy - 0.5)
                sy = int(np.floor(fy))
                for r in (min(max(sy, 0), g['hc'] - 1), min(max(sy + 1, 0), g['hc'] - 1)):
                    if g['SY'] == 2:
                        assert 0 <= r - cwy0 < CWR, (H, W, mode, y)
            for x in range(max(x0, 0), min(x0 + g['TW'], W)):
                fx = np.float32((x + 0.5) * up_sx - 0.5)
                sx = max(int(np.floor(fx)), 0)
                copy = sx + 1 >= g['wc']
                sx = min(sx, g['wc'] - 1)
                assert 0 <= sx - cwx0 < CWC and (copy or sx + 1 - cwx0 < CWC), (H, W, mode, x)
    assert (covered == 1).all()


def sizes():
    out = set()
    for v in golden().values():
        h, w, mode = v['shape'][0], v['shape'][1], v['mode']
        # odd sizes with subsampling run the untiled general-geometry kernels (jds_gen.hip)
        if (mode != '4:4:4' and w % 2) or (mode == '4:2:0' and h % 2):
            continue
        out.add((h, w, mode))
    rng = np.random.default_rng(0)
    for _ in range(60):
        mode = ('4:4:4', '4:2:2', '4:2:0')[rng.integers(3)]
        h, w = int(rng.integers(1, 200)), int(rng.integers(1, 200))
        if mode != '4:4:4':
            w += w % 2
        if mode == '4:2:0':
            h += h % 2
        out.add((h, w, mode))
    return sorted(out)


@pytest.mark.parametrize('h,w,mode', [s for s in sizes() if s[0] * s[1] <= 600 * 600])
def test_tile_windows_cover_every_tap(h, w, mode):
    check_geometry(h, w, mode)
