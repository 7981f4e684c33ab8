"""CPU ORACLE — test infrastructure only, never part of the product.

Baseline JPEG entropy coding of the reference's quantised coefficients
("real entropy coding ... using ZIGZAG_ORDER
(utils/constants.py:18-27, currently unused)").  The reference stops at an
estimate (utils/metrics.py:51-92, "no entropy coding"); this module defines
what the MI355X entropy coder (csrc/jds_entropy.hip) must produce, byte for
byte, and checks it:

* stream: ITU-T T.81 baseline sequential JFIF, 8-bit, Huffman, one
  quantisation table (the reference quantises all three planes with the luma
  table, engines/pipeline.py:43), the standard Huffman tables of T.81 Annex K.3
  (K.3-K.6: luma tables for Y, chroma tables for Cb/Cr), three
  NON-interleaved scans (Y, Cb, Cr).  A non-interleaved scan visits a
  component's blocks in raster order over ceil(w/8) x ceil(h/8) blocks, which
  is exactly the reference's block order and count
  (engines/block_processor.py:19-31 after pad_to_multiple), so the reference's
  all_quantized_coeffs (engines/pipeline.py:56,99) is the scan content as is;
  its reflect padding only fills blocks a decoder crops.
* coefficient scale: the reference's orthonormal dctn (dct_engine.py:7-9) with
  the -128 level shift is T.81's FDCT, and round(c/Q) its quantiser, so a
  standard decoder reconstructs the reference's image (up to its own IDCT /
  upsampling precision).
* entropy coding per T.81 F.1.2: DC difference (predictor reset to 0 at the
  start of each scan), category + magnitude bits; AC run/size symbols in
  zigzag order (ZIGZAG_ORDER), ZRL for runs > 15, EOB after the last nonzero
  coefficient unless it is coefficient 63; each scan padded with 1-bits to a
  byte boundary; 0xFF bytes followed by a stuffed 0x00.

Pinning: the Huffman tables are checked against the DHT segments libjpeg
writes (Pillow's encoder), the stream is decoded by libjpeg (Pillow) and by
decode_jfif below (coefficients round-trip exactly); see
tests/test_entropy_cpu.py.  There is no reference encoder: the bitstream
itself is "parity unpinned" against the reference, which has none.
"""
from __future__ import annotations

from typing import Dict, List, Sequence, Tuple

import numpy as np

# utils/constants.py:18-27 (row-major index of the k-th zigzag coefficient)
ZIGZAG = np.array([
    0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5,
    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6, 7, 14, 21, 28,
    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63], dtype=np.int64)

# T.81 Annex K.3, tables K.3 - K.6: (BITS[1..16], HUFFVAL)
DC_LUMA = ([0, 1, 5, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0, 0, 0], list(range(12)))
DC_CHROMA = ([0, 3, 1, 1, 1, 1, 1, 1, 1, 1, 1, 0, 0, 0, 0, 0], list(range(12)))
AC_LUMA = ([0, 2, 1, 3, 3, 2, 4, 3, 5, 5, 4, 4, 0, 0, 1, 0x7d], [
    0x01, 0x02, 0x03, 0x00, 0x04, 0x11, 0x05, 0x12, 0x21, 0x31, 0x41, 0x06, 0x13, 0x51, 0x61, 0x07,
    0x22, 0x71, 0x14, 0x32, 0x81, 0x91, 0xa1, 0x08, 0x23, 0x42, 0xb1, 0xc1, 0x15, 0x52, 0xd1, 0xf0,
    0x24, 0x33, 0x62, 0x72, 0x82, 0x09, 0x0a, 0x16, 0x17, 0x18, 0x19, 0x1a, 0x25, 0x26, 0x27, 0x28,
    0x29, 0x2a, 0x34, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48, 0x49,
    0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68, 0x69,
    0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x83, 0x84, 0x85, 0x86, 0x87, 0x88, 0x89,
    0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5, 0xa6, 0xa7,
    0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3, 0xc4, 0xc5,
    0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda, 0xe1, 0xe2,
    0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf1, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8,
    0xf9, 0xfa])
AC_CHROMA = ([0, 2, 1, 2, 4, 4, 3, 4, 7, 5, 4, 4, 0, 1, 2, 0x77], [
    0x00, 0x01, 0x02, 0x03, 0x11, 0x04, 0x05, 0x21, 0x31, 0x06, 0x12, 0x41, 0x51, 0x07, 0x61, 0x71,
    0x13, 0x22, 0x32, 0x81, 0x08, 0x14, 0x42, 0x91, 0xa1, 0xb1, 0xc1, 0x09, 0x23, 0x33, 0x52, 0xf0,
    0x15, 0x62, 0x72, 0xd1, 0x0a, 0x16, 0x24, 0x34, 0xe1, 0x25, 0xf1, 0x17, 0x18, 0x19, 0x1a, 0x26,
    0x27, 0x28, 0x29, 0x2a, 0x35, 0x36, 0x37, 0x38, 0x39, 0x3a, 0x43, 0x44, 0x45, 0x46, 0x47, 0x48,
    0x49, 0x4a, 0x53, 0x54, 0x55, 0x56, 0x57, 0x58, 0x59, 0x5a, 0x63, 0x64, 0x65, 0x66, 0x67, 0x68,
    0x69, 0x6a, 0x73, 0x74, 0x75, 0x76, 0x77, 0x78, 0x79, 0x7a, 0x82, 0x83, 0x84, 0x85, 0x86, 0x87,
    0x88, 0x89, 0x8a, 0x92, 0x93, 0x94, 0x95, 0x96, 0x97, 0x98, 0x99, 0x9a, 0xa2, 0xa3, 0xa4, 0xa5,
    0xa6, 0xa7, 0xa8, 0xa9, 0xaa, 0xb2, 0xb3, 0xb4, 0xb5, 0xb6, 0xb7, 0xb8, 0xb9, 0xba, 0xc2, 0xc3,
    0xc4, 0xc5, 0xc6, 0xc7, 0xc8, 0xc9, 0xca, 0xd2, 0xd3, 0xd4, 0xd5, 0xd6, 0xd7, 0xd8, 0xd9, 0xda,
    0xe2, 0xe3, 0xe4, 0xe5, 0xe6, 0xe7, 0xe8, 0xe9, 0xea, 0xf2, 0xf3, 0xf4, 0xf5, 0xf6, 0xf7, 0xf8,
    0xf9, 0xfa])
for _bits, _vals in (DC_LUMA, DC_CHROMA, AC_LUMA, AC_CHROMA):
    assert sum(_bits) == len(_vals)

SAMPLING = {'4:4:4': 0x11, '4:2:2': 0x21, '4:2:0': 0x22}   # Y's (H << 4 | V); Cb, Cr are 0x11


def huffman_codes(table) -> Dict[int, Tuple[int, int]]:
    """T.81 Annex C (Generate_size_table / Generate_code_table): symbol -> (code, length)."""
    bits, vals = table
    codes, code, k = {}, 0, 0
    for length in range(1, 17):
        for _ in range(bits[length - 1]):
            codes[vals[k]] = (code, length)
            code += 1
            k += 1
        code <<= 1
    return codes


def category(v: int) -> int:
    """SSSS: bit length of |v| (T.81 F.1.2.1)."""
    return int(abs(int(v))).bit_length()


class BitWriter:
    def __init__(self):
        self.out = bytearray()
        self.acc = 0
        self.n = 0
        self.bits = 0

    def put(self, code: int, length: int):
        if length == 0:
            return
        self.acc = (self.acc << length) | (code & ((1 << length) - 1))
        self.n += length
        self.bits += length
        while self.n >= 8:
            self.n -= 8
            self.out.append((self.acc >> self.n) & 0xFF)
        self.acc &= (1 << self.n) - 1

    def flush(self) -> bytes:
        """Pad with 1-bits to a byte boundary (T.81 F.1.2.3), then stuff 0x00 after every 0xFF."""
        if self.n:
            pad = 8 - self.n
            self.put((1 << pad) - 1, pad)
            self.bits -= pad
        raw = bytes(self.out)
        return raw.replace(b'\xff', b'\xff\x00')


def block_symbols(zz: np.ndarray, pred: int):
    """(code-class, symbol, magnitude, magnitude length) tuples of one zigzag block (T.81 F.1.2)."""
    out = []
    diff = int(zz[0]) - pred
    s = category(diff)
    out.append(('dc', s, diff if diff >= 0 else diff - 1, s))
    run = 0
    last = int(np.flatnonzero(zz[1:])[-1]) + 1 if np.any(zz[1:]) else 0
    for k in range(1, last + 1):
        v = int(zz[k])
        if v == 0:
            run += 1
            continue
        while run > 15:
            out.append(('ac', 0xF0, 0, 0))
            run -= 16
        s = category(v)
        out.append(('ac', (run << 4) | s, v if v >= 0 else v - 1, s))
        run = 0
    if last < 63:
        out.append(('ac', 0x00, 0, 0))
    return out


def encode_scan(blocks: np.ndarray, chroma: bool) -> Tuple[bytes, int]:
    """Entropy-coded segment of one non-interleaved scan: blocks (n, 64) int16 in
    row-major coefficient order.  Returns (stuffed bytes, entropy-coded bits
    before padding)."""
    dc = huffman_codes(DC_CHROMA if chroma else DC_LUMA)
    ac = huffman_codes(AC_CHROMA if chroma else AC_LUMA)
    w = BitWriter()
    zzb = np.asarray(blocks, dtype=np.int64).reshape(-1, 64)[:, ZIGZAG]
    pred = 0
    for b in zzb:
        for cls, sym, mag, mlen in block_symbols(b, pred):
            code, length = (dc if cls == 'dc' else ac)[sym]
            w.put(code, length)
            w.put(mag, mlen)
        pred = int(b[0])
    bits = w.bits
    return w.flush(), bits


def block_bits(blocks: np.ndarray, chroma: bool) -> np.ndarray:
    """Entropy-coded bits of every block of a scan (vectorised; the per-block
    count the GPU's first pass computes)."""
    dcl = huffman_codes(DC_CHROMA if chroma else DC_LUMA)
    acl = huffman_codes(AC_CHROMA if chroma else AC_LUMA)
    dc_len = np.array([dcl[s][1] for s in range(12)])
    ac_len = np.zeros(256, np.int64)
    for s, (_, ln) in acl.items():
        ac_len[s] = ln
    zz = np.asarray(blocks, dtype=np.int64).reshape(-1, 64)[:, ZIGZAG]
    n = zz.shape[0]
    pred = np.concatenate([[0], zz[:-1, 0]])
    diff = zz[:, 0] - pred
    cat = lambda a: np.where(a == 0, 0, np.floor(np.log2(np.maximum(np.abs(a), 1))).astype(np.int64) + 1)
    s_dc = cat(diff)
    bits = dc_len[s_dc] + s_dc
    ac = zz[:, 1:]
    nz = ac != 0
    k = np.arange(1, 64)
    # previous nonzero AC index (0 = none) for each position
    idx = np.where(nz, k[None, :], 0)
    prev = np.maximum.accumulate(np.concatenate([np.zeros((n, 1), np.int64), idx[:, :-1]], axis=1), axis=1)
    run = k[None, :] - prev - 1
    s_ac = cat(ac)
    sym = ((run & 15) << 4) | s_ac
    per = np.where(nz, (run >> 4) * ac_len[0xF0] + ac_len[sym] + s_ac, 0)
    bits = bits + per.sum(axis=1)
    bits = bits + np.where(nz[:, -1], 0, ac_len[0x00])
    return bits.astype(np.int64)


def jfif_headers(H: int, W: int, mode: str, qtable: np.ndarray) -> bytes:
    """SOI, APP0 (JFIF 1.01), DQT (table 0, zigzag order), SOF0, DHT x4."""
    q = np.asarray(qtable, dtype=np.float64).reshape(64)
    qz = q[ZIGZAG]
    if not (np.all(qz >= 1) and np.all(qz <= 255) and np.all(qz == np.floor(qz))):
        raise ValueError('baseline JPEG needs integer quantisation steps in [1, 255]')
    out = bytearray(b'\xff\xd8')
    out += b'\xff\xe0\x00\x10JFIF\x00\x01\x01\x00\x00\x01\x00\x01\x00\x00'
    out += b'\xff\xdb\x00\x43\x00' + bytes(int(v) for v in qz)
    out += b'\xff\xc0\x00\x11\x08' + int(H).to_bytes(2, 'big') + int(W).to_bytes(2, 'big') + b'\x03'
    out += bytes([1, SAMPLING[mode], 0, 2, 0x11, 0, 3, 0x11, 0])
    for tc_th, (bits, vals) in ((0x00, DC_LUMA), (0x10, AC_LUMA), (0x01, DC_CHROMA), (0x11, AC_CHROMA)):
        out += b'\xff\xc4' + (3 + 16 + len(vals)).to_bytes(2, 'big') + bytes([tc_th]) + bytes(bits) + bytes(vals)
    return bytes(out)


def sos(component: int) -> bytes:
    """SOS for one component (1 = Y with tables 0/0, 2/3 = Cb/Cr with tables 1/1), Ss=0 Se=63 Ah=Al=0."""
    return b'\xff\xda\x00\x08\x01' + bytes([component, 0x00 if component == 1 else 0x11, 0, 63, 0])


def encode_jfif(coeffs: np.ndarray, H: int, W: int, mode: str, qtable: np.ndarray,
                ny: int, nc: int) -> Tuple[bytes, List[int]]:
    """The whole file for one frame: coeffs = all_quantized_coeffs (Y blocks,
    Cb blocks, Cr blocks, 64 each); ny / nc = luma / per-plane chroma block counts.
    Returns (file bytes, [entropy-coded bits of the Y, Cb, Cr scans])."""
    c = np.asarray(coeffs).reshape(-1, 64)
    assert c.shape[0] == ny + 2 * nc
    out = bytearray(jfif_headers(H, W, mode, qtable))
    bits = []
    for comp, (lo, hi) in enumerate(((0, ny), (ny, ny + nc), (ny + nc, ny + 2 * nc)), start=1):
        seg, nb = encode_scan(c[lo:hi], chroma=comp > 1)
        out += sos(comp) + seg
        bits.append(nb)
    out += b'\xff\xd9'
    return bytes(out), bits


# --- decoder (round-trip check of the oracle itself) -----------------------

class BitReader:
    def __init__(self, data: bytes):
        self.d = data
        self.p = 0
        self.acc = 0
        self.n = 0

    def bit(self) -> int:
        if self.n == 0:
            b = self.d[self.p]
            self.p += 1
            if b == 0xFF:
                assert self.d[self.p] == 0x00, 'marker inside entropy-coded data'
                self.p += 1
            self.acc, self.n = b, 8
        self.n -= 1
        return (self.acc >> self.n) & 1

    def bits(self, k: int) -> int:
        v = 0
        for _ in range(k):
            v = (v << 1) | self.bit()
        return v


def _extend(v: int, s: int) -> int:
    return v - (1 << s) + 1 if s and v < (1 << (s - 1)) else v


def decode_scan(data: bytes, nblocks: int, chroma: bool) -> np.ndarray:
    """Inverse of encode_scan: (nblocks, 64) int16 in row-major order."""
    dec = []
    for t in (DC_CHROMA if chroma else DC_LUMA, AC_CHROMA if chroma else AC_LUMA):
        dec.append({(l, c): s for s, (c, l) in huffman_codes(t).items()})
    r = BitReader(data)

    def symbol(table):
        code, length = 0, 0
        while True:
            code = (code << 1) | r.bit()
            length += 1
            if (length, code) in table:
                return table[(length, code)]
            assert length < 16, 'bad Huffman code'

    out = np.zeros((nblocks, 64), np.int64)
    pred = 0
    for b in range(nblocks):
        zz = np.zeros(64, np.int64)
        s = symbol(dec[0])
        pred = pred + _extend(r.bits(s), s)
        zz[0] = pred
        k = 1
        while k < 64:
            rs = symbol(dec[1])
            run, s = rs >> 4, rs & 15
            if s == 0:
                if run == 15:
                    k += 16
                    continue
                break
            k += run
            zz[k] = _extend(r.bits(s), s)
            k += 1
        out[b, ZIGZAG] = zz
    return out.astype(np.int16)


def decode_jfif(data: bytes) -> Dict[str, object]:
    """Parse a file written by encode_jfif: geometry, qtable (row-major) and the coefficients."""
    assert data[:2] == b'\xff\xd8'
    p, info, scans = 2, {}, []
    while True:
        assert data[p] == 0xFF
        m = data[p + 1]
        if m == 0xD9:
            break
        ln = int.from_bytes(data[p + 2:p + 4], 'big')
        seg = data[p + 4:p + 2 + ln]
        if m == 0xDB:
            q = np.zeros(64)
            q[ZIGZAG] = np.frombuffer(seg[1:65], np.uint8)
            info['qtable'] = q.reshape(8, 8)
        elif m == 0xC0:
            info['H'] = int.from_bytes(seg[1:3], 'big')
            info['W'] = int.from_bytes(seg[3:5], 'big')
            info['sampling'] = seg[7]
        p += 2 + ln
        if m == 0xDA:
            e = p
            while not (data[e] == 0xFF and data[e + 1] != 0x00):
                e += 1
            scans.append((seg[1], data[p:e]))
            p = e
    H, W, smp = info['H'], info['W'], info['sampling']
    hmax, vmax = smp >> 4, smp & 15
    ny = ((H + 7) // 8) * ((W + 7) // 8)
    hc, wc = -(-H // vmax), -(-W // hmax)
    nc = ((hc + 7) // 8) * ((wc + 7) // 8)
    coeffs = [decode_scan(d, ny if comp == 1 else nc, comp != 1) for comp, d in scans]
    info['coeffs'] = np.concatenate([c.reshape(-1) for c in coeffs])
    return info
