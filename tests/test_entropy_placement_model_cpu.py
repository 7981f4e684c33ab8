"""Host model of the single-pass entropy coder's placement (csrc/jds_entropy.hip:
es_place, k_ent_place, k_ent_fix): segments of up to 64 blocks, each lane's bit string
placed at its offset, words shared by several lanes written once by the lane
holding their first bit with the others' bits gathered by the segmented OR,
a segment's first word handed to the fix-up when the previous segment holds
its first bit (or, fused as k_ent_place does by default, completed by the
previous segment from this segment's leading bits), the scan's last byte
padded with 1-bits and the 0xFF bytes counted per owning segment.  The model follows the kernel's index arithmetic
step for step; the test checks that the assembled words equal the plain
concatenated stream and that the 0xFF counts add up, over ragged block counts
and bit lengths (blocks of 4 bits -- several per word -- up to 300 bits).
The GPU kernels themselves are pinned byte for byte by test_gpu_entropy.py."""
import random

import pytest


def _place_scan(nbits_list, seed, fuse=False):
    rng = random.Random(seed)
    blocks = [[rng.randint(0, 1) for _ in range(nb)] for nb in nbits_list]
    # make 0xFF bytes common enough to exercise the counts
    for blk in blocks:
        if rng.random() < 0.3:
            for i in range(len(blk)):
                blk[i] = 1 if rng.random() < 0.9 else blk[i]
    stream = [b for blk in blocks for b in blk]
    total = len(stream)
    raw = [None] * ((total + 31) // 32 + 2)
    nseg = (len(blocks) + 63) // 64
    headw, ffs, ranges = {}, [0] * nseg, []
    pre = 0
    for g in range(nseg):
        blk = blocks[g * 64:(g + 1) * 64]
        nb = [len(b) for b in blk]
        A = sum(nb)
        W0, W1 = pre, pre + A
        ranges.append((W0, W1))
        last_seg = g == nseg - 1
        nv = len(blk)
        fz = fuse and not last_seg
        tailx, Wn = 0, 0
        if fz:  # k_ent_place: the next segment's lanes that start inside word W1 >> 5
            nbl = blocks[(g + 1) * 64:(g + 2) * 64]
            nbn = [len(b) for b in nbl] + [0] * (64 - len(nbl))
            sh1 = W1 & 31
            ex = 0
            for l in range(64):
                p = sh1 + ex
                if sh1 and nbn[l] and p < 32:
                    w0 = int(''.join(map(str, (nbl[l] + [0] * 32)[:32])), 2)
                    tailx |= w0 >> p
                ex += nbn[l]
            An = sum(nbn)
            if g + 2 == nseg and sh1 and ((W1 + An - 1) >> 5) == ((W1 - 1) >> 5):
                Wn = W1 + An
        o = [W0 + sum(nb[:l]) for l in range(nv)]

        def words(l):
            bits = blk[l] + [0] * ((-len(blk[l])) % 32)
            return [int(''.join(map(str, bits[i:i + 32])), 2) for i in range(0, len(bits), 32)]
        st = [words(l) for l in range(nv)]

        def stw(l, j):
            return st[l][j] if j < len(st[l]) else 0
        sh = [x & 31 for x in o]
        hw = [x >> 5 for x in o]
        tw = [(o[l] + nb[l] - 1) >> 5 for l in range(nv)]
        single = [hw[l] == tw[l] for l in range(nv)]
        hv = [stw(l, 0) >> sh[l] for l in range(nv)]
        c = [((o[l] + nb[l]) & 31) != 0 and (l + 1 < nv or fz) for l in range(nv)]
        X = hv + [0] * (64 - nv)
        F = [1 if (single[l] and c[l]) else 0 for l in range(nv)] + [0] * (64 - nv)
        if fz and F[63]:
            X[63] |= tailx
            F[63] = 0
        d = 1
        while d < 8:  # log-step segmented suffix OR (the kernel's shuffles; spans of 8 lanes)
            Xn = [X[l + d] if l + d < 64 else X[l] for l in range(64)]
            Fn = [F[l + d] if l + d < 64 else F[l] for l in range(64)]
            for l in range(64):
                if F[l] and l + d < 64:
                    X[l] |= Xn[l]
                    F[l] = Fn[l]
            d *= 2
        wlast = (W1 - 1) >> 5
        open_end = (not fz) and (not last_seg) and (W1 & 31)
        Wend = W1 if last_seg else Wn
        ffc = 0

        def pad(v, widx):
            used = Wend - 32 * widx
            pb = (8 - (used & 7)) & 7
            if pb:
                v |= ((1 << pb) - 1) << (32 - used - pb)
            return v, (used + 7) >> 3

        def ff(v, n):
            return sum(1 for b in range(4) if b < n and ((v >> (24 - 8 * b)) & 255) == 255)

        def put(widx, v):
            nonlocal ffc
            n4 = 4
            if Wend and widx == wlast:
                v, n4 = pad(v, widx)
            assert raw[widx] is None, ('word written twice', widx)
            raw[widx] = v
            if not (open_end and widx == wlast):
                ffc += ff(v, n4)
        for l in range(nv):
            in_tail = (tailx if (fz and l == 63) else X[l + 1]) if c[l] else 0
            own_head = sh[l] == 0
            nout = tw[l] - hw[l]
            if own_head and not single[l]:
                put(hw[l], hv[l])
            prev = stw(l, 0)
            for j in range(1, nout):
                cur = stw(l, j)
                put(hw[l] + j, ((prev << 32 | cur) >> sh[l]) & 0xFFFFFFFF)
                prev = cur
            tv = hv[l] if single[l] else ((prev << 32 | stw(l, nout)) >> sh[l]) & 0xFFFFFFFF
            if not single[l] or own_head:
                put(tw[l], tv | in_tail)
            if l == 0 and not own_head and not (fuse and g > 0):
                headw[g] = X[0]
        ffs[g] = ffc
        pre = W1
    for g in range(1, nseg if not fuse else 1):  # k_ent_fix
        W0, W1 = ranges[g]
        if W0 & 31:
            w = W0 >> 5
            v = raw[w] | headw[g]
            n4 = 4
            if g == nseg - 1 and ((W1 - 1) >> 5) == w:
                used = W1 - 32 * w
                pb = (8 - (used & 7)) & 7
                if pb:
                    v |= ((1 << pb) - 1) << (32 - used - pb)
                n4 = (used + 7) >> 3
            raw[w] = v
            ffs[g - 1] += sum(1 for b in range(4) if b < n4 and ((v >> (24 - 8 * b)) & 255) == 255)
    bits = stream + [1] * ((-total) % 8)  # T.81 F.1.2.3 padding
    ref = bytes(int(''.join(map(str, bits[i:i + 8])), 2) for i in range(0, len(bits), 8))
    got = b''.join(raw[i].to_bytes(4, 'big') for i in range((len(ref) + 3) // 4))[:len(ref)]
    return got, ref, sum(ffs)


@pytest.mark.parametrize('fuse', [False, True])
@pytest.mark.parametrize('seed', range(60))
def test_placement_model_equals_concatenation(seed, fuse):
    rng = random.Random(seed)
    nblk = rng.choice([1, 2, 63, 64, 65, 127, 128, 129, 200, 300])
    kind = rng.choice(['small', 'mixed', 'big', 'min'])
    if kind == 'min':  # every block at the 4-bit minimum: 8 lanes inside one word (the longest OR chains)
        nb = [4 if rng.random() < 0.9 else rng.randint(5, 40) for _ in range(nblk)]
    elif kind == 'small':
        nb = [rng.randint(4, 12) for _ in range(nblk)]
    elif kind == 'big':
        nb = [rng.randint(30, 300) for _ in range(nblk)]
    else:
        nb = [rng.choice([4, 5, 6, 31, 32, 33, 64, 100]) for _ in range(nblk)]
    got, ref, nff = _place_scan(nb, seed, fuse)
    assert got == ref
    assert nff == ref.count(0xFF)
