"""Test-side BC6H block decoder, written from the BC6H format description
(the Direct3D 11 BC6H specification: mode table, per-mode header bit layouts,
endpoint sign extension and inverse transform, unquantisation, 3/4-bit
interpolation weights, final 31/64 (unsigned) or 31/32 (signed) scaling), not
from this project's encoder (gfx_imagecompress_amd/csrc/gic_bc6h.hip) or its
CPU restatement (oracle/orc_bc6h.c).  It shares no code or table with either:
the tests use it as an independent reader of their blocks
(tests/test_bc6h_decode.py).

decode_block(block16, signed) -> dict with the mode (1-14), partition,
quantised endpoints after the inverse transform, per-texel indices, and the 16
texels as 16-bit half patterns (uint16, 3 channels).
"""
from __future__ import annotations

import numpy as np

# mode number: (mode bits value, mode bit count, endpoint bits, delta bits (r, g, b), transformed, regions)
MODES = {
    1: (0x00, 2, 10, (5, 5, 5), True, 2),
    2: (0x01, 2, 7, (6, 6, 6), True, 2),
    3: (0x02, 5, 11, (5, 4, 4), True, 2),
    4: (0x06, 5, 11, (4, 5, 4), True, 2),
    5: (0x0A, 5, 11, (4, 4, 5), True, 2),
    6: (0x0E, 5, 9, (5, 5, 5), True, 2),
    7: (0x12, 5, 8, (6, 5, 5), True, 2),
    8: (0x16, 5, 8, (5, 6, 5), True, 2),
    9: (0x1A, 5, 8, (5, 5, 6), True, 2),
    10: (0x1E, 5, 6, (6, 6, 6), False, 2),
    11: (0x03, 5, 10, (10, 10, 10), False, 1),
    12: (0x07, 5, 11, (9, 9, 9), True, 1),
    13: (0x0B, 5, 12, (8, 8, 8), True, 1),
    14: (0x0F, 5, 16, (4, 4, 4), True, 1),
}

# Header layouts after the mode bits, in storage order (block bit ascending).
# "r0 9 0" = field r0, bits 9 down to 0 stored lowest first; "r0 10 15" (modes
# 13 and 14) = the reversed form, bit 15 stored first.  Endpoint names: r0/g0/b0
# and r1.. are region 0's two endpoints, r2.. and r3.. region 1's.
_LAYOUT_TEXT = {
    1: "g2 4 4, b2 4 4, b3 4 4, r0 9 0, g0 9 0, b0 9 0, r1 4 0, g3 4 4, g2 3 0, g1 4 0, b3 0 0, g3 3 0, "
       "b1 4 0, b3 1 1, b2 3 0, r2 4 0, b3 2 2, r3 4 0, b3 3 3",
    2: "g2 5 5, g3 4 4, g3 5 5, r0 6 0, b3 0 0, b3 1 1, b2 4 4, g0 6 0, b2 5 5, b3 2 2, g2 4 4, b0 6 0, "
       "b3 3 3, b3 5 5, b3 4 4, r1 5 0, g2 3 0, g1 5 0, g3 3 0, b1 5 0, b2 3 0, r2 5 0, r3 5 0",
    3: "r0 9 0, g0 9 0, b0 9 0, r1 4 0, r0 10 10, g2 3 0, g1 3 0, g0 10 10, b3 0 0, g3 3 0, b1 3 0, "
       "b0 10 10, b3 1 1, b2 3 0, r2 4 0, b3 2 2, r3 4 0, b3 3 3",
    4: "r0 9 0, g0 9 0, b0 9 0, r1 3 0, r0 10 10, g3 4 4, g2 3 0, g1 4 0, g0 10 10, g3 3 0, b1 3 0, "
       "b0 10 10, b3 1 1, b2 3 0, r2 3 0, b3 0 0, b3 2 2, r3 3 0, g2 4 4, b3 3 3",
    5: "r0 9 0, g0 9 0, b0 9 0, r1 3 0, r0 10 10, b2 4 4, g2 3 0, g1 3 0, g0 10 10, b3 0 0, g3 3 0, "
       "b1 4 0, b0 10 10, b2 3 0, r2 3 0, b3 1 1, b3 2 2, r3 3 0, b3 4 4, b3 3 3",
    6: "r0 8 0, b2 4 4, g0 8 0, g2 4 4, b0 8 0, b3 4 4, r1 4 0, g3 4 4, g2 3 0, g1 4 0, b3 0 0, g3 3 0, "
       "b1 4 0, b3 1 1, b2 3 0, r2 4 0, b3 2 2, r3 4 0, b3 3 3",
    7: "r0 7 0, g3 4 4, b2 4 4, g0 7 0, b3 2 2, g2 4 4, b0 7 0, b3 3 3, b3 4 4, r1 5 0, g2 3 0, g1 4 0, "
       "b3 0 0, g3 3 0, b1 4 0, b3 1 1, b2 3 0, r2 5 0, r3 5 0",
    8: "r0 7 0, b3 0 0, b2 4 4, g0 7 0, g2 5 5, g2 4 4, b0 7 0, g3 5 5, b3 4 4, r1 4 0, g3 4 4, g2 3 0, "
       "g1 5 0, g3 3 0, b1 4 0, b3 1 1, b2 3 0, r2 4 0, b3 2 2, r3 4 0, b3 3 3",
    9: "r0 7 0, b3 1 1, b2 4 4, g0 7 0, b2 5 5, g2 4 4, b0 7 0, b3 5 5, b3 4 4, r1 4 0, g3 4 4, g2 3 0, "
       "g1 4 0, b3 0 0, g3 3 0, b1 5 0, b2 3 0, r2 4 0, b3 2 2, r3 4 0, b3 3 3",
    10: "r0 5 0, g3 4 4, b3 0 0, b3 1 1, b2 4 4, g0 5 0, g2 5 5, b2 5 5, b3 2 2, g2 4 4, b0 5 0, g3 5 5, "
        "b3 3 3, b3 5 5, b3 4 4, r1 5 0, g2 3 0, g1 5 0, g3 3 0, b1 5 0, b2 3 0, r2 5 0, r3 5 0",
    11: "r0 9 0, g0 9 0, b0 9 0, r1 9 0, g1 9 0, b1 9 0",
    12: "r0 9 0, g0 9 0, b0 9 0, r1 8 0, r0 10 10, g1 8 0, g0 10 10, b1 8 0, b0 10 10",
    13: "r0 9 0, g0 9 0, b0 9 0, r1 7 0, r0 10 11, g1 7 0, g0 10 11, b1 7 0, b0 10 11",
    14: "r0 9 0, g0 9 0, b0 9 0, r1 3 0, r0 10 15, g1 3 0, g0 10 15, b1 3 0, b0 10 15",
}


def _parse_layout(text):
    out = []
    for item in text.split(","):
        name, a, b = item.split()
        a, b = int(a), int(b)
        bits = list(range(b, a + 1)) if a >= b else list(range(b, a - 1, -1))
        out.append((name, bits))
    return out


LAYOUTS = {m: _parse_layout(t) for m, t in _LAYOUT_TEXT.items()}

# two-region partitions 0-31: bit t = region of texel t (t = 4 * row + column)
PARTITIONS = [
    0xCCCC, 0x8888, 0xEEEE, 0xECC8, 0xC880, 0xFEEC, 0xFEC8, 0xEC80,
    0xC800, 0xFFEC, 0xFE80, 0xE800, 0xFFE8, 0xFF00, 0xFFF0, 0xF000,
    0xF710, 0x008E, 0x7100, 0x08CE, 0x008C, 0x7310, 0x3100, 0x8CCE,
    0x088C, 0x3110, 0x6666, 0x366C, 0x17E8, 0x0FF0, 0x718E, 0x399C,
]
# the region-1 anchor texel of each partition (its index is stored with one bit less)
ANCHORS = [15] * 16 + [15, 2, 8, 2, 2, 8, 8, 15, 2, 8, 2, 2, 8, 8, 2, 2]

W3 = [0, 9, 18, 27, 37, 46, 55, 64]
W4 = [0, 4, 9, 13, 17, 21, 26, 30, 34, 38, 43, 47, 51, 55, 60, 64]


class _Bits:
    def __init__(self, block):
        self.v = int.from_bytes(bytes(bytearray(block)), "little")
        self.pos = 0

    def take(self, n):
        r = (self.v >> self.pos) & ((1 << n) - 1)
        self.pos += n
        return r


def _sext(x, bits):
    return x - (1 << bits) if x & (1 << (bits - 1)) else x


def _unquantize(x, bits, signed):
    if not signed:
        if bits >= 15:
            return x
        if x == 0:
            return 0
        if x == (1 << bits) - 1:
            return 0xFFFF
        return ((x << 16) + 0x8000) >> bits
    if bits >= 16:
        return x
    neg = x < 0
    x = -x if neg else x
    if x == 0:
        u = 0
    elif x >= (1 << (bits - 1)) - 1:
        u = 0x7FFF
    else:
        u = ((x << 15) + 0x4000) >> (bits - 1)
    return -u if neg else u


def _finish(v, signed):
    """the interpolated value as a 16-bit half pattern"""
    if not signed:
        return (v * 31) >> 6
    h = -(((-v) * 31) >> 5) if v < 0 else (v * 31) >> 5
    return (0x8000 | (-h)) if h < 0 else h


def mode_of(block):
    b0 = int(block[0])
    if (b0 & 3) < 2:
        return 1 + (b0 & 3)
    m5 = b0 & 0x1F
    for k, v in MODES.items():
        if v[1] == 5 and v[0] == m5:
            return k
    return 0   # reserved mode: the block decodes to zero


def decode_block(block, signed=False):
    block = np.asarray(block, dtype=np.uint8)
    mode = mode_of(block)
    if mode == 0:
        return {"mode": 0, "texels": np.zeros((16, 3), np.uint16)}
    mval, mbits, epb, dbits, transformed, regions = MODES[mode]
    rd = _Bits(block)
    rd.take(mbits)
    f = {}
    for name, bits in LAYOUTS[mode]:
        for bit in bits:
            f[name] = f.get(name, 0) | (rd.take(1) << bit)
    partition = rd.take(5) if regions == 2 else 0
    header = 82 if regions == 2 else 65
    assert rd.pos == header, (mode, rd.pos)
    nends = 2 * regions
    ep = [[f.get(f"{c}{e}", 0) for c in "rgb"] for e in range(nends)]
    # sign extension and the inverse transform
    for c in range(3):
        if signed:
            ep[0][c] = _sext(ep[0][c], epb)
        for e in range(1, nends):
            if transformed:
                d = _sext(ep[e][c], dbits[c])
                v = (ep[0][c] + d) & ((1 << epb) - 1)
                ep[e][c] = _sext(v, epb) if signed else v
            elif signed:
                ep[e][c] = _sext(ep[e][c], epb)
    # indices
    ib = 3 if regions == 2 else 4
    pmask = PARTITIONS[partition] if regions == 2 else 0
    anchors = {0, ANCHORS[partition]} if regions == 2 else {0}
    idx = []
    for t in range(16):
        idx.append(rd.take(ib - 1 if t in anchors else ib))
    assert rd.pos == 128
    weights = W3 if ib == 3 else W4
    unq = [[_unquantize(ep[e][c], epb, signed) for c in range(3)] for e in range(nends)]
    tex = np.zeros((16, 3), np.uint16)
    for t in range(16):
        r = (pmask >> t) & 1
        a, b = unq[2 * r], unq[2 * r + 1]
        w = weights[idx[t]]
        for c in range(3):
            tex[t, c] = _finish(((64 - w) * a[c] + w * b[c] + 32) >> 6, signed)
    return {"mode": mode, "partition": partition, "regions": regions, "endpoint_bits": epb,
            "endpoints": ep, "unquantized": unq, "indices": idx, "texels": tex}


def half_to_float(h):
    return np.asarray(h, np.uint16).view(np.float16).astype(np.float32)
