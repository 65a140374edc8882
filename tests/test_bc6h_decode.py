"""BC6H blocks read back by an independent decoder (tests/bc6h_decode.py,
written from the BC6H format description, sharing no code or table with the
encoder or its CPU restatement).

The GPU kernels are bit-identical to oracle/orc_bc6h.c (tests/test_gpu_bc6h.py),
so the CPU tests here read the restatement's blocks; test_gpu_bc6h.py's
test_bc6h_gpu_blocks_decode_independently reads the kernels' own.  What this
pins, beyond the two restatements agreeing with each other:
  * header layout, endpoint transform and index packing: a block's decoded
    texels reproduce the encoder's own error (unsigned: within one half-unit
    per channel value, the encoder's palette scales endpoints by 31/64 before
    interpolating where the format interpolates first), and its decoded
    endpoints lie within 0.6 of a quantisation step (the bin centre, plus the
    quantiser bias; 1 step for the end codes) of the pattern search's float
    endpoints (orc_bc6h_pattern, either endpoint order);
  * the signed path's known reference behaviour: QuantizeToInt
    (amd_hdr_encode.cpp:83-115) divides the ORIGINAL signed value and then
    negates a negative one again, so a negative endpoint is stored as its
    magnitude -- decoded signed endpoints match |float endpoint|, and random-
    sign blocks decode to non-negative ramps.  The reference's own error for
    signed blocks is computed with unsigned unquantisation
    (decompress_endpoints2's issigned is never set) and is not a decode error,
    so signed blocks are checked by endpoints and by a relative L1 bound on
    positive data.
"""
import ctypes

import numpy as np
import pytest

import bc6h_decode as D
import oracle_lib
from gfx_imagecompress_amd import synth


def _tile(img):
    h, w, _ = img.shape
    bx, by = w // 4, h // 4
    return img[:by * 4, :bx * 4].reshape(by, 4, bx, 4, 4).transpose(0, 2, 1, 3, 4).reshape(-1, 64)


def _random_blocks(n, seed, signed=False):
    rng = np.random.default_rng(seed)
    scale = np.exp2(rng.uniform(-10, 5, size=(n, 1)))
    b = rng.random((n, 64)) * scale
    if signed:
        b = b * np.where(rng.random((n, 64)) < 0.5, -1.0, 1.0)
    return b.astype(np.float32)


def _half_int(x):
    """half patterns as the encoder's integer space: +bits, or -(magnitude bits)"""
    u = np.asarray(x, np.float16).view(np.uint16).astype(np.int64)
    return np.where(u & 0x8000, -(u & 0x7FFF), u)


def _input_half_int(block, signed):
    v = np.asarray(block, np.float32).reshape(16, 4)[:, :3]
    h = _half_int(np.abs(v).astype(np.float16))
    # texels below 0.00001 (amd_bc6h_body.cpp:1539-1573): 0 unsigned, -|half| signed
    return np.where(v < 0.00001, -h if signed else 0, h)


def _pattern_endpoints(block, signed, shape):
    fep = (ctypes.c_float * 12)()
    idx = (ctypes.c_int * 32)()
    cnt = (ctypes.c_int * 2)()
    b = np.ascontiguousarray(block, np.float32)
    oracle_lib.lib().orc_bc6h_pattern(b.ctypes.data, int(signed), int(shape), ctypes.addressof(fep),
                                      ctypes.addressof(idx), ctypes.addressof(cnt))
    return np.array(fep[:], np.float64).reshape(2, 2, 3)


def _finish(v, signed):
    if not signed:
        return (v * 31) >> 6
    return -(((-v) * 31) >> 5) if v < 0 else (v * 31) >> 5


def _endpoint_distance(d, fep, signed):
    """largest distance, in quantisation steps, of a region's decoded endpoints
    from the pattern state's (the closer endpoint order).  Codes decode to
    their bin centre (<= 0.6 step away: half a step plus the quantiser's bias
    and the unquantise/31-64 rounding), except the end codes 0 and the
    largest, which decode to the range ends (<= 1 step)."""
    bits = d["endpoint_bits"]
    step = (1 << (16 - bits)) * (31 / 32 if signed else 31 / 64)
    top = (1 << (bits - 1)) - 1 if signed else (1 << bits) - 1
    ref = np.abs(fep) if signed else fep
    worst = 0.0
    for r in range(d["regions"]):
        q = np.array([d["endpoints"][2 * r + e] for e in range(2)])
        a = np.array([[_finish(v, signed) for v in d["unquantized"][2 * r + e]] for e in range(2)], np.float64)
        allow = np.where((q == 0) | (np.abs(q) >= top), 1.0, 0.6)
        scaled = [np.max(np.abs(a - ref[r]) / (allow * step)), np.max(np.abs(a[::-1] - ref[r]) / (allow[::-1] * step))]
        worst = max(worst, min(scaled))
    return worst


def test_tables_agree_with_the_oracle_anchors():
    pos = ctypes.c_int()
    for s in range(32):
        anchor = oracle_lib.lib().orc_bc6h_anchor(s, ctypes.byref(pos))
        assert anchor == D.ANCHORS[s], s
        assert (D.PARTITIONS[s] >> D.ANCHORS[s]) & 1 == 1 and D.PARTITIONS[s] & 1 == 0, s


def test_layouts_cover_every_header_bit():
    for m, (_, mbits, epb, dbits, transformed, regions) in D.MODES.items():
        fields = {}
        for name, bits in D.LAYOUTS[m]:
            for b in bits:
                assert b not in fields.setdefault(name, set()), (m, name, b)
                fields[name].add(b)
        n = sum(len(v) for v in fields.values())
        assert mbits + n + (5 if regions == 2 else 0) == (82 if regions == 2 else 65), m
        for c, ch in enumerate("rgb"):
            assert fields[f"{ch}0"] == set(range(epb)), (m, ch)
            for e in range(1, 2 * regions):   # deltas, or (modes 10, 11) full endpoints of that width
                assert fields[f"{ch}{e}"] == set(range(dbits[c])), (m, ch, e)


def _blocks_unsigned():
    return np.concatenate([_tile(synth.hdr_rgba(64, 32, seed=3)), _random_blocks(256, 7)]).astype(np.float32)


def test_unsigned_blocks_decode_to_the_encoder_error():
    blocks = _blocks_unsigned()
    out, err = oracle_lib.bc6h_blocks(blocks, False)
    modes = set()
    for k in range(len(out)):
        d = D.decode_block(out[k], False)
        modes.add(d["mode"])
        assert 1 <= d["mode"] <= 10, (k, d["mode"])    # CompressBlock emits two-region modes only
        dec = np.abs(_input_half_int(blocks[k], False) - _half_int(d["texels"].view(np.float16))).sum()
        assert abs(dec - float(err[k])) <= 48, (k, d["mode"], dec, float(err[k]))
        assert _endpoint_distance(d, _pattern_endpoints(blocks[k], False, d["partition"]), False) <= 1.0, k
    assert len(modes) >= 3, modes


def test_unsigned_hdr_ramp_round_trip():
    blocks = _tile(synth.hdr_rgba(64, 32, seed=3)).astype(np.float32)
    out, _ = oracle_lib.bc6h_blocks(blocks, False)
    for k in range(len(out)):
        d = D.decode_block(out[k], False)
        a = _input_half_int(blocks[k], False)
        rel = np.abs(a - _half_int(d["texels"].view(np.float16))).sum() / max(1, np.abs(a).sum())
        assert rel <= 0.02, (k, d["mode"], rel)


@pytest.mark.parametrize("data", ["positive", "random_sign"])
def test_signed_blocks_decode_to_the_magnitude_endpoints(data):
    if data == "positive":
        blocks = _tile(synth.hdr_rgba(64, 32, seed=3)).astype(np.float32)
    else:
        blocks = np.concatenate([_tile(synth.hdr_rgba(64, 32, seed=3, signed=True)),
                                 _random_blocks(128, 9, signed=True)]).astype(np.float32)
    out, _ = oracle_lib.bc6h_blocks(blocks, True)
    for k in range(len(out)):
        d = D.decode_block(out[k], True)
        assert 1 <= d["mode"] <= 10, (k, d["mode"])
        assert _endpoint_distance(d, _pattern_endpoints(blocks[k], True, d["partition"]), True) <= 1.0, k
        if data == "positive":
            a = _input_half_int(blocks[k], True)
            rel = np.abs(a - _half_int(d["texels"].view(np.float16))).sum() / max(1, np.abs(a).sum())
            assert rel <= 0.06, (k, d["mode"], rel)
        else:
            # the stored endpoints are magnitudes
            assert min(min(e) for e in d["endpoints"]) >= 0, (k, d["endpoints"])
