"""GPU parity tests for BC6H against the CPU restatement.

The HIP kernels (gfx_imagecompress_amd/csrc/gic_bc6h.hip) and oracle/orc_bc6h.c
both restate BC6HBlockEncoder::CompressBlock at the image API's quality 1.0
(src/amd_bc6h_body.cpp:1521-1652, src/amd_hdr_encode.cpp) in single precision
and the reference's operation order: blocks and encoder errors must be
bit-identical.  Parity against the reference itself is unpinned: its
Math_Float2Half (al2o3_cmath) is un-vendored and taken as IEEE binary16
round-to-nearest-even, and no reference fixture holds BC6H output.
"""
import ctypes

import numpy as np
import pytest

import gfx_imagecompress_amd as gic
import oracle_lib
from gfx_imagecompress_amd import synth

pytestmark = pytest.mark.gpu


def _gpu_blocks(blocks, signed=False):
    import torch
    t = torch.from_numpy(np.ascontiguousarray(blocks, np.float32).reshape(-1, 64)).cuda()
    n = t.shape[0]
    dst = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    err = torch.zeros(n, dtype=torch.float64, device="cuda")
    gic.encode_blocks_f32(gic.FMT_BC6H_SF if signed else gic.FMT_BC6H, t, dst, block_err=err)
    torch.cuda.synchronize()
    return dst.cpu().numpy().reshape(-1, 16), err.cpu().numpy()


def _report(a, b):
    bad = np.nonzero((a != b).any(axis=1))[0]
    return f"{len(bad)} of {len(a)} blocks differ, first {bad[:8].tolist()}"


def _check(blocks, signed=False):
    got, gerr = _gpu_blocks(blocks, signed)
    ref, rerr = oracle_lib.bc6h_blocks(blocks, signed)
    assert np.array_equal(got, ref), _report(got, ref)
    assert np.array_equal(gerr, rerr.astype(np.float64)), "encoder errors differ"
    return got


def _random_blocks(n, seed, signed=False):
    rng = np.random.default_rng(seed)
    scale = np.exp2(rng.uniform(-10, 5, size=(n, 1)))
    b = rng.random((n, 64)) * scale
    if signed:
        b = b * np.where(rng.random((n, 64)) < 0.5, -1.0, 1.0)
    return b.astype(np.float32)


def _tile_blocks(img):
    h, w, _ = img.shape
    bx, by = w // 4, h // 4
    return img[:by * 4, :bx * 4].reshape(by, 4, bx, 4, 4).transpose(0, 2, 1, 3, 4).reshape(-1, 64)


@pytest.mark.parametrize("signed", [False, True])
def test_bc6h_random_blocks(gpu, signed):
    _check(_random_blocks(768, 11 + signed, signed), signed)


@pytest.mark.parametrize("signed", [False, True])
def test_bc6h_hdr_image_blocks(gpu, signed):
    img = synth.hdr_rgba(128, 64, seed=3, signed=signed)
    got = _check(_tile_blocks(img), signed)
    # every mode the pattern search can reach shows up on the HDR ramp
    modes = got[:, 0] & 0x1f
    assert len(np.unique(modes)) >= 4


def test_bc6h_special_blocks(gpu):
    """Solid blocks, two colours, identical subsets, values past the half
    range (F16 infinity), tiny values below the 0.00001 cut, negative texels
    on the unsigned path (clamped to 0 by the conversion) and zero blocks."""
    rng = np.random.default_rng(5)
    bl = []
    for v in (0.0, 1e-6, 0.5, 1.0, 3.25, 70000.0, 1e9):
        bl.append(np.full(64, v, np.float32))
    for _ in range(16):   # two colours in a random texel split
        a, b = rng.random(4) * 4, rng.random(4) * 4
        m = rng.random(16) < 0.5
        bl.append(np.where(m[:, None], a, b).astype(np.float32).reshape(64))
    for _ in range(16):   # gradients along one axis
        t = np.linspace(0, 1, 16)[:, None]
        bl.append((rng.random(4) * 2 + t * rng.random(4) * 8).astype(np.float32).reshape(64))
    for _ in range(16):   # mixed signs and tiny values on the unsigned path
        b = (rng.random(64) - 0.3) * np.exp2(rng.uniform(-20, 2))
        bl.append(b.astype(np.float32))
    blocks = np.stack(bl)
    _check(blocks, False)
    _check(blocks, True)


def test_bc6h_float_image_ragged(gpu):
    """FLOAT32 source through gic_hip_encode_rows_src (edge clamp, 2 slices,
    3 channels) against the oracle on the same clamped blocks."""
    import torch
    w, h, s = 37, 23, 2
    img = np.stack([synth.hdr_rgba(w, h, seed=9 + i)[..., :3] for i in range(s)])
    src = torch.from_numpy(np.ascontiguousarray(img).reshape(-1)).cuda()
    bx, by = (w + 3) // 4, (h + 3) // 4
    dst = torch.zeros(bx * by * s * 16, dtype=torch.uint8, device="cuda")
    err = torch.zeros(bx * by * s, dtype=torch.float64, device="cuda")
    gic.encode_device_src(gic.FMT_BC6H, gic.SRC_FLOAT32, src, w, h, s, 3, dst, gic.Options(), block_err=err)
    torch.cuda.synchronize()
    ys = np.minimum(np.arange(by * 4), h - 1)
    xs = np.minimum(np.arange(bx * 4), w - 1)
    pad = np.ones((s, by * 4, bx * 4, 4), np.float32)
    pad[..., :3] = img[:, ys][:, :, xs]
    blocks = np.concatenate([_tile_blocks(pad[i]) for i in range(s)])
    ref, rerr = oracle_lib.bc6h_blocks(blocks)
    got = dst.cpu().numpy().reshape(-1, 16)
    assert np.array_equal(got, ref), _report(got, ref)
    assert np.array_equal(err.cpu().numpy(), rerr.astype(np.float64))


def test_bc6h_unorm8_image(gpu):
    """An 8-bit RGBA source (texels v / 255.0f, the reference's float read)."""
    img = synth.g1(64, 32)
    import torch
    src = torch.from_numpy(img.copy()).cuda()
    dst = torch.zeros(16 * 8 * 16, dtype=torch.uint8, device="cuda")
    gic.encode_device(gic.FMT_BC6H, src, 64, 32, 1, 4, dst)
    torch.cuda.synchronize()
    blocks = _tile_blocks(img.astype(np.float32) / np.float32(255.0))
    ref, _ = oracle_lib.bc6h_blocks(blocks)
    got = dst.cpu().numpy().reshape(-1, 16)
    assert np.array_equal(got, ref), _report(got, ref)


def test_bc6h_image_api(gpu):
    """Image_CompressAMDBC6H on an R32G32B32A32_SFLOAT image: the stand-in
    header marks that format signed, so the destination is DXBC6H_SFLOAT (25)
    and the signed encoder runs (amd_bc6h_compressor.cpp:19-25); bytes equal to
    the block path, a DDS with the DX10 header."""
    lib = gic.library()
    lib.Image_CreateNoClear.restype = ctypes.c_void_p
    lib.Image_CreateNoClear.argtypes = [ctypes.c_uint32] * 4 + [ctypes.c_int]
    lib.Image_RawDataPtr.argtypes = [ctypes.c_void_p]
    lib.Image_RawDataPtr.restype = ctypes.c_void_p
    lib.Image_Destroy.argtypes = [ctypes.c_void_p]
    lib.Image_CompressAMDBC6H.restype = ctypes.c_void_p
    lib.Image_CompressAMDBC6H.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    w, h = 20, 12
    img = synth.hdr_rgba(w, h, seed=4)
    p = lib.Image_CreateNoClear(w, h, 1, 1, 9)   # R32G32B32A32_SFLOAT
    ctypes.memmove(lib.Image_RawDataPtr(p), img.tobytes(), img.nbytes)
    q = lib.Image_CompressAMDBC6H(p, None, None, None)
    assert q
    import struct
    hdr = ctypes.string_at(q, 32)
    assert struct.unpack_from("<III", hdr, 8) == (20, 12, 1)
    assert struct.unpack_from("<I", hdr, 24)[0] == 25   # TinyImageFormat_DXBC6H_SFLOAT
    data = ctypes.string_at(lib.Image_RawDataPtr(q), 5 * 3 * 16)
    got = np.frombuffer(data, np.uint8).reshape(-1, 16)
    ref, _ = oracle_lib.bc6h_blocks(_tile_blocks(img), signed=True)
    assert np.array_equal(got, ref), _report(got, ref)
    lib.gic_save_dds.argtypes = [ctypes.c_void_p, ctypes.c_char_p]
    import os
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "bc6h.dds")
        assert lib.gic_save_dds(q, path.encode()) == gic.GIC_OK
        raw = open(path, "rb").read()
        assert raw[84:88] == b"DX10" and struct.unpack_from("<I", raw, 128)[0] == 96   # BC6H_SF16
        assert raw[148:] == data
    lib.Image_Destroy(q)
    lib.Image_Destroy(p)


def test_bc6h_gpu_blocks_decode_independently(gpu):
    """The kernels' own blocks read by the format-description decoder
    (tests/bc6h_decode.py; tests/test_bc6h_decode.py holds the reasoning):
    unsigned blocks decode to texels whose error is the kernels' reported
    block error within one unit per channel value."""
    import bc6h_decode as D
    from test_bc6h_decode import _half_int, _input_half_int
    blocks = np.concatenate([_tile_blocks(synth.hdr_rgba(64, 32, seed=5)), _random_blocks(128, 13)])
    got, gerr = _gpu_blocks(blocks)
    for k in range(len(got)):
        d = D.decode_block(got[k], False)
        assert 1 <= d["mode"] <= 10, (k, d["mode"])
        dec = np.abs(_input_half_int(blocks[k], False) - _half_int(d["texels"].view(np.float16))).sum()
        assert abs(dec - gerr[k]) <= 48, (k, d["mode"], dec, gerr[k])


@pytest.mark.parametrize("signed", [False, True])
def test_bc6h_device_decoder_matches_the_test_decoder(gpu, signed):
    """gic_hip_decode_bc6h (the product's decoder, its own transcription of the
    format's layouts) gives the same half texels as tests/bc6h_decode.py on the
    kernels' blocks of a ragged HDR image, every mode the encoder reaches."""
    import torch
    import bc6h_decode as D
    w, h = 70, 38
    img = synth.hdr_rgba(w, h, seed=9, signed=signed)
    src = torch.from_numpy(img.reshape(-1).copy()).cuda()
    bx, by = (w + 3) // 4, (h + 3) // 4
    fmt = gic.FMT_BC6H_SF if signed else gic.FMT_BC6H
    dst = torch.zeros(bx * by * 16, dtype=torch.uint8, device="cuda")
    gic.encode_device_src(fmt, gic.SRC_FLOAT32, src, w, h, 1, 4, dst)
    out = torch.zeros(h * w * 4, dtype=torch.int16, device="cuda")
    gic.decode_bc6h_device(fmt, dst, w, h, 1, out)
    torch.cuda.synchronize()
    blocks = dst.cpu().numpy().reshape(by, bx, 16)
    got = out.cpu().numpy().view(np.uint16).reshape(h, w, 4)
    assert (got[:, :, 3] == 0x3C00).all()
    for y in range(by):
        for x in range(bx):
            d = D.decode_block(blocks[y, x], signed)
            want = d["texels"].reshape(4, 4, 3)
            ys, xs = min(4, h - 4 * y), min(4, w - 4 * x)
            assert np.array_equal(got[4 * y:4 * y + ys, 4 * x:4 * x + xs, :3], want[:ys, :xs]), (y, x, d["mode"])


def test_bc6h_full_image_round_trip(gpu):
    """Full-size property check: a 1024^2 HDR ramp encoded and decoded on the GPU
    reproduces its input within 2 % relative L1 per block (half-float integer
    space), the bound tests/test_bc6h_decode.py pins on the restatement."""
    import torch
    n = 1024
    img = synth.hdr_rgba(n, n, seed=1)
    src = torch.from_numpy(img.reshape(-1).copy()).cuda()
    dst = torch.zeros((n // 4) ** 2 * 16, dtype=torch.uint8, device="cuda")
    gic.encode_device_src(gic.FMT_BC6H, gic.SRC_FLOAT32, src, n, n, 1, 4, dst)
    out = torch.zeros(n * n * 4, dtype=torch.int16, device="cuda")
    gic.decode_bc6h_device(gic.FMT_BC6H, dst, n, n, 1, out)
    torch.cuda.synchronize()
    dec = out.cpu().numpy().view(np.uint16).reshape(n, n, 4)[:, :, :3].astype(np.int64)
    want = np.where(img[:, :, :3] < 0.00001, 0, img[:, :, :3].astype(np.float16).view(np.uint16)).astype(np.int64)
    d = np.abs(dec - want).reshape(n // 4, 4, n // 4, 4, 3).sum(axis=(1, 3, 4))
    m = want.reshape(n // 4, 4, n // 4, 4, 3).sum(axis=(1, 3, 4))
    rel = d / np.maximum(m, 1)
    assert rel.max() <= 0.02, float(rel.max())
