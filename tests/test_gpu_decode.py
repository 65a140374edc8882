"""GPU BCn decoder (gic_hip_decode) against independent decoders.

BC7: the oracle's decoder (oracle/orc_bc7.c orc_bc7_decode, the BPTC format),
bit-exact on encoder output and on random 16-byte blocks (every mode, the
reserved mode included).  BC1-BC5: the numpy decoder below, written from the
format description with the conventions gic.h states.  Round trips: the
decoded 8K encodes of the bench textures against their sources (PSNR floor).
"""
import ctypes

import numpy as np
import pytest

import gfx_imagecompress_amd as gic
import oracle_lib
from gfx_imagecompress_amd import synth
from test_gpu_parity import gpu_encode

pytestmark = pytest.mark.gpu


def _np_colour(b8, four_only):
    w0 = b8[:, 0:4].copy().view(np.uint32)[:, 0]
    w1 = b8[:, 4:8].copy().view(np.uint32)[:, 0]
    c0, c1 = (w0 & 0xffff).astype(np.int64), (w0 >> 16).astype(np.int64)

    def rgb(c):
        r, g, b = (c >> 11) & 31, (c >> 5) & 63, c & 31
        return np.stack([(r << 3) | (r >> 2), (g << 2) | (g >> 4), (b << 3) | (b >> 2)], -1)
    e0, e1 = rgb(c0), rgb(c1)
    four = np.ones_like(c0, bool) if four_only else c0 > c1
    p2 = np.where(four[:, None], (2 * e0 + e1 + 1) // 3, (e0 + e1 + 1) // 2)
    p3 = np.where(four[:, None], (e0 + 2 * e1 + 1) // 3, 0)
    pal = np.stack([e0, e1, p2, p3], 1)                        # (n, 4, 3)
    alpha = np.full((len(c0), 4), 255, np.int64)
    alpha[:, 3] = np.where(four, 255, 0)
    idx = (w1[:, None] >> (2 * np.arange(16))) & 3
    rgbv = np.take_along_axis(pal, idx[:, :, None].astype(np.int64), 1)
    a = np.take_along_axis(alpha, idx.astype(np.int64), 1)
    return np.concatenate([rgbv, a[:, :, None]], -1)


def _np_scalar(b8):
    e0, e1 = b8[:, 0].astype(np.int64), b8[:, 1].astype(np.int64)
    bits = np.zeros(len(b8), np.uint64)
    for k in range(6):
        bits |= b8[:, 2 + k].astype(np.uint64) << np.uint64(8 * k)
    idx = ((bits[:, None] >> (np.uint64(3) * np.arange(16, dtype=np.uint64))) & np.uint64(7)).astype(np.int64)
    k = np.arange(8)
    eight = (e0 > e1)[:, None]
    pal8 = ((8 - k) * e0[:, None] + (k - 1) * e1[:, None] + 3) // 7
    pal6 = ((6 - k) * e0[:, None] + (k - 1) * e1[:, None] + 2) // 5
    pal6[:, 6], pal6[:, 7] = 0, 255
    pal = np.where(eight, pal8, pal6)
    pal[:, 0], pal[:, 1] = e0, e1
    return np.take_along_axis(pal, idx, 1)


def np_decode(fmt, blocks):
    """(n, bytes) blocks -> (n, 16, 4) RGBA."""
    b = np.ascontiguousarray(blocks, np.uint8)
    if fmt == 1:
        return _np_colour(b, False)
    if fmt == 4:
        r = _np_scalar(b)
        z = np.zeros_like(r)
        return np.stack([r, z, z, np.full_like(r, 255)], -1)
    if fmt == 5:
        r, g = _np_scalar(b[:, :8]), _np_scalar(b[:, 8:])
        return np.stack([r, g, np.zeros_like(r), np.full_like(r, 255)], -1)
    out = _np_colour(b[:, 8:], True)
    if fmt == 3:
        out[:, :, 3] = _np_scalar(b[:, :8])
    else:
        a = b[:, :8].copy().view(np.uint64)[:, 0]
        out[:, :, 3] = ((a[:, None] >> (np.uint64(4) * np.arange(16, dtype=np.uint64))) & np.uint64(15)).astype(
            np.int64) * 17
    return out


def gpu_decode(fmt, blocks, w, h, s=1):
    import torch
    bt = torch.from_numpy(np.ascontiguousarray(blocks, np.uint8).reshape(-1)).cuda()
    out = torch.full((s * h * w * 4,), 7, dtype=torch.uint8, device="cuda")
    gic.decode_device(fmt, bt, w, h, s, out)
    torch.cuda.synchronize()
    return out.cpu().numpy().reshape(s, h, w, 4)


def _to_blocks(img):
    """(S, H, W, 4) with H, W multiples of 4 -> (S*by*bx, 16, 4) row-major blocks."""
    s, h, w, _ = img.shape
    return img.reshape(s, h // 4, 4, w // 4, 4, 4).transpose(0, 1, 3, 2, 4, 5).reshape(-1, 16, 4)


@pytest.mark.parametrize("fmt", [1, 2, 3, 4, 5])
def test_decode_bcx_random_blocks(gpu, fmt):
    rng = np.random.default_rng(100 + fmt)
    bb = gic.block_bytes(fmt)
    blocks = rng.integers(0, 256, (64 * 16, bb), dtype=np.uint8)
    blocks[::7, :4] = blocks[::7, 2:6]   # some equal / ordered endpoint pairs
    got = _to_blocks(gpu_decode(fmt, blocks, 256, 64))
    assert np.array_equal(got, np_decode(fmt, blocks))


def test_decode_bc7_random_and_encoded_blocks(gpu):
    rng = np.random.default_rng(7)
    rand = rng.integers(0, 256, (1024, 16), dtype=np.uint8)
    rand[::9, 0] = 0                      # reserved mode
    enc = gpu_encode(7, synth.noise_rgba(64, 64, seed=3, alpha=True))
    for blocks in (rand, enc):
        n = len(blocks)
        got = _to_blocks(gpu_decode(7, blocks, 64, n // 16 * 4))
        ref = oracle_lib.bc7_decode(blocks).astype(np.int64)
        assert np.array_equal(got, ref)


@pytest.mark.parametrize("fmt", [1, 2, 3, 4, 5, 7])
def test_decode_ragged_edges_and_slices(gpu, fmt):
    """37x23 with 2 slices: edge blocks write only the texels inside."""
    w, h, s = 37, 23, 2
    bx, by = (w + 3) // 4, (h + 3) // 4
    rng = np.random.default_rng(fmt)
    blocks = rng.integers(0, 256, (s * bx * by, gic.block_bytes(fmt)), dtype=np.uint8)
    got = gpu_decode(fmt, blocks, w, h, s)
    full = (oracle_lib.bc7_decode(blocks).astype(np.int64) if fmt == 7 else np_decode(fmt, blocks))
    full = full.reshape(s, by, bx, 4, 4, 4).transpose(0, 1, 3, 2, 4, 5).reshape(s, by * 4, bx * 4, 4)
    assert np.array_equal(got, full[:, :h, :w])


@pytest.mark.parametrize("fmt", [1, 3, 4, 5, 7])
def test_encode_decode_round_trip_psnr(gpu, fmt):
    """Decoded encodes of the bench textures stay close to their sources."""
    n = 512 if fmt == 7 else 2048
    if fmt in (4, 5):
        src = synth.height_field(n, n, seed=1)[..., None] if fmt == 4 else synth.normal_map(synth.height_field(n, n))
        opts = gic.Options(bc4_channel=0)
    else:
        src = synth.g1(n, n)
        opts = None
    blocks = gpu_encode(fmt, src, opts)
    dec = gpu_decode(fmt, blocks, n, n)[0].astype(np.float64)
    c = src.shape[-1]
    d = dec[..., :c] - src.astype(np.float64)
    psnr = 10 * np.log10(255.0 ** 2 / max(float((d * d).mean()), 1e-9))
    floor = {1: 33.0, 3: 33.0, 4: 40.0, 5: 40.0, 7: 40.0}[fmt]
    assert psnr > floor, psnr


def test_host_decompress_image(gpu):
    """gic_decompress_image on the result of the reference host API
    Image_CompressAMDBC3: equals the device decode of the same blocks."""
    lib = gic.library()
    img = synth.noise_rgba(40, 24, seed=5, alpha=True)
    blocks = gpu_encode(3, img)
    lib.Image_CreateNoClear.restype = ctypes.c_void_p
    lib.Image_RawDataPtr.argtypes = [ctypes.c_void_p]
    lib.Image_RawDataPtr.restype = ctypes.c_void_p
    lib.Image_Destroy.argtypes = [ctypes.c_void_p]
    p = lib.Image_CreateNoClear(40, 24, 1, 1, 22)   # TinyImageFormat_DXBC3_UNORM
    ctypes.memmove(lib.Image_RawDataPtr(p), blocks.tobytes(), blocks.nbytes)
    q = lib.gic_decompress_image(p)
    assert q
    out = np.ctypeslib.as_array(ctypes.cast(lib.Image_RawDataPtr(q), ctypes.POINTER(ctypes.c_uint8)),
                                (24, 40, 4)).copy()
    lib.Image_Destroy(q)
    lib.Image_Destroy(p)
    assert np.array_equal(out, gpu_decode(3, blocks, 40, 24)[0])
