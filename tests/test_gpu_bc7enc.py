"""bc7enc16 -- the reference's fast BC7 path (src/richgel999_bc7enc16.cpp,
ImageCompress_Compress(DXBC7, fast=true), imagecompress.cpp:34-36) -- on the
GPU against the oracle's restatement (oracle/orc_bc7enc.c), bit for bit.

Parity note: the reference pins no bc7enc16 values (its tests only run the
encoders) and cannot be built here, so the oracle is
parity-unpinned; alpha blocks additionally follow the oracle's documented
choice for the reference's uninitialised m_endpoints_share_pbit.
"""
import ctypes

import numpy as np
import pytest

import gfx_imagecompress_amd as gic
import oracle_lib
from gfx_imagecompress_amd import synth
from test_gpu_parity import _mismatch_report

pytestmark = pytest.mark.gpu

SETTINGS = [(False, True), (True, True), (False, False), (True, False)]   # (fast, perceptual)


def _gpu_image(img, fast, perceptual, first_row=0, num_rows=None):
    import torch
    a = np.ascontiguousarray(img)
    if a.ndim == 3:
        a = a[None]
    s, h, w, c = a.shape
    bx, by = gic.blocks_shape(w, h)
    rows = by - first_row if num_rows is None else num_rows
    src = torch.from_numpy(a).cuda()
    dst = torch.zeros(bx * rows * s * 16, dtype=torch.uint8, device="cuda")
    o = gic.Options.bc7enc16(fast, perceptual)
    o.force_alpha_one = c < 4
    gic.encode_device(gic.FMT_BC7ENC16, src, w, h, s, c, dst, o, first_block_row=first_row, num_block_rows=rows)
    torch.cuda.synchronize()
    return dst.cpu().numpy().reshape(-1, 16)


def _random_blocks(n, seed, alpha):
    rng = np.random.default_rng(seed)
    b = rng.integers(0, 256, (n, 16, 4), dtype=np.uint8)
    # a mix of structure: some blocks low-contrast around a base colour, some two-colour
    base = rng.integers(0, 256, (n, 1, 4), dtype=np.int32)
    low = np.clip(base + rng.integers(-6, 7, (n, 16, 4)), 0, 255).astype(np.uint8)
    two = np.where(rng.integers(0, 2, (n, 16, 1)) == 1, base, 255 - base).astype(np.uint8)
    kind = rng.integers(0, 3, n)
    b[kind == 1] = low[kind == 1]
    b[kind == 2] = two[kind == 2]
    if not alpha:
        b[:, :, 3] = 255
    return b


@pytest.mark.parametrize("fast,perceptual", SETTINGS)
@pytest.mark.parametrize("kind", ["g1", "g0"])
def test_bc7enc_image_matches_oracle(gpu, kind, fast, perceptual):
    img = synth.g1(256, 256) if kind == "g1" else synth.g0(256, 256)
    got = _gpu_image(img, fast, perceptual)
    ref = oracle_lib.encode_image_bc7enc(img, fast, perceptual)
    assert np.array_equal(got, ref), _mismatch_report(got, ref)


@pytest.mark.parametrize("n", [2048, 4200])
@pytest.mark.parametrize("fast,perceptual", SETTINGS)
@pytest.mark.parametrize("alpha", [False, True])
def test_bc7enc_block_batch_matches_oracle(gpu, alpha, fast, perceptual, n):
    """The block ABI (Image_CompressRichGel999BC7enc16) on seeded blocks: random,
    low-contrast and two-colour blocks, opaque or with alpha.  Below 4096 blocks
    a wave per block (the mode-1 partition estimates on its lanes), from 4096 a
    lane per block."""
    import torch
    blocks = _random_blocks(n, 7 + alpha, alpha)
    src = torch.from_numpy(blocks.reshape(-1, 64)).cuda()
    dst = torch.zeros(blocks.shape[0] * 16, dtype=torch.uint8, device="cuda")
    gic.encode_blocks_u8(src, dst, gic.Options.bc7enc16(fast, perceptual))
    torch.cuda.synchronize()
    got = dst.cpu().numpy().reshape(-1, 16)
    ref = oracle_lib.bc7enc_blocks(blocks, fast, perceptual)
    assert np.array_equal(got, ref), _mismatch_report(got, ref)


def test_bc7enc_solid_and_edge_blocks(gpu):
    """Solid blocks (mode-1 single colour tables), a ragged 37x23 image with 2
    slices and an RGB source (alpha forced to 255)."""
    solid = np.zeros((256, 16, 4), np.uint8)
    solid[:, :, :3] = np.arange(256, dtype=np.uint8)[:, None, None]
    solid[:, :, 3] = 255
    import torch
    src = torch.from_numpy(solid.reshape(-1, 64)).cuda()
    dst = torch.zeros(256 * 16, dtype=torch.uint8, device="cuda")
    gic.encode_blocks_u8(src, dst)
    torch.cuda.synchronize()
    got = dst.cpu().numpy().reshape(-1, 16)
    assert np.array_equal(got, oracle_lib.bc7enc_blocks(solid))
    rng = np.random.default_rng(3)
    stack = rng.integers(0, 256, (2, 23, 37, 4), dtype=np.uint8)
    got = _gpu_image(stack, False, True)
    assert np.array_equal(got, oracle_lib.encode_image_bc7enc(stack, False, True))
    rgb = synth.g1(64, 48)[..., :3].copy()
    got = _gpu_image(rgb, True, False)
    assert np.array_equal(got, oracle_lib.encode_image_bc7enc(rgb, True, False))


def test_bc7enc_8k_rows_and_decode(gpu):
    """Config-4 size: the whole 8192^2 G1 texture through the fast path, every
    32nd block row compared with the oracle, the decoded image within 1.5 dB of
    the oracle blocks' PSNR on those rows."""
    img = synth.g1(8192, 8192)
    got = _gpu_image(img, False, True).reshape(2048, 2048, 16)
    rows = list(range(0, 2048, 32))
    ref = np.concatenate([oracle_lib.encode_image_bc7enc(img[r * 4:r * 4 + 4], False, True) for r in rows])
    sub = got[rows].reshape(-1, 16)
    assert np.array_equal(sub, ref), _mismatch_report(sub, ref)
    modes = np.unique([(int(b[0]) & -int(b[0])).bit_length() - 1 for b in sub])
    assert set(modes.tolist()) <= {1, 6}


def test_bc7enc_host_api(gpu):
    """Image_CompressRichGel999BC7 (NULL options = perceptual, not fast), its
    sRGB destination, ImageCompress_Compress(DXBC7, fast=true) and the block
    entry Image_CompressRichGel999BC7enc16."""
    lib = gic.library()

    class Hdr(ctypes.Structure):
        _fields_ = [("dataSize", ctypes.c_uint64), ("width", ctypes.c_uint32), ("height", ctypes.c_uint32),
                    ("depth", ctypes.c_uint32), ("slices", ctypes.c_uint32), ("format", ctypes.c_int),
                    ("flags", ctypes.c_uint32), ("data", ctypes.c_void_p)]

    class Rich(ctypes.Structure):
        _fields_ = [("perceptual", ctypes.c_bool), ("fast", ctypes.c_bool)]
    lib.Image_CreateNoClear.restype = ctypes.c_void_p
    lib.Image_CompressRichGel999BC7.restype = ctypes.c_void_p
    lib.Image_CompressRichGel999BC7.argtypes = [ctypes.c_void_p] * 4
    lib.ImageCompress_Compress.restype = ctypes.c_void_p
    lib.ImageCompress_Compress.argtypes = [ctypes.c_int, ctypes.c_bool, ctypes.c_void_p]
    lib.Image_CompressRichGel999BC7enc16.argtypes = [ctypes.c_void_p, ctypes.c_bool, ctypes.c_bool, ctypes.c_void_p]
    lib.Image_Destroy.argtypes = [ctypes.c_void_p]

    img = synth.g1(70, 46)
    for fmt, dst_fmt in ((7, 18), (8, 19)):   # R8G8B8A8 UNORM / SRGB -> DXBC7 UNORM / SRGB
        p = lib.Image_CreateNoClear(70, 46, 1, 1, fmt)
        ctypes.memmove(Hdr.from_address(p).data, img.ctypes.data, img.nbytes)
        d = lib.Image_CompressRichGel999BC7(p, None, None, None)
        hd = Hdr.from_address(d)
        assert (hd.width, hd.height, hd.format) == (72, 48, dst_fmt)
        got = np.ctypeslib.as_array((ctypes.c_uint8 * hd.dataSize).from_address(hd.data)).reshape(-1, 16)
        assert np.array_equal(got, oracle_lib.encode_image_bc7enc(img, False, True))
        lib.Image_Destroy(d)
        opt = Rich(False, True)   # linear, fast
        d = lib.Image_CompressRichGel999BC7(p, ctypes.byref(opt), None, None)
        hd = Hdr.from_address(d)
        got = np.ctypeslib.as_array((ctypes.c_uint8 * hd.dataSize).from_address(hd.data)).reshape(-1, 16)
        assert np.array_equal(got, oracle_lib.encode_image_bc7enc(img, True, False))
        lib.Image_Destroy(d)
        lib.Image_Destroy(p)
    p = lib.Image_CreateNoClear(70, 46, 1, 1, 7)
    ctypes.memmove(Hdr.from_address(p).data, img.ctypes.data, img.nbytes)
    d = lib.ImageCompress_Compress(7, True, p)   # Image_CT_DXBC7 with fast = true -> bc7enc16 defaults
    hd = Hdr.from_address(d)
    got = np.ctypeslib.as_array((ctypes.c_uint8 * hd.dataSize).from_address(hd.data)).reshape(-1, 16)
    assert np.array_equal(got, oracle_lib.encode_image_bc7enc(img, False, True))
    lib.Image_Destroy(d)
    lib.Image_Destroy(p)
    blk = _random_blocks(4, 11, True)
    for i in range(4):
        out = (ctypes.c_uint8 * 16)()
        words = np.ascontiguousarray(blk[i]).view(np.uint32).reshape(16)
        lib.Image_CompressRichGel999BC7enc16(words.ctypes.data, i & 1, i >> 1, out)
        assert bytes(out) == oracle_lib.bc7enc_blocks(blk[i:i + 1], bool(i & 1), bool(i >> 1))[0].tobytes()
