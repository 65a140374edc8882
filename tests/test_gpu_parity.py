"""GPU parity tests: the HIP kernels (through the C ABI) against the oracle.

Bar: bit-exact for BC1/BC4/BC5.  Inputs are seeded; sizes
where the oracle finishes in seconds are compared block-for-block, the 8K
configurations likewise (the oracle runs multi-threaded).
"""
import ctypes
import json
import os

import numpy as np
import pytest

import gfx_imagecompress_amd as gic
import oracle_lib
from gfx_imagecompress_amd import synth

pytestmark = pytest.mark.gpu
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def gpu_encode(fmt, img, options=None, first_row=0, num_rows=None, err=False):
    import torch
    a = np.ascontiguousarray(img, dtype=np.uint8)
    if a.ndim == 2:
        a = a[:, :, None]
    if a.ndim == 3:
        a = a[None]
    s, h, w, c = a.shape
    bx, by = gic.blocks_shape(w, h)
    rows = by - first_row if num_rows is None else num_rows
    src = torch.from_numpy(a).cuda()
    dst = torch.zeros(bx * rows * s * gic.block_bytes(fmt), dtype=torch.uint8, device="cuda")
    e = torch.zeros(bx * rows * s, dtype=torch.float64, device="cuda") if err else None
    opts = options or gic.Options()
    if fmt in (gic.FMT_BC1, gic.FMT_BC7) and c < 4:
        opts.force_alpha_one = True
    gic.encode_device(fmt, src, w, h, s, c, dst, opts, first_block_row=first_row, num_block_rows=rows,
                      block_err=e)
    torch.cuda.synchronize()
    out = dst.cpu().numpy().reshape(-1, gic.block_bytes(fmt))
    return (out, e.cpu().numpy()) if err else out


def _manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def _golden_case(name):
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(GOLDEN, "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    for n, fmt, img, kw in mg.cases():
        if n == name:
            return fmt, img, kw
    raise KeyError(name)


def _mismatch_report(a, b):
    bad = np.nonzero((a != b).any(axis=1))[0]
    return f"{len(bad)} of {len(a)} blocks differ, first {bad[:8].tolist()}"


@pytest.mark.parametrize("name", sorted(k for k in _manifest() if not k.startswith("bc7")))
def test_golden_bcx(gpu, name):
    fmt, img, kw = _golden_case(name)
    opts = gic.Options(bc4_channel=kw.get("bc4_channel", 1))
    out = gpu_encode(fmt, img, opts)
    ref = np.fromfile(os.path.join(GOLDEN, name + ".bin"), np.uint8).reshape(out.shape)
    assert np.array_equal(out, ref), _mismatch_report(out, ref)


@pytest.mark.parametrize("w,h", [(1, 1), (3, 5), (5, 3), (4, 4), (7, 9), (257, 257), (130, 66)])
def test_bc1_edges_and_npot(gpu, w, h):
    img = synth.noise_rgba(w, h, seed=w * 131 + h, alpha=True)
    out = gpu_encode(gic.FMT_BC1, img)
    ref = oracle_lib.encode_image(1, img)
    assert np.array_equal(out, ref), _mismatch_report(out, ref)


@pytest.mark.parametrize("channels", [1, 2, 3, 4])
def test_bc1_bc5_channel_layouts(gpu, channels):
    img = synth.noise_rgba(48, 40, seed=channels)[..., :channels]
    for fmt in (1, 5):
        if fmt == 5 and channels < 2:
            continue
        out = gpu_encode(fmt, img)
        ref = oracle_lib.encode_image(fmt, img)
        assert np.array_equal(out, ref), (fmt, _mismatch_report(out, ref))


def _k_colour_blocks(bx, by, kmax, seed):
    """An image whose block (x, y) has exactly k = k(x, y) distinct colours,
    k in 1..kmax: each texel takes one of the block's k random palette entries,
    every entry used at least once."""
    rng = np.random.default_rng(seed)
    img = np.zeros((by * 4, bx * 4, 4), np.uint8)
    img[..., 3] = 255
    for y in range(by):
        for x in range(bx):
            k = int(rng.integers(1, kmax + 1))
            pal = rng.integers(0, 256, size=(k, 3), dtype=np.uint8)
            sel = np.concatenate([np.arange(k), rng.integers(0, k, size=16 - k)])
            rng.shuffle(sel)
            img[y * 4:(y + 1) * 4, x * 4:(x + 1) * 4, :3] = pal[sel].reshape(4, 4, 3)
    return img


@pytest.mark.parametrize("kmax", [3, 8, 9, 12, 16])
def test_bc1_wave_unique_colour_counts(gpu, kmax):
    """The 8x8 endpoint search evaluates entries only up to the largest unique-
    colour count of the wave's blocks (64 consecutive blocks of a block row):
    waves whose blocks all have <= 8 colours skip the whole second half, waves
    mixing 1..kmax stop at the largest.  Bit-exact against the oracle either way."""
    img = _k_colour_blocks(128, 6, kmax, seed=kmax)
    out = gpu_encode(gic.FMT_BC1, img)
    ref = oracle_lib.encode_image(1, img)
    assert np.array_equal(out, ref), _mismatch_report(out, ref)


def test_bc1_solid_and_transparent_blocks(gpu):
    img = np.zeros((16, 16, 4), np.uint8)
    img[:8, :8] = (10, 200, 30, 255)        # solid colour
    img[:8, 8:] = (0, 0, 0, 0)              # fully transparent
    img[8:, :8] = (255, 255, 255, 255)      # solid white
    img[8:, 8:, :3] = 77
    img[8:, 8:, 3] = np.arange(64).reshape(8, 8) * 4  # alpha ramp across the threshold
    out = gpu_encode(gic.FMT_BC1, img)
    assert np.array_equal(out, oracle_lib.encode_image(1, img))


def test_bc1_block_api_arbitrary_floats(gpu):
    """Image_CompressAMDBC1Block / AlphaSingleModeBlock on float inputs that do
    not come from 8-bit texels (the general block-level contract)."""
    lib = gic.library()
    rng = np.random.default_rng(5)
    for k in range(64):
        blk = rng.random((16, 4), dtype=np.float32)
        if k % 4 == 0:
            blk[:, 3] = 1.0
        out = np.zeros(8, np.uint8)
        lib.Image_CompressAMDBC1Block(blk.ctypes.data_as(ctypes.c_void_p), False, False, 1,
                                      ctypes.c_float(128 / 255.0), out.ctypes.data_as(ctypes.c_void_p))
        assert out.tobytes() == oracle_lib.bc1_block(blk), k
        v = rng.random(16, dtype=np.float32)
        out4 = np.zeros(8, np.uint8)
        lib.Image_CompressAMDAlphaSingleModeBlock(v.ctypes.data_as(ctypes.c_void_p),
                                                  out4.ctypes.data_as(ctypes.c_void_p))
        assert out4.tobytes() == oracle_lib.bc4_block(v), k


def test_block_api_status(gpu):
    """The void block entry points report their outcome through
    gic_block_last_status(): 0 after a good call; adaptive colour weights (UB in
    the reference, not implemented) give GIC_EUNSUP and a zero block."""
    lib = gic.library()
    lib.gic_block_last_status.restype = ctypes.c_int
    blk = np.random.default_rng(9).random((16, 4), dtype=np.float32)
    out = np.full(8, 0xAB, np.uint8)
    lib.Image_CompressAMDBC1Block(blk.ctypes.data_as(ctypes.c_void_p), False, False, 1,
                                  ctypes.c_float(0.0), out.ctypes.data_as(ctypes.c_void_p))
    assert lib.gic_block_last_status() == gic.GIC_OK
    assert out.tobytes() == oracle_lib.bc1_block(blk, threshold=0.0)
    lib.Image_CompressAMDBC1Block(blk.ctypes.data_as(ctypes.c_void_p), True, False, 1,
                                  ctypes.c_float(0.0), out.ctypes.data_as(ctypes.c_void_p))
    assert lib.gic_block_last_status() == gic.GIC_EUNSUP
    assert not out.any()


def test_bc1_refinement_steps_option(gpu):
    img = synth.g1(64, 64)
    for steps in (0, 2, 3):
        out = gpu_encode(gic.FMT_BC1, img, gic.Options(refinement_steps=steps))
        blocks = [oracle_lib.bc1_block(_block_f32(img, bx, by), steps=steps)
                  for by in range(16) for bx in range(16)]
        assert np.array_equal(out, np.frombuffer(b"".join(blocks), np.uint8).reshape(-1, 8)), steps


@pytest.mark.parametrize("steps", [1, 2])
def test_bc1_b3d_refinement_option(gpu, steps):
    """AMD b3DRefinement (Refine3D's joint 6-D jitter, amd_bcx_body.cpp:808-932):
    BC1 image path on G1 and the BC3 colour half / float block path on noise."""
    import torch
    img = synth.g1(32, 32) if steps == 1 else synth.g1(16, 16)
    n = (img.shape[0] // 4) * (img.shape[1] // 4)
    out = gpu_encode(gic.FMT_BC1, img, gic.Options(refinement_steps=steps, b3d_refinement=True))
    side = img.shape[1] // 4
    blocks = [oracle_lib.bc1_block(_block_f32(img, bx, by), steps=steps, b3d=True)
              for by in range(img.shape[0] // 4) for bx in range(side)]
    assert np.array_equal(out, np.frombuffer(b"".join(blocks), np.uint8).reshape(-1, 8))
    assert n == len(blocks)
    rng = np.random.default_rng(40 + steps)
    fb = rng.random((32, 16, 4), dtype=np.float32)
    fb[::2] = np.round(fb[::2] * 255) / np.float32(255.0)
    t = torch.from_numpy(fb.reshape(-1, 64)).cuda()
    for fmt in (gic.FMT_BC1, gic.FMT_BC3):
        dst = torch.zeros(32 * gic.block_bytes(fmt), dtype=torch.uint8, device="cuda")
        gic.encode_blocks_f32(fmt, t, dst, gic.Options(refinement_steps=steps, b3d_refinement=True))
        torch.cuda.synchronize()
        got = dst.cpu().numpy().reshape(32, -1)
        for i, b in enumerate(fb):
            ref = oracle_lib.bc1_block(b, steps=steps, b3d=True) if fmt == gic.FMT_BC1 else \
                oracle_lib.bc23_block(fmt, b, steps=steps, b3d=True)
            assert got[i].tobytes() == ref, (fmt, i)


def _block_f32(img, bx, by):
    return img[by * 4:by * 4 + 4, bx * 4:bx * 4 + 4].reshape(16, 4).astype(np.float32) / np.float32(255.0)


def test_row_shards_and_slices_match_full(gpu):
    stack = np.stack([synth.g1(96, 80, seed=s) for s in range(3)])
    full = gpu_encode(gic.FMT_BC1, stack).reshape(3, 20, 24, 8)
    part = gpu_encode(gic.FMT_BC1, stack, first_row=7, num_rows=5).reshape(3, 5, 24, 8)
    assert np.array_equal(full[:, 7:12], part)
    ref = oracle_lib.encode_image(1, stack).reshape(3, 20, 24, 8)
    assert np.array_equal(full, ref)


def test_bc4_channel_select(gpu):
    img = synth.noise_rgba(32, 32, seed=11)
    for ch in range(4):
        out = gpu_encode(gic.FMT_BC4, img, gic.Options(bc4_channel=ch))
        assert np.array_equal(out, oracle_lib.encode_image(4, img, bc4_channel=ch)), ch


def test_host_image_api(gpu):
    """Image_CompressAMDBC1 / BC5 through the reference-compatible host API."""
    lib = gic.library()

    class Hdr(ctypes.Structure):
        _fields_ = [("dataSize", ctypes.c_uint64), ("width", ctypes.c_uint32), ("height", ctypes.c_uint32),
                    ("depth", ctypes.c_uint32), ("slices", ctypes.c_uint32), ("format", ctypes.c_int),
                    ("flags", ctypes.c_uint32), ("data", ctypes.c_void_p)]
    lib.Image_CreateNoClear.restype = ctypes.c_void_p
    lib.Image_CompressAMDBC1.restype = ctypes.c_void_p
    lib.Image_CompressAMDBC1.argtypes = [ctypes.c_void_p] * 5
    lib.Image_CompressAMDBC5.restype = ctypes.c_void_p
    lib.Image_CompressAMDBC5.argtypes = [ctypes.c_void_p] * 3
    lib.Image_Destroy.argtypes = [ctypes.c_void_p]
    img = synth.reference_pattern_rgb(257, 257)[..., :3].copy()
    p = lib.Image_CreateNoClear(257, 257, 1, 1, 5)    # R8G8B8_UNORM
    ctypes.memmove(Hdr.from_address(p).data, img.ctypes.data, img.nbytes)

    progress = []
    CB = ctypes.CFUNCTYPE(ctypes.c_bool, ctypes.c_void_p, ctypes.c_float)
    cb = CB(lambda user, pct: progress.append(pct) or False)
    d = lib.Image_CompressAMDBC1(p, None, None, ctypes.cast(cb, ctypes.c_void_p), None)
    assert d
    hd = Hdr.from_address(d)
    assert (hd.width, hd.height, hd.format) == (260, 260, 10)
    got = np.ctypeslib.as_array((ctypes.c_uint8 * hd.dataSize).from_address(hd.data)).reshape(-1, 8)
    assert np.array_equal(got, oracle_lib.encode_image(1, img))
    assert len(progress) == 65 and progress[0] == 0.0
    lib.Image_Destroy(d)
    # abort via progress callback -> NULL
    stop = CB(lambda user, pct: pct > 50)
    assert not lib.Image_CompressAMDBC1(p, None, None, ctypes.cast(stop, ctypes.c_void_p), None)
    d5 = lib.Image_CompressAMDBC5(p, None, None)
    h5 = Hdr.from_address(d5)
    got5 = np.ctypeslib.as_array((ctypes.c_uint8 * h5.dataSize).from_address(h5.data)).reshape(-1, 16)
    assert np.array_equal(got5, oracle_lib.encode_image(5, img))
    lib.Image_Destroy(d5)
    lib.Image_Destroy(p)


@pytest.mark.parametrize("fmt,kind", [(1, "g1"), (1, "g0"), (4, "height"), (5, "normal")])
def test_full_8k_bit_exact(gpu, fmt, kind):
    """Configs 2 and 3 at full size, every block compared with the oracle."""
    n = 8192
    if kind == "g1":
        img = synth.g1(n, n)
    elif kind == "g0":
        img = synth.g0(n, n)
    elif kind == "height":
        img = synth.height_field(n, n, seed=1)
    else:
        img = synth.normal_map(synth.height_field(n, n, seed=1))
    opts = gic.Options(bc4_channel=0)
    out = gpu_encode(fmt, img, opts)
    ref = oracle_lib.encode_image(fmt, img, bc4_channel=0)
    assert np.array_equal(out, ref), _mismatch_report(out, ref)


@pytest.mark.parametrize("fmt", [2, 3])
def test_bc23_images(gpu, fmt):
    """BC2 / BC3 (amd_bc2/bc3_compressor.cpp): alpha half and the 4-colour RGB
    half vs the oracle, on alpha noise, alpha patterns, an RGB source (alpha
    forced to 1) and a ragged 37x23 edge case."""
    for img in (synth.noise_rgba(48, 40, seed=21, alpha=True), synth.reference_pattern_rgb(64, 64, alpha_ramp=True),
                synth.reference_pattern_rgb(37, 23, punch_through=True), synth.g1(64, 32)[..., :3]):
        out = gpu_encode(fmt, img)
        ref = oracle_lib.encode_image(fmt, img)
        assert np.array_equal(out, ref), _mismatch_report(out, ref)


@pytest.mark.parametrize("n", [97, 4100])
def test_bc4_block_batch_f32(gpu, n):
    """Block-level BC4 (the batched Image_CompressAMDAlphaSingleModeBlock): below
    4096 blocks two waves per block (bc4_blocks_wave_kernel: the 8- and 6-value
    ramp modes on one wave each, the grid and climb spread over the lanes), from
    4096 one lane per block; both bit-exact vs the
    oracle on noise, 8-bit grid values, solid and two-value blocks and blocks at
    the FIXED-mode extremes (0 / 1)."""
    import torch
    rng = np.random.default_rng(n)
    v = rng.random((n, 16), dtype=np.float32)
    v[::3] = np.round(v[::3] * 255) / np.float32(255.0)
    v[1::7] = v[1::7, :1]                                            # solid
    v[2::7] = np.where(rng.random((len(v[2::7]), 16)) < 0.5, v[2::7, :1], v[2::7, 1:2])   # two values
    v[3::7, :5] = 0.0                                                # extremes: 6-value mode's fixed 0 / 255
    v[3::7, 5:9] = 1.0
    v[4::7] = v[4::7] * np.float32(0.15) + np.float32(0.4)          # narrow range: climb without the grid
    t = torch.from_numpy(v).cuda()
    dst = torch.zeros(n * 8, dtype=torch.uint8, device="cuda")
    gic.encode_blocks_f32(gic.FMT_BC4, t, dst)
    torch.cuda.synchronize()
    got = dst.cpu().numpy().reshape(-1, 8)
    for i in range(n):
        assert got[i].tobytes() == oracle_lib.bc4_block(v[i]), i


@pytest.mark.parametrize("n", [97, 4100])
@pytest.mark.parametrize("steps,thr", [(1, 0.0), (1, 128 / 255.0), (2, 0.5)])
def test_bc1_block_batch_f32(gpu, n, steps, thr):
    """Block-level BC1 (the batched Image_CompressAMDBC1Block): below 4096 blocks
    one wave per block (bc1_blocks_wave_kernel: the 8x8 endpoint candidates on
    the wave's lanes, each Refine channel pass's (2 steps + 1)^2 jitters spread
    over them), from 4096 one lane per block; bit-exact vs the oracle on noise,
    8-bit grid values, solid blocks, alpha below / above the threshold."""
    import torch
    rng = np.random.default_rng(1000 * steps + n)
    blocks = rng.random((n, 16, 4), dtype=np.float32)
    blocks[::3] = np.round(blocks[::3] * 255) / np.float32(255.0)
    blocks[1::5] = blocks[1::5, :1]                      # solid blocks
    blocks[2::5, :, 3] = 1.0                             # opaque
    t = torch.from_numpy(blocks.reshape(-1, 64)).cuda()
    dst = torch.zeros(n * 8, dtype=torch.uint8, device="cuda")
    gic.encode_blocks_f32(gic.FMT_BC1, t, dst, gic.Options(refinement_steps=steps, bc1_alpha_threshold=thr))
    torch.cuda.synchronize()
    got = dst.cpu().numpy().reshape(-1, 8)
    for i in range(n):
        assert got[i].tobytes() == oracle_lib.bc1_block(blocks[i], steps=steps, threshold=thr), i


@pytest.mark.parametrize("n", [96, 4100])
@pytest.mark.parametrize("fmt", [2, 3])
def test_bc23_block_batch_f32(gpu, fmt, n):
    """Block-level BC2/BC3 on arbitrary float blocks (the batched form of the
    component-block API, Image_CompressAMDRGBSingleModeBlock / ...AlphaSingleModeBlock):
    a wave per block below 4096 blocks, a lane per block from 4096."""
    import torch
    rng = np.random.default_rng(fmt + n)
    blocks = rng.random((n, 16, 4), dtype=np.float32)
    blocks[::3] = np.round(blocks[::3] * 255) / np.float32(255.0)
    blocks[1::5] = blocks[1::5, :1]                      # solid blocks
    t = torch.from_numpy(blocks.reshape(-1, 64)).cuda()
    dst = torch.zeros(n * 16, dtype=torch.uint8, device="cuda")
    gic.encode_blocks_f32(fmt, t, dst)
    torch.cuda.synchronize()
    got = dst.cpu().numpy().reshape(-1, 16)
    for i, b in enumerate(blocks):
        assert got[i].tobytes() == oracle_lib.bc23_block(fmt, b), i


def test_bc3_full_8k_bit_exact(gpu):
    """BC3 over a whole 8192^2 RGBA8 texture with a noisy alpha channel."""
    n = 8192
    img = synth.g1(n, n)
    img[..., 3] = synth.g1(n, n, seed=5)[..., 0]
    out = gpu_encode(3, img)
    ref = oracle_lib.encode_image(3, img)
    assert np.array_equal(out, ref), _mismatch_report(out, ref)


def _float_blocks(tex, w, h):
    """(H, W, 4) float texels -> (by*bx, 16, 4) blocks with ReadNxNBlockF's edge clamp."""
    bx, by = (w + 3) // 4, (h + 3) // 4
    ys = np.minimum(np.arange(by * 4), h - 1)
    xs = np.minimum(np.arange(bx * 4), w - 1)
    t = tex[ys][:, xs]
    return t.reshape(by, 4, bx, 4, 4).transpose(0, 2, 1, 3, 4).reshape(-1, 16, 4).astype(np.float32)


@pytest.mark.parametrize("fmt", [4, 5])
def test_snorm8_sources_bc45(gpu, fmt):
    """R8_SNORM / R8G8_SNORM sources (amd_bc4/bc5_compressor.cpp:16-19): texels
    max(v / 127.0f, -1.0f), encoded like the reference's float block path."""
    import torch
    w, h, c = 30, 22, (1 if fmt == 4 else 2)
    rng = np.random.default_rng(fmt)
    img = rng.integers(-128, 128, (h, w, c), dtype=np.int8)
    img[:8] = np.clip(np.arange(w) * 9 - 128, -128, 127).astype(np.int8)[None, :, None]   # ramps
    src = torch.from_numpy(img.copy()).cuda()
    bx, by = (w + 3) // 4, (h + 3) // 4
    dst = torch.zeros(bx * by * gic.block_bytes(fmt), dtype=torch.uint8, device="cuda")
    gic.encode_device_src(fmt, gic.SRC_SNORM8, src, w, h, 1, c, dst, gic.Options(bc4_channel=0))
    torch.cuda.synchronize()
    got = dst.cpu().numpy().reshape(-1, gic.block_bytes(fmt))
    tex = np.zeros((h, w, 4), np.float32)
    tex[..., 3] = 1.0
    tex[..., :c] = np.maximum(img.astype(np.float32) / np.float32(127.0), np.float32(-1.0))
    blocks = _float_blocks(tex, w, h)
    for i, b in enumerate(blocks):
        ref = oracle_lib.bc4_block(b[:, 0])
        if fmt == 5:
            ref += oracle_lib.bc4_block(b[:, 1])
        assert got[i].tobytes() == ref, i


@pytest.mark.parametrize("fmt", [1, 3, 7])
def test_float32_sources(gpu, fmt):
    """R32G32B32A32_SFLOAT sources: float texels as stored through the float
    block encoders (BC1/BC3 with values outside [0, 1] too; BC7 inside it:
    the reference indexes its 256-entry single-point tables with floor/ceil
    of the texel, amd_shake.cpp:627-635, out of bounds for other values)."""
    import torch
    w, h = 21, 13 if fmt == 7 else 26
    rng = np.random.default_rng(10 + fmt)
    tex = rng.random((h, w, 4), dtype=np.float32)
    if fmt != 7:
        tex = tex * np.float32(1.2) - np.float32(0.1)
    tex[:, :, 3] = np.where(rng.random((h, w)) < 0.8, np.float32(1.0), tex[:, :, 3])
    src = torch.from_numpy(tex.copy()).cuda()
    bx, by = (w + 3) // 4, (h + 3) // 4
    dst = torch.zeros(bx * by * gic.block_bytes(fmt), dtype=torch.uint8, device="cuda")
    gic.encode_device_src(fmt, gic.SRC_FLOAT32, src, w, h, 1, 4, dst)
    torch.cuda.synchronize()
    got = dst.cpu().numpy().reshape(-1, gic.block_bytes(fmt))
    for i, b in enumerate(_float_blocks(tex, w, h)):
        if fmt == 1:
            ref = oracle_lib.bc1_block(b)
        elif fmt == 3:
            ref = oracle_lib.bc23_block(3, b)
        else:
            ref = oracle_lib.bc7_block(b)[0]
        assert got[i].tobytes() == ref, i


def test_host_api_snorm_source_gives_snorm_destination(gpu):
    """Image_CompressAMDBC4 on an R8_SNORM image returns a DXBC4_SNORM image
    (amd_bc4_compressor.cpp:16-19) with the device path's blocks."""
    import torch
    lib = gic.library()
    lib.Image_CreateNoClear.restype = ctypes.c_void_p
    lib.Image_RawDataPtr.argtypes = [ctypes.c_void_p]
    lib.Image_RawDataPtr.restype = ctypes.c_void_p
    lib.Image_Destroy.argtypes = [ctypes.c_void_p]
    lib.Image_CompressAMDBC4.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    lib.Image_CompressAMDBC4.restype = ctypes.c_void_p
    rng = np.random.default_rng(3)
    img = rng.integers(-128, 128, (16, 24, 1), dtype=np.int8)
    p = lib.Image_CreateNoClear(24, 16, 1, 1, 2)   # R8_SNORM
    ctypes.memmove(lib.Image_RawDataPtr(p), img.tobytes(), img.nbytes)
    q = lib.Image_CompressAMDBC4(p, None, None)
    assert q
    fmt_field = ctypes.c_int.from_address(q + 24).value
    assert fmt_field == 15   # TinyImageFormat_DXBC4_SNORM
    out = np.ctypeslib.as_array(ctypes.cast(lib.Image_RawDataPtr(q), ctypes.POINTER(ctypes.c_uint8)), (192,)).copy()
    src = torch.from_numpy(img.copy()).cuda()
    dst = torch.zeros(24 * 8, dtype=torch.uint8, device="cuda")
    gic.encode_device_src(4, gic.SRC_SNORM8, src, 24, 16, 1, 1, dst)   # channel 1 (Q1): of an R8 source, zeros
    torch.cuda.synchronize()
    assert out.tobytes() == dst.cpu().numpy().tobytes()
    lib.Image_Destroy(q)
    lib.Image_Destroy(p)


def _special_blocks(kind, n=48, seed=0):
    """Float blocks in [0, 1) with some texels replaced by values the reference
    reads unclamped (block_utils.cpp:7-41): huge finite (their x255 scale or
    the search's hi - lo differences overflow to inf), +-inf, or NaN."""
    rng = np.random.default_rng(seed)
    b = rng.random((n, 16, 4), dtype=np.float32)
    b[::2, :, 3] = 1.0
    vals = {"huge": [1e36, 3.0e38, -3.0e38, 2.0e37], "inf": [np.inf, -np.inf], "nan": [np.nan]}[kind]
    for i in range(n):
        for _ in range(1 + i % 3):
            t, c = int(rng.integers(16)), int(rng.integers(4 if i % 4 == 3 else 3))
            b[i, t, c] = np.float32(vals[int(rng.integers(len(vals)))])
    return b


@pytest.mark.parametrize("kind", ["huge", "inf", "nan"])
def test_bc1_bc3_non_finite_float_texels(gpu, kind):
    """Huge, infinite and NaN float texels through the BC1 block API
    (Image_CompressAMDBC1Block), and through the FLOAT32 source path for BC1
    and BC3, against the oracle (the search's fast division by 3 returns +-inf
    and NaN as IEEE division does, gic_fastdiv.h)."""
    import torch
    lib = gic.library()
    blocks = _special_blocks(kind)
    for i, blk in enumerate(blocks):
        out = np.zeros(8, np.uint8)
        lib.Image_CompressAMDBC1Block(np.ascontiguousarray(blk).ctypes.data_as(ctypes.c_void_p), False, False, 1,
                                      ctypes.c_float(128 / 255.0), out.ctypes.data_as(ctypes.c_void_p))
        assert out.tobytes() == oracle_lib.bc1_block(blk), (kind, i)
        # each channel as a BC4 block (the one-wave kernel: lane-parallel sort with
        # the register sort for NaN blocks, register value table)
        for c in range(4):
            v = np.ascontiguousarray(blk.reshape(16, 4)[:, c])
            out4 = np.zeros(8, np.uint8)
            lib.Image_CompressAMDAlphaSingleModeBlock(v.ctypes.data_as(ctypes.c_void_p),
                                                      out4.ctypes.data_as(ctypes.c_void_p))
            assert out4.tobytes() == oracle_lib.bc4_block(v), (kind, i, c)
    # the same blocks as a 4 x 12-block FLOAT32 image
    tex = blocks.reshape(4, 12, 4, 4, 4).transpose(0, 2, 1, 3, 4).reshape(16, 48, 4)
    src = torch.from_numpy(np.ascontiguousarray(tex)).cuda()
    for fmt in (1, 3):
        dst = torch.zeros(48 * gic.block_bytes(fmt), dtype=torch.uint8, device="cuda")
        gic.encode_device_src(fmt, gic.SRC_FLOAT32, src, 48, 16, 1, 4, dst)
        torch.cuda.synchronize()
        got = dst.cpu().numpy().reshape(-1, gic.block_bytes(fmt))
        for i, b in enumerate(_float_blocks(tex, 48, 16)):
            ref = oracle_lib.bc1_block(b) if fmt == 1 else oracle_lib.bc23_block(3, b)
            assert got[i].tobytes() == ref, (kind, fmt, i)
