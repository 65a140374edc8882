"""CPU tests of the C-ABI boundary: the HIP library loads and exports every
function declared in include/*/*.h.  No compute calls (no GPU here)."""
import ctypes
import glob
import os
import re

import gfx_imagecompress_amd as gic

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared_functions():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        src = re.sub(r"//[^\n]*", "", src)
        for m in re.finditer(r"([A-Za-z_][A-Za-z0-9_]*)\s*\(", src):
            name = m.group(1)
            prefix = src[max(0, m.start() - 200):m.start()]
            if name in ("if", "sizeof", "defined") or "typedef" in prefix.split(";")[-1]:
                continue
            if re.search(r"(AL2O3_EXTERN_C|\bint|\bvoid|\buint32_t|const char \*|\bbool|Image_ImageHeader const \*|"
                         r"Image_CompressType|\bvoid \*)\s*\**\s*$", prefix.split(";")[-1].split("\n")[-1]):
                names.add(name)
    return names


def test_header_parse_finds_api():
    names = _declared_functions()
    for must in ("Image_CompressAMDBC1", "Image_CompressAMDBC7", "Image_CompressAMDBC1Block",
                 "gic_hip_encode", "gic_hip_encode_rows", "Image_CreateNoClear"):
        assert must in names, must


def test_library_exports_every_declared_symbol():
    lib = gic.library()
    missing = [n for n in sorted(_declared_functions()) if not hasattr(lib, n)]
    assert not missing, missing


def test_default_options_match_reference():
    o = gic._COptions()
    gic.library().gic_default_options(ctypes.byref(o))
    assert o.struct_size == ctypes.sizeof(gic._COptions)
    assert abs(o.bc1_alpha_threshold - 128 / 255.0) < 1e-7
    assert o.refinement_steps == 1 and o.bc4_channel == 1 and o.bc7_mode_mask == 0xFF
    assert o.colour_restrict == 1 and o.alpha_restrict == 1 and o.bc7_quality == 1.0
    # bc7enc16: Image_CompressDefaultRichGel99Options {perceptual = true, fast = false} (richgel999_bc7enc16.cpp:13-19)
    assert (o.bc7enc_perceptual, o.bc7enc_uber_level, o.bc7enc_max_partitions) == (1, 4, 64)
    assert o.bc7enc_least_squares == 1 and o.bc7enc_filterbank == 1
    py = gic.Options().to_c()
    assert bytes(py) == bytes(o), "Python Options defaults drift from gic_default_options"


def test_block_bytes_and_argument_checks():
    lib = gic.library()
    assert lib.gic_block_bytes(1) == 8 and lib.gic_block_bytes(4) == 8
    assert lib.gic_block_bytes(5) == 16 and lib.gic_block_bytes(7) == 16
    # invalid arguments are rejected before any HIP call
    assert lib.gic_hip_encode(1, None, 4, 4, 1, 4, 16, None, None, None, None) == gic.GIC_EINVAL
    o = gic.Options(adaptive_weights=True).to_c()
    assert lib.gic_hip_encode(1, 16, 4, 4, 1, 4, 16, ctypes.byref(o), 16, None, None) == gic.GIC_EUNSUP
    assert lib.gic_block_bytes(gic.FMT_BC7ENC16) == 16
    o = gic.Options(bc7enc_uber_level=5).to_c()
    assert lib.gic_hip_encode(gic.FMT_BC7ENC16, 16, 4, 4, 1, 4, 16, ctypes.byref(o), 16, None, None) == gic.GIC_EINVAL
    assert lib.gic_hip_encode_blocks_u8(gic.FMT_BC7, 16, 1, None, 16, None) == gic.GIC_EINVAL
    assert lib.gic_hip_encode_blocks_u8(gic.FMT_BC7ENC16, None, 1, None, 16, None) == gic.GIC_EINVAL
    for bound in (float("nan"), -1.0, 70000.0):   # bc7_mse_bound: NaN, negative, above 255^2
        o = gic.Options(bc7_mse_bound=bound).to_c()
        assert lib.gic_hip_encode(gic.FMT_BC7, 16, 4, 4, 1, 4, 16, ctypes.byref(o), 16, None, None) == gic.GIC_EINVAL
    # BC6H decoder: BC6H formats only, RGBA16F rows of at least width * 8 bytes
    assert lib.gic_hip_decode_bc6h(gic.FMT_BC7, 16, 4, 4, 1, 16, 32, None) == gic.GIC_EINVAL
    assert lib.gic_hip_decode_bc6h(gic.FMT_BC6H, 16, 4, 4, 1, 16, 31, None) == gic.GIC_EINVAL
    assert lib.gic_hip_decode_bc6h(gic.FMT_BC6H, None, 4, 4, 1, 16, 32, None) == gic.GIC_EINVAL
    assert lib.gic_hip_decode(gic.FMT_BC6H, 16, 4, 4, 1, 16, 16, None) == gic.GIC_EINVAL


def test_image_model_and_pick_type():
    lib = gic.library()
    lib.Image_CreateNoClear.restype = ctypes.c_void_p
    lib.Image_Destroy.argtypes = [ctypes.c_void_p]

    class Hdr(ctypes.Structure):
        _fields_ = [("dataSize", ctypes.c_uint64), ("width", ctypes.c_uint32), ("height", ctypes.c_uint32),
                    ("depth", ctypes.c_uint32), ("slices", ctypes.c_uint32), ("format", ctypes.c_int),
                    ("flags", ctypes.c_uint32), ("data", ctypes.c_void_p)]
    # 257x257 DXBC1 pads to 260x260 (tests/test_imagecompress.cpp:169-170)
    p = lib.Image_CreateNoClear(257, 257, 1, 1, 10)  # TinyImageFormat_DXBC1_RGB_UNORM
    h = Hdr.from_address(p)
    assert (h.width, h.height, h.dataSize) == (260, 260, 65 * 65 * 8)
    lib.ImageCompress_PickCompressionType.argtypes = [ctypes.c_int, ctypes.c_void_p]
    lib.Image_Destroy(p)
    q = lib.Image_CreateNoClear(8, 8, 1, 1, 7)  # R8G8B8A8_UNORM
    assert lib.ImageCompress_PickCompressionType(0x10, q) == 7  # DXBC7 when allowed
    assert lib.ImageCompress_PickCompressionType(0x1, q) == 3   # DXBC3 for alpha sources
    lib.Image_Destroy(q)


def test_dds_writer_headers(tmp_path):
    """gic_save_dds (host only): legacy FourCC header for BC1, DX10 header for
    BC7 with the DXGI format, block data verbatim after the header."""
    import struct
    lib = gic.library()
    lib.Image_CreateNoClear.restype = ctypes.c_void_p
    lib.Image_Destroy.argtypes = [ctypes.c_void_p]
    lib.Image_RawDataPtr.argtypes = [ctypes.c_void_p]
    lib.Image_RawDataPtr.restype = ctypes.c_void_p
    for fmt_id, want_fourcc, dxgi, bb in ((10, b"DXT1", None, 8), (18, b"DX10", 98, 16), (19, b"DX10", 99, 16)):
        p = lib.Image_CreateNoClear(20, 12, 1, 1, fmt_id)
        n = 5 * 3 * bb
        payload = bytes((i * 7) & 255 for i in range(n))
        ctypes.memmove(lib.Image_RawDataPtr(p), payload, n)
        path = str(tmp_path / f"t{fmt_id}.dds")
        assert lib.gic_save_dds(p, path.encode()) == gic.GIC_OK
        data = open(path, "rb").read()
        assert data[:4] == b"DDS "
        size, flags, h, w, pitch = struct.unpack_from("<5I", data, 4)
        # DDSD_LINEARSIZE: total bytes of the top-level image; DDSD_MIPMAPCOUNT with one level
        assert (size, h, w, pitch) == (124, 12, 20, 5 * 3 * bb)
        assert flags & 0x80000 and flags & 0x20000
        assert struct.unpack_from("<I", data, 4 + 24)[0] == 1
        assert data[4 + 80:4 + 84] == want_fourcc
        off = 128
        if dxgi is not None:
            assert struct.unpack_from("<5I", data, 128)[:2] == (dxgi, 3)
            off += 20
        assert data[off:] == payload
        lib.Image_Destroy(p)
    # not a block format
    q = lib.Image_CreateNoClear(8, 8, 1, 1, 7)
    assert lib.gic_save_dds(q, str(tmp_path / "x.dds").encode()) == gic.GIC_EINVAL
    lib.Image_Destroy(q)
