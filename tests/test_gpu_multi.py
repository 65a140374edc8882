"""gic_encode_multi: the multi-GPU split of the reference's block loop behind the C ABI.

The box has one GPU, so the multi-device lists here name device 0 several
times: every rank still uploads only the source rows its range reads, encodes
them on its own stream from its own host thread, and the gather (peer copies
for a repeated device; RCCL over distinct devices) places each piece at its
reference-order offset.  The result must equal the single-call encode byte for
byte -- ragged row counts, several slices (ranges crossing slice boundaries),
the edge clamp of the last block row, the float source path.  The RCCL gather
itself needs distinct devices: it is exercised on an 8-GPU node only.
"""
import os

import numpy as np
import pytest

import gfx_imagecompress_amd as gic
from gfx_imagecompress_amd import synth
from test_gpu_parity import gpu_encode

pytestmark = pytest.mark.gpu


def _multi(fmt, img, devices, options=None, src_type=0, peer=False):
    import torch
    a = img if img.ndim == 4 else img[None]
    s, h, w, _ = a.shape
    bx, by = gic.blocks_shape(w, h)
    dst = torch.zeros(bx * by * s * gic.block_bytes(fmt), dtype=torch.uint8, device="cuda")
    rep = gic.encode_multi(fmt, a, devices, dst, options, src_type=src_type, peer_copy=peer)
    return dst.cpu().numpy().reshape(-1, gic.block_bytes(fmt)), rep


@pytest.mark.parametrize("fmt", [gic.FMT_BC1, gic.FMT_BC4, gic.FMT_BC5, gic.FMT_BC7ENC16])
def test_multi_equals_single_call(gpu, fmt):
    """3 slices of 203 x 141 (36 block rows each, 108 slice-major rows over 1, 3
    and 5 ranks: ranges of 36 / 22 rows that start and end inside slices)."""
    img = np.stack([synth.noise_rgba(203, 141, seed=7 + k) for k in range(3)])
    if fmt in (gic.FMT_BC4, gic.FMT_BC5):
        img = np.ascontiguousarray(img[..., :2])
    opts = gic.Options(bc4_channel=0)
    ref = gpu_encode(fmt, img, opts)
    for devs in ([0], [0, 0, 0], [0, 0, 0, 0, 0]):
        got, rep = _multi(fmt, img, devs, opts)
        assert np.array_equal(got, ref), (fmt, devs, int((got != ref).any(axis=1).sum()))
        assert rep["ranks"] == len(devs) and not rep["rccl"]
        bb = gic.block_bytes(fmt)
        first0, n0 = gic.multi_split(36 * 3, len(devs), 0)
        assert rep["gathered_bytes"] == (36 * 3 - n0) * 51 * bb


def test_multi_bc7_matches_single_call(gpu):
    """BC7 (the reference search) over 2 ranks: each rank's BC7 call returns with
    its work complete (the H4 decision), so the ranks run on separate host
    threads; the pieces land in order."""
    img = synth.g1(64, 24)
    ref = gpu_encode(gic.FMT_BC7, img)
    got, rep = _multi(gic.FMT_BC7, img, [0, 0])
    assert np.array_equal(got, ref)
    assert rep["gathered_bytes"] == 3 * 16 * 16


def test_multi_float_source(gpu):
    """FLOAT32 texels (BC6H) go through the same split: the device gathers its
    rows into float blocks and encodes them."""
    hdr = synth.hdr_rgba(64, 52, seed=5)
    import torch
    src = torch.from_numpy(hdr.reshape(-1).copy()).cuda()
    ref = torch.zeros(16 * 13 * 16, dtype=torch.uint8, device="cuda")
    gic.encode_device_src(gic.FMT_BC6H, gic.SRC_FLOAT32, src, 64, 52, 1, 4, ref)
    got, _ = _multi(gic.FMT_BC6H, hdr, [0, 0, 0], src_type=gic.SRC_FLOAT32)
    assert np.array_equal(got, ref.cpu().numpy().reshape(-1, 16))


def _image_api(lib, name, img, *extra):
    """Image_CompressAMD<name> on an R8G8B8A8_UNORM header holding img (H,W,4)."""
    import ctypes
    h, w, _ = img.shape
    p = lib.Image_CreateNoClear(w, h, 1, 1, 7)   # R8G8B8A8_UNORM
    ctypes.memmove(lib.Image_RawDataPtr(p), img.tobytes(), img.nbytes)
    fn = getattr(lib, "Image_CompressAMD" + name)
    fn.restype = ctypes.c_void_p
    fn.argtypes = [ctypes.c_void_p] * (1 + len(extra) + 2)
    q = fn(p, *extra, None, None)
    assert q
    bb = 8 if name == "BC1" else 16
    out = np.frombuffer(ctypes.string_at(lib.Image_RawDataPtr(q), ((w + 3) // 4) * ((h + 3) // 4) * bb),
                        np.uint8).reshape(-1, bb).copy()
    lib.Image_Destroy(q)
    lib.Image_Destroy(p)
    return out


def test_image_api_with_gic_devices(gpu, monkeypatch):
    """Image_CompressAMDBC1 / BC7 (the reference's C entry points) with
    GIC_DEVICES listing more than one device take the multi-device path and
    return the single-device bytes."""
    import ctypes
    lib = gic.library()
    lib.Image_CreateNoClear.restype = ctypes.c_void_p
    lib.Image_CreateNoClear.argtypes = [ctypes.c_uint32] * 4 + [ctypes.c_int]
    lib.Image_RawDataPtr.argtypes = [ctypes.c_void_p]
    lib.Image_RawDataPtr.restype = ctypes.c_void_p
    lib.Image_Destroy.argtypes = [ctypes.c_void_p]
    img = np.ascontiguousarray(synth.noise_rgba(96, 42, seed=3))
    small = np.ascontiguousarray(synth.g1(32, 12))
    ref1 = _image_api(lib, "BC1", img, None, None)
    ref7 = _image_api(lib, "BC7", small, None)
    assert np.array_equal(ref1, gpu_encode(gic.FMT_BC1, img))
    monkeypatch.setenv("GIC_DEVICES", "0,0,0")
    assert np.array_equal(_image_api(lib, "BC1", img, None, None), ref1)
    assert np.array_equal(_image_api(lib, "BC7", small, None), ref7)
    r = gic._MultiReport()
    assert lib.gic_multi_last_report(ctypes.byref(r)) == 0 and r.ranks == 3
    assert lib.gic_multi_release() == 0


def test_multi_rejects_bad_arguments(gpu):
    import torch
    img = synth.g1(16, 16)
    dst = torch.zeros(16 * 8, dtype=torch.uint8, device="cuda")
    with pytest.raises(gic.GicError):
        gic.encode_multi(gic.FMT_BC1, img, [99], dst)
    with pytest.raises(gic.GicError):
        gic.encode_multi(gic.FMT_BC1, img, [], dst)


# ---------------------------------------------------------------------------
# the host-image pipeline (gic_pipeline.cpp): upload / encode / download overlap


def _progress_run(fmt, img, entry=None, abort_at=None, options=None):
    seen = []

    def cb(pct):
        seen.append(pct)
        return abort_at is not None and pct > abort_at
    out = gic.compress_host(fmt, img, options, progress=cb, entry=entry)
    return out, seen


@pytest.mark.parametrize("mode", ["pageable", "staged", "register"])
def test_host_pipeline_modes_and_pieces(gpu, monkeypatch, mode):
    """Every upload mode, cut into many pieces (GIC_PIECE_BLOCKS), over three
    slices whose pieces end inside and at slice ends: the same bytes as the
    device path, and the report counts the pieces."""
    img = np.stack([synth.noise_rgba(203, 141, seed=11 + k) for k in range(3)])
    ref = gpu_encode(gic.FMT_BC1, img).reshape(3, 36, 51, 8)
    monkeypatch.setenv("GIC_H2D", mode)
    monkeypatch.setenv("GIC_PIECE_BLOCKS", str(51 * 5))   # 5 block rows a piece: 8 per slice
    got = gic.compress_host(gic.FMT_BC1, img, gic.Options())
    assert np.array_equal(got, ref)
    rep = gic.host_report()
    assert rep["devices"] == 1 and rep["pieces"] == 3 * 8
    assert rep["h2d_mode"] == ["pageable", "staged", "register"].index(mode)
    assert rep["total_ms"] > 0 and rep["h2d_ms"] > 0 and rep["encode_ms"] > 0 and rep["d2h_ms"] > 0


def test_host_pipeline_progress_sequence_single_and_multi(gpu, monkeypatch):
    """Image_CompressAMDBC1 with a progress callback: one device, and
    GIC_DEVICES=0,0,0 (three lanes, every lane downloading its rows straight
    into the host image) -- the same bytes and exactly the reference's per-row
    sequence 100 * (y * bx) / (bx * by), slice by slice, in order
    (amd_bc1_compressor.cpp:64-68); a callback returning true gives NULL."""
    img = np.stack([synth.noise_rgba(96, 42, seed=21 + k) for k in range(2)])
    bx, by = 24, 11
    want = [np.float32(100.0) * np.float32(y * bx) / np.float32(bx * by) for _ in range(2) for y in range(by)]
    monkeypatch.setenv("GIC_PIECE_BLOCKS", str(bx * 2))
    ref, seq = _progress_run(gic.FMT_BC1, img, entry="Image_CompressAMDBC1")
    assert ref is not None and np.array_equal(ref, gpu_encode(gic.FMT_BC1, img).reshape(2, by, bx, 8))
    assert np.array_equal(np.array(seq, np.float32), np.array(want, np.float32))
    for devs in ("0,0,0", "0,0,0,0,0"):
        monkeypatch.setenv("GIC_DEVICES", devs)
        got, seq = _progress_run(gic.FMT_BC1, img, entry="Image_CompressAMDBC1")
        assert np.array_equal(got, ref), devs
        assert np.array_equal(np.array(seq, np.float32), np.array(want, np.float32)), devs
        assert gic.host_report()["devices"] == len(devs.split(","))
        out, seq = _progress_run(gic.FMT_BC1, img, entry="Image_CompressAMDBC1", abort_at=50.0)
        assert out is None and seq[-1] > 50.0 and len(seq) < len(want)
    # BC7 through its wrapper over three lanes
    small = np.ascontiguousarray(synth.g1(32, 12))
    monkeypatch.setenv("GIC_DEVICES", "0,0,0")
    got7, seq7 = _progress_run(gic.FMT_BC7, small, entry="Image_CompressAMDBC7")
    assert np.array_equal(got7.reshape(-1, 16), gpu_encode(gic.FMT_BC7, small))
    assert len(seq7) == 3
    assert gic.library().gic_multi_release() == 0


def test_compress_image_options(gpu):
    """gic_compress_image takes every option: the BC7 bounded exit through the
    host path equals the device path's blocks with the same options."""
    img = np.ascontiguousarray(synth.g1(64, 32))
    o = gic.Options(bc7_mse_bound=0.5)
    got = gic.compress_host(gic.FMT_BC7, img, o)
    assert np.array_equal(got.reshape(-1, 16), gpu_encode(gic.FMT_BC7, img, o))
    got5 = gic.compress_host(gic.FMT_BC5, np.ascontiguousarray(img[..., :2]), gic.Options())
    assert np.array_equal(got5.reshape(-1, 16), gpu_encode(gic.FMT_BC5, np.ascontiguousarray(img[..., :2])))


def test_encode_multi_checks_dst_device_and_dtype(gpu):
    import torch
    img = synth.g1(16, 16)
    dst = torch.zeros(16 * 8, dtype=torch.uint8, device="cuda")
    with pytest.raises(gic.GicError):
        gic.encode_multi(gic.FMT_BC1, img.astype(np.float32), [0], dst)   # float data, UNORM8 source type
    with pytest.raises(gic.GicError):
        gic.encode_multi(gic.FMT_BC1, img, [0], torch.zeros(16 * 8, dtype=torch.uint8))   # host dst
