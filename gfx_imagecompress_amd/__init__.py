"""gfx_imagecompress_amd -- MI355X-native BCn block compressor.

Python mirror of the reference's ``Image_Compress*`` operator interface
(DeanoC/gfx_imagecompress ``include/gfx_imagecompress/imagecompress.h``) over
the C ABI of ``lib/libgfx_imagecompress_amd.so`` (HIP kernels for gfx950).

* :func:`encode_device` -- the batched device entry (``gic_hip_encode_rows``):
  inputs already resident in HBM (torch tensors), asynchronous on a stream.
* :func:`compress_bc1` / :func:`compress_bc4` / :func:`compress_bc5` /
  :func:`compress_bc7` -- host-array convenience wrappers with the reference
  wrappers' defaults (``amd_bc{1,4,5,7}_compressor.cpp``).

There is no CPU fallback: if the shared library or a GPU is missing every
compression call raises :class:`GicError`.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, replace

__all__ = [
    "GicError", "Options", "FMT_BC1", "FMT_BC2", "FMT_BC3", "FMT_BC4", "FMT_BC5", "FMT_BC6H", "FMT_BC6H_SF",
    "FMT_BC7", "FMT_BC7ENC16", "compress_bc6h",
    "library", "encode_blocks_u8", "compress_bc7_fast", "iter_cap_hits", "set_iter_cap", "nonterminating_loops",
    "last_h4_report", "encode_multi", "multi_split",
    "block_bytes", "blocks_shape", "encode_device", "encode_device_src", "encode_blocks_f32", "decode_device", "compress_bc1", "compress_bc2",
    "compress_bc3", "compress_bc4", "compress_bc5", "compress_bc7", "LIB_PATH",
]

FMT_BC1, FMT_BC2, FMT_BC3, FMT_BC4, FMT_BC5, FMT_BC7 = 1, 2, 3, 4, 5, 7
FMT_BC7ENC16 = 8   # BC7 by bc7enc16, the reference's fast encoder (richgel999_bc7enc16.cpp)
FMT_BC6H, FMT_BC6H_SF = 6, 9   # BC6H unsigned / signed half floats (amd_bc6h_body.cpp, BC6HBlockEncoder)
_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GIC_LIBRARY") or os.path.join(_HERE, "lib", "libgfx_imagecompress_amd.so")

GIC_OK, GIC_EINVAL, GIC_EUNSUP, GIC_EHIP = 0, -1, -2, -3
_ERRS = {GIC_EINVAL: "invalid argument", GIC_EUNSUP: "unsupported option", GIC_EHIP: "HIP runtime error"}


class GicError(RuntimeError):
    """Raised when the HIP library is missing or a call fails."""


class _COptions(ctypes.Structure):
    _fields_ = [
        ("struct_size", ctypes.c_uint32),
        ("bc1_alpha_threshold", ctypes.c_float),
        ("refinement_steps", ctypes.c_uint8),
        ("b3d_refinement", ctypes.c_uint8),
        ("adaptive_weights", ctypes.c_uint8),
        ("bc4_channel", ctypes.c_uint8),
        ("bc7_mode_mask", ctypes.c_uint8),
        ("colour_restrict", ctypes.c_uint8),
        ("alpha_restrict", ctypes.c_uint8),
        ("force_alpha_one", ctypes.c_uint8),
        ("bc7_quality", ctypes.c_float),
        ("bc7_performance", ctypes.c_float),
        ("bc7_shake_ranks", ctypes.c_uint32),
        ("bc7enc_perceptual", ctypes.c_uint8),
        ("bc7enc_uber_level", ctypes.c_uint8),
        ("bc7enc_max_partitions", ctypes.c_uint8),
        ("bc7enc_least_squares", ctypes.c_uint8),
        ("bc7enc_filterbank", ctypes.c_uint8),
        ("bc7_mse_bound", ctypes.c_float),
    ]


@dataclass
class Options:
    """Mirror of ``gic_options`` with the reference defaults.

    bc1_alpha_threshold: ``Image_CompressBC1Options.AlphaThreshold / 255``
    (amd_bc1_compressor.cpp:57; alpha-aware even when UseAlpha is false).
    refinement_steps: ``Image_CompressAMDBackendOptions.RefinementSteps``.
    bc4_channel: the reference BC4 wrapper reads channel 1 (green).
    """

    bc1_alpha_threshold: float = 128 / 255.0
    refinement_steps: int = 1
    b3d_refinement: bool = False
    adaptive_weights: bool = False
    bc4_channel: int = 1
    bc7_mode_mask: int = 0xFF
    colour_restrict: bool = True
    alpha_restrict: bool = True
    force_alpha_one: bool = False
    bc7_quality: float = 1.0
    bc7_performance: float = 1.0
    bc7_shake_ranks: int = 0
    # bc7enc16 (FMT_BC7ENC16): the image API's defaults (perceptual, fast = false -> uber level 4)
    bc7enc_perceptual: bool = True
    bc7enc_uber_level: int = 4
    bc7enc_max_partitions: int = 64
    bc7enc_least_squares: bool = True
    bc7enc_filterbank: bool = True
    # BC7 bounded exit: blocks whose cheap probe decodes within this MSE are final (0 = off)
    bc7_mse_bound: float = 0.0

    def to_c(self) -> _COptions:
        o = _COptions()
        o.struct_size = ctypes.sizeof(_COptions)
        o.bc1_alpha_threshold = float(self.bc1_alpha_threshold)
        o.refinement_steps = int(self.refinement_steps)
        o.b3d_refinement = int(bool(self.b3d_refinement))
        o.adaptive_weights = int(bool(self.adaptive_weights))
        o.bc4_channel = int(self.bc4_channel)
        o.bc7_mode_mask = int(self.bc7_mode_mask)
        o.colour_restrict = int(bool(self.colour_restrict))
        o.alpha_restrict = int(bool(self.alpha_restrict))
        o.force_alpha_one = int(bool(self.force_alpha_one))
        o.bc7_quality = float(self.bc7_quality)
        o.bc7_performance = float(self.bc7_performance)
        o.bc7_shake_ranks = int(self.bc7_shake_ranks)
        o.bc7enc_perceptual = int(bool(self.bc7enc_perceptual))
        o.bc7enc_uber_level = int(self.bc7enc_uber_level)
        o.bc7enc_max_partitions = int(self.bc7enc_max_partitions)
        o.bc7enc_least_squares = int(bool(self.bc7enc_least_squares))
        o.bc7enc_filterbank = int(bool(self.bc7enc_filterbank))
        o.bc7_mse_bound = float(self.bc7_mse_bound)
        return o

    @staticmethod
    def bc7enc16(fast: bool = False, perceptual: bool = True) -> "Options":
        """The settings Image_CompressRichGel999BC7enc16 derives from its
        (fast, perceptual) arguments (richgel999_bc7enc16.cpp:73-89)."""
        return Options(bc7enc_perceptual=perceptual, bc7enc_uber_level=0 if fast else 4)


class _MultiReport(ctypes.Structure):
    _fields_ = [("ranks", ctypes.c_int), ("rccl", ctypes.c_int), ("encode_ms_max", ctypes.c_double),
                ("gather_ms", ctypes.c_double), ("gathered_bytes", ctypes.c_uint64)]


class _HostReport(ctypes.Structure):
    _fields_ = [("devices", ctypes.c_int), ("pieces", ctypes.c_int), ("h2d_mode", ctypes.c_int),
                ("total_ms", ctypes.c_double), ("h2d_ms", ctypes.c_double), ("encode_ms", ctypes.c_double),
                ("d2h_ms", ctypes.c_double)]


class _ImageHeader(ctypes.Structure):   # include/gfx_image/image.h
    _fields_ = [("dataSize", ctypes.c_uint64), ("width", ctypes.c_uint32), ("height", ctypes.c_uint32),
                ("depth", ctypes.c_uint32), ("slices", ctypes.c_uint32), ("format", ctypes.c_int),
                ("flags", ctypes.c_uint32), ("data", ctypes.c_void_p)]


PROGRESS_FUNC = ctypes.CFUNCTYPE(ctypes.c_bool, ctypes.c_void_p, ctypes.c_float)

_lib = None


def library() -> ctypes.CDLL:
    """Load the HIP shared library (raises GicError if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise GicError(f"{LIB_PATH} missing: run `make -C gfx_imagecompress_amd` "
                       "(or __graft_entry__.build()); there is no CPU fallback")
    lib = ctypes.CDLL(LIB_PATH)
    vp, u32, sz = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_size_t
    lib.gic_hip_encode_rows.argtypes = [ctypes.c_int, vp, u32, u32, u32, u32, sz, u32, u32,
                                        ctypes.POINTER(_COptions), vp, vp, vp]
    lib.gic_hip_encode_rows.restype = ctypes.c_int
    lib.gic_hip_encode_rows_src.argtypes = [ctypes.c_int, ctypes.c_int, vp, u32, u32, u32, u32, sz, u32, u32,
                                            ctypes.POINTER(_COptions), vp, vp, vp]
    lib.gic_hip_encode_rows_src.restype = ctypes.c_int
    lib.gic_hip_encode.argtypes = [ctypes.c_int, vp, u32, u32, u32, u32, sz,
                                   ctypes.POINTER(_COptions), vp, vp, vp]
    lib.gic_hip_encode.restype = ctypes.c_int
    lib.gic_hip_encode_blocks_f32.argtypes = [ctypes.c_int, vp, u32, ctypes.POINTER(_COptions), vp, vp, vp]
    lib.gic_hip_encode_blocks_f32.restype = ctypes.c_int
    lib.gic_hip_encode_blocks_u8.argtypes = [ctypes.c_int, vp, u32, ctypes.POINTER(_COptions), vp, vp]
    lib.gic_hip_encode_blocks_u8.restype = ctypes.c_int
    lib.gic_hip_decode.argtypes = [ctypes.c_int, vp, u32, u32, u32, vp, sz, vp]
    lib.gic_hip_decode.restype = ctypes.c_int
    lib.gic_hip_decode_bc6h.argtypes = [ctypes.c_int, vp, u32, u32, u32, vp, sz, vp]
    lib.gic_hip_decode_bc6h.restype = ctypes.c_int
    lib.gic_decompress_image.argtypes = [vp]
    lib.gic_decompress_image.restype = vp
    lib.gic_save_dds.argtypes = [vp, ctypes.c_char_p]
    lib.gic_save_dds.restype = ctypes.c_int
    lib.gic_default_options.argtypes = [ctypes.POINTER(_COptions)]
    lib.gic_default_options.restype = None
    lib.gic_block_bytes.argtypes = [ctypes.c_int]
    lib.gic_block_bytes.restype = u32
    lib.gic_last_hip_error.restype = ctypes.c_int
    lib.gic_version.restype = ctypes.c_char_p
    lib.gic_iter_cap_hits.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    lib.gic_iter_cap_hits.restype = ctypes.c_int
    lib.gic_set_iter_cap.argtypes = [ctypes.c_int]
    lib.gic_set_iter_cap.restype = ctypes.c_int
    lib.gic_nonterminating_loops.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    lib.gic_nonterminating_loops.restype = ctypes.c_int
    lib.gic_last_h4_report.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32)]
    lib.gic_last_h4_report.restype = ctypes.c_int
    lib.gic_encode_multi.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32,
                                     ctypes.c_uint32, ctypes.c_uint32, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int,
                                     ctypes.POINTER(ctypes.c_int), ctypes.c_void_p, ctypes.c_uint32]
    lib.gic_encode_multi.restype = ctypes.c_int
    lib.gic_multi_last_report.argtypes = [ctypes.POINTER(_MultiReport)]
    lib.gic_multi_last_report.restype = ctypes.c_int
    lib.gic_multi_release.restype = ctypes.c_int
    lib.gic_multi_split.argtypes = [ctypes.c_uint64, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_uint64),
                                    ctypes.POINTER(ctypes.c_uint64)]
    lib.gic_multi_split.restype = ctypes.c_int
    lib.gic_last_bc7_stages.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_int)]
    lib.gic_last_bc7_stages.restype = ctypes.c_int
    lib.gic_last_host_report.argtypes = [ctypes.POINTER(_HostReport)]
    lib.gic_last_host_report.restype = ctypes.c_int
    lib.gic_compress_image.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(_COptions), ctypes.c_void_p,
                                       ctypes.c_void_p]
    lib.gic_compress_image.restype = ctypes.c_void_p
    lib.Image_CreateNoClear.argtypes = [ctypes.c_uint32] * 4 + [ctypes.c_int]
    lib.Image_CreateNoClear.restype = ctypes.c_void_p
    lib.Image_Destroy.argtypes = [ctypes.c_void_p]
    lib.Image_Destroy.restype = None
    for name in ("Image_CompressAMDBC1",):
        getattr(lib, name).argtypes = [ctypes.c_void_p] * 5
        getattr(lib, name).restype = ctypes.c_void_p
    for name in ("Image_CompressAMDBC2", "Image_CompressAMDBC3", "Image_CompressAMDBC7", "Image_CompressAMDBC6H",
                 "Image_CompressRichGel999BC7"):
        getattr(lib, name).argtypes = [ctypes.c_void_p] * 4
        getattr(lib, name).restype = ctypes.c_void_p
    for name in ("Image_CompressAMDBC4", "Image_CompressAMDBC5"):
        getattr(lib, name).argtypes = [ctypes.c_void_p] * 3
        getattr(lib, name).restype = ctypes.c_void_p
    _lib = lib
    return lib


def _check(rc: int) -> None:
    if rc != GIC_OK:
        extra = ""
        if rc == GIC_EHIP:
            extra = f" (hipError {library().gic_last_hip_error()})"
        raise GicError(f"gic call failed: {_ERRS.get(rc, rc)}{extra}")


def iter_cap_hits(reset: bool = False) -> int:
    """Quantiser loops stopped at the iteration cap on the current device
    (gic_iter_cap_hits).  BC7: each stop marks its block, which
    the same call encodes again through the uncapped general path (see
    :func:`last_h4_report`); BC6H: the loop's per-loop cap."""
    n = ctypes.c_ulonglong(0)
    _check(library().gic_iter_cap_hits(ctypes.byref(n), 1 if reset else 0))
    return int(n.value)


def set_iter_cap(cap: int) -> None:
    """The iteration cap (rounds past the never-reset counter's exhaustion;
    < 0 restores the default 4096).  A test hook."""
    _check(library().gic_set_iter_cap(int(cap)))


def nonterminating_loops(reset: bool = False) -> int:
    """Quantiser loops proven cyclic (the reference would never return on
    their blocks) on the current device (gic_nonterminating_loops)."""
    n = ctypes.c_ulonglong(0)
    _check(library().gic_nonterminating_loops(ctypes.byref(n), 1 if reset else 0))
    return int(n.value)


def last_h4_report() -> tuple[int, int]:
    """(blocks re-run after a cap stop, loops proven cyclic) of this thread's
    last BC7 call (gic_last_h4_report)."""
    a, b = ctypes.c_uint32(0), ctypes.c_uint32(0)
    _check(library().gic_last_h4_report(ctypes.byref(a), ctypes.byref(b)))
    return int(a.value), int(b.value)


def encode_multi(fmt: int, image, devices, dst, options: Options | None = None, src_type: int = 0,
                 peer_copy: bool = False) -> dict:
    """gic_encode_multi: the block rows of a host image stack (numpy (S,H,W,C)
    or (H,W,C); uint8, int8 or float32 per ``src_type``) split over ``devices``
    of this process, one gather into ``dst`` (a uint8 tensor on devices[0]).
    Returns the call's report (ranks, rccl, encode_ms_max, gather_ms,
    gathered_bytes)."""
    import numpy as np
    a = np.ascontiguousarray(image)
    if a.ndim == 3:
        a = a[None]
    s, h, w, c = a.shape
    bx, by = blocks_shape(w, h)
    want = {SRC_UNORM8: np.uint8, SRC_SNORM8: np.int8, SRC_FLOAT32: np.float32}.get(src_type)
    if want is None or a.dtype != want:
        raise GicError(f"source type {src_type} needs a {want} image, got {a.dtype}")
    if not dst.is_cuda or dst.numel() * dst.element_size() < bx * by * s * block_bytes(fmt):
        raise GicError("dst must be a device tensor holding the whole image's blocks")
    if not devices or dst.device.index != devices[0]:
        raise GicError(f"dst must live on devices[0] ({devices[0] if devices else None}), not {dst.device}")
    devs = (ctypes.c_int * len(devices))(*devices)
    opts = (options or Options()).to_c()
    rc = library().gic_encode_multi(fmt, src_type, a.ctypes.data, w, h, s, c, w * c * a.itemsize, ctypes.byref(opts),
                                    len(devices), devs, dst.data_ptr(), 1 if peer_copy else 0)
    _check(rc)
    r = _MultiReport()
    _check(library().gic_multi_last_report(ctypes.byref(r)))
    return {"ranks": r.ranks, "rccl": bool(r.rccl), "encode_ms_max": r.encode_ms_max, "gather_ms": r.gather_ms,
            "gathered_bytes": int(r.gathered_bytes)}


# TinyImageFormat of a host source (include/gfx_image/image.h)
_HOST_FORMATS = {("u1", 1): 1, ("i1", 1): 2, ("u1", 2): 3, ("i1", 2): 4, ("u1", 3): 5, ("u1", 4): 7,
                 ("f4", 4): 9}


def _host_header(lib, a):
    """An Image_ImageHeader (library-allocated) holding the (S,H,W,C) array a."""
    s, h, w, c = a.shape
    key = (a.dtype.kind + str(a.dtype.itemsize), c)
    if key not in _HOST_FORMATS:
        raise GicError(f"no host image format for {a.dtype} with {c} channels")
    p = lib.Image_CreateNoClear(w, h, 1, s, _HOST_FORMATS[key])
    if not p:
        raise GicError("Image_CreateNoClear failed")
    ctypes.memmove(_ImageHeader.from_address(p).data, a.ctypes.data, a.nbytes)
    return p


def last_bc7_stages() -> list[int]:
    """Blocks entering each stage of this thread's last BC7 call
    (gic_last_bc7_stages): [all, after the direct mode-6 fit, after the mode-6
    probe, after mode 3, after mode 1, after mode 4] with the bounded exit, [all]
    without."""
    arr, n = (ctypes.c_uint32 * 6)(), ctypes.c_int(0)
    _check(library().gic_last_bc7_stages(arr, ctypes.byref(n)))
    return [int(arr[k]) for k in range(n.value)]


def host_report() -> dict:
    """gic_last_host_report: this thread's last host-image call (devices,
    pieces, h2d_mode, total_ms and the upload / encode / download spans)."""
    r = _HostReport()
    _check(library().gic_last_host_report(ctypes.byref(r)))
    return {k: getattr(r, k) for k, _ in _HostReport._fields_}


class HostImage:
    """A host image (Image_ImageHeader allocated by the library) holding a numpy
    array (H,W,C) or (S,H,W,C), uint8 / int8 / float32 (C = 4 for float), for
    repeated host-path calls.  ``last_call_ms`` is the C call alone (host clock)."""

    def __init__(self, image):
        import numpy as np
        a = np.ascontiguousarray(image)
        if a.ndim == 2:
            a = a[:, :, None]
        if a.ndim == 3:
            a = a[None]
        self.shape = a.shape
        self.ptr = _host_header(library(), a)
        self.last_call_ms = 0.0

    def compress(self, fmt: int, options: Options | None = None, progress=None, entry: str | None = None):
        """``gic_compress_image`` with explicit options, or with ``entry`` one of
        the reference's own wrappers (e.g. ``"Image_CompressAMDBC1"``, NULL
        options).  ``progress``: None or callable(pct) -> bool (True aborts).
        Returns (S,by,bx,bytes) uint8 blocks, or None when aborted."""
        import time
        import numpy as np
        lib = library()
        s, h, w, _ = self.shape
        bx, by = blocks_shape(w, h)
        cb = PROGRESS_FUNC(lambda user, pct: bool(progress(pct))) if progress else None
        cbp = ctypes.cast(cb, ctypes.c_void_p) if cb else None
        opts = (options or Options()).to_c()
        t0 = time.perf_counter()
        if entry is None:
            out = lib.gic_compress_image(self.ptr, fmt, ctypes.byref(opts), cbp, None)
        else:
            fn = getattr(lib, entry)
            extra = {5: [None, None], 4: [None], 3: []}[len(fn.argtypes)]
            out = fn(self.ptr, *extra, cbp, None)
        self.last_call_ms = (time.perf_counter() - t0) * 1e3
        if not out:
            return None
        hd = _ImageHeader.from_address(out)
        blocks = np.ctypeslib.as_array((ctypes.c_uint8 * hd.dataSize).from_address(hd.data)).copy()
        lib.Image_Destroy(out)
        return blocks.reshape(s, by, bx, -1)

    def close(self):
        if self.ptr:
            library().Image_Destroy(self.ptr)
            self.ptr = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def compress_host(fmt: int, image, options: Options | None = None, progress=None, entry: str | None = None):
    """The host-image path (host image in, host blocks out) through the C ABI,
    one call: see :class:`HostImage`.  The call's timing is :func:`host_report`."""
    with HostImage(image) as hi:
        return hi.compress(fmt, options, progress, entry)


def multi_split(rows_total: int, ndev: int, i: int) -> tuple[int, int]:
    """(first slice-major block row, rows) of device i in gic_encode_multi."""
    a, b = ctypes.c_uint64(0), ctypes.c_uint64(0)
    _check(library().gic_multi_split(rows_total, ndev, i, ctypes.byref(a), ctypes.byref(b)))
    return int(a.value), int(b.value)


def block_bytes(fmt: int) -> int:
    return 8 if fmt in (FMT_BC1, FMT_BC4) else 16


def blocks_shape(width: int, height: int) -> tuple[int, int]:
    """(block columns, block rows) of an image, edge blocks included."""
    return (width + 3) // 4, (height + 3) // 4


def _stream_handle(stream) -> int | None:
    if stream is None:
        import torch
        return torch.cuda.current_stream().cuda_stream
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream


def encode_device(fmt: int, src, width: int, height: int, slices: int, channels: int, dst,
                  options: Options | None = None, first_block_row: int = 0,
                  num_block_rows: int | None = None, block_err=None, stream=None,
                  row_pitch: int | None = None) -> None:
    """Asynchronously encode an 8-bit image stack resident in HBM.

    src: uint8 CUDA tensor holding ``slices*height`` rows of ``row_pitch`` bytes.
    dst: uint8 CUDA tensor receiving ``bx*num_block_rows*slices`` blocks.
    Launched on ``stream`` (default: torch's current stream).
    """
    import torch
    if not (src.is_cuda and dst.is_cuda):
        raise GicError("encode_device needs device (HBM) tensors; there is no CPU path")
    bx, by = blocks_shape(width, height)
    nrows = by - first_block_row if num_block_rows is None else num_block_rows
    pitch = width * channels if row_pitch is None else row_pitch
    need = bx * nrows * slices * block_bytes(fmt)
    if dst.numel() * dst.element_size() < need:
        raise GicError(f"dst too small: {dst.numel() * dst.element_size()} < {need}")
    if src.numel() * src.element_size() < pitch * height * slices:
        raise GicError("src too small for the given shape")
    if block_err is not None and (block_err.dtype != torch.float64 or block_err.numel() < bx * nrows * slices):
        raise GicError("block_err must be float64 with one entry per block")
    opts = (options or Options()).to_c()
    rc = library().gic_hip_encode_rows(fmt, src.data_ptr(), width, height, slices, channels, pitch,
                                       first_block_row, nrows, ctypes.byref(opts), dst.data_ptr(),
                                       block_err.data_ptr() if block_err is not None else None,
                                       _stream_handle(stream))
    _check(rc)


SRC_UNORM8, SRC_SNORM8, SRC_FLOAT32 = 0, 1, 2


def encode_device_src(fmt: int, src_type: int, src, width: int, height: int, slices: int, channels: int, dst,
                      options: Options | None = None, first_block_row: int = 0, num_block_rows: int | None = None,
                      block_err=None, stream=None) -> None:
    """gic_hip_encode_rows_src: like :func:`encode_device` for SNORM8 (int8
    tensor) or FLOAT32 (float32 tensor) sources, rows packed without padding."""
    import torch
    if not (src.is_cuda and dst.is_cuda):
        raise GicError("encode_device_src needs device (HBM) tensors; there is no CPU path")
    want = {SRC_UNORM8: torch.uint8, SRC_SNORM8: torch.int8, SRC_FLOAT32: torch.float32}[src_type]
    if src.dtype != want or not src.is_contiguous():
        raise GicError(f"source must be a contiguous {want} tensor for source type {src_type}")
    bx, by = blocks_shape(width, height)
    nrows = by - first_block_row if num_block_rows is None else num_block_rows
    if src.numel() < width * height * slices * channels:
        raise GicError("src too small for the given shape")
    if dst.numel() * dst.element_size() < bx * nrows * slices * block_bytes(fmt):
        raise GicError("dst too small")
    if block_err is not None and (block_err.dtype != torch.float64 or block_err.numel() < bx * nrows * slices):
        raise GicError("block_err must be float64 with one entry per block")
    opts = (options or Options()).to_c()
    rc = library().gic_hip_encode_rows_src(fmt, src_type, src.data_ptr(), width, height, slices, channels,
                                           width * channels * src.element_size(), first_block_row, nrows,
                                           ctypes.byref(opts), dst.data_ptr(),
                                           block_err.data_ptr() if block_err is not None else None,
                                           _stream_handle(stream))
    _check(rc)


def encode_blocks_f32(fmt: int, blocks, dst, options: Options | None = None, block_err=None, stream=None) -> None:
    """Block-level batch: blocks is a float32 CUDA tensor (n,64) for BC1/BC2/BC3/BC7 or (n,16) for BC4.

    The batched form of ``Image_CompressAMDBC1Block`` / ``Image_CompressAMDAlphaSingleModeBlock`` /
    ``Image_CompressAMDMultiModeLDRBlock`` (reference imagecompress.h:117-136).
    """
    import torch
    if fmt not in (FMT_BC1, FMT_BC2, FMT_BC3, FMT_BC4, FMT_BC6H, FMT_BC6H_SF, FMT_BC7, FMT_BC7ENC16):
        raise GicError(f"encode_blocks_f32: format {fmt} has no block-level entry "
                       f"(BC1, BC2, BC3, BC4, BC6H, BC6H_SF, BC7, BC7ENC16)")
    if not (blocks.is_cuda and dst.is_cuda):
        raise GicError("encode_blocks_f32 needs device (HBM) tensors; there is no CPU path")
    if blocks.dtype != torch.float32 or not blocks.is_contiguous():
        raise GicError("blocks must be a contiguous float32 tensor")
    per = 16 if fmt == FMT_BC4 else 64
    if blocks.dim() != 2 or blocks.shape[1] != per:
        raise GicError(f"blocks must have shape (n, {per}) for format {fmt}, got {tuple(blocks.shape)}")
    n = blocks.shape[0]
    if n == 0:
        return
    if not dst.is_contiguous() or dst.numel() * dst.element_size() < n * block_bytes(fmt):
        raise GicError(f"dst too small or not contiguous: need {n * block_bytes(fmt)} bytes")
    if block_err is not None and (not block_err.is_cuda or block_err.dtype != torch.float64
                                  or not block_err.is_contiguous() or block_err.numel() < n):
        raise GicError("block_err must be a contiguous float64 device tensor with one entry per block")
    opts = (options or Options()).to_c()
    rc = library().gic_hip_encode_blocks_f32(fmt, blocks.data_ptr(), n, ctypes.byref(opts), dst.data_ptr(),
                                             block_err.data_ptr() if block_err is not None else None,
                                             _stream_handle(stream))
    _check(rc)


def encode_blocks_u8(blocks, dst, options: Options | None = None, stream=None) -> None:
    """bc7enc16 at its block ABI (``Image_CompressRichGel999BC7enc16``, reference
    imagecompress.h:139-142): blocks is a uint8 CUDA tensor (n, 64) of RGBA8
    texels (or int32/uint32 (n, 16) packed words); dst receives n 16-byte BC7 blocks."""
    import torch
    if not (blocks.is_cuda and dst.is_cuda):
        raise GicError("encode_blocks_u8 needs device (HBM) tensors; there is no CPU path")
    if not blocks.is_contiguous() or blocks.dim() != 2 or blocks.numel() * blocks.element_size() != blocks.shape[0] * 64:
        raise GicError("blocks must be a contiguous (n, 64) uint8 or (n, 16) 32-bit tensor")
    n = blocks.shape[0]
    if n == 0:
        return
    if not dst.is_contiguous() or dst.numel() * dst.element_size() < n * 16:
        raise GicError(f"dst too small or not contiguous: need {n * 16} bytes")
    opts = (options or Options()).to_c()
    _check(library().gic_hip_encode_blocks_u8(FMT_BC7ENC16, blocks.data_ptr(), n, ctypes.byref(opts),
                                              dst.data_ptr(), _stream_handle(stream)))


def decode_device(fmt: int, blocks, width: int, height: int, slices: int, out, row_pitch: int | None = None,
                  stream=None) -> None:
    """Asynchronously decode BCn blocks (uint8 CUDA tensor, row-major per slice)
    into ``out`` (uint8 CUDA tensor of slices*height rows of row_pitch bytes,
    RGBA8) -- gic_hip_decode."""
    if not (blocks.is_cuda and out.is_cuda):
        raise GicError("decode_device needs device (HBM) tensors; there is no CPU path")
    bx, by = blocks_shape(width, height)
    if blocks.numel() * blocks.element_size() < bx * by * slices * block_bytes(fmt):
        raise GicError("blocks tensor too small for the given shape")
    pitch = width * 4 if row_pitch is None else row_pitch
    if not out.is_contiguous() or out.numel() * out.element_size() < pitch * height * slices:
        raise GicError("out tensor too small for the given shape")
    _check(library().gic_hip_decode(fmt, blocks.data_ptr(), width, height, slices, out.data_ptr(), pitch,
                                    _stream_handle(stream)))


def decode_bc6h_device(fmt: int, blocks, width: int, height: int, slices: int, out, row_pitch: int | None = None,
                       stream=None) -> None:
    """Asynchronously decode BC6H blocks (uint8 CUDA tensor) into ``out`` (a CUDA
    tensor of slices*height rows of row_pitch bytes, 4 half floats per texel,
    alpha 1.0) -- gic_hip_decode_bc6h."""
    if not (blocks.is_cuda and out.is_cuda):
        raise GicError("decode_bc6h_device needs device (HBM) tensors; there is no CPU path")
    bx, by = blocks_shape(width, height)
    if blocks.numel() * blocks.element_size() < bx * by * slices * 16:
        raise GicError("blocks tensor too small for the given shape")
    pitch = width * 8 if row_pitch is None else row_pitch
    if not out.is_contiguous() or out.numel() * out.element_size() < pitch * height * slices:
        raise GicError("out tensor too small for the given shape")
    _check(library().gic_hip_decode_bc6h(fmt, blocks.data_ptr(), width, height, slices, out.data_ptr(), pitch,
                                         _stream_handle(stream)))


def _host_compress(fmt: int, image, options: Options):
    """numpy (H,W,C) or (S,H,W,C) uint8 -> numpy uint8 blocks (S,by,bx,bytes)."""
    import numpy as np
    import torch
    a = np.ascontiguousarray(image)
    if a.dtype != np.uint8:
        raise GicError("8-bit sources only")
    if a.ndim == 2:
        a = a[:, :, None]
    if a.ndim == 3:
        a = a[None]
    s, h, w, c = a.shape
    bx, by = blocks_shape(w, h)
    dev = torch.device("cuda", torch.cuda.current_device())
    src = torch.from_numpy(a).to(dev)
    dst = torch.empty(bx * by * s * block_bytes(fmt), dtype=torch.uint8, device=dev)
    encode_device(fmt, src, w, h, s, c, dst, options)
    torch.cuda.synchronize()
    return dst.cpu().numpy().reshape(s, by, bx, block_bytes(fmt))


def compress_bc1(image, options: Options | None = None):
    """Image_CompressAMDBC1 (amd_bc1_compressor.cpp:11-71) on a host array."""
    o = options or Options()
    if image.ndim >= 3 and image.shape[-1] < 4:
        o = replace(o, force_alpha_one=True)   # the caller's Options stay untouched
    return _host_compress(FMT_BC1, image, o)


def compress_bc2(image, options: Options | None = None):
    """Image_CompressAMDBC2 (amd_bc2_compressor.cpp:11-58): explicit alpha + 4-colour RGB."""
    o = options or Options()
    if image.ndim >= 3 and image.shape[-1] < 4:
        o = replace(o, force_alpha_one=True)
    return _host_compress(FMT_BC2, image, o)


def compress_bc3(image, options: Options | None = None):
    """Image_CompressAMDBC3 (amd_bc3_compressor.cpp:11-58): interpolated alpha + 4-colour RGB."""
    o = options or Options()
    if image.ndim >= 3 and image.shape[-1] < 4:
        o = replace(o, force_alpha_one=True)
    return _host_compress(FMT_BC3, image, o)


def compress_bc4(image, options: Options | None = None):
    """Image_CompressAMDBC4 (amd_bc4_compressor.cpp:11-50): channel 1 by default."""
    return _host_compress(FMT_BC4, image, options or Options())


def compress_bc5(image, options: Options | None = None):
    """Image_CompressAMDBC5 (amd_bc5_compressor.cpp:11-56)."""
    return _host_compress(FMT_BC5, image, options or Options())


def compress_bc7(image, options: Options | None = None):
    """Image_CompressAMDBC7 (amd_bc7_compressor.cpp:25-81)."""
    o = options or Options()
    if image.ndim >= 3 and image.shape[-1] < 4:
        o = replace(o, force_alpha_one=True)
    return _host_compress(FMT_BC7, image, o)


def compress_bc6h(image, signed: bool = False):
    """Image_CompressAMDBC6H (amd_bc6h_compressor.cpp:11-56) on a host float32
    array (H,W,C) or (S,H,W,C): BC6H unsigned (signed=False, DXBC6H_UFLOAT) or
    signed (the encoder's path for signed sources, DXBC6H_SFLOAT).  Returns
    (S,by,bx,16) uint8 blocks."""
    import numpy as np
    import torch
    a = np.ascontiguousarray(image, dtype=np.float32)
    if a.ndim == 2:
        a = a[:, :, None]
    if a.ndim == 3:
        a = a[None]
    s, h, w, c = a.shape
    bx, by = blocks_shape(w, h)
    dev = torch.device("cuda", torch.cuda.current_device())
    src = torch.from_numpy(a).to(dev)
    dst = torch.empty(bx * by * s * 16, dtype=torch.uint8, device=dev)
    encode_device_src(FMT_BC6H_SF if signed else FMT_BC6H, SRC_FLOAT32, src.reshape(-1), w, h, s, c, dst,
                      Options(force_alpha_one=c < 4))
    torch.cuda.synchronize()
    return dst.cpu().numpy().reshape(s, by, bx, 16)


def compress_bc7_fast(image, options: Options | None = None):
    """Image_CompressRichGel999BC7 (richgel999_bc7enc16.cpp:21-71): bc7enc16 with
    the image API's defaults (perceptual, uber level 4) unless options say otherwise."""
    o = options or Options()
    if image.ndim >= 3 and image.shape[-1] < 4:
        o = replace(o, force_alpha_one=True)
    return _host_compress(FMT_BC7ENC16, image, o)
