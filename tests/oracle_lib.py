"""ctypes binding of the CPU restatement (oracle/liboracle_bcn.so).

TEST INFRASTRUCTURE ONLY: tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg are the only users; the product never loads the oracle.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "liboracle_bcn.so")

_lib = None


def build() -> str:
    if not os.path.exists(ORACLE_SO):
        subprocess.run(["make", "-C", ORACLE_DIR, "-s"], check=True)
    return ORACLE_SO


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        _lib = ctypes.CDLL(build())
        vp = ctypes.c_void_p
        _lib.orc_encode_image.argtypes = [ctypes.c_int, vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                          ctypes.c_uint32, ctypes.c_int, ctypes.c_int32, ctypes.c_int32,
                                          ctypes.c_int, vp, vp]
        _lib.orc_encode_image.restype = ctypes.c_int
        _lib.orc_encode_image_bc7.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                              ctypes.c_int32, ctypes.c_int32, ctypes.c_int, ctypes.c_float,
                                              ctypes.c_uint8, vp, vp]
        _lib.orc_encode_image_bc7.restype = ctypes.c_int
        _lib.orc_encode_image_bc7_ex.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                                 ctypes.c_uint32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int,
                                                 ctypes.c_float, ctypes.c_uint8, ctypes.c_int, vp, vp]
        _lib.orc_encode_image_bc7_ex.restype = ctypes.c_int
        _lib.orc_encode_image_bc7_perf.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                                   ctypes.c_uint32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int,
                                                   ctypes.c_float, ctypes.c_uint8, ctypes.c_float, vp, vp]
        _lib.orc_encode_image_bc7_perf.restype = ctypes.c_int
        _lib.orc_bc7_opt_quant_trace.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp, ctypes.c_int]
        _lib.orc_bc7_opt_quant_trace.restype = ctypes.c_double
        _lib.orc_bc7_opt_quant.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp, ctypes.c_int]
        _lib.orc_bc7_opt_quant.restype = ctypes.c_double
        _lib.orc_bc7_trace_len.argtypes = [ctypes.c_int, ctypes.c_int]
        _lib.orc_bc7_trace_len.restype = ctypes.c_int
        _lib.orc_bc1_block.argtypes = [vp, ctypes.c_int, ctypes.c_float, vp]
        _lib.orc_bc4_block.argtypes = [vp, vp]
        _lib.orc_rgb4_block.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp]
        _lib.orc_bc1_block_ex.argtypes = [vp, ctypes.c_int, ctypes.c_float, ctypes.c_int, vp]
        _lib.orc_explicit_alpha_block.argtypes = [vp, vp]
        _lib.orc_bc7_block.argtypes = [vp, ctypes.c_uint8, ctypes.c_int, ctypes.c_float, ctypes.c_int,
                                       ctypes.c_int, ctypes.c_float, vp]
        _lib.orc_bc7_block.restype = ctypes.c_double
        _lib.orc_bc7_block_ex.argtypes = [vp, ctypes.c_uint8, ctypes.c_int, ctypes.c_float, ctypes.c_int,
                                          ctypes.c_int, ctypes.c_float, ctypes.c_int, vp]
        _lib.orc_bc7_block_ex.restype = ctypes.c_double
        _lib.orc_fnv1a64.argtypes = [vp, ctypes.c_size_t]
        _lib.orc_fnv1a64.restype = ctypes.c_uint64
        _lib.orc_bc7_shake_ramp.argtypes = [ctypes.c_int] * 5
        _lib.orc_bc7_shake_ramp.restype = ctypes.c_int
        _lib.orc_bc7_decode.argtypes = [vp, vp]
        _lib.orc_bc7_decode_n.argtypes = [vp, ctypes.c_size_t, vp]
        _lib.orc_bc7enc_block.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp]
        _lib.orc_encode_image_bc7enc.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                                 ctypes.c_uint32, ctypes.c_int, ctypes.c_int, vp]
        _lib.orc_encode_image_bc7enc.restype = ctypes.c_int
        _lib.orc_encode_image_bc7enc_rows.argtypes = [vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                                      ctypes.c_uint32, ctypes.c_int32, ctypes.c_int32, ctypes.c_int,
                                                      ctypes.c_int, ctypes.c_int, vp]
        _lib.orc_encode_image_bc7enc_rows.restype = ctypes.c_int
        _lib.orc_bc7_set_probe_init.argtypes = [ctypes.c_int]
        _lib.orc_bc7_set_probe_init.restype = None
        _lib.orc_bc7_fit6.argtypes = [vp, vp]
        _lib.orc_bc7_fit6.restype = ctypes.c_double
        _lib.orc_encode_bc6h_blocks.argtypes = [vp, ctypes.c_int, ctypes.c_int, ctypes.c_int, vp, vp]
        _lib.orc_encode_bc6h_blocks.restype = ctypes.c_int
        _lib.orc_bc6h_block.argtypes = [vp, ctypes.c_int, vp]
        _lib.orc_bc6h_block.restype = ctypes.c_float
        _lib.orc_bc6h_set_cap.argtypes = [ctypes.c_int]
        _lib.orc_bc6h_set_cap.restype = None
        _lib.orc_bc6h_h4_counts.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.POINTER(ctypes.c_ulonglong)]
        _lib.orc_bc6h_h4_counts.restype = None
        _lib.orc_float_to_half.argtypes = [ctypes.c_float]
        _lib.orc_float_to_half.restype = ctypes.c_uint16
        _lib.orc_bc6h_anchor.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
        _lib.orc_bc6h_anchor.restype = ctypes.c_int
        _lib.orc_bc6h_ev_p.restype = ctypes.c_int
        _lib.orc_bc6h_pattern.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp, vp, vp]
        _lib.orc_bc6h_pattern.restype = ctypes.c_float
    return _lib


def block_bytes(fmt: int) -> int:
    return 8 if fmt in (1, 4) else 16


def encode_image(fmt: int, img: np.ndarray, bc4_channel: int = 1, first_row: int = -1, num_rows: int = -1,
                 threads: int = 0, want_err: bool = False):
    """img: (H,W,C) or (S,H,W,C) uint8.  Returns uint8 blocks (S*rows*bx, bytes) [, errors]."""
    a = np.ascontiguousarray(img, dtype=np.uint8)
    if a.ndim == 2:
        a = a[:, :, None]
    if a.ndim == 3:
        a = a[None]
    s, h, w, c = a.shape
    bx, by = (w + 3) // 4, (h + 3) // 4
    rows = by - max(first_row, 0) if num_rows < 0 else num_rows
    out = np.zeros((s * rows * bx, block_bytes(fmt)), np.uint8)
    err = np.zeros(s * rows * bx, np.float64) if want_err else None
    threads = threads or min(os.cpu_count() or 1, 16)
    rc = lib().orc_encode_image(fmt, a.ctypes.data, w, h, s, c, bc4_channel, first_row, num_rows, threads,
                                out.ctypes.data, err.ctypes.data if want_err else None)
    if rc != 0:
        raise RuntimeError(f"oracle encode failed ({rc})")
    return (out, err) if want_err else out


def encode_image_bc7(img: np.ndarray, quality: float = 1.0, mode_mask: int = 0xFF, first_row: int = -1,
                     num_rows: int = -1, threads: int = 0, want_err: bool = False, shake_ranks: int = 0,
                     performance: float = 1.0):
    """BC7 over an image with the encoder quality / ModeMask of the block API;
    shake_ranks > 0 models the GPU's pruned search (gic_options.bc7_shake_ranks)."""
    a = np.ascontiguousarray(img, dtype=np.uint8)
    if a.ndim == 2:
        a = a[:, :, None]
    if a.ndim == 3:
        a = a[None]
    s, h, w, c = a.shape
    bx, by = (w + 3) // 4, (h + 3) // 4
    rows = by - max(first_row, 0) if num_rows < 0 else num_rows
    out = np.zeros((s * rows * bx, 16), np.uint8)
    err = np.zeros(s * rows * bx, np.float64) if want_err else None
    threads = threads or min(os.cpu_count() or 1, 16)
    if performance != 1.0:
        if shake_ranks:
            raise ValueError("the oracle models performance < 1 with the reference search only")
        rc = lib().orc_encode_image_bc7_perf(a.ctypes.data, w, h, s, c, first_row, num_rows, threads, quality,
                                             mode_mask, performance, out.ctypes.data,
                                             err.ctypes.data if want_err else None)
    else:
        rc = lib().orc_encode_image_bc7_ex(a.ctypes.data, w, h, s, c, first_row, num_rows, threads, quality,
                                           mode_mask, shake_ranks, out.ctypes.data,
                                           err.ctypes.data if want_err else None)
    if rc != 0:
        raise RuntimeError(f"oracle encode failed ({rc})")
    return (out, err) if want_err else out


def bc1_block(block: np.ndarray, steps: int = 1, threshold: float = 128 / 255.0, b3d: bool = False) -> bytes:
    b = np.ascontiguousarray(block, dtype=np.float32).reshape(64)
    out = np.zeros(8, np.uint8)
    lib().orc_bc1_block_ex(b.ctypes.data, steps, threshold, int(b3d), out.ctypes.data)
    return out.tobytes()


def bc4_block(values: np.ndarray) -> bytes:
    v = np.ascontiguousarray(values, dtype=np.float32).reshape(16)
    out = np.zeros(8, np.uint8)
    lib().orc_bc4_block(v.ctypes.data, out.ctypes.data)
    return out.tobytes()


def bc23_block(fmt: int, block: np.ndarray, steps: int = 1, b3d: bool = False) -> bytes:
    """BC2 (fmt 2) / BC3 (fmt 3) block from 16 RGBA float texels: alpha half, colour half."""
    b = np.ascontiguousarray(block, dtype=np.float32).reshape(64)
    a = np.ascontiguousarray(b.reshape(16, 4)[:, 3])
    out = np.zeros(16, np.uint8)
    if fmt == 3:
        lib().orc_bc4_block(a.ctypes.data, out.ctypes.data)
    else:
        lib().orc_explicit_alpha_block(a.ctypes.data, out.ctypes.data)
    col = np.zeros(8, np.uint8)
    lib().orc_rgb4_block(b.ctypes.data, steps, int(b3d), col.ctypes.data)
    out[8:] = col
    return out.tobytes()


def bc7_block(block: np.ndarray, mode_mask: int = 0xFF):
    b = np.ascontiguousarray(block, dtype=np.float32).reshape(64)
    out = np.zeros(16, np.uint8)
    e = lib().orc_bc7_block(b.ctypes.data, mode_mask, 1, 1.0, 1, 1, 1.0, out.ctypes.data)
    return out.tobytes(), e


def bc7_blocks_ex(blocks: np.ndarray, mode_mask: int = 0xFF, colour_restrict: bool = True, shake_ranks: int = 0,
                  has_alpha: bool = True) -> np.ndarray:
    """orc_bc7_block_ex over (n, 16, 4) uint8 blocks (texels as v / 255.0f, the
    image driver's conversion), with the encoder's colour restriction and the
    GPU's shake-rank cap selectable."""
    b = np.ascontiguousarray(blocks, dtype=np.uint8).reshape(-1, 64)
    out = np.zeros((b.shape[0], 16), np.uint8)
    for k in range(b.shape[0]):
        f = (b[k].astype(np.float32) / np.float32(255.0)).astype(np.float32)
        lib().orc_bc7_block_ex(f.ctypes.data, mode_mask, int(has_alpha), 1.0, int(colour_restrict), 1, 1.0,
                               shake_ranks, out[k].ctypes.data)
    return out


def bc7_fit6_blocks(blocks: np.ndarray) -> tuple[np.ndarray, np.ndarray]:
    """orc_bc7_fit6 (the bounded exit's direct mode-6 fit, gic_bc7.hip k_fit6)
    over (n, 16, 4) uint8 blocks: (packed blocks, palette squared errors)."""
    b = np.ascontiguousarray(blocks, dtype=np.uint8).reshape(-1, 64)
    out = np.zeros((b.shape[0], 16), np.uint8)
    err = np.zeros(b.shape[0])
    for k in range(b.shape[0]):
        f = (b[k].astype(np.float32) / np.float32(255.0)).astype(np.float32)
        err[k] = lib().orc_bc7_fit6(f.ctypes.data, out[k].ctypes.data)
    return out, err


def encode_image_bc7enc(img: np.ndarray, fast: bool = False, perceptual: bool = True) -> np.ndarray:
    """bc7enc16 over an 8-bit image (Image_CompressRichGel999BC7's block loop)."""
    a = np.ascontiguousarray(img, dtype=np.uint8)
    if a.ndim == 2:
        a = a[:, :, None]
    if a.ndim == 3:
        a = a[None]
    s, h, w, c = a.shape
    out = np.zeros((s * ((h + 3) // 4) * ((w + 3) // 4), 16), np.uint8)
    if lib().orc_encode_image_bc7enc(a.ctypes.data, w, h, s, c, int(fast), int(perceptual), out.ctypes.data) != 0:
        raise RuntimeError("oracle bc7enc16 encode failed")
    return out


def encode_image_bc7enc_rows(img: np.ndarray, first_row: int, num_rows: int, threads: int = 0, fast: bool = False,
                             perceptual: bool = True) -> np.ndarray:
    """bc7enc16 on a block-row range through the oracle's thread pool (CPU baseline)."""
    a = np.ascontiguousarray(img, dtype=np.uint8)
    if a.ndim == 3:
        a = a[None]
    s, h, w, c = a.shape
    out = np.zeros((s * num_rows * ((w + 3) // 4), 16), np.uint8)
    threads = threads or min(os.cpu_count() or 1, 16)
    if lib().orc_encode_image_bc7enc_rows(a.ctypes.data, w, h, s, c, first_row, num_rows, threads, int(fast),
                                          int(perceptual), out.ctypes.data) != 0:
        raise RuntimeError("oracle bc7enc16 encode failed")
    return out


def bc7enc_blocks(rgba: np.ndarray, fast: bool = False, perceptual: bool = True) -> np.ndarray:
    """bc7enc16 on (n, 16, 4) uint8 blocks (Image_CompressRichGel999BC7enc16)."""
    b = np.ascontiguousarray(rgba, dtype=np.uint8).reshape(-1, 64)
    out = np.zeros((b.shape[0], 16), np.uint8)
    for i in range(b.shape[0]):
        lib().orc_bc7enc_block(b[i].ctypes.data, int(fast), int(perceptual), out[i].ctypes.data)
    return out


def bc6h_blocks(blocks: np.ndarray, signed: bool = False, threads: int = 0):
    """BC6HBlockEncoder::CompressBlock (quality 1.0) on (n, 64) float RGBA blocks:
    ((n, 16) uint8 blocks, (n,) float32 encoder errors)."""
    b = np.ascontiguousarray(blocks, dtype=np.float32).reshape(-1, 64)
    out = np.zeros((b.shape[0], 16), np.uint8)
    err = np.zeros(b.shape[0], np.float32)
    threads = threads or min(os.cpu_count() or 1, 16)
    lib().orc_encode_bc6h_blocks(b.ctypes.data, b.shape[0], int(signed), threads, out.ctypes.data, err.ctypes.data)
    return out, err


def bc6h_set_cap(cap: int) -> None:
    """The oracle's per-loop H4 cap of optQuantAnD_f (< 0 = the default 4096)."""
    lib().orc_bc6h_set_cap(int(cap))


def bc6h_h4_counts() -> tuple[int, int]:
    """Cumulative (proven cycles, cap stops) of the oracle's BC6H quantiser loops."""
    a, b = ctypes.c_ulonglong(0), ctypes.c_ulonglong(0)
    lib().orc_bc6h_h4_counts(ctypes.byref(a), ctypes.byref(b))
    return int(a.value), int(b.value)


def bc7_decode(blocks: np.ndarray) -> np.ndarray:
    """(n,16) uint8 -> (n,16,4) uint8 RGBA."""
    b = np.ascontiguousarray(blocks, dtype=np.uint8).reshape(-1, 16)
    out = np.zeros((b.shape[0], 16, 4), np.uint8)
    lib().orc_bc7_decode_n(b.ctypes.data, b.shape[0], out.ctypes.data)
    return out


def fnv1a64(data: np.ndarray) -> int:
    a = np.ascontiguousarray(data).view(np.uint8)
    return int(lib().orc_fnv1a64(a.ctypes.data, a.size))
