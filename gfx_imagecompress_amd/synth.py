"""Synthetic texture generators shared by tests and bench.py.

G0: RGBA8 gradient, R = x*255/(W-1), G = y*255/(H-1), B = (x+y)*255/(W+H-2),
    A = 255 (integer division; for 256x256 this is the survey's G0 exactly).
G1: G0 plus per-pixel noise n in [-8, 8] added to R, G and B, clamped.  The
    noise is a counter-based hash of the pixel index so it can be generated
    in parallel on the host (numpy) or on the device (torch) identically.
HEIGHT / NORMAL: value-noise height field (R8) and its central-difference
    normal map (RG8) for the BC4/BC5 configuration.
All generators return arrays shaped (H, W, C) or (S, H, W, C).
"""
from __future__ import annotations

import numpy as np

_M32 = 0xFFFFFFFF


def _mix32(x):
    """lowbias32 integer hash (works on numpy uint64 or torch int64 arrays)."""
    x = x & _M32
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & _M32
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & _M32
    x = x ^ (x >> 16)
    return x


def g0(width: int, height: int) -> np.ndarray:
    y, x = np.mgrid[0:height, 0:width].astype(np.int64)
    img = np.empty((height, width, 4), np.uint8)
    img[..., 0] = x * 255 // max(width - 1, 1)
    img[..., 1] = y * 255 // max(height - 1, 1)
    img[..., 2] = (x + y) * 255 // max(width + height - 2, 1)
    img[..., 3] = 255
    return img


def g1(width: int, height: int, seed: int = 0x9E3779B9) -> np.ndarray:
    img = g0(width, height).astype(np.int64)
    idx = np.arange(width * height, dtype=np.uint64).reshape(height, width)
    n = (_mix32(idx ^ np.uint64(seed)).astype(np.int64) % 17) - 8
    img[..., :3] += n[..., None]
    return np.clip(img, 0, 255).astype(np.uint8)


def g1_torch(width: int, height: int, slices: int = 1, seed: int = 0x9E3779B9, device="cuda"):
    """Device-side G1 (bit-identical to :func:`g1` per slice; slice s uses seed+s)."""
    import torch
    y = torch.arange(height, device=device, dtype=torch.int64).view(height, 1)
    x = torch.arange(width, device=device, dtype=torch.int64).view(1, width)
    out = torch.empty((slices, height, width, 4), dtype=torch.uint8, device=device)
    r = x * 255 // max(width - 1, 1)
    g = y * 255 // max(height - 1, 1)
    b = (x + y) * 255 // max(width + height - 2, 1)
    idx = y * width + x
    for s in range(slices):
        n = (_mix32(idx ^ ((seed + s) & _M32)) % 17) - 8
        out[s, ..., 0] = (r + n).clamp(0, 255).to(torch.uint8)
        out[s, ..., 1] = (g + n).clamp(0, 255).to(torch.uint8)
        out[s, ..., 2] = (b + n).clamp(0, 255).to(torch.uint8)
        out[s, ..., 3] = 255
    return out


def g2(width: int, height: int, seed: int = 0x9E3779B9) -> np.ndarray:
    """G0 plus independent noise per channel: n_c in [-8, 8] for R, G, B from
    three hashes of the pixel index.  G1's single n moves a texel along the grey
    axis, so its blocks stay nearly collinear; G2's noise is isotropic in RGB,
    a harder case for BC7's line fits (the bounded exit's second content)."""
    img = g0(width, height).astype(np.int64)
    idx = np.arange(width * height, dtype=np.uint64).reshape(height, width)
    for c in range(3):
        key = np.uint64((seed + 0x632BE5AB * (c + 1)) & _M32)
        img[..., c] += (_mix32(idx ^ key).astype(np.int64) % 17) - 8
    return np.clip(img, 0, 255).astype(np.uint8)


def g2_torch(width: int, height: int, seed: int = 0x9E3779B9, device="cuda"):
    """Device-side G2 (bit-identical to :func:`g2`), shape (1, H, W, 4)."""
    import torch
    y = torch.arange(height, device=device, dtype=torch.int64).view(height, 1)
    x = torch.arange(width, device=device, dtype=torch.int64).view(1, width)
    base = (x * 255 // max(width - 1, 1), y * 255 // max(height - 1, 1),
            (x + y) * 255 // max(width + height - 2, 1))
    idx = y * width + x
    out = torch.empty((1, height, width, 4), dtype=torch.uint8, device=device)
    for c in range(3):
        n = (_mix32(idx ^ ((seed + 0x632BE5AB * (c + 1)) & _M32)) % 17) - 8
        out[0, ..., c] = (base[c] + n).clamp(0, 255).to(torch.uint8)
    out[0, ..., 3] = 255
    return out


def noise_rgba(width: int, height: int, seed: int = 1, alpha: bool = False) -> np.ndarray:
    rng = np.random.default_rng(seed)
    img = rng.integers(0, 256, size=(height, width, 4), dtype=np.uint8)
    if not alpha:
        img[..., 3] = 255
    return img


def height_field(width: int, height: int, seed: int = 1, octaves: int = 5) -> np.ndarray:
    """Value-noise fBm height map, quantised to uint8 (H, W)."""
    rng = np.random.default_rng(seed)
    acc = np.zeros((height, width), np.float64)
    amp, total = 1.0, 0.0
    for o in range(octaves):
        cells = 4 << o
        grid = rng.random((cells + 1, cells + 1))
        ys = np.linspace(0, cells, height, endpoint=False)
        xs = np.linspace(0, cells, width, endpoint=False)
        y0 = ys.astype(np.int64)
        x0 = xs.astype(np.int64)
        fy = (ys - y0)[:, None]
        fx = (xs - x0)[None, :]
        fy = fy * fy * (3 - 2 * fy)
        fx = fx * fx * (3 - 2 * fx)
        a = grid[y0][:, x0]
        b = grid[y0][:, x0 + 1]
        c = grid[y0 + 1][:, x0]
        d = grid[y0 + 1][:, x0 + 1]
        acc += amp * ((a * (1 - fx) + b * fx) * (1 - fy) + (c * (1 - fx) + d * fx) * fy)
        total += amp
        amp *= 0.5
    return np.clip(np.round(acc / total * 255.0), 0, 255).astype(np.uint8)


def normal_map(h8: np.ndarray) -> np.ndarray:
    """RG8 normal map from a height field (central differences)."""
    h = h8.astype(np.float64) / 255.0
    dx = (np.roll(h, -1, axis=1) - np.roll(h, 1, axis=1)) * 4.0
    dy = (np.roll(h, -1, axis=0) - np.roll(h, 1, axis=0)) * 4.0
    n = np.stack([-dx, -dy, np.ones_like(h)], axis=-1)
    n /= np.linalg.norm(n, axis=-1, keepdims=True)
    rg = np.round((n[..., :2] * 0.5 + 0.5) * 255.0)
    return np.clip(rg, 0, 255).astype(np.uint8)


def reference_pattern_rgb(width: int, height: int, punch_through: bool = False, alpha_ramp: bool = False):
    """The reference tests' checker patterns (tests/test_imagecompress.cpp:50-120), RGBA8."""
    y, x = np.mgrid[0:height, 0:width]
    img = np.zeros((height, width, 4), np.uint8)
    img[..., 1] = 255
    img[..., 3] = 255
    red = ((x // 2) & 2).astype(bool) | ((y // 2) & 2).astype(bool)
    img[red] = (255, 0, 0, 255)
    blue = ((x // 3) % 3).astype(bool) & ((y // 3) % 3).astype(bool)
    img[blue] = (0, 0, 255, 255)
    if punch_through:
        img[(x > width // 2) & (y > height // 2)] = (0, 0, 0, 0)
    if alpha_ramp:
        a = (x.astype(np.float32) / np.float32(width))
        img[..., 3] = np.clip(np.round(a * 255.0), 0, 255).astype(np.uint8)
    return img


def hdr_rgba(width: int, height: int, seed: int = 1, signed: bool = False) -> np.ndarray:
    """HDR float32 RGBA (H, W, 4) for BC6H: an exponential ramp over 12 stops
    (2^-8 .. 2^4) times a smooth hue, with 3 % multiplicative noise and a few
    bright highlights; signed = values in [-range, range] (sign from a hash)."""
    y, x = np.mgrid[0:height, 0:width].astype(np.float64)
    u = x / max(width - 1, 1)
    v = y / max(height - 1, 1)
    lum = np.exp2(-8.0 + 12.0 * u)
    idx = np.arange(width * height, dtype=np.uint64).reshape(height, width)
    h = _mix32(idx ^ np.uint64(seed & _M32)).astype(np.float64) / 4294967296.0
    noise = 1.0 + 0.03 * (2.0 * h - 1.0)
    img = np.empty((height, width, 4), np.float32)
    img[..., 0] = lum * (0.6 + 0.4 * v) * noise
    img[..., 1] = lum * (0.4 + 0.6 * (1 - v)) * noise
    img[..., 2] = lum * (0.3 + 0.7 * np.abs(u - v)) * noise
    hi = h > 0.995
    img[hi, :3] *= 8.0
    if signed:
        sgn = np.where(_mix32(idx ^ np.uint64((seed * 7 + 3) & _M32)) & 1, -1.0, 1.0)
        img[..., :3] *= sgn[..., None]
    img[..., 3] = 1.0
    return img
