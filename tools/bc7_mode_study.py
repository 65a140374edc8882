"""Per-mode BC7 cost and decoded error on the 8K G1 texture (a block-row band):
for the full mode mask and each single mode, the encode time (HIP events) and
every block's decoded SSE (RGBA, 0..255 units).  Input for the error-bound
exit study (which blocks a cheap stage already brings within the per-block
MSE contract's absolute slack).

    python tools/bc7_mode_study.py [--rows 256] [--out gpurun_out/mode_study.npz]
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import gfx_imagecompress_amd as gic          # noqa: E402
from gfx_imagecompress_amd import synth      # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=256)
    ap.add_argument("--size", type=int, default=8192)
    ap.add_argument("--shake-ranks", type=int, default=0)
    ap.add_argument("--no-colour-restrict", action="store_true", help="let opaque blocks use modes 4-7")
    ap.add_argument("--masks", default="", help="comma-separated hex mode masks (default: ff and each mode)")
    ap.add_argument("--out", default="gpurun_out/mode_study.npz")
    a = ap.parse_args()
    size, rows = a.size, a.rows
    img = synth.g1(size, size)[: rows * 4]
    src = torch.from_numpy(np.ascontiguousarray(img)).cuda()
    bx = size // 4
    n = bx * rows
    dst = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
    dec = torch.empty(rows * 4 * size * 4, dtype=torch.uint8, device="cuda")
    ref = src.reshape(rows, 4, bx, 4, 4).permute(0, 2, 1, 3, 4).reshape(n, 64).to(torch.int32)
    out = {}
    s = torch.cuda.current_stream()
    masks = [int(x, 16) for x in a.masks.split(",")] if a.masks else [0xFF] + [1 << m for m in range(8)]
    for mask in masks:
        o = gic.Options(bc7_mode_mask=mask, bc7_shake_ranks=a.shake_ranks, colour_restrict=not a.no_colour_restrict)
        gic.encode_device(gic.FMT_BC7, src, size, rows * 4, 1, 4, dst, o)   # warm (tables, workspaces)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        gic.encode_device(gic.FMT_BC7, src, size, rows * 4, 1, 4, dst, o)
        e1.record(s)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1)
        gic.decode_device(gic.FMT_BC7, dst, size, rows * 4, 1, dec)
        torch.cuda.synchronize()
        d = dec.reshape(rows, 4, bx, 4, 4).permute(0, 2, 1, 3, 4).reshape(n, 64).to(torch.int32)
        sse = ((d - ref) ** 2).sum(dim=1)
        out[f"sse_{mask:02x}"] = sse.cpu().numpy()
        out[f"ms_{mask:02x}"] = np.float64(ms)
        out[f"blk_{mask:02x}"] = dst.cpu().numpy().reshape(-1, 16) if mask == 0xFF else np.zeros(0)
        print(f"mask {mask:02x}: {ms:9.2f} ms, mean MSE {sse.double().mean().item() / 64:.4f}, "
              f"MSE<=0.5 {(sse <= 32).double().mean().item():.4f}", flush=True)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    np.savez_compressed(a.out, **out)


if __name__ == "__main__":
    main()
