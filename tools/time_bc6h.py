"""Time BC6H (unsigned and signed) on a synthetic HDR float32 texture on the GPU.

    python tools/time_bc6h.py [--size 1024] [--reps 3]
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
    ap.add_argument("--size", type=int, default=1024)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--only", choices=["signed", "unsigned"], default=None)
    a = ap.parse_args()
    n = a.size
    for signed in (False, True):
        if a.only and (a.only == "signed") != signed:
            continue
        img = synth.hdr_rgba(n, n, seed=1, signed=signed)
        src = torch.from_numpy(img.reshape(-1).copy()).cuda()
        nb = (n // 4) ** 2
        dst = torch.empty(nb * 16, dtype=torch.uint8, device="cuda")
        fmt = gic.FMT_BC6H_SF if signed else gic.FMT_BC6H
        gic.encode_device_src(fmt, gic.SRC_FLOAT32, src, n, 64, 1, 4, dst)
        torch.cuda.synchronize()
        s = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(a.reps):
            gic.encode_device_src(fmt, gic.SRC_FLOAT32, src, n, n, 1, 4, dst)
        e1.record(s)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / a.reps
        import hashlib
        dig = hashlib.sha1(dst.cpu().numpy().tobytes()).hexdigest()[:16]
        print(f"{os.environ.get('GIC_LIBRARY', '')} BC6H {'signed' if signed else 'unsigned'} {n}x{n}: {ms:.1f} ms = "
              f"{n * n / ms / 1e3:.2f} Mpix/s, {nb / ms * 1e3:.0f} blocks/s  digest {dig}", flush=True)


if __name__ == "__main__":
    main()
