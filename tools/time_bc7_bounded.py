"""Time the BC7 bounded-exit path (and the exact one) on a block-row band of
the 8K G1 texture; run under rocprofv3 --kernel-trace --stats with
GIC_BC7_SINGLE_STREAM=1 for a per-kernel split of the probe and the full
search.

    python tools/time_bc7_bounded.py [--rows 256] [--bound 0.5] [--shake-ranks 0]
"""
import argparse
import hashlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import gfx_imagecompress_amd as gic          # noqa: E402
from gfx_imagecompress_amd import synth      # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=256)
    ap.add_argument("--size", type=int, default=8192)
    ap.add_argument("--bound", type=float, default=0.5)
    ap.add_argument("--shake-ranks", type=int, default=0)
    ap.add_argument("--no-warm", action="store_true",
                    help="skip the 4-row warm-up pass (a --pmc run then counts exactly one pass)")
    a = ap.parse_args()
    size, rows = a.size, a.rows
    src = torch.from_numpy(np.ascontiguousarray(synth.g1(size, size)[: rows * 4])).cuda()
    dst = torch.empty((size // 4) * rows * 16, dtype=torch.uint8, device="cuda")
    o = gic.Options(bc7_mse_bound=a.bound, bc7_shake_ranks=a.shake_ranks)
    if not a.no_warm:
        gic.encode_device(gic.FMT_BC7, src, size, 16, 1, 4, dst, o)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    gic.encode_device(gic.FMT_BC7, src, size, rows * 4, 1, 4, dst, o)
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    print(f"bound {a.bound} shake_ranks {a.shake_ranks}: {rows} block rows in {ms:.1f} ms = "
          f"{size * rows * 4 / ms / 1e3:.2f} Mpix/s, output sha1 {hashlib.sha1(dst.cpu().numpy().tobytes()).hexdigest()[:16]}",
          flush=True)


if __name__ == "__main__":
    main()
