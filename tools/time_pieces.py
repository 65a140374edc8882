"""How the BC1 / BC7 encode time of the 8K G1 texture (resident in HBM) depends
on how many launches (pieces of block rows) it is cut into -- the cost side of
the host pipeline's piece size (gic_pipeline.cpp piece_rows).

    python tools/time_pieces.py [--fmt 1] [--bound 0.5] [--cuts 1,2,4,8,16,32]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import gfx_imagecompress_amd as gic          # noqa: E402
from gfx_imagecompress_amd import synth      # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fmt", type=int, default=1)
    ap.add_argument("--bound", type=float, default=0.5)
    ap.add_argument("--cuts", default="1,2,4,8,16,32")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--streams", type=int, default=1, help="pieces round-robin over this many streams")
    a = ap.parse_args()
    size, by = 8192, 2048
    src = synth.g1_torch(size, size, 1, seed=0x9E3779B9)
    bb = gic.block_bytes(a.fmt)
    dst = torch.empty(by * 2048 * bb, dtype=torch.uint8, device="cuda")
    o = gic.Options(bc7_mse_bound=a.bound) if a.fmt == 7 else gic.Options()
    s = torch.cuda.current_stream()
    ss = [torch.cuda.Stream() for _ in range(a.streams)]
    for cut in [int(c) for c in a.cuts.split(",")]:
        per = (by + cut - 1) // cut
        best = 1e30
        for _ in range(a.reps if a.fmt != 7 else 2):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record(s)
            for q in ss:
                q.wait_event(e0)
            for k, r0 in enumerate(range(0, by, per)):
                n = min(per, by - r0)
                gic.encode_device(a.fmt, src, size, size, 1, 4, dst[r0 * 2048 * bb:], o, r0, n, stream=ss[k % len(ss)])
            for q in ss:
                s.wait_stream(q)
            e1.record(s)
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1))
        print(f"fmt {a.fmt}, {a.streams} stream(s): {cut:3d} pieces of {per:4d} block rows: {best:8.3f} ms", flush=True)


if __name__ == "__main__":
    main()
