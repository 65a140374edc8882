"""Does writing the blocks straight into pinned host memory (the host-image
pipeline's zero-copy outputs) slow the BC1 encode?  8K G1 resident in HBM, the
image in N pieces over two streams, blocks to a device buffer vs a pinned host
buffer (hipHostMalloc'd memory is addressable by the kernels).

    python tools/time_zc.py [--pieces 16]
"""
import argparse
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import gfx_imagecompress_amd as gic          # noqa: E402
from gfx_imagecompress_amd import synth      # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pieces", type=int, default=16)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    size, by = 8192, 2048
    src = synth.g1_torch(size, size, 1, seed=0x9E3779B9)
    nbytes = by * 2048 * 8
    dev_dst = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    host_dst = torch.empty(nbytes, dtype=torch.uint8, pin_memory=True)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    opts = gic.Options().to_c()
    lib = gic.library()
    rows = by // a.pieces

    def run(ptr):
        for k in range(a.pieces):
            s = streams[k % 2]
            rc = lib.gic_hip_encode_rows(1, src.data_ptr(), size, size, 1, 4, size * 4, k * rows, rows,
                                         ctypes.byref(opts), ptr + k * rows * 2048 * 8, None,
                                         ctypes.c_void_p(s.cuda_stream))
            assert rc == 0, rc

    # an unrelated 256 MiB upload running beside the encode (the pipeline's H2D traffic)
    up_src = torch.empty(size * size * 4, dtype=torch.uint8, pin_memory=True)
    up_dst = torch.empty(size * size * 4, dtype=torch.uint8, device="cuda")
    up_stream = torch.cuda.Stream()
    for name, ptr, copy in (("device", dev_dst.data_ptr(), False), ("pinned host", host_dst.data_ptr(), False),
                            ("device, beside a 256 MiB upload", dev_dst.data_ptr(), True),
                            ("pinned host, beside a 256 MiB upload", host_dst.data_ptr(), True)):
        best = 1e9
        for _ in range(a.reps):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(streams[0])
            streams[1].wait_stream(streams[0])
            if copy:
                up_stream.wait_stream(streams[0])
                with torch.cuda.stream(up_stream):
                    up_dst.copy_(up_src, non_blocking=True)
            run(ptr)
            streams[0].wait_stream(streams[1])
            e1.record(streams[0])
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1))
        print(f"{a.pieces} pieces, blocks to {name}: {best:.3f} ms", flush=True)
    torch.cuda.synchronize()
    print("identical:", bool(torch.equal(dev_dst.cpu(), host_dst)))
    # the pipeline's shape without its threads: piece k's rows uploaded (pinned
    # source, one stream) into the buffer the kernels read, its encode waiting on
    # that upload's event; then the same with the whole source resident
    host_src = src.cpu().pin_memory()
    slab = torch.empty_like(src)
    row_bytes = size * 4 * 4 * rows
    flat_h, flat_d = host_src.view(-1), slab.view(-1)
    for name, wait in (("piecewise upload + encode (event per piece)", True), ("resident, same launches", False)):
        best = 1e9
        for _ in range(a.reps):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(streams[0])
            streams[1].wait_stream(streams[0])
            up_stream.wait_stream(streams[0])
            evs = []
            for k in range(a.pieces):
                if wait:
                    with torch.cuda.stream(up_stream):
                        flat_d[k * row_bytes:(k + 1) * row_bytes].copy_(flat_h[k * row_bytes:(k + 1) * row_bytes],
                                                                        non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(up_stream)
                    evs.append(ev)
            for k in range(a.pieces):
                s = streams[k % 2]
                if wait:
                    s.wait_event(evs[k])
                rc = lib.gic_hip_encode_rows(1, slab.data_ptr() if wait else src.data_ptr(), size, size, 1, 4,
                                             size * 4, k * rows, rows, ctypes.byref(opts),
                                             host_dst.data_ptr() + k * rows * 2048 * 8, None,
                                             ctypes.c_void_p(s.cuda_stream))
                assert rc == 0, rc
            streams[0].wait_stream(streams[1])
            e1.record(streams[0])
            torch.cuda.synchronize()
            best = min(best, e0.elapsed_time(e1))
        print(f"{a.pieces} pieces, {name}: {best:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
