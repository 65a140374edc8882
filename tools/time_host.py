"""The bench's host-image leg alone (bench.host_api_leg): Image_CompressAMDBC1
and the BC7 bounded exit on the 8K G1 host image, end to end, every upload mode.

    python tools/time_host.py [--no-bc7]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
import bench                                 # noqa: E402
import gfx_imagecompress_amd as gic          # noqa: E402
from gfx_imagecompress_amd import synth      # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--no-bc7", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    size = 8192
    src = synth.g1_torch(size, size, 1, seed=bench.G1_SEED, device=dev)
    dst = torch.empty((size // 4) ** 2 * 8, dtype=torch.uint8, device=dev)
    s = torch.cuda.current_stream()
    for _ in range(3):
        gic.encode_device(1, src, size, size, 1, 4, dst, gic.Options(), stream=s)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(10):
        gic.encode_device(1, src, size, size, 1, 4, dst, gic.Options(), stream=s)
    e1.record(s)
    torch.cuda.synchronize()
    args = argparse.Namespace(bc7_rows=0 if a.no_bc7 else -1)
    print(json.dumps(bench.host_api_leg(args, gic, src, size, dev, e0.elapsed_time(e1) / 10), indent=1))


if __name__ == "__main__":
    main()
