"""Piece plan sweep of the host-image pipeline: Image_CompressAMDBC1 on the 8K
G1 host image end to end for (first piece, later pieces) block counts set
through GIC_PIECE_FIRST / GIC_PIECE_BLOCKS, beside the device-resident kernel.

    python tools/time_host_pieces.py [--plans 262144:262144,131072:1048576,...]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
import bench                                 # noqa: E402
import gfx_imagecompress_amd as gic          # noqa: E402
from gfx_imagecompress_amd import synth      # noqa: E402

# first:per[:encode streams[:upload mode[:hooks]]], hooks '+'-separated from
# poll, inline_up, nopop, nocopy, zc_nc (gic_pipeline.cpp GIC_PIPE_*)
DEFAULT = ("262144:262144:2,262144:262144:2:register:zc_nc,262144:262144:2:pageable:zc_nc,"
           "524288:524288:2:register:zc_nc,131072:131072:2:register:zc_nc,262144:262144:2,"
           "262144:262144:2:register:nocopy,262144:262144:2:register:nocopy+nopop+poll+inline_up")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--plans", default=DEFAULT)
    ap.add_argument("--reps", type=int, default=5)
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
    kern = e0.elapsed_time(e1) / 10
    want = dst.cpu().numpy()
    host = np.ascontiguousarray(src[0].cpu().numpy())
    hi = gic.HostImage(host)
    rows = []
    try:
        for plan in a.plans.split(","):
            first, per, *rest = plan.split(":")
            os.environ["GIC_PIECE_FIRST"], os.environ["GIC_PIECE_BLOCKS"] = first, per
            os.environ["GIC_ENC_STREAMS"] = rest[0] if rest else "2"
            os.environ["GIC_H2D"] = rest[1] if len(rest) > 1 else "register"
            hooks = rest[2].split("+") if len(rest) > 2 and rest[2] else []
            for h in ("POLL", "INLINE_UP", "NOPOP", "NOCOPY", "ZC_NC"):
                os.environ["GIC_PIPE_" + h] = "1" if h.lower() in hooks else "0"
            times, best, ok = [], None, True
            for _ in range(1 + a.reps):
                got = hi.compress(1, entry="Image_CompressAMDBC1")
                ok = ok and np.array_equal(got.reshape(-1), want) if "nocopy" not in hooks else ok
                rep = gic.host_report()
                times.append(hi.last_call_ms)
                if best is None or rep["total_ms"] < best["total_ms"]:
                    best = rep
            e2e = min(times[1:])
            rows.append({"first": int(first), "per": int(per), "streams": os.environ["GIC_ENC_STREAMS"],
                         "hooks": "+".join(hooks),
                         "h2d": os.environ["GIC_H2D"], "pieces": best["pieces"], "e2e_ms": round(e2e, 3),
                         "h2d_ms": round(best["h2d_ms"], 3), "encode_ms": round(best["encode_ms"], 3),
                         "d2h_ms": round(best["d2h_ms"], 3), "e2e_over_kernel": round(e2e / kern, 3),
                         "bytes_equal": bool(ok)})
            print(json.dumps(rows[-1]), flush=True)
    finally:
        hi.close()
    print(json.dumps({"kernel_ms": round(kern, 4)}))


if __name__ == "__main__":
    main()
