"""BC4 / BC5 kernel time on the bench's 8K inputs: BC4 of the height map (R8),
BC4 of each channel of the normal map (RG8, channel 0 and 1) and BC5 of the
normal map -- separates the per-channel cost of the data from the kernel.
    python tools/time_bc45.py [reps]"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import gfx_imagecompress_amd as gic
from gfx_imagecompress_amd import synth

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
n = 8192
h = synth.height_field(n, n, seed=1)
srcs = {"height R8": (torch.from_numpy(h[None, :, :, None].copy()).cuda(), 1),
        "normal RG8": (torch.from_numpy(synth.normal_map(h)[None].copy()).cuda(), 2)}
dst = torch.empty((n // 4) ** 2 * 16, dtype=torch.uint8, device="cuda")


def t(fmt, src, ch, channel):
    o = gic.Options(bc4_channel=channel)
    gic.encode_device(fmt, src, n, n, 1, ch, dst, o)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        gic.encode_device(fmt, src, n, n, 1, ch, dst, o)
    e.record()
    torch.cuda.synchronize()
    import hashlib
    t.dig = hashlib.sha1(dst.cpu().numpy().tobytes()).hexdigest()[:12]
    return s.elapsed_time(e) / reps


for name, (src, ch) in srcs.items():
    for c in range(ch):
        ms = t(4, src, ch, c)
        print(f"{os.environ.get('GIC_LIBRARY', '')} BC4 {name} channel {c}: {ms:.4f} ms  digest {t.dig}", flush=True)
ms = t(5, srcs['normal RG8'][0], 2, 0)
print(f"{os.environ.get('GIC_LIBRARY', '')} BC5 normal RG8: {ms:.4f} ms  digest {t.dig}", flush=True)
