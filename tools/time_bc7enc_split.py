import os, sys
sys.path.insert(0, '/root/repo')
import torch
import gfx_imagecompress_amd as gic
from gfx_imagecompress_amd import synth
n = 8192
src = torch.from_numpy(synth.g1(n, n)[None].copy()).cuda()
dst = torch.empty((n // 4) ** 2 * 16, dtype=torch.uint8, device="cuda")
for uber in (0, 1, 2, 3, 4):
    for mp in (64, 1):
        o = gic.Options(bc7enc_uber_level=uber, bc7enc_max_partitions=mp)
        gic.encode_device(gic.FMT_BC7ENC16, src, n, n, 1, 4, dst, o); torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(3): gic.encode_device(gic.FMT_BC7ENC16, src, n, n, 1, 4, dst, o)
        e.record(); torch.cuda.synchronize()
        print(f"uber {uber} max_parts {mp}: {s.elapsed_time(e)/3:.2f} ms", flush=True)
