"""Time BC1 on the 8192^2 G1 texture with the library GIC_LIBRARY names and
write its blocks' FNV-1a digest (compare variants against the default build).
    GIC_LIBRARY=path python tools/time_bc1.py [reps]"""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
import gfx_imagecompress_amd as gic
from gfx_imagecompress_amd import synth

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
n = 8192
src = torch.from_numpy(synth.g1(n, n)[None].copy()).cuda()
dst = torch.empty((n // 4) ** 2 * 8, dtype=torch.uint8, device="cuda")
gic.encode_device(gic.FMT_BC1, src, n, n, 1, 4, dst)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(reps):
    gic.encode_device(gic.FMT_BC1, src, n, n, 1, 4, dst)
e.record()
torch.cuda.synchronize()
ms = s.elapsed_time(e) / reps
h = dst.cpu().numpy()
d = int(np.frombuffer(h.tobytes(), dtype=np.uint64).astype(np.uint64).sum() % (1 << 61))
print(f"{os.environ.get('GIC_LIBRARY', 'default')}: {ms:.3f} ms  {n * n / ms / 1e3:.1f} Mpix/s  digest {d}", flush=True)
