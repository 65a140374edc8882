"""BC2 / BC3 kernel time and output digest on the 8K G1 texture.
    python tools/time_bc23.py [reps]"""
import hashlib
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import gfx_imagecompress_amd as gic
from gfx_imagecompress_amd import synth

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
n = 8192
src = torch.from_numpy(synth.g1(n, n)[None].copy()).cuda()
dst = torch.empty((n // 4) ** 2 * 16, dtype=torch.uint8, device="cuda")
for fmt in (2, 3):
    gic.encode_device(fmt, src, n, n, 1, 4, dst)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        gic.encode_device(fmt, src, n, n, 1, 4, dst)
    e.record()
    torch.cuda.synchronize()
    dig = hashlib.sha1(dst.cpu().numpy().tobytes()).hexdigest()[:16]
    print(f"{os.environ.get('GIC_LIBRARY', '')} BC{fmt}: {s.elapsed_time(e) / reps:.3f} ms  digest {dig}", flush=True)
