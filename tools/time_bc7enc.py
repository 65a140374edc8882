"""Time the bc7enc16 kernels on an 8192^2 G1 texture (all four settings)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import gfx_imagecompress_amd as gic
from gfx_imagecompress_amd import synth

n = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
img = synth.g1(n, n)
src = torch.from_numpy(img[None].copy()).cuda()
dst = torch.empty((n // 4) ** 2 * 16, dtype=torch.uint8, device="cuda")
for fast, perc in ((False, True), (True, True), (False, False), (True, False)):
    o = gic.Options.bc7enc16(fast, perc)
    gic.encode_device(gic.FMT_BC7ENC16, src, n, n, 1, 4, dst, o)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(3):
        gic.encode_device(gic.FMT_BC7ENC16, src, n, n, 1, 4, dst, o)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / 3
    import hashlib
    dig = hashlib.sha1(dst.cpu().numpy().tobytes()).hexdigest()[:16]
    print(f"{os.environ.get('GIC_LIBRARY', '')} fast={fast} perceptual={perc}: {ms:.2f} ms  "
          f"{n * n / ms / 1e3:.1f} Mpix/s  digest {dig}", flush=True)
