"""Section timing of the BC7 wave shakers (needs a -DGIC_PROFILE build in GIC_LIBRARY)."""
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import gfx_imagecompress_amd as gic
from gfx_imagecompress_amd import synth

lib = gic.library()
lib.gic_debug_profile.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
n = 8192
rows = int(sys.argv[1]) if len(sys.argv) > 1 else 8
src = synth.g1_torch(n, n, 1, seed=0x9E3779B9, device="cuda")
dst = torch.empty((n // 4) * rows * 16, dtype=torch.uint8, device="cuda")
buf = (ctypes.c_ulonglong * 32)()
gic.encode_device(7, src, n, n, 1, 4, dst, gic.Options(), 0, rows)
torch.cuda.synchronize()
lib.gic_debug_profile(buf, 1)
gic.encode_device(7, src, n, n, 1, 4, dst, gic.Options(), 0, rows)
torch.cuda.synchronize()
lib.gic_debug_profile(buf, 0)
names = {0: "c.collapse", 1: "c.ls", 2: "c.pass_setup", 3: "c.build_ramp", 4: "c.texels", 5: "c.tail",
         6: "c.combo/iter", 8: "w.collapse", 9: "w.ls", 10: "w.chan_setup", 11: "w.texels", 12: "w.reduce+comb",
         13: "w.rq_tail", 14: "w.combo", 15: "w.rq_unpack+ramp", 16: "w.rq_nearest", 17: "w.rq_wsum",
         18: "c.moments", 19: "c.exp_table", 20: "w.moments", 21: "w.exp_table"}
tot = sum(buf[i] for i in names)
for i, nm in names.items():
    print(f"{nm:16s} {buf[i] / 1e9:10.3f} Gcyc {100.0 * buf[i] / tot:6.1f}%")
counts = {22: "corner passes walked", 23: "corner texel pairs", 24: "corner passes cut", 25: "corner passes deduped",
          26: "corner expansions", 27: "corner texels of walked passes", 28: "corner passes skipping the min",
          29: "corners() calls"}
for i, nm in counts.items():
    print(f"{nm:32s} {buf[i]:14d}")
