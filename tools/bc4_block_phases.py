"""Phase timing of the one-wave BC4 block kernel (needs an instrumented build in
GIC_LIBRARY that prints s_memtime stamps of block 0's wave).
    GIC_LIBRARY=gpurun_var/bc4ph/lib.so python tools/bc4_block_phases.py"""
import ctypes
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import gfx_imagecompress_amd as gic

lib = gic.library()
rng = np.random.default_rng(1)
for _ in range(4):
    blk = rng.random(16, dtype=np.float32)
    out = (ctypes.c_uint8 * 8)()
    lib.Image_CompressAMDAlphaSingleModeBlock(blk.ctypes.data_as(ctypes.c_void_p), out)
