"""Phase timing of the one-wave BC1 block kernel (needs the instrumented
gpurun_var/bc1ph build: s_memtime stamps of wave 0 printed by block 0).
    GIC_LIBRARY=gpurun_var/bc1ph/lib.so python tools/bc1_block_phases.py"""
import ctypes
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import gfx_imagecompress_amd as gic

lib = gic.library()
rng = np.random.default_rng(1)
for _ in range(4):
    blk = rng.random(64, dtype=np.float32)
    blk[3::4] = 1.0
    out = (ctypes.c_uint8 * 8)()
    lib.Image_CompressAMDBC1Block(blk.ctypes.data_as(ctypes.c_void_p), ctypes.c_bool(False), ctypes.c_bool(False),
                                  ctypes.c_uint8(1), ctypes.c_float(0.0), out)
