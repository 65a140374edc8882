"""Debug helper: per-mode BC7 GPU vs oracle comparison on a small image."""
import sys, os
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
import gfx_imagecompress_amd as gic
from gfx_imagecompress_amd import synth
import oracle_lib

img = synth.noise_rgba(16, 16, seed=3, alpha=True)
blocks = img.reshape(4, 4, 4, 4, 4).transpose(0, 2, 1, 3, 4).reshape(16, 16, 4).astype(np.float32) / np.float32(255.0)
t = torch.from_numpy(blocks.reshape(16, 64).copy()).cuda()
for mask in (0xFF, 0x10, 0x20, 0x40, 0x80):
    dst = torch.zeros(16 * 16, dtype=torch.uint8, device="cuda")
    gic.encode_blocks_f32(gic.FMT_BC7, t, dst, gic.Options(bc7_mode_mask=mask))
    torch.cuda.synchronize()
    got = dst.cpu().numpy().reshape(16, 16)
    bad = []
    for i in range(16):
        ref, _ = oracle_lib.bc7_block(blocks[i], mask)
        if got[i].tobytes() != ref:
            bad.append((i, got[i].tobytes().hex(), ref.hex()))
    print("mask %02x: %d bad" % (mask, len(bad)))
    for b in bad[:3]:
        print("   ", b)
