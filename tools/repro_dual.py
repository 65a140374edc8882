"""Repro for the merged dual-index quantiser build (DESIGN.md note): BC7 with
mode masks 0x10/0x20/0xFF on noise blocks, GPU vs oracle; prints mismatches.
Run with GIC_LIBRARY=<variant lib.so>."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
import gfx_imagecompress_amd as gic  # noqa: E402
from gfx_imagecompress_amd import synth  # noqa: E402
import oracle_lib  # noqa: E402

print("lib", gic.LIB_PATH)
sets = {
    "noise16_alpha": synth.noise_rgba(16, 16, seed=3, alpha=True),
    "noise64_alpha": synth.noise_rgba(64, 64, seed=5, alpha=True),
    "noise64_opaque": synth.noise_rgba(64, 64, seed=6, alpha=False),
    "g1_64": synth.g1(64, 64),
}
total_bad = 0
for name, img in sets.items():
    h, w = img.shape[:2]
    nb = (h // 4) * (w // 4)
    blocks = img.reshape(h // 4, 4, w // 4, 4, 4).transpose(0, 2, 1, 3, 4).reshape(nb, 64).astype(np.float32) / np.float32(255)
    t = torch.from_numpy(np.ascontiguousarray(blocks)).cuda()
    for mask in (0x10, 0x20, 0x30, 0xFF):
        dst = torch.zeros(nb * 16, dtype=torch.uint8, device="cuda")
        gic.encode_blocks_f32(gic.FMT_BC7, t, dst, gic.Options(bc7_mode_mask=mask))
        torch.cuda.synchronize()
        got = dst.cpu().numpy().reshape(nb, 16)
        bad = []
        for i in range(nb):
            ref, _ = oracle_lib.bc7_block(blocks[i], mask)
            if got[i].tobytes() != ref:
                bad.append(i)
        total_bad += len(bad)
        print(f"{name} mask {mask:02x}: {len(bad)}/{nb} differ {bad[:10]}", flush=True)
        for i in bad[:2]:
            ref, _ = oracle_lib.bc7_block(blocks[i], mask)
            print("   block", i, "gpu", got[i].tobytes().hex(), "ref", ref.hex(), "texels", img.reshape(-1)[:0])
            print("   ", (blocks[i] * 255).astype(int).reshape(16, 4).tolist())
print("TOTAL_BAD", total_bad)
