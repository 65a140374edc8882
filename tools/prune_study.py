#!/usr/bin/env python3
"""BC7 search-pruning study (instrumentation; reads the oracle's trace).

Builds tools/prune_study.c with the oracle sources (-DORC_TRACE) into /tmp,
encodes a block sample of the 8192^2 G1 texture at default quality and saves
per-(mode, rank) quantiser and shaken errors to an .npz for policy simulation.
Usage: python tools/prune_study.py OUT.npz [rows...]
"""
import ctypes
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gfx_imagecompress_amd import synth  # noqa: E402

SO = "/tmp/study/libstudy.so"


def build():
    os.makedirs("/tmp/study", exist_ok=True)
    o = os.path.join(ROOT, "oracle")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-fno-fast-math", "-fPIC", "-pthread", "-std=gnu11",
                    "-DORC_TRACE", "-shared", "-o", SO, os.path.join(ROOT, "tools", "prune_study.c"),
                    os.path.join(o, "orc_bc7.c"), os.path.join(o, "orc_bcx.c"), os.path.join(o, "orc_image.c"), os.path.join(o, "orc_bc7enc.c"),
                    os.path.join(o, "orc_bc6h.c"),
                    "-lm", "-I", o], check=True)


def blocks_of(img, rows, step=1):
    h, w, _ = img.shape
    bx = w // 4
    out = []
    for r in rows:
        t = img[r * 4:r * 4 + 4].reshape(4, bx, 4, 4).transpose(1, 0, 2, 3).reshape(bx, 64)
        out.append(t[::step])
    return (np.concatenate(out).astype(np.float32) / np.float32(255.0)).astype(np.float32)


def run(blocks, threads):
    lib = ctypes.CDLL(SO)
    n = blocks.shape[0]
    q = np.zeros((n, 8, 8)); s = np.zeros((n, 8, 8)); m = np.zeros((n, 8)); p = np.zeros((n, 8, 8), np.int32)
    best = np.zeros(n); out = np.zeros((n, 16), np.uint8); allq = np.zeros((n, 8, 64))
    vp = ctypes.c_void_p
    lib.study.argtypes = [vp, ctypes.c_int, ctypes.c_int, vp, vp, vp, vp, vp, vp, vp]
    b = np.ascontiguousarray(blocks)
    lib.study(b.ctypes.data, n, threads, q.ctypes.data, s.ctypes.data, m.ctypes.data, p.ctypes.data,
              best.ctypes.data, out.ctypes.data, allq.ctypes.data)
    return dict(q=q, s=s, m=m, p=p, best=best, out=out, allq=allq)


if __name__ == "__main__":
    build()
    dst = sys.argv[1]
    rows = [int(x) for x in sys.argv[2:]] or [0, 512, 1024, 1536]
    img = synth.g1(8192, 8192)
    blk = blocks_of(img, rows, step=2)
    t0 = time.time()
    r = run(blk, os.cpu_count() or 1)
    print(f"{blk.shape[0]} blocks in {time.time() - t0:.1f}s")
    np.savez_compressed(dst, blocks=blk, **r)
