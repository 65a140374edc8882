"""Study: how much of the BC7 mode-0/1 shaking could an exact lower bound prune?

Builds the oracle with -DORC_TRACE (per-rank shaken errors), encodes a random
sample of G1 8K blocks, and for every shaken (mode, rank) compares a lower
bound on any encoding's error for that partition with the block's final error.
Study tool only (loads the oracle); not part of the product or the tests.
"""
import ctypes
import os
import re
import subprocess
import sys
from multiprocessing import Pool

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
LIB = "/tmp/liboracle_trace.so"
TRACE_T = ctypes.CFUNCTYPE(None, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_double,
                           ctypes.POINTER(ctypes.c_double))


def build():
    o = os.path.join(ROOT, "oracle")
    subprocess.run(["gcc", "-O2", "-ffp-contract=off", "-fPIC", "-pthread", "-std=gnu11", "-DORC_TRACE", "-shared",
                    "-o", LIB, f"{o}/orc_bcx.c", f"{o}/orc_bc7.c", f"{o}/orc_image.c", "-lm"], check=True)


def shapes():
    t = open(os.path.join(ROOT, "oracle", "bc7_tables.h")).read()
    out = {}
    for name, k in (("kBc7Shape2", 2), ("kBc7Shape3", 3)):
        body = re.search(name + r"\[64\] = \{(.*?)\};", t, re.S).group(1)
        out[k] = [int(v, 16) for v in re.findall(r"0x([0-9a-f]+)u", body)]
    return out


SUBSETS = {0: 3, 1: 2, 2: 3, 3: 2, 6: 1, 7: 2}
SH = None
LIBH = None


def line_lb(x, delta):
    n = len(x)
    if n <= 1:
        return 0.0
    c = x - x.mean(0)
    s = c.T @ c
    w = np.linalg.eigvalsh(s)
    r = max(0.0, float(w.sum() - w[-1]))
    if r <= 4 * n * delta * delta:
        return 0.0
    return r - 2 * delta * np.sqrt(n * r)


def work(blocks):
    global SH, LIBH
    if LIBH is None:
        LIBH = ctypes.CDLL(LIB)
        SH = shapes()
    recs = []

    def cb(kind, mode, rank, part, err, sub):
        recs.append((kind, mode, rank, part, err))

    f = TRACE_T(cb)
    ctypes.c_void_p.in_dll(LIBH, "orc_bc7_trace").value = ctypes.cast(f, ctypes.c_void_p).value
    LIBH.orc_bc7_block.restype = ctypes.c_double
    out = []
    for blk in blocks:
        recs.clear()
        inN = (blk.astype(np.float32) / np.float32(255.0)).astype(np.float32)
        o = (ctypes.c_uint8 * 16)()
        best = LIBH.orc_bc7_block(inN.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint8(0xFF), 0, ctypes.c_float(1.0),
                                  1, 1, ctypes.c_float(1.0), o)
        x = blk.reshape(16, 4)[:, :3].astype(np.float64)
        modes = {r[1]: r[4] for r in recs if r[0] == 1}
        ranks = []
        for kind, mode, rank, part, err in recs:
            if kind != 0 or mode not in (0, 1):
                continue
            ns = SUBSETS[mode]
            lb = 0.0
            for s in range(ns):
                sel = [t for t in range(16) if ((SH[ns][part] >> (2 * t)) & 3) == s]
                lb += line_lb(x[sel], np.sqrt(3) / 2)
            ranks.append((mode, rank, err, lb))
        out.append((best, modes, ranks))
    return out


def main():
    from gfx_imagecompress_amd import synth
    build()
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    rows = 64
    img = synth.g1(8192, 8192)[:4 * rows]
    rng = np.random.default_rng(1)
    bx = rng.integers(0, 2048, n)
    by = rng.integers(0, rows, n)
    blocks = [img[4 * y:4 * y + 4, 4 * x:4 * x + 4].copy() for x, y in zip(bx, by)]
    chunks = [blocks[i::8] for i in range(8)]
    with Pool(8) as p:
        res = sum(p.map(work, chunks), [])
    tot = prunable = viol = 0
    staged = 0
    wins = {}
    for best, modes, ranks in res:
        wm = min(modes, key=lambda m: (modes[m], [6, 4, 3, 1, 2, 0, 7, 5].index(m)))
        wins[wm] = wins.get(wm, 0) + 1
        # staged incumbent: everything except mode 0/1 ranks >= 1
        inc = min([v for m, v in modes.items() if m not in (0, 1)] +
                  [e for (m, r, e, lb) in ranks if r == 0])
        for m, r, e, lb in ranks:
            tot += 1
            viol += lb > e + 1e-9
            prunable += lb > best
            staged += r >= 1 and lb > inc
    print(f"blocks {len(res)} mode wins {sorted(wins.items())}")
    print(f"mode0/1 rank shakes {tot}: LB violations {viol}, prunable vs final {prunable} ({prunable / tot:.1%}),"
          f" staged (rank>=1 vs incumbent) {staged} ({staged / tot:.1%})")
    gaps = [lb / e for _, _, ranks in res for (m, r, e, lb) in ranks if e > 0]
    print("LB/err quantiles", np.quantile(gaps, [0.1, 0.5, 0.9]))
    rel = [e / best for best, _, ranks in res for (m, r, e, lb) in ranks if best > 0]
    print("err/final quantiles", np.quantile(rel, [0.1, 0.25, 0.5, 0.75, 0.9]))


if __name__ == "__main__":
    main()
