#!/usr/bin/env python3
"""Audit of the gfx950 machine code in the built library.

Extracts the device code objects of lib/libgfx_imagecompress_amd.so
(llvm-objdump --offloading), disassembles them and reports, per kernel:
  * scalar loads whose address comes straight from v_readfirstlane_b32 with no
    waterfall loop: a load the compiler believed wave-uniform.  This is the
    signature of the round-1 dual-index quantiser fault (a lane-divergent index
    into the __constant__ mode table folded into an s_load, so every lane read
    the first lane's cluster count; DESIGN.md "Dual-index quantiser fault").
    The kernels must have none;
  * scalar-cache writes (s_store / s_buffer_store / s_scratch_store / scalar
    atomics / s_dcache_wb), which this project never emits;
  * scratch (private segment) use, reported for information;
  * per-kernel resources from the code objects' metadata notes (VGPRs,
    SGPRs, their spill counts, private and LDS bytes, waves per SIMD the
    VGPR count allows) and the v_writelane_b32 count of each kernel (SGPR
    spill stores go through v_writelane into a VGPR lane, reloads through
    v_readlane).
Usage: python tools/isa_audit.py [lib.so]   -> exit 1 on a finding.
"""
from __future__ import annotations

import os
import re
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "gfx_imagecompress_amd", "lib", "libgfx_imagecompress_amd.so")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"

_FUNC = re.compile(r"^[0-9a-f]+ <(\S+)>:$")
_RFL = re.compile(r"v_readfirstlane_b32 s(\d+), v")
_SLOAD = re.compile(r"\bs_(?:load|buffer_load)_\w+ s[\[\d:\]]+, s\[(\d+):(\d+)\]")
_SSTORE = re.compile(r"\b(s_store_|s_buffer_store_|s_scratch_store_|s_atomic_|s_buffer_atomic_|s_dcache_wb|"
                     r"s_dcache_discard)")
_SCRATCH = re.compile(r"\bscratch_(load|store)_")


def disassemble(lib: str) -> list[str]:
    tmp = tempfile.mkdtemp(prefix="gic_isa_")
    try:
        dst = os.path.join(tmp, "lib.so")
        shutil.copy(lib, dst)
        subprocess.run([OBJDUMP, "--offloading", dst], cwd=tmp, check=True, capture_output=True)
        out = []
        for f in sorted(os.listdir(tmp)):
            if "amdgcn" in f and "gfx950" in f:
                out += subprocess.run([OBJDUMP, "-d", os.path.join(tmp, f)], check=True, capture_output=True,
                                      text=True).stdout.split("\n")
        return out
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


def resources(lib: str) -> dict:
    """{kernel symbol: {vgpr, sgpr, vgpr_spill, sgpr_spill, private, lds, waves}}
    from the gfx950 code objects' AMDGPU metadata notes."""
    tmp = tempfile.mkdtemp(prefix="gic_res_")
    out = {}
    try:
        dst = os.path.join(tmp, "lib.so")
        shutil.copy(lib, dst)
        subprocess.run([OBJDUMP, "--offloading", dst], cwd=tmp, check=True, capture_output=True)
        for f in sorted(os.listdir(tmp)):
            if "amdgcn" not in f or "gfx950" not in f:
                continue
            notes = subprocess.run([READELF, "--notes", os.path.join(tmp, f)], check=True, capture_output=True,
                                   text=True).stdout
            for m in re.split(r"\n\s+- \.agpr_count", notes):
                nm = re.search(r"\.symbol:\s+(\S+)\.kd", m)
                if not nm:
                    continue

                def g(k):
                    mm = re.search(re.escape(k) + r":\s+(\d+)", m)
                    return int(mm.group(1)) if mm else 0
                v = g(".vgpr_count")
                out[nm.group(1)] = {"vgpr": v, "sgpr": g(".sgpr_count"), "vgpr_spill": g(".vgpr_spill_count"),
                                    "sgpr_spill": g(".sgpr_spill_count"),
                                    "private": g(".private_segment_fixed_size"),
                                    "lds": g(".group_segment_fixed_size"),
                                    "waves": min(8, 512 // max(8, (v + 7) // 8 * 8))}
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    return out


def audit(lines: list[str]) -> dict:
    """{'uniform_loads': [(kernel, text)], 'scalar_stores': [...], 'scratch': {kernel: count}, 'kernels': n}"""
    res = {"uniform_loads": [], "scalar_stores": [], "scratch": {}, "kernels": 0, "writelane": {}}
    kern = "?"
    for i, line in enumerate(lines):
        m = _FUNC.match(line)
        if m:
            kern = m.group(1)
            res["kernels"] += 1
            continue
        if _SSTORE.search(line):
            res["scalar_stores"].append((kern, line.split("//")[0].strip()))
        if _SCRATCH.search(line):
            res["scratch"][kern] = res["scratch"].get(kern, 0) + 1
        if "v_writelane_b32" in line:
            res["writelane"][kern] = res["writelane"].get(kern, 0) + 1
        m = _RFL.search(line)
        if not m:
            continue
        r = int(m.group(1))
        # a waterfall loop compares the read value back against the lanes
        # (v_cmp ... s[r]) and branches back; a straight readfirstlane ->
        # s_load is the miscompile signature
        window = lines[i + 1:i + 6]
        if any("v_cmp" in w and f"s{r}" in w for w in window):
            continue
        for w in window:
            ms = _SLOAD.search(w)
            if ms and int(ms.group(1)) in (r, r - 1):
                res["uniform_loads"].append((kern, w.split("//")[0].strip()))
                break
    return res


def main() -> int:
    lib = sys.argv[1] if len(sys.argv) > 1 else LIB
    res = audit(disassemble(lib))
    print(f"{res['kernels']} device functions")
    for k, n in sorted(res["scratch"].items(), key=lambda kv: -kv[1]):
        print(f"  scratch ops {n:6d}  {k[:100]}")
    rs = resources(lib)
    print("kernel resources (VGPRs, waves/SIMD by VGPRs, spills, private/LDS bytes, v_writelane count):")
    for k, r in sorted(rs.items()):
        print(f"  vgpr {r['vgpr']:3d} ({r['waves']} w)  sgpr {r['sgpr']:3d}  vspill {r['vgpr_spill']:3d}  "
              f"sspill {r['sgpr_spill']:4d}  priv {r['private']:4d}  lds {r['lds']:6d}  "
              f"writelane {res['writelane'].get(k, 0):4d}  {k[:90]}")
    for kind in ("uniform_loads", "scalar_stores"):
        for k, t in res[kind]:
            print(f"FINDING {kind}: {k[:80]}: {t}")
    return 1 if res["uniform_loads"] or res["scalar_stores"] else 0


if __name__ == "__main__":
    sys.exit(main())
