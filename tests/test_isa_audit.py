"""Machine-code audit of the built gfx950 library (CPU only: disassembly).

No kernel may contain a scalar load whose address is a bare v_readfirstlane of
a VGPR (the signature of the round-1 dual-index quantiser fault: a
lane-divergent constant-table index emitted as a wave-uniform load), and no
kernel may write through the scalar data cache.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import isa_audit  # noqa: E402


@pytest.fixture(scope="module")
def isa():
    if not os.path.exists(isa_audit.OBJDUMP):
        pytest.skip("llvm-objdump not in this image")
    if not os.path.exists(isa_audit.LIB):
        pytest.skip("library not built")
    return isa_audit.audit(isa_audit.disassemble(isa_audit.LIB))


def test_library_has_device_code(isa):
    assert isa["kernels"] >= 15


def test_no_scalarised_divergent_loads(isa):
    assert isa["uniform_loads"] == [], isa["uniform_loads"][:5]


def test_no_scalar_cache_writes(isa):
    assert isa["scalar_stores"] == [], isa["scalar_stores"][:5]


def test_detector_flags_the_fault_signature():
    lines = ["0000000000001000 <k>:",
             "\tv_readfirstlane_b32 s4, v8  // x",
             "\tv_readfirstlane_b32 s5, v9  // x",
             "\ts_load_dword s4, s[4:5], 0x20  // x",
             "0000000000002000 <w>:",
             "\tv_readfirstlane_b32 s4, v8  // x",
             "\tv_cmp_eq_u32_e32 vcc, s4, v8  // waterfall",
             "\ts_load_dword s4, s[4:5], 0x20  // x"]
    res = isa_audit.audit(lines)
    assert [k for k, _ in res["uniform_loads"]] == ["k"]
