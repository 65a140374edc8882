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


@pytest.fixture(scope="module")
def res():
    if not os.path.exists(isa_audit.READELF) or not os.path.exists(isa_audit.LIB):
        pytest.skip("llvm-readelf or the library missing")
    return isa_audit.resources(isa_audit.LIB)


def _kernel(res, part):
    ks = [k for k in res if part in k]
    assert ks, part
    return res[ks[0]]


def test_bc7_fast_shakers_run_eight_waves(res):
    """The fast BC7 wave kernels (quant_single_point_d deferred to the slow
    kernels, bc7_wave.inc FAST) fit 8 waves per SIMD.  k_shake_wave<8> spills
    one VGPR (8 B of scratch per lane) at 64 VGPRs; the spill-free 7-wave
    build measured 2.4 % slower on the exact 256-row run
    (profiles/r04a_bc7_exact256_ab.txt), so the bound allows that one."""
    for part in ("k_shake_waveILi8E", "k_shake_waveILi4E", "k_dual_waveE"):
        r = _kernel(res, part)
        assert r["waves"] == 8 and r["vgpr_spill"] <= 1 and r["private"] <= 8, (part, r)


def test_bc4_bc5_image_kernels_use_no_scratch_arrays(res):
    """CompBlock1's running arrays live in LDS columns, not scratch; the kernels
    run at least 6 waves per SIMD with at most a few spilled VGPRs."""
    for part, waves in (("bc45_image_kernelILi4E", 6), ("bc45_image_kernelILi5E", 6)):
        r = _kernel(res, part)
        assert r["waves"] >= waves and r["private"] <= 32 and r["vgpr_spill"] <= 4, (part, r)


def test_bc1_default_kernel_runs_four_waves_without_scratch(res):
    """RefinementSteps == 1 (the default) has its own BC1 kernel whose Refine
    sweeps the LDS-parked colours once per candidate set (refine_pass3): no
    scratch, so the kernel's HBM traffic is the texels in and the blocks out
    (profiles/traffic_bc1.json)."""
    r = _kernel(res, "bc1_image_kernelILb0ELb1E")
    assert r["waves"] >= 4 and r["private"] == 0 and r["vgpr_spill"] == 0, r


def test_quant_sub_runs_three_waves(res):
    """k_quant_sub (f64 quantiser, latency bound) fits 3 waves per SIMD with
    the indices packed in bytes and the lattice offsets in LDS."""
    r = _kernel(res, "k_quant_subE")
    assert r["waves"] >= 3 and r["private"] <= 64, r
