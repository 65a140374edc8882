"""CPU check of the BC1 search's exact division by 3 (csrc/gic_fastdiv.h,
compiled for the host) against IEEE float division on a stride of all float
inputs; the exhaustive GPU check (tools/rcp_check.hip) is logged in
profiles/r03d_fastdiv_check.txt."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_div3_rn_equals_ieee_division(tmp_path):
    exe = str(tmp_path / "fastdiv_check")
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-std=c++17", os.path.join(ROOT, "tests", "fastdiv_check.cpp"),
                    "-o", exe], check=True)
    out = subprocess.run([exe, "7"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout + out.stderr
    assert out.stdout.startswith("0/")
