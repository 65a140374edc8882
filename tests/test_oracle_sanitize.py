"""AddressSanitizer + UndefinedBehaviorSanitizer run of the CPU restatement
("race detection / sanitizers").

The oracle is the sole checker of every parity claim, so it is built once
with -fsanitize=address,undefined (oracle/Makefile `sanitize`) and a driver
(oracle/sanitize_main.c) runs every entry -- BC1-BC5 image loops, BC7 exact /
staged / pruned / performance < 1, bc7enc16, the block entries, BC6H signed
and unsigned -- through the pthread pools on small seeded inputs.  Any
ASan report or UBSan runtime error fails the test.  CPU only.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_oracle_under_asan_ubsan():
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "-s", "sanitize"], check=True)
    # verify_asan_link_order=0: the environment may preload other libraries
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:verify_asan_link_order=0",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    r = subprocess.run([os.path.join(ROOT, "oracle", "_san", "oracle_san")], env=env, capture_output=True, text=True,
                       timeout=900)
    log = r.stdout + r.stderr
    assert r.returncode == 0, log[-4000:]
    assert "runtime error" not in log and "AddressSanitizer" not in log, log[-4000:]
    assert "rc=0" in r.stdout
