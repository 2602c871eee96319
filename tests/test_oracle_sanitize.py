"""The CPU oracle under AddressSanitizer + UndefinedBehaviorSanitizer: `make -C oracle sanitize`
builds otslam_oracle.cpp with -fsanitize=address,undefined and drives every entry point on a small synthetic scene
(oracle/sanitize_check.cpp).  Any sanitizer report fails the run."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("make") is None, reason="needs g++ and make")
def test_oracle_asan_ubsan():
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "sanitize"], capture_output=True, text=True,
                       timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "ERROR: AddressSanitizer" not in out and "runtime error" not in out, out[-4000:]
    assert out.strip().splitlines()[-1] == "OK"
