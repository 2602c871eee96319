"""The reciprocal-table division of the FAST integrate kernels (csrc/tsdf.hip k_batch_integrate<C64, true>) is exact:
q0 = RN(a*y), q = fma(fma(-b, q0, a), y, q0) with y = RN(1/b) equals the IEEE quotient a/b for every integer
divisor b in [1, 4096].  binary32 (tsdf mean): every 16th significand of a in [1, 2) against every b (the full
exhaustive run, stride 1, is recorded in DESIGN.md); binary64 (colour mean): random and near-boundary a per b.
Host arithmetic only (g++, strict IEEE: -ffp-contract=off); no GPU."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_markstein_reciprocal_table_exact(tmp_path):
    exe = str(tmp_path / "markstein_check")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-fopenmp",
                    os.path.join(ROOT, "tools", "markstein_check.cpp"), "-o", exe], check=True, timeout=300)
    r = subprocess.run([exe, "16", "20000"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.strip().splitlines()[-1] == "OK"
