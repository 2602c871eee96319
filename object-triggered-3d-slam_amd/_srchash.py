"""Source hash of the HIP library: sha256 (16 hex) over csrc/*.hip, csrc/*.h, csrc/Makefile and include/*.h.

Shared by the build (csrc/Makefile compiles it into libotslam_hip.so, returned by ot_version()) and by
_lib.load(), which refuses a library whose compiled-in hash differs from the sources beside it (a stale build).
Standalone on purpose: `python3 _srchash.py` runs without importing the package (no torch, no ctypes).
"""
from __future__ import annotations

import hashlib
import os

_HERE = os.path.dirname(os.path.abspath(__file__))


def compute(pkg_dir: str = _HERE) -> str:
    h = hashlib.sha256()
    csrc = os.path.join(pkg_dir, "csrc")
    inc = os.path.join(os.path.dirname(pkg_dir), "include")
    files = sorted(f for f in os.listdir(csrc) if f.endswith((".hip", ".h")) or f == "Makefile")
    paths = [os.path.join(csrc, f) for f in files] + sorted(os.path.join(inc, f) for f in os.listdir(inc)
                                                            if f.endswith(".h"))
    for p in paths:
        h.update(os.path.basename(p).encode())
        with open(p, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(compute())
