"""Run a Python script or module against a kernel-variant build (A/B timing; tools only, never the product).

    python tools/with_variant.py <name|base> bench.py --steps 5 ...
    python tools/with_variant.py <name|base> -m pytest tests/test_gpu_tsdf.py -m gpu

<name> selects object-triggered-3d-slam_amd/variants/libotslam_<name>.so (built by tools/variants.sh build);
"base" runs the product library unchanged.
"""
import importlib
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
name, rest = sys.argv[1], sys.argv[2:]
L = importlib.import_module("object-triggered-3d-slam_amd._lib")
if name != "base":
    L.use_variant(os.path.join(ROOT, "object-triggered-3d-slam_amd", "variants", f"libotslam_{name}.so"))
if rest[0] == "-m":
    sys.argv = [rest[1]] + rest[2:]
    runpy.run_module(rest[1], run_name="__main__", alter_sys=True)
else:
    sys.argv = rest
    sys.path.insert(0, os.path.dirname(os.path.abspath(rest[0])))
    runpy.run_path(rest[0], run_name="__main__")
