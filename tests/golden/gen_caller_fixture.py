"""Generate tests/golden/caller_fixture.json by RUNNING the reference scripts (read from /root/reference) against
a recording `open3d` stub on the deterministic datasets of dataset.py.

Run once in the build container (the GPU box has no /root/reference):
    python tests/golden/gen_caller_fixture.py
Only the recorded call logs (paths relative to the dataset root, arguments, extrinsic matrices, written point
arrays) are committed; no reference source is copied.  The hard-coded dataset paths at the top of each script
(e.g. reconstruct_rgbd_filter.py:11) are redirected to a temporary directory before execution.
"""
from __future__ import annotations

import json
import os
import re
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import dataset  # noqa: E402
import recorder  # noqa: E402

REF = "/root/reference"
SCRIPTS = {
    "reconstruct_rgbd_filter": ("3d_model/reconstruct_rgbd_filter.py", "scan", {"base_dir": ""}),
    "reconstruct_rgbd": ("3d_model/reconstruct_rgbd.py", "scan", {"base_dir": ""}),
    "multi_reconstruct_rgbd_filter": ("3d_model/multi_reconstruct_rgbd_filter.py", "scan", {"base_dir": ""}),
    "reconstruct_rgbd_gt": ("3d_model/reconstruct_rgbd_gt.py", "scan", {"base_dir": ""}),
    "check_one_frame": ("3d_model/check_one_frame.py", "scan", {"base_dir": ""}),
    "hybrid_map": ("fusion/hybrid_map.py", "map", {"map_base": "map", "obj_dir": "objects",
                                                    "save_path": "out/hybrid_map_selective.ply"}),
}


def run_script(rel, root, assigns):
    src = open(os.path.join(REF, rel)).read()
    for var, sub in assigns.items():
        target = os.path.join(root, sub) if sub else root
        src, n = re.subn(rf"(?m)^{var}\s*=\s*\".*\"\s*$", f"{var} = {target!r}", src)
        assert n == 1, (rel, var)
    rec = recorder.Recorder(root)
    saved = {k: sys.modules.get(k) for k in ("open3d", "cv2")}
    sys.modules["open3d"] = recorder.make_open3d(rec)
    sys.modules["cv2"] = recorder.make_cv2()
    try:
        exec(compile(src, os.path.join(REF, rel), "exec"), {"__name__": "__main__", "__file__": rel})
    except Exception as exc:  # e.g. reconstruct_rgbd.py has no per-frame try/except: the script dies
        rec.log("exception", type=type(exc).__name__)
    finally:
        for k, v in saved.items():
            if v is None:
                sys.modules.pop(k, None)
            else:
                sys.modules[k] = v
    return rec.calls


def main():
    out = {}
    for name, (rel, kind, assigns) in SCRIPTS.items():
        with tempfile.TemporaryDirectory() as root:
            if kind == "scan":
                dataset.write_scan_dataset(root)
            else:
                dataset.write_map_dataset(root)
            out[name] = run_script(rel, root, assigns)
    path = os.path.join(HERE, "caller_fixture.json")
    with open(path, "w") as f:
        json.dump({"generated_by": "tests/golden/gen_caller_fixture.py (reference scripts executed against a "
                                   "recording open3d stub)", "scripts": {k: v[0] for k, v in SCRIPTS.items()},
                   "calls": out}, f)
    print(f"wrote {path}: " + ", ".join(f"{k}={len(v)} calls" for k, v in out.items()))


if __name__ == "__main__":
    main()
