"""Deterministic on-disk datasets in the reference layout, used both to capture the caller fixture from the
reference scripts and to replay it against this repo's restated callers (the file CONTENTS that matter to the
callers are the pose text files and the map; images only need to exist)."""
from __future__ import annotations

import os

import numpy as np


def _rigid(rng):
    a = rng.uniform(-np.pi, np.pi, 3)
    cz, sz, cy, sy, cx, sx = np.cos(a[0]), np.sin(a[0]), np.cos(a[1]), np.sin(a[1]), np.cos(a[2]), np.sin(a[2])
    R = np.array([[cz, -sz, 0], [sz, cz, 0], [0, 0, 1]]) @ np.array([[cy, 0, sy], [0, 1, 0], [-sy, 0, cy]]) @ \
        np.array([[1, 0, 0], [0, cx, -sx], [0, sx, cx]])
    T = np.eye(4)
    T[:3, :3], T[:3, 3] = R, rng.uniform(-2, 2, 3)
    return T


def write_scan_dataset(base):
    """Object_0: frames 1..11 (lexical order 1,10,11,2,...); Object_1: colour/depth 1..3 but poses 1 and 3 only
    (the reference pairs lists by index, so frame 2 gets pose 3 and frame 3 raises IndexError -> skipped);
    gt_* frames 0..2 for reconstruct_rgbd_gt.py; color_0000/depth_0000 for check_one_frame.py."""
    rng = np.random.default_rng(1234)
    for sub in ("color", "depth", "poses"):
        os.makedirs(os.path.join(base, sub), exist_ok=True)

    def touch(p):
        with open(p, "wb") as f:
            f.write(b"\0")

    for label, frames, pose_frames in (("Object_0", range(1, 12), range(1, 12)), ("Object_1", range(1, 4), (1, 3))):
        for i in frames:
            touch(os.path.join(base, "color", f"{label}_{i}.jpg"))
            touch(os.path.join(base, "depth", f"{label}_{i}.png"))
        for i in pose_frames:
            np.savetxt(os.path.join(base, "poses", f"{label}_{i}.txt"), _rigid(rng), fmt="%.6f")
    for i in range(3):
        touch(os.path.join(base, "color", f"gt_color_{i}.jpg"))
        touch(os.path.join(base, "depth", f"gt_depth_{i}.png"))
        np.savetxt(os.path.join(base, "poses", f"gt_pose_{i}.txt"), _rigid(rng), fmt="%.6f")
    touch(os.path.join(base, "color", "color_0000.png"))
    touch(os.path.join(base, "depth", "depth_0000.png"))


def write_map_dataset(base):
    """A 37x53 PGM with ~15 % occupied pixels (values < 100), its YAML, and two small object PLYs (ASCII)."""
    from PIL import Image

    rng = np.random.default_rng(99)
    os.makedirs(os.path.join(base, "map"), exist_ok=True)
    os.makedirs(os.path.join(base, "objects"), exist_ok=True)
    img = rng.integers(100, 256, size=(37, 53)).astype(np.uint8)
    occ = rng.uniform(size=img.shape) < 0.15
    img[occ] = rng.integers(0, 100, size=int(occ.sum())).astype(np.uint8)
    img[0, 0], img[5, 7] = 99, 100  # threshold edge: 99 occupied, 100 free
    Image.fromarray(img, mode="L").save(os.path.join(base, "map", "map_selective.pgm"))
    with open(os.path.join(base, "map", "map_selective.yaml"), "w") as f:
        f.write("image: map_selective.pgm\nresolution: 0.05\norigin: [-12.35, -7.6, 0.0]\nnegate: 0\n"
                "occupied_thresh: 0.65\nfree_thresh: 0.196\n")
    for name, n in (("Object_1.ply", 7), ("Object_0.ply", 5)):
        pts = rng.uniform(-1, 1, size=(n, 3))
        with open(os.path.join(base, "objects", name), "w") as f:
            f.write(f"ply\nformat ascii 1.0\nelement vertex {n}\nproperty double x\nproperty double y\n"
                    f"property double z\nend_header\n")
            for p in pts:
                f.write(f"{p[0]!r} {p[1]!r} {p[2]!r}\n")
