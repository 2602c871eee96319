"""Hybrid-map fusion (fusion/hybrid_map.py) on the MI355X facade.

  create_map_cloud  <- hybrid_map.py:25-60   occupied pixels (img < 100) -> (ox + c*res, oy + (h-1-r)*res, 0)
                       in row-major order; one stable-compaction kernel (ot_occupancy_to_points) replaces the
                       reference's per-pixel Python loop; painted 0.2 grey.
  load_all_objects  <- hybrid_map.py:62-96   sorted *.ply, mesh fallback sampled to 15000 points, painted red,
                       concatenated in file order.
  build_hybrid_map  <- hybrid_map.py:98-124  map cloud first, then the objects; written as one PLY.
Multi-GPU merge of per-rank object clouds (RCCL all-gather) lives in distributed.py.
"""
from __future__ import annotations

import ctypes as C
import glob
import importlib
import os

import numpy as np


def _default_o3d():
    return importlib.import_module(__package__)


def read_map(yaml_file, pgm_file):
    """(img uint8 [h][w], resolution, (ox, oy)) from a ROS map_server YAML + PGM (cv2.imread -> PIL here)."""
    import yaml
    from PIL import Image as PILImage

    with open(yaml_file) as f:
        meta = yaml.safe_load(f)
    with PILImage.open(pgm_file) as im:
        img = np.array(im.convert("L"), dtype=np.uint8)
    origin = meta["origin"]
    return img, float(meta["resolution"]), (float(origin[0]), float(origin[1]))


def occupancy_points(img, resolution, origin, threshold=100):
    """GPU kernel: occupied pixel centres as float64 (Q, 3) device tensor, row-major order."""
    from . import _device as D
    from . import _lib as L

    h, w = img.shape
    d = D.to_device(np.ascontiguousarray(img, dtype=np.uint8))
    out = D.empty((h * w, 3), "float64")
    n = C.c_int64(0)
    L.call("ot_occupancy_to_points", D.ptr(d), int(h), int(w), int(threshold), float(resolution), float(origin[0]),
           float(origin[1]), D.ptr(out), C.byref(n), D.stream_ptr())
    return out[:n.value]


def create_map_cloud(yaml_file, pgm_file, o3d=None, threshold=100):
    o3d = o3d or _default_o3d()
    if not os.path.exists(yaml_file) or not os.path.exists(pgm_file):
        return None
    img, res, origin = read_map(yaml_file, pgm_file)
    pcd = o3d.geometry.PointCloud()
    pcd.points = occupancy_points(img, res, origin, threshold)
    pcd.paint_uniform_color([0.2, 0.2, 0.2])
    return pcd


def load_all_objects(directory, o3d=None, fallback_samples=15000):
    o3d = o3d or _default_o3d()
    files = sorted(glob.glob(os.path.join(directory, "*.ply")))
    if not files:
        return None
    combined = o3d.geometry.PointCloud()
    for path in files:
        try:
            pcd = o3d.io.read_point_cloud(path)
            if len(pcd.points) == 0:
                pcd = o3d.io.read_triangle_mesh(path).sample_points_uniformly(number_of_points=fallback_samples)
            pcd.paint_uniform_color([1.0, 0.0, 0.0])
            combined += pcd
        except Exception as exc:  # reference: report and continue
            print(f"Error loading {path}: {exc}")
    return combined


def build_hybrid_map(yaml_file, pgm_file, obj_dir, save_path, o3d=None):
    """main() of hybrid_map.py without the viewer: returns the merged cloud (also written to save_path)."""
    o3d = o3d or _default_o3d()
    map_pcd = create_map_cloud(yaml_file, pgm_file, o3d)
    if map_pcd is None:
        return None
    objs = load_all_objects(obj_dir, o3d)
    merged = map_pcd if (objs is None or len(objs.points) == 0) else map_pcd + objs
    os.makedirs(os.path.dirname(os.path.abspath(save_path)), exist_ok=True)
    o3d.io.write_point_cloud(save_path, merged)
    return merged
