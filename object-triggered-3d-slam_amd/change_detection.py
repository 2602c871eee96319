"""Change detection against a saved map — SURVEY.md §8(f) rank 2, BASELINE configs[4] ("diff vs saved map").

Host-side mirrors of the reference's change-detection code, backed by the HIP kernels of libotslam_hip.so:

* ``smart_paste(base_img, overlay_img, x, y, w, h)`` — fusion/2d_selective_merge.py:58-69 (same signature; the
  base grid is updated in place and returned, as the reference does).
* ``ChangeDetector`` — ros2_ws/src/lidar_detection/src/diff_node.cpp (ChangeDetectorNode): the node's parameters
  (distance_threshold, time_threshold, grid_resolution, decay_rate) and its per-scan callback, with the beam
  comparison batched over many scans on the GPU and the time-decayed evidence grid kept in native host code.
* ``voxel_key_diff(new, old, voxel_size, origin)`` — added / removed lattice cells of an object cloud versus the
  saved map's cloud (the 3-D half of configs[4]'s diff).
* ``virtual_scan(grid, resolution, origin, template, poses)`` — ros2_ws/src/lidar_detection/src/virtual_scan_node.cpp
  (VirtualScanNode): the scan the saved map would return at each robot pose (the diff node's /virtual_scan input),
  ray-marched per beam on the GPU; ``occupancy_from_pgm`` / ``tf2_get_yaw`` prepare its inputs.

Every compute call goes through the C ABI; there is no CPU implementation in this module.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _device as D
from . import _lib as L

UNKNOWN_PIXEL = 205  # 2d_selective_merge.py:63
PASTE_THRESHOLD = 5  # 2d_selective_merge.py:64


def smart_paste(base_img, overlay_img, x, y, w, h, unknown=UNKNOWN_PIXEL, threshold=PASTE_THRESHOLD):
    """2d_selective_merge.py:58-69: cells of ``overlay_img`` inside the rectangle that carry data (outside
    unknown ± threshold) overwrite ``base_img``.  Updates ``base_img`` (uint8 numpy array) in place and returns
    it; a rectangle reaching outside the image leaves it unchanged."""
    n_changed = _paste(base_img, overlay_img, x, y, w, h, unknown, threshold)
    del n_changed
    return base_img


def merge_maps(old_map, new_map, unknown=UNKNOWN_PIXEL, threshold=PASTE_THRESHOLD):
    """Whole-map smart_paste of a new occupancy grid onto the saved one.  Returns (merged copy, changed cells)."""
    out = np.array(old_map, dtype=np.uint8, copy=True)
    h, w = out.shape
    n = _paste(out, new_map, 0, 0, w, h, unknown, threshold)
    return out, n


def _paste(base_img, overlay_img, x, y, w, h, unknown, threshold):
    base = np.asarray(base_img)
    if base.dtype != np.uint8 or base.ndim != 2:
        raise RuntimeError("[smart_paste] base_img must be a 2-D uint8 grid")
    over = np.ascontiguousarray(overlay_img, dtype=np.uint8)
    if over.shape != base.shape:
        raise RuntimeError("[smart_paste] overlay_img must have the base grid's shape")
    hh, ww = base.shape
    if x < 0 or y < 0 or x + w > ww or y + h > hh or w <= 0 or h <= 0:
        return 0
    db = D.to_device(np.ascontiguousarray(base))
    do = D.to_device(over)
    n = C.c_int64(0)
    L.call("ot_grid_smart_paste", D.ptr(db), D.ptr(do), hh, ww, int(x), int(y), int(w), int(h), int(unknown),
           int(threshold), C.byref(n), D.stream_ptr())
    base[...] = D.to_host(db)
    return n.value


def voxel_key_diff(new_cloud, old_cloud, voxel_size, origin):
    """Lattice cells floor((p - origin) / voxel_size) occupied by ``new_cloud`` but not ``old_cloud`` (added) and
    the converse (removed); int32 [k][3] each, sorted lexicographically.  Clouds: PointCloud or (n, 3) arrays."""
    a = _xyz_dev(new_cloud)
    b = _xyz_dev(old_cloud)
    n, m = int(a.shape[0]), int(b.shape[0])
    added = D.empty((max(n, 1), 3), "int32")
    removed = D.empty((max(m, 1), 3), "int32")
    na, nr = C.c_int64(0), C.c_int64(0)
    o = (C.c_double * 3)(*[float(v) for v in origin])
    L.call("ot_voxel_key_diff", D.ptr(a) if n else None, n, D.ptr(b) if m else None, m, float(voxel_size), o,
           D.ptr(added), C.byref(na), D.ptr(removed), C.byref(nr), D.stream_ptr())
    return D.to_host(added[:na.value]), D.to_host(removed[:nr.value])


def voxel_key_diff_multi(new_clouds, old_clouds, voxel_size, origin):
    """voxel_key_diff for many objects in one pass (object j of new_clouds vs object j of old_clouds).  Returns
    (added, removed) as int32 [k][4] = (object, x, y, z), sorted by object then cell."""
    if len(new_clouds) != len(old_clouds):
        raise RuntimeError("[voxel_key_diff] new and old object lists differ in length")
    import torch

    def cat(clouds):
        parts = [_xyz_dev(c) for c in clouds]
        off = np.zeros(len(parts) + 1, np.int64)
        off[1:] = np.cumsum([int(p.shape[0]) for p in parts])
        xyz = torch.cat(parts, 0).contiguous() if parts else D.empty((0, 3), "float64")
        return xyz, off

    a, oa = cat(new_clouds)
    b, ob = cat(old_clouds)
    added = D.empty((max(int(oa[-1]), 1), 4), "int32")
    removed = D.empty((max(int(ob[-1]), 1), 4), "int32")
    na, nr = C.c_int64(0), C.c_int64(0)
    o = (C.c_double * 3)(*[float(v) for v in origin])
    L.call("ot_voxel_key_diff_multi", D.ptr(a) if oa[-1] else None, oa.ctypes.data_as(C.c_void_p),
           D.ptr(b) if ob[-1] else None, ob.ctypes.data_as(C.c_void_p), len(new_clouds), float(voxel_size), o,
           D.ptr(added), C.byref(na), D.ptr(removed), C.byref(nr), D.stream_ptr())
    return D.to_host(added[:na.value]), D.to_host(removed[:nr.value])


def _xyz_dev(c):
    if hasattr(c, "_xyz"):
        return c._xyz.dev()
    a = np.ascontiguousarray(np.asarray(c, dtype=np.float64).reshape(-1, 3))
    return D.to_device(a)


@dataclass
class LaserScan:
    """The sensor_msgs/LaserScan fields the change detector reads."""

    ranges: np.ndarray
    angle_min: float
    angle_increment: float
    range_max: float = float("inf")


class ChangeDetector:
    """ChangeDetectorNode (diff_node.cpp): compares each real scan with the virtual scan rendered from the saved
    map.  ``scan_callback`` handles one scan pair; ``process`` a batch of pairs (one GPU launch for all beams, then
    the evidence-grid updates in scan order).  Outputs are the node's two published clouds — added (new) and
    removed (gone) cells above time_threshold — as float32 (k, 3) arrays sorted by cell."""

    SEARCH_WINDOW = 20  # diff_node.cpp:113, :143

    def __init__(self, distance_threshold=0.5, time_threshold=2.0, grid_resolution=0.1, decay_rate=0.5):
        self.distance_threshold = float(distance_threshold)
        self.time_threshold = float(time_threshold)
        self.grid_resolution = float(grid_resolution)
        self.decay_rate = float(decay_rate)
        self._grids = []
        for _ in range(2):
            g = C.c_void_p()
            L.call("ot_change_grid_create", self.time_threshold, self.decay_rate, self.grid_resolution, C.byref(g))
            self._grids.append(g)

    def __del__(self):
        for g in getattr(self, "_grids", []):
            try:
                L.call("ot_change_grid_destroy", g)
            except Exception:
                pass

    def scan_callback(self, real_scan: LaserScan, virtual_scan: LaserScan, pose, dt):
        """One scan pair (pose = map<-sensor as (tx, ty, tz, qx, qy, qz, qw)); returns (added, removed)."""
        if len(real_scan.ranges) != len(virtual_scan.ranges):  # diff_node.cpp:87
            return self.published()
        return self.process(np.asarray(real_scan.ranges, np.float32)[None], np.asarray(virtual_scan.ranges,
                            np.float32)[None], real_scan, virtual_scan, np.asarray(pose, np.float64)[None], [dt])

    def process(self, real_ranges, virtual_ranges, real_meta: LaserScan, virtual_meta: LaserScan, poses, dts):
        """Batch of B scan pairs: ranges float32 [B][N], poses [B][7], dts [B] (seconds since the previous scan)."""
        flags_new, flags_gone, keys_new, keys_gone = self.flag_beams(real_ranges, virtual_ranges, real_meta,
                                                                     virtual_meta, poses)
        for b, dt in enumerate(dts):
            for g, k, f in ((self._grids[0], keys_new[b], flags_new[b]), (self._grids[1], keys_gone[b], flags_gone[b])):
                k = np.ascontiguousarray(k, np.int32)
                f = np.ascontiguousarray(f, np.uint8)
                L.call("ot_change_grid_update", g, k.ctypes.data_as(C.c_void_p), f.ctypes.data_as(C.c_void_p),
                       f.shape[0], float(dt))
        return self.published()

    def flag_beams(self, real_ranges, virtual_ranges, real_meta: LaserScan, virtual_meta: LaserScan, poses):
        """GPU part: per-beam new / gone flags and map-grid cells for B scans (diff_node.cpp:103-160)."""
        R = _as_dev(real_ranges, np.float32)
        V = _as_dev(virtual_ranges, np.float32)
        if R.shape != V.shape or R.dim() != 2:
            raise RuntimeError("[ChangeDetector] real and virtual ranges must both be [n_scans][n_beams]")
        B, N = int(R.shape[0]), int(R.shape[1])
        P = np.ascontiguousarray(np.asarray(poses, np.float64).reshape(B, 7))
        fn, fg = D.empty((B, N), "uint8"), D.empty((B, N), "uint8")
        kn, kg = D.empty((B, N, 2), "int32"), D.empty((B, N, 2), "int32")
        L.call("ot_scan_diff", D.ptr(R), D.ptr(V), B, N, float(real_meta.angle_min), float(real_meta.angle_increment),
               float(real_meta.range_max), float(virtual_meta.angle_min), float(virtual_meta.angle_increment),
               self.distance_threshold, self.SEARCH_WINDOW, P.ctypes.data_as(C.c_void_p), self.grid_resolution,
               D.ptr(fn), D.ptr(fg), D.ptr(kn), D.ptr(kg), D.stream_ptr())
        return D.to_host(fn), D.to_host(fg), D.to_host(kn), D.to_host(kg)

    def published(self):
        """(added, removed): cells above time_threshold as float32 (x*res + res/2, y*res + res/2, 0)."""
        out = []
        for g in self._grids:
            n = C.c_int64(0)
            L.call("ot_change_grid_publish", g, None, 0, C.byref(n))
            xyz = np.zeros((n.value, 3), np.float32)
            if n.value:
                L.call("ot_change_grid_publish", g, xyz.ctypes.data_as(C.c_void_p), n.value, C.byref(n))
            out.append(xyz)
        return out[0], out[1]


def tf2_get_yaw(qx, qy, qz, qw):
    """tf2::getYaw(quaternion) (tf2/utils.h: Matrix3x3(q).getEulerYPR): yaw of the rotation matrix of q."""
    d = qx * qx + qy * qy + qz * qz + qw * qw
    s = 2.0 / d
    xs, ys, zs = qx * s, qy * s, qz * s
    wz, xx, xy = qw * zs, qx * xs, qx * ys
    yy, zz = qy * ys, qz * zs
    m00, m10, m20 = 1.0 - (yy + zz), xy + wz, qx * zs - qw * ys
    if abs(m20) >= 1:  # gimbal lock: tf2 returns yaw 0
        return 0.0
    cp = np.cos(-np.arcsin(m20))
    return float(np.arctan2(m10 / cp, m00 / cp))


def occupancy_from_pgm(img, negate=0, occupied_thresh=0.65, free_thresh=0.196):
    """map_server's trinary PGM -> OccupancyGrid data (int8: 100 occupied, 0 free, -1 unknown)."""
    v = np.asarray(img, dtype=np.float64)
    p = v / 255.0 if negate else (255.0 - v) / 255.0
    out = np.full(v.shape, -1, np.int8)
    out[p > occupied_thresh] = 100
    out[p < free_thresh] = 0
    return out[::-1].copy()  # PGM row 0 is the top of the map; OccupancyGrid row 0 is the bottom (origin)


def virtual_scan(grid, resolution, origin, template: LaserScan, poses, n_beams=None):
    """virtual_scan_node.cpp:245-292 (VirtualScanNode, "copycat" mode): the LaserScan the saved map would produce
    at each robot pose, with the template scan's angles and range_max.  grid: OccupancyGrid int8 [h][w]
    (row 0 at origin); poses [B][3] = (x, y, yaw).  Returns float32 ranges [B][n_beams] (+inf = no hit)."""
    g = _as_dev(grid, np.int8)
    if g.dim() != 2:
        raise RuntimeError("[VirtualScan] grid must be [height][width]")
    P = np.ascontiguousarray(np.asarray(poses, np.float64).reshape(-1, 3))
    n = int(n_beams if n_beams is not None else len(template.ranges))
    out = D.empty((P.shape[0], n), "float32")
    L.call("ot_virtual_scan", D.ptr(g), int(g.shape[0]), int(g.shape[1]), float(resolution), float(origin[0]),
           float(origin[1]), P.shape[0], n, float(template.angle_min), float(template.angle_increment),
           float(template.range_max), P.ctypes.data_as(C.c_void_p), D.ptr(out), D.stream_ptr())
    return D.to_host(out)


def _as_dev(a, dtype):
    if D.is_tensor(a):
        return a.contiguous()
    return D.to_device(np.ascontiguousarray(np.asarray(a, dtype=dtype)))
