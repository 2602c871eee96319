"""Batched configs[2] filter chain (device-resident): many RGB-D frames through the per-frame Open3D sequence

    rgbd = RGBDImage.create_from_color_and_depth(color, depth, depth_scale, depth_trunc)     (check_one_frame.py:22-25)
    pcd = PointCloud.create_from_rgbd_image(rgbd, intrinsic, extrinsic)                       (check_one_frame.py:27)
    down = pcd.voxel_down_sample(voxel_size)                                                  (check_one_frame.py:28)
    kept, ind = down.remove_statistical_outlier(nb_neighbors, std_ratio)                     (north_star, A.7)

in one C-ABI call per batch (ot_rgbd_filter_run).  Results equal the per-frame calls bit for bit; the batch form
exists because the per-frame chain is bound by its host round trips, not by the GPU.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _device as D
from . import _lib as L
from .geometry import PointCloud, _Arr


class RGBDFilterBatch:
    def __init__(self, intrinsic, max_frames=32, depth_scale=1000.0, depth_trunc=5.0, voxel_size=0.005,
                 nb_neighbors=20, std_ratio=2.0):
        D.require_gpu()
        self._intr = L.intrinsics_struct(intrinsic)
        self._h = C.c_void_p()
        L.call("ot_rgbd_filter_create", C.byref(self._intr), int(max_frames), float(depth_scale), float(depth_trunc),
               float(voxel_size), int(nb_neighbors), float(std_ratio), C.byref(self._h))
        self.max_frames = int(max_frames)
        self._keep = None
        self.n_frames = 0

    def __del__(self):
        h = getattr(self, "_h", None)
        if h and h.value:
            try:
                L.load().ot_rgbd_filter_destroy(h)
            except Exception:
                pass
            self._h = C.c_void_p()

    def run(self, depth, color, extrinsics):
        """depth uint16 [F][h][w], color uint8 [F][h][w][3] (numpy or device tensors), extrinsics float64 [F][4][4]."""
        d = D.to_device(depth, "uint16" if not D.is_tensor(depth) else None)
        c = D.to_device(color, "uint8" if not D.is_tensor(color) else None)
        ext = np.ascontiguousarray(np.asarray(extrinsics, np.float64).reshape(-1, 16))
        F = ext.shape[0]
        if d.shape[0] != F or c.shape[0] != F:
            raise RuntimeError("[rgbd_filter] depth / color / extrinsics frame counts differ")
        if tuple(d.shape[1:]) != (self._intr.height, self._intr.width) or \
                tuple(c.shape[1:]) != (self._intr.height, self._intr.width, 3):
            raise RuntimeError("[CreatePointCloudFromRGBDImage] Unsupported image format.")
        self._keep = (d, c)
        L.call("ot_rgbd_filter_run", self._h, F, D.ptr(d), D.ptr(c), ext.ctypes.data_as(C.c_void_p), D.stream_ptr())
        self.n_frames = F
        n = F + 1
        po, vo, ko = (np.zeros(n, np.int64) for _ in range(3))
        P, K, KK = C.c_int64(0), C.c_int64(0), C.c_int64(0)
        L.call("ot_rgbd_filter_sizes", self._h, C.byref(P), C.byref(K), C.byref(KK), po.ctypes.data_as(C.c_void_p),
               vo.ctypes.data_as(C.c_void_p), ko.ctypes.data_as(C.c_void_p))
        self.points, self.voxels, self.kept = P.value, K.value, KK.value
        self.point_offsets, self.voxel_offsets, self.kept_offsets = po, vo, ko
        return self

    def frame(self, f):
        """(kept PointCloud with colours, kept indices) of frame f — remove_statistical_outlier's return value."""
        n = int(self.kept_offsets[f + 1] - self.kept_offsets[f])
        xyz, rgb, idx = D.empty((n, 3), "float64"), D.empty((n, 3), "float64"), D.empty((n,), "int64")
        L.call("ot_rgbd_filter_copy", self._h, int(f), D.ptr(xyz), D.ptr(rgb), D.ptr(idx), None, None, None,
               D.stream_ptr())
        pcd = PointCloud()
        pcd._xyz, pcd._rgb = _Arr(dev=xyz), _Arr(dev=rgb)
        return pcd, D.to_host(idx).tolist()

    def voxel_cloud(self, f):
        """frame f's voxel_down_sample output (points + colours) and its mean kNN distances."""
        n = int(self.voxel_offsets[f + 1] - self.voxel_offsets[f])
        xyz, rgb, avg = D.empty((n, 3), "float64"), D.empty((n, 3), "float64"), D.empty((n,), "float64")
        L.call("ot_rgbd_filter_copy", self._h, int(f), None, None, None, D.ptr(xyz), D.ptr(rgb), D.ptr(avg),
               D.stream_ptr())
        pcd = PointCloud()
        pcd._xyz, pcd._rgb = _Arr(dev=xyz), _Arr(dev=rgb)
        return pcd, D.to_host(avg)
