"""CPU ORACLE bindings — TEST INFRASTRUCTURE ONLY.

Loads oracle/libotslam_oracle.so (a strict-IEEE C++ restatement of the Open3D algorithms on the reference hot
path; see otslam_oracle.cpp for the parity status: *parity unpinned* vs Open3D, which is absent here).
Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.  The product
package (object-triggered-3d-slam_amd/) never imports it.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libotslam_oracle.so")
_lib = None

_d = C.c_double
_i64 = C.c_int64
_i32 = C.c_int
_p = C.c_void_p


def build(force: bool = False) -> str:
    src = os.path.join(_HERE, "otslam_oracle.cpp")
    if force or not os.path.exists(_LIB_PATH) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src):
        subprocess.run(["make", "-C", _HERE], check=True, stdout=subprocess.DEVNULL)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = C.CDLL(_LIB_PATH)
        sig = {
            "oro_inverse4": (None, [_p, _p]),
            "oro_depth_to_float": (None, [_p, _p, _i64, _d, _d]),
            "oro_depth_multiplier": (None, [_i32, _i32, _d, _d, _d, _d, _p]),
            "oro_unproject": (_i64, [_p, _p, _i32, _i32, _d, _d, _d, _d, _p, _i32, _p, _p]),
            "oro_voxel_down_sample": (_i64, [_p, _p, _p, _i64, _d, _p, _p, _p, _p]),
            "oro_tsdf_create": (_p, [_d, _d, _i32, _i32]),
            "oro_tsdf_destroy": (None, [_p]),
            "oro_tsdf_integrate": (_i64, [_p, _p, _p, _i32, _i32, _d, _d, _d, _d, _p]),
            "oro_tsdf_num_units": (_i64, [_p]),
            "oro_tsdf_total_updates": (_i64, [_p]),
            "oro_tsdf_unit_integrations": (_i64, [_p]),
            "oro_tsdf_export": (None, [_p, _p, _p, _p, _p]),
            "oro_tsdf_extract_mesh": (None, [_p, C.POINTER(_i64), C.POINTER(_i64)]),
            "oro_tsdf_fetch_mesh": (None, [_p, _p, _p, _p]),
            "oro_mesh_vertex_normals": (None, [_p, _i64, _p, _i64, _p]),
            "oro_mesh_sample_uniform": (_i32, [_p, _p, _p, _i64, _p, _i64, _i64, C.c_uint64, _p, _p, _p]),
            "oro_mesh_surface_area": (C.c_double, [_p, _p, _i64]),
            "oro_filter_min_z": (_i64, [_p, _p, _i64, _d, _p, _p]),
            "oro_remove_statistical_outlier": (_i64, [_p, _i64, _i32, _d, _p, _p]),
            "oro_remove_radius_outlier": (_i64, [_p, _i64, _i32, _d, _p]),
            "oro_occupancy_to_points": (_i64, [_p, _i32, _i32, _i32, _d, _d, _d, _p]),
            "oro_point_cloud_distance": (None, [_p, _i64, _p, _i64, _p]),
            "oro_scan_diff": (None, [_p, _p, _i32, _i32, C.c_float, C.c_float, C.c_float, C.c_float, C.c_float, _d,
                                     _i32, _p, _d, _p, _p, _p, _p]),
            "oro_change_grid_run": (_i64, [_p, _p, _i32, _i32, _p, _d, _d, _d, _p]),
            "oro_virtual_scan": (None, [_p, _i32, _i32, C.c_float, C.c_float, C.c_float, _i32, _i32, C.c_float,
                                        C.c_float, C.c_float, _p, _p]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _c(a, dtype):
    return None if a is None else np.ascontiguousarray(a, dtype=dtype)


def inverse4(m):
    m = _c(m, np.float64)
    out = np.empty((4, 4), np.float64)
    lib().oro_inverse4(_ptr(m), _ptr(out))
    return out


def depth_to_float(depth_u16, depth_scale=1000.0, depth_trunc=3.0):
    d = _c(depth_u16, np.uint16)
    out = np.empty(d.shape, np.float32)
    lib().oro_depth_to_float(_ptr(d), _ptr(out), d.size, depth_scale, depth_trunc)
    return out


def depth_multiplier(w, h, fx, fy, cx, cy):
    out = np.empty((h, w), np.float32)
    lib().oro_depth_multiplier(w, h, fx, fy, cx, cy, _ptr(out))
    return out


def unproject(depth_f32, color, intr, extrinsic=None, stride=1):
    """PointCloud.create_from_rgbd_image / create_from_depth_image. intr = (w, h, fx, fy, cx, cy)."""
    w, h, fx, fy, cx, cy = intr
    d = _c(depth_f32, np.float32)
    col = _c(color, np.uint8)
    ext = _c(np.eye(4) if extrinsic is None else extrinsic, np.float64)
    cap = ((h + stride - 1) // stride) * ((w + stride - 1) // stride)
    xyz = np.empty((cap, 3), np.float64)
    rgb = np.empty((cap, 3), np.float64) if col is not None else None
    n = lib().oro_unproject(_ptr(d), _ptr(col), w, h, fx, fy, cx, cy, _ptr(ext), stride, _ptr(xyz), _ptr(rgb))
    return xyz[:n].copy(), (rgb[:n].copy() if rgb is not None else None)


def voxel_down_sample(xyz, rgb, voxel_size, normals=None):
    p = _c(xyz, np.float64)
    c = _c(rgb, np.float64)
    nn = _c(normals, np.float64)
    n = p.shape[0]
    ox = np.empty((max(n, 1), 3), np.float64)
    oc = np.empty((max(n, 1), 3), np.float64) if c is not None else None
    on = np.empty((max(n, 1), 3), np.float64) if nn is not None else None
    ok = np.empty((max(n, 1), 3), np.int32)
    k = lib().oro_voxel_down_sample(_ptr(p), _ptr(c), _ptr(nn), n, voxel_size, _ptr(ox), _ptr(oc), _ptr(on), _ptr(ok))
    if k < 0:
        raise RuntimeError("[VoxelDownSample] voxel_size <= 0." if k == -1 else "[VoxelDownSample] voxel_size is too small.")
    return ox[:k].copy(), (oc[:k].copy() if oc is not None else None), ok[:k].copy(), (on[:k].copy() if on is not None else None)


class TSDF:
    """ScalableTSDFVolume restatement (units sorted by key on export)."""

    def __init__(self, voxel_length=0.01, sdf_trunc=0.04, color_type=1, stride=4):
        self.h = lib().oro_tsdf_create(voxel_length, sdf_trunc, color_type, stride)

    def __del__(self):
        if getattr(self, "h", None):
            lib().oro_tsdf_destroy(self.h)
            self.h = None

    def integrate(self, depth_f32, color, intr, extrinsic):
        w, h, fx, fy, cx, cy = intr
        d = _c(depth_f32, np.float32)
        col = _c(color, np.uint8)
        ext = _c(extrinsic, np.float64)
        return lib().oro_tsdf_integrate(self.h, _ptr(d), _ptr(col), w, h, fx, fy, cx, cy, _ptr(ext))

    def num_units(self):
        return lib().oro_tsdf_num_units(self.h)

    def total_updates(self):
        return lib().oro_tsdf_total_updates(self.h)

    def unit_integrations(self):
        return lib().oro_tsdf_unit_integrations(self.h)

    def export(self):
        u = self.num_units()
        keys = np.empty((u, 3), np.int32)
        tsdf = np.empty((u, 4096), np.float32)
        weight = np.empty((u, 4096), np.float32)
        color = np.empty((u, 4096, 3), np.float64)
        lib().oro_tsdf_export(self.h, _ptr(keys), _ptr(tsdf), _ptr(weight), _ptr(color))
        return keys, tsdf, weight, color

    def extract_triangle_mesh(self):
        nv, nt = C.c_int64(0), C.c_int64(0)
        lib().oro_tsdf_extract_mesh(self.h, C.byref(nv), C.byref(nt))
        V = np.empty((nv.value, 3), np.float64)
        VC = np.empty((nv.value, 3), np.float64)
        T = np.empty((nt.value, 3), np.int32)
        lib().oro_tsdf_fetch_mesh(self.h, _ptr(V), _ptr(VC), _ptr(T))
        return V, VC, T


def vertex_normals(V, T):
    V = _c(V, np.float64)
    T = _c(T, np.int32)
    N = np.empty_like(V)
    lib().oro_mesh_vertex_normals(_ptr(V), V.shape[0], _ptr(T), T.shape[0], _ptr(N))
    return N


def surface_area(V, T):
    V = _c(V, np.float64)
    T = _c(T, np.int32)
    return float(lib().oro_mesh_surface_area(_ptr(V), _ptr(T), T.shape[0]))


def sample_points_uniformly(V, T, n_points, seed, VN=None, VC=None):
    V = _c(V, np.float64)
    T = _c(T, np.int32)
    VN = _c(VN, np.float64)
    VC = _c(VC, np.float64)
    P = np.empty((n_points, 3), np.float64)
    PN = np.empty((n_points, 3), np.float64) if VN is not None else None
    PC = np.empty((n_points, 3), np.float64) if VC is not None else None
    rc = lib().oro_mesh_sample_uniform(_ptr(V), _ptr(VN), _ptr(VC), V.shape[0], _ptr(T), T.shape[0], n_points,
                                       seed, _ptr(P), _ptr(PN), _ptr(PC))
    if rc != 0:
        raise RuntimeError("[SamplePointsUniformly] invalid input")
    return P, PN, PC


def filter_min_z(xyz, rgb, zmin):
    p = _c(xyz, np.float64)
    c = _c(rgb, np.float64)
    ox = np.empty_like(p)
    oc = np.empty_like(c) if c is not None else None
    k = lib().oro_filter_min_z(_ptr(p), _ptr(c), p.shape[0], zmin, _ptr(ox), _ptr(oc))
    return ox[:k].copy(), (oc[:k].copy() if oc is not None else None)


def batch_cell_shift(nb_neighbors):
    """log2 of the SOR cell edge in voxels of the batched configs[2] chain (filter_batch.hip fb_cell_shift): the
    largest m <= 4 with 4^m <= 2 t, t = max(0.9 k, 2) -- the power of two nearest sqrt(t) in ratio (ties up); 2 for
    nb_neighbors = 20."""
    t = max(0.9 * nb_neighbors, 2.0)
    m = 0
    while m < 4 and 4.0 ** (m + 1) <= 2.0 * t:
        m += 1
    return m


def cell_major_order(keys, m):
    """Permutation that puts a voxel cloud (voxel_down_sample's integer keys (kx, ky, kz), any order) in the batched
    chain's canonical order: lexicographic by the cell (kx, ky, kz) >> m, then by the voxel inside the cell.  Open3D
    emits its voxels in hash-map order; the batch's order is the SOR grid's cell order (filter_batch.hip)."""
    k = np.asarray(keys, np.int64).reshape(-1, 3)
    c, l = k >> m, k & ((1 << m) - 1)
    return np.lexsort((l[:, 2], l[:, 1], l[:, 0], c[:, 2], c[:, 1], c[:, 0]))


def remove_statistical_outlier(xyz, nb_neighbors, std_ratio):
    p = _c(xyz, np.float64)
    n = p.shape[0]
    idx = np.empty(max(n, 1), np.int64)
    avg = np.empty(max(n, 1), np.float64)
    k = lib().oro_remove_statistical_outlier(_ptr(p), n, nb_neighbors, std_ratio, _ptr(idx), _ptr(avg))
    if k < 0:
        raise RuntimeError("Illegal input parameters")
    return idx[:k].copy(), avg[:n].copy()


def remove_radius_outlier(xyz, nb_points, radius):
    p = _c(xyz, np.float64)
    n = p.shape[0]
    idx = np.empty(max(n, 1), np.int64)
    k = lib().oro_remove_radius_outlier(_ptr(p), n, nb_points, radius, _ptr(idx))
    if k < 0:
        raise RuntimeError("Illegal input parameters")
    return idx[:k].copy()


def occupancy_to_points(img, threshold, res, ox, oy):
    im = _c(img, np.uint8)
    h, w = im.shape
    out = np.empty((h * w, 3), np.float64)
    k = lib().oro_occupancy_to_points(_ptr(im), h, w, threshold, res, ox, oy, _ptr(out))
    return out[:k].copy()


def point_cloud_distance(src, tgt):
    """PointCloud.compute_point_cloud_distance (eval_cone.py:99,103): exhaustive float64 1-NN distances."""
    a = _c(src, np.float64).reshape(-1, 3)
    b = _c(tgt, np.float64).reshape(-1, 3)
    out = np.empty(max(a.shape[0], 1), np.float64)
    lib().oro_point_cloud_distance(_ptr(a), a.shape[0], _ptr(b), b.shape[0], _ptr(out))
    return out[:a.shape[0]].copy()


def smart_paste(base_img, overlay_img, x, y, w, h, unknown=205, threshold=5):
    """2d_selective_merge.py:58-69 restated with numpy (returns a new array; out-of-image rectangle: unchanged)."""
    out = np.array(base_img, dtype=np.uint8, copy=True)
    hi_, wi_ = out.shape
    if x < 0 or y < 0 or x + w > wi_ or y + h > hi_:
        return out
    new = np.asarray(overlay_img, dtype=np.uint8)[y:y + h, x:x + w].astype(np.int64)
    known = (new < unknown - threshold) | (new > unknown + threshold)
    roi = out[y:y + h, x:x + w]
    roi[known] = new[known].astype(np.uint8)
    return out


def voxel_key_diff(new_xyz, old_xyz, voxel_size, origin):
    """Lattice-key set difference: (keys of new absent from old, keys of old absent from new), each sorted."""
    def keys(p):
        p = np.asarray(p, np.float64).reshape(-1, 3)
        k = np.floor((p - np.asarray(origin, np.float64)) / voxel_size).astype(np.int64)
        return np.unique(k, axis=0) if len(k) else np.zeros((0, 3), np.int64)

    a, b = keys(new_xyz), keys(old_xyz)
    sa = {tuple(r) for r in a.tolist()}
    sb = {tuple(r) for r in b.tolist()}
    added = np.array(sorted(sa - sb), np.int64).reshape(-1, 3)
    removed = np.array(sorted(sb - sa), np.int64).reshape(-1, 3)
    return added.astype(np.int32), removed.astype(np.int32)


def scan_diff(real, virt, r_amin, r_inc, r_max, v_amin, v_inc, thresh, window, poses, grid_res):
    """diff_node.cpp:103-160 per beam of a batch of scans (see otslam_oracle.cpp)."""
    R = _c(real, np.float32)
    V = _c(virt, np.float32)
    B, N = R.shape
    P = _c(poses, np.float64).reshape(B, 7)
    nf, gf = np.zeros((B, N), np.uint8), np.zeros((B, N), np.uint8)
    nk, gk = np.zeros((B, N, 2), np.int32), np.zeros((B, N, 2), np.int32)
    lib().oro_scan_diff(_ptr(R), _ptr(V), B, N, r_amin, r_inc, r_max, v_amin, v_inc, thresh, window, _ptr(P),
                        grid_res, _ptr(nf), _ptr(gf), _ptr(nk), _ptr(gk))
    return nf, gf, nk, gk


def change_grid_run(keys, flags, dts, time_thresh, decay_rate, grid_res):
    """updateGrid over the scans in order, then publishCloud's cells (float32 [k][3], sorted by (x, y))."""
    K = _c(keys, np.int32)
    F = _c(flags, np.uint8)
    B, N = F.shape
    D = _c(dts, np.float64)
    n = lib().oro_change_grid_run(_ptr(K), _ptr(F), B, N, _ptr(D), time_thresh, decay_rate, grid_res, None)
    out = np.zeros((max(n, 1), 3), np.float32)
    lib().oro_change_grid_run(_ptr(K), _ptr(F), B, N, _ptr(D), time_thresh, decay_rate, grid_res, _ptr(out))
    return out[:n].copy()


def virtual_scan(grid, resolution, origin_x, origin_y, n_beams, angle_min, angle_increment, range_max, poses):
    """virtual_scan_node.cpp:245-292 for poses [B][3] (x, y, yaw): float32 ranges [B][n_beams]."""
    g = _c(grid, np.int8)
    h, w = g.shape
    P = _c(poses, np.float64).reshape(-1, 3)
    out = np.empty((P.shape[0], n_beams), np.float32)
    lib().oro_virtual_scan(_ptr(g), h, w, resolution, origin_x, origin_y, P.shape[0], n_beams, angle_min,
                           angle_increment, range_max, _ptr(P), _ptr(out))
    return out
