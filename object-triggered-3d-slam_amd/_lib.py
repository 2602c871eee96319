"""ctypes binding of the C ABI in include/otslam.h (libotslam_hip.so, built in-tree for gfx950).

This is the only way the facade reaches the hot path.  There is no CPU fallback: if the library is missing or
no HIP device is present, every compute call raises RuntimeError.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# the product library; A/B timing of kernel variants goes through tools/with_variant.py (use_variant), never through
# the product's environment
LIB_PATH = os.path.join(_HERE, "libotslam_hip.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "otslam.h")

OT_OK = 0
OT_ERR_INVALID_ARGUMENT = 1
OT_ERR_UNSUPPORTED_FORMAT = 2
OT_ERR_CAPACITY = 3
OT_ERR_HIP = 4

OT_COLOR_NONE = 0
OT_COLOR_RGB8 = 1


class ot_intrinsics(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("fx", C.c_double), ("fy", C.c_double),
                ("cx", C.c_double), ("cy", C.c_double)]


class ot_mesh_sample_job(C.Structure):
    _fields_ = [("vertices", C.c_void_p), ("vertex_normals", C.c_void_p), ("vertex_colors", C.c_void_p),
                ("n_vertices", C.c_int64), ("triangles", C.c_void_p), ("n_triangles", C.c_int64),
                ("out_xyz", C.c_void_p), ("out_normals", C.c_void_p), ("out_colors", C.c_void_p)]


_p = C.c_void_p
_d = C.c_double
_i32 = C.c_int32
_i64 = C.c_int64
_pi64 = C.POINTER(C.c_int64)
_pint = C.POINTER(ot_intrinsics)

# name -> argtypes (restype is int32 status unless listed in _RESTYPES)
SIGNATURES = {
    "ot_last_error": [],
    "ot_version": [],
    "ot_abi_version": [],
    "ot_depth_to_float": [_p, _p, _i64, _d, _d, _p],
    "ot_depth_multiplier": [_pint, _p, _p],
    "ot_unproject": [_p, _p, _pint, _p, _i32, _p, _p, _i64, _pi64, _p],
    "ot_voxel_down_sample": [_p, _p, _p, _i64, _d, _p, _p, _p, _p, _pi64, _p],
    "ot_remove_statistical_outlier": [_p, _i64, _i32, _d, _p, _p, _pi64, _p],
    "ot_remove_radius_outlier": [_p, _i64, _i32, _d, _p, _pi64, _p],
    "ot_compute_point_cloud_distance": [_p, _i64, _p, _i64, _p, _p],
    "ot_filter_min_z": [_p, _p, _i64, _d, _p, _p, _pi64, _p],
    "ot_gather_rows3": [_p, _p, _i64, _p, _p],
    "ot_tsdf_create": [_d, _d, _i32, _i32, _i32, _i64, C.POINTER(_p)],
    "ot_tsdf_destroy": [_p],
    "ot_tsdf_reset": [_p],
    "ot_tsdf_reset_async": [_p, _p],
    "ot_tsdf_integrate": [_p, _p, _p, _pint, _p, _p],
    "ot_tsdf_integrate_u16": [_p, _p, _p, _pint, _p, _d, _d, _p],
    "ot_tsdf_integrate_u16_frames": [_p, _i32, _p, _p, _pint, _p, _d, _d, _p],
    "ot_tsdf_flush": [_p, _p],
    "ot_tsdf_set_batch": [_p, _i32],
    "ot_tsdf_set_frontend_overlap": [_p, _i32],
    "ot_tsdf_pending_frames": [_p, _p],
    "ot_tsdf_num_units": [_p, _pi64, _p],
    "ot_tsdf_counters": [_p, _pi64, _pi64, _p],
    "ot_tsdf_set_color_precision": [_p, _i32],
    "ot_tsdf_get_color_precision": [_p, _p],
    "ot_tsdf_export_color64": [_p, _i64, _p, _p],
    "ot_tsdf_set_profiling": [_p, _i32],
    "ot_tsdf_kernel_time": [_p, C.POINTER(C.c_double), _pi64],
    "ot_tsdf_frontend_time": [_p, C.POINTER(C.c_double), _pi64],
    "ot_tsdf_export_units": [_p, _i64, _p, _p, _p, _p, _p],
    "ot_tsdf_import_units": [_p, _i64, _p, _p, _p, _p, _p],
    "ot_tsdf_import_units_color64": [_p, _i64, _p, _p, _p, _p, _p],
    "ot_tsdf_set_shard": [_p, _i32, _i32],
    "ot_tsdf_set_shard_block": [_p, _i32],
    "ot_tsdf_set_shard_sector": [_p, _i32, _i32, _d, _d],
    "ot_tsdf_batch_stats": [_p, _pi64, _pi64, _pi64],
    "ot_tsdf_border_destinations": [_p, _i64, _p, _p, _p],
    "ot_tsdf_mesh_serial": [_p, _pi64],
    "ot_tsdf_mesh_vertex_normals": [_p, _i64, _p, _i64, _p, _i64, _p, _p],
    "ot_tsdf_export_border": [_p, _i64, _p, _p, _p, _p, _pi64, _p],
    "ot_tsdf_import_border": [_p, _i64, _p, _p, _p, _p, _p],
    "ot_tsdf_fetch_mesh_keys": [_p, _p, _p, _p],
    "ot_tsdf_extract_triangle_mesh": [_p, _pi64, _pi64, _p],
    "ot_tsdf_fetch_triangle_mesh": [_p, _p, _p, _p, _p],
    "ot_tsdf_extract_triangle_mesh_count": [_p, _pi64, _pi64, _p],
    "ot_tsdf_emit_triangle_mesh": [_p, _p, _p, _p, _p],
    "ot_tsdf_extract_triangle_mesh_into": [_p, _p, _p, _p, _i64, _i64, _pi64, _pi64, _p],
    "ot_tsdf_extract_sample_min_z": [_p, _p, _p, _p, _i64, _i64, _p, _p, _i64, C.c_uint64, _d, _p, _p, _pi64, _pi64,
                                     _pi64, _p],
    "ot_mesh_compute_vertex_normals": [_p, _i64, _p, _i64, _p, _p],
    "ot_mesh_sample_points_uniformly": [_p, _p, _p, _i64, _p, _i64, _i64, C.c_uint64, _p, _p, _p, _p],
    "ot_mesh_sample_points_uniformly_batch": [_p, _i32, _i64, C.c_uint64, _p],
    "ot_mesh_sample_points_min_z": [_p, _i32, _i64, C.c_uint64, _d, _pi64, _p],
    "ot_mesh_sample_points_min_z_async": [_p, _i32, _i64, C.c_uint64, _d, _p],
    "ot_mesh_sample_points_min_z_wait": [_i32, _pi64],
    "ot_mesh_sample_points_uniformly_after": [_p, _i32, _i64, C.c_uint64, _p, _p],
    "ot_mesh_get_surface_area": [_p, _i64, _p, _i64, C.POINTER(C.c_double), _p],
    "ot_occupancy_to_points": [_p, _i32, _i32, _i32, _d, _d, _d, _p, _pi64, _p],
    "ot_grid_smart_paste": [_p, _p, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _i32, _pi64, _p],
    "ot_voxel_key_diff": [_p, _i64, _p, _i64, _d, _p, _p, _pi64, _p, _pi64, _p],
    "ot_voxel_key_diff_multi": [_p, _p, _p, _p, _i32, _d, _p, _p, _pi64, _p, _pi64, _p],
    "ot_scan_diff": [_p, _p, _i32, _i32, C.c_float, C.c_float, C.c_float, C.c_float, C.c_float, _d, _i32, _p, _d,
                     _p, _p, _p, _p, _p],
    "ot_virtual_scan": [_p, _i32, _i32, C.c_float, C.c_float, C.c_float, _i32, _i32, C.c_float, C.c_float,
                        C.c_float, _p, _p, _p],
    "ot_change_grid_create": [_d, _d, _d, C.POINTER(_p)],
    "ot_change_grid_destroy": [_p],
    "ot_change_grid_update": [_p, _p, _p, _i64, _d],
    "ot_change_grid_publish": [_p, _p, _i64, _pi64],
    "ot_rgbd_filter_create": [_pint, _i32, _d, _d, _d, _i32, _d, C.POINTER(_p)],
    "ot_rgbd_filter_destroy": [_p],
    "ot_rgbd_filter_run": [_p, _i32, _p, _p, _p, _p],
    "ot_rgbd_filter_sizes": [_p, _pi64, _pi64, _pi64, _p, _p, _p],
    "ot_rgbd_filter_outputs": [_p, C.POINTER(_p), C.POINTER(_p), C.POINTER(_p), C.POINTER(_p), C.POINTER(_p),
                               C.POINTER(_p)],
    "ot_rgbd_filter_copy": [_p, _i32, _p, _p, _p, _p, _p, _p, _p],
}
_RESTYPES = {"ot_last_error": C.c_char_p, "ot_version": C.c_char_p, "ot_abi_version": C.c_int32,
             "otx_alloc_count": C.c_longlong}

_lib = None
_lock = threading.Lock()


class OTError(RuntimeError):
    """Raised for any non-OK status; message mirrors Open3D's utility::LogError text."""


# test hooks exported by the library but outside the drop-in boundary (not declared in include/otslam.h)
TEST_SIGNATURES = {
    "otx_serial_chain_f64": [_p, _i64, _i32, _p, _pi64, _p],
    "otx_chain_walk_trace": [_p, _i64, _i32, _p, _p, _i32, _p],
    "otx_tsdf_stats": [_p, _p],
    "otx_unit_sort_radix": [_i32],
    "otx_sor_netfill": [_i32],
    "otx_integrate_fine": [_i32],
    "otx_touch_stage_blocks": [_i32],
    "otx_touch_frames": [_i32],
    "otx_split_frontend": [_i32],
    "otx_defer_integrate": [_i32],
    "otx_integrate_depth": [_i32],
    "otx_mc_emit_fork": [_i32],
    "otx_normals_at": [_i32],
    "otx_sampler_hi_stream": [_i32],
    "otx_sort_pairs_u64_u32": [_p, _p, _p, _p, _i64, _i32, _p],
    "otx_sort_segments_u32_u32": [_p, _p, _p, _p, _p, _i32, _i32, _p],
    "otx_alloc_count": [],
}


def use_variant(path: str) -> None:
    """Test / tool hook: load a kernel-variant build from object-triggered-3d-slam_amd/variants/ instead of the
    product library (A/B timing).  Must run before the first load(); the product never calls it."""
    global LIB_PATH
    path = os.path.abspath(path)
    if os.path.dirname(path) != os.path.join(_HERE, "variants"):
        raise RuntimeError(f"variant libraries live in {os.path.join(_HERE, 'variants')}: {path}")
    if _lib is not None:
        raise RuntimeError("use_variant() after the library was loaded")
    LIB_PATH = path


def load():
    """Load libotslam_hip.so (raises RuntimeError, never falls back)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"HIP extension missing: {LIB_PATH} (run __graft_entry__.build())")
        lib = C.CDLL(LIB_PATH)
        lib.ot_version.argtypes, lib.ot_version.restype = [], C.c_char_p
        built, src = library_source_hash(lib), source_hash()
        if built != src:  # binary provenance: the .so must be the build of the sources beside it
            raise RuntimeError(f"stale HIP library {LIB_PATH}: built from sources {built or '(no hash)'}, "
                               f"sources here are {src} (run __graft_entry__.build())")
        missing = []
        for name, argtypes in {**SIGNATURES, **TEST_SIGNATURES}.items():
            try:
                f = getattr(lib, name)
            except AttributeError:
                missing.append(name)
                continue
            f.argtypes = argtypes
            f.restype = _RESTYPES.get(name, C.c_int32)
        lib._ot_missing = set(missing)
        _lib = lib
    return _lib


def call(name, *args):
    lib = load()
    if name in lib._ot_missing:
        raise RuntimeError(f"{LIB_PATH} does not export {name} (stale build?)")
    st = getattr(lib, name)(*args)
    if st != OT_OK:
        msg = lib.ot_last_error().decode(errors="replace")
        raise OTError(msg or f"{name} failed with status {st}")
    return st


def alloc_count() -> int:
    """Device allocations made so far by the library's grow-only buffers (test / bench hook)."""
    return int(load().otx_alloc_count())


def intrinsics_struct(intr) -> ot_intrinsics:
    return ot_intrinsics(int(intr.width), int(intr.height), float(intr.fx), float(intr.fy), float(intr.cx),
                         float(intr.cy))


def source_hash() -> str:
    """sha256 (16 hex) over the HIP sources, headers and Makefile the library is built from (_srchash.py): tags
    measurements (profiles/pmc_traffic.json) with the build they were taken on; the Makefile compiles the same hash
    into the library (ot_version), and load() refuses a library built from other sources."""
    from . import _srchash

    return _srchash.compute()


def library_source_hash(lib) -> str:
    """The source hash compiled into a loaded library (ot_version() ends with ' src=<hash>'), '' if absent."""
    ver = lib.ot_version().decode(errors="replace")
    return ver.rsplit(" src=", 1)[1].strip() if " src=" in ver else ""
