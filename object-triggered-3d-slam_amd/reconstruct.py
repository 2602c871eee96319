"""Restated callers of the reference's offline reconstruction scripts (3d_model/*.py), running on this package.

Each function keeps the reference's file discovery, frame order, pose convention, Open3D call sequence,
constants and skip-on-error behaviour, but takes the Open3D-shaped module as a parameter (`o3d`, default: this
package) so the same code runs on the MI355X facade, or on a recording stub in the caller-parity test
(tests/test_callers.py against the fixture captured from the reference scripts themselves).

  get_unique_object_names  <- reconstruct_rgbd_filter.py:39-58
  reconstruct_object       <- reconstruct_rgbd_filter.py:60-141 (output="points") and
                              reconstruct_rgbd.py:60-119 (output="mesh")
  reconstruct_range        <- multi_reconstruct_rgbd_filter.py:51-137
  reconstruct_gt           <- reconstruct_rgbd_gt.py:28-98
  run_all                  <- reconstruct_rgbd_filter.py:143-157 / reconstruct_rgbd.py:121-135
  check_one_frame          <- check_one_frame.py:1-31
"""
from __future__ import annotations

import glob
import importlib
import os
import sys
from dataclasses import dataclass, field

import numpy as np

from .synth import T_FIX, T_FIX_GT


def _default_o3d():
    return importlib.import_module(__package__)


@dataclass
class ScanConfig:
    """Module-level constants of the reference scripts (reconstruct_rgbd_filter.py:11-37)."""
    base_dir: str
    width: int = 640
    height: int = 480
    fx: float = 565.6009
    fy: float = 565.6009
    cx: float = 320.5
    cy: float = 240.5
    voxel_length: float = 0.01          # :82
    sdf_trunc: float = 0.04             # :83
    depth_scale: float = 1000.0         # :100
    depth_trunc: float = 3.0            # :101
    z_filter: float = 0.03              # :22
    n_samples: int = 100000             # :123
    t_fix: np.ndarray = field(default_factory=lambda: T_FIX.copy())
    sample_seed: int = 0                # this build's seeded sampler (Open3D's is unseeded)

    @property
    def color_dir(self):
        return os.path.join(self.base_dir, "color")

    @property
    def depth_dir(self):
        return os.path.join(self.base_dir, "depth")

    @property
    def pose_dir(self):
        return os.path.join(self.base_dir, "poses")

    @property
    def save_dir(self):
        return os.path.join(self.base_dir, "3d_reconst")


def _log(msg, log):
    if log:
        print(msg, file=sys.stdout)


def get_unique_object_names(cfg: ScanConfig):
    """Object labels = colour file name minus its last `_<n>` token, sorted (reconstruct_rgbd_filter.py:39-58)."""
    labels = set()
    for path in glob.glob(os.path.join(cfg.color_dir, "*.jpg")):
        tokens = os.path.basename(path).split("_")
        if len(tokens) >= 2:
            labels.add("_".join(tokens[:-1]))
    return sorted(labels)


def _frame_lists(cfg: ScanConfig, label: str):
    """Per-object file lists in LEXICAL order (sorted(glob)), as the reference builds them (:68-70)."""
    pick = lambda d, ext: sorted(glob.glob(os.path.join(d, f"{label}_*.{ext}")))
    return pick(cfg.color_dir, "jpg"), pick(cfg.depth_dir, "png"), pick(cfg.pose_dir, "txt")


def _intrinsic(o3d, cfg):
    return o3d.camera.PinholeCameraIntrinsic(cfg.width, cfg.height, cfg.fx, cfg.fy, cfg.cx, cfg.cy)


def _new_volume(o3d, cfg):
    integ = o3d.pipelines.integration
    return integ.ScalableTSDFVolume(voxel_length=cfg.voxel_length, sdf_trunc=cfg.sdf_trunc,
                                    color_type=integ.TSDFVolumeColorType.RGB8)


def _integrate_frame(o3d, cfg, volume, intrinsic, colors, depths, poses, i):
    """Frame i: decode, extrinsic = inv(pose_ros @ T_fix), RGBD with depth_scale/trunc, integrate (:91-105).
    The three lists are indexed in the reference's order (colour, depth, pose), so a short pose list fails
    after both images were read — the same side effects as the reference's IndexError path."""
    color = o3d.io.read_image(colors[i])
    depth = o3d.io.read_image(depths[i])
    pose_ros = np.loadtxt(poses[i])
    extrinsic = np.linalg.inv(pose_ros @ cfg.t_fix)
    rgbd = o3d.geometry.RGBDImage.create_from_color_and_depth(
        color, depth, depth_scale=cfg.depth_scale, depth_trunc=cfg.depth_trunc, convert_rgb_to_intensity=False)
    volume.integrate(rgbd, intrinsic, extrinsic)


def _mesh_empty(mesh):
    """The reference's `len(mesh.vertices) == 0` (reconstruct_rgbd_filter.py:115-117).  On this package's mesh it reads
    the row count only (TriangleMesh.has_vertices, also Open3D API): `mesh.vertices` would hand out a writable host view,
    which settles the deferred vertex normals and copies V to the host and back."""
    has = getattr(mesh, "has_vertices", None)
    return (not has()) if callable(has) else len(mesh.vertices) == 0


def _filtered_cloud(o3d, cfg, mesh):
    """sample_points_uniformly(N) then keep z >= threshold, points and colours only (:123-132).  This package's
    facade does both in one pass (TriangleMesh.sample_points_min_z: the same cloud); Open3D takes the reference's
    steps."""
    if hasattr(mesh, "sample_points_min_z"):
        return mesh.sample_points_min_z(cfg.n_samples, cfg.z_filter, cfg.sample_seed)
    pcd = mesh.sample_points_uniformly(number_of_points=cfg.n_samples)
    pts = np.asarray(pcd.points)
    cols = np.asarray(pcd.colors)
    keep = pts[:, 2] >= cfg.z_filter
    out = o3d.geometry.PointCloud()
    out.points = o3d.utility.Vector3dVector(pts[keep])
    out.colors = o3d.utility.Vector3dVector(cols[keep])
    return out


def reconstruct_object(label: str, cfg: ScanConfig, o3d=None, output: str = "points", log: bool = False):
    """Reconstruct one object; returns the written path (or None when nothing was produced).

    output="points": reconstruct_rgbd_filter.py — per-frame errors are skipped (:89,108-109), the mesh is
    sampled and Z-filtered and written as a point cloud.  output="mesh": reconstruct_rgbd.py — no error
    skipping, the mesh itself is written."""
    o3d = o3d or _default_o3d()
    colors, depths, poses = _frame_lists(cfg, label)
    n = len(colors)
    if n == 0:
        _log(f"No files found for {label}", log)
        return None
    os.makedirs(cfg.save_dir, exist_ok=True)
    intrinsic = _intrinsic(o3d, cfg)
    volume = _new_volume(o3d, cfg)
    for i in range(n):
        if output == "mesh":
            _integrate_frame(o3d, cfg, volume, intrinsic, colors, depths, poses, i)
            continue
        try:
            _integrate_frame(o3d, cfg, volume, intrinsic, colors, depths, poses, i)
        except Exception as exc:  # reference: print and skip the frame
            _log(f"Skipping frame {i + 1} due to error: {exc}", log)
    path = os.path.join(cfg.save_dir, f"{label}.ply")
    fused = getattr(volume, "extract_mesh_and_sample_min_z", None)
    if output == "points" and fused is not None:
        # this package: :112-132 (extract, normals, sample, Z mask) in one host call, the same cloud
        mesh, cloud = fused(cfg.n_samples, cfg.z_filter, cfg.sample_seed)
        if cloud is None:
            _log("Mesh is empty", log)
            return None
        o3d.io.write_point_cloud(path, cloud)
        return path
    mesh = volume.extract_triangle_mesh()
    mesh.compute_vertex_normals()
    if output == "mesh":
        o3d.io.write_triangle_mesh(path, mesh)
        return path
    if _mesh_empty(mesh):
        _log("Mesh is empty", log)
        return None
    o3d.io.write_point_cloud(path, _filtered_cloud(o3d, cfg, mesh))
    return path


def reconstruct_range(name: str, start: int, end: int, cfg: ScanConfig, file_prefix: str = "Object_0", o3d=None,
                      log: bool = False):
    """multi_reconstruct_rgbd_filter.py:51-137: frames `<prefix>_<i>` for i in [start, end] in NUMERIC order;
    a missing colour file is skipped, any other per-frame error is reported and skipped."""
    o3d = o3d or _default_o3d()
    os.makedirs(cfg.save_dir, exist_ok=True)
    intrinsic = _intrinsic(o3d, cfg)
    volume = _new_volume(o3d, cfg)
    done = 0
    for i in range(start, end + 1):
        stem = f"{file_prefix}_{i}"
        cpath = os.path.join(cfg.color_dir, stem + ".jpg")
        if not os.path.exists(cpath):
            _log(f"File missing {stem}.jpg, skipping", log)
            continue
        try:
            _integrate_frame(o3d, cfg, volume, intrinsic, [cpath], [os.path.join(cfg.depth_dir, stem + ".png")],
                             [os.path.join(cfg.pose_dir, stem + ".txt")], 0)
            done += 1
        except Exception as exc:
            _log(f"Error on frame {i}: {exc}", log)
    if done == 0:
        return None
    path = os.path.join(cfg.save_dir, f"{name}.ply")
    fused = getattr(volume, "extract_mesh_and_sample_min_z", None)
    if fused is not None:  # this package: extract, normals, sample and Z mask in one host call
        mesh, cloud = fused(cfg.n_samples, cfg.z_filter, cfg.sample_seed)
        if cloud is None:
            return None
        o3d.io.write_point_cloud(path, cloud)
        return path
    mesh = volume.extract_triangle_mesh()
    mesh.compute_vertex_normals()
    if _mesh_empty(mesh):
        return None
    o3d.io.write_point_cloud(path, _filtered_cloud(o3d, cfg, mesh))
    return path


def reconstruct_gt(cfg: ScanConfig, o3d=None, log: bool = False):
    """reconstruct_rgbd_gt.py:28-98: gt_color*/gt_depth*/gt_pose* files, the alternative T_fix, mesh output."""
    o3d = o3d or _default_o3d()
    pick = lambda d, pat: sorted(glob.glob(os.path.join(d, pat)))
    colors = pick(cfg.color_dir, "gt_color*.jpg")
    depths = pick(cfg.depth_dir, "gt_depth*.png")
    poses = pick(cfg.pose_dir, "gt_pose*.txt")
    if not colors:
        return None
    gcfg = ScanConfig(**{**cfg.__dict__, "t_fix": T_FIX_GT.copy()})
    os.makedirs(cfg.save_dir, exist_ok=True)
    intrinsic = _intrinsic(o3d, gcfg)
    volume = _new_volume(o3d, gcfg)
    for i in range(len(colors)):
        _integrate_frame(o3d, gcfg, volume, intrinsic, colors, depths, poses, i)
    mesh = volume.extract_triangle_mesh()
    mesh.compute_vertex_normals()
    path = os.path.join(cfg.save_dir, "object_reconst_gt.ply")
    o3d.io.write_triangle_mesh(path, mesh)
    return path


def run_all(cfg: ScanConfig, o3d=None, output: str = "points", objects=None, log: bool = False):
    """main(): every object label in sorted order, one reconstruction each (objects are independent —
    the multi-GPU driver shards this list, see distributed.py)."""
    labels = get_unique_object_names(cfg) if objects is None else objects
    return {label: reconstruct_object(label, cfg, o3d=o3d, output=output, log=log) for label in labels}


def check_one_frame(base_dir: str, o3d=None, cfg: ScanConfig = None, show: bool = True):
    """check_one_frame.py:1-31: one RGB-D frame of the object scan (color/color_0000.png, depth/depth_0000.png) ->
    create_from_color_and_depth(depth_scale 1000, depth_trunc 5.0) -> create_from_rgbd_image (identity extrinsic)
    -> voxel_down_sample(0.01) -> draw_geometries (headless here: visualization.draw_geometries).  Returns the cloud."""
    o3d = o3d or _default_o3d()
    cfg = cfg or ScanConfig(base_dir=base_dir)
    color_path = os.path.join(base_dir, "color/color_0000.png")
    depth_path = os.path.join(base_dir, "depth/depth_0000.png")
    intrinsics = _intrinsic(o3d, cfg)
    color_raw = o3d.io.read_image(color_path)
    depth_raw = o3d.io.read_image(depth_path)
    rgbd = o3d.geometry.RGBDImage.create_from_color_and_depth(color_raw, depth_raw, depth_scale=cfg.depth_scale,
                                                              depth_trunc=5.0, convert_rgb_to_intensity=False)
    pcd = o3d.geometry.PointCloud.create_from_rgbd_image(rgbd, intrinsics)
    pcd = pcd.voxel_down_sample(0.01)
    if show:
        o3d.visualization.draw_geometries([pcd])
    return pcd
