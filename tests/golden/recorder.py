"""A recording stand-in for the `open3d` (and `cv2`) modules: every call the reference callers make on the hot
path is logged with its arguments, so the SAME call log can be produced by (a) the reference scripts themselves
(tests/golden/gen_caller_fixture.py, run once in the build container) and (b) this repo's restated callers
(tests/test_callers.py).  No arithmetic of Open3D is emulated; fake objects return deterministic arrays so the
reference's own numpy code (extrinsic inversion, Z mask, occupancy loop, concatenation) runs for real.
"""
from __future__ import annotations

import os
import types

import numpy as np


class Recorder:
    def __init__(self, base):
        self.base = os.path.abspath(base)
        self.calls = []

    def rel(self, p):
        p = os.path.abspath(str(p))
        return os.path.relpath(p, self.base) if p.startswith(self.base) else p

    def log(self, call, **kw):
        self.calls.append({"call": call, **kw})


class FakeImage:
    def __init__(self, path):
        self.path = path


class FakeRGBD:
    def __init__(self, color, depth):
        self.color, self.depth = color, depth


class FakeCloud:
    def __init__(self, rec, points=None, colors=None):
        self._rec = rec
        self.points = np.zeros((0, 3)) if points is None else np.asarray(points, np.float64)
        self.colors = np.zeros((0, 3)) if colors is None else np.asarray(colors, np.float64)

    def paint_uniform_color(self, c):
        self.colors = np.tile(np.asarray(c, np.float64).reshape(1, 3), (len(self.points), 1))
        self._rec.log("paint_uniform_color", color=[float(x) for x in c], n=len(self.points))
        return self

    def __iadd__(self, other):  # PointCloud::operator+= (colours kept only when both sides have them)
        had = len(self.points) > 0
        keep_c = (not had or len(self.colors) > 0) and len(other.colors) > 0
        self.colors = np.concatenate([self.colors if had else np.zeros((0, 3)), other.colors]) if keep_c else np.zeros((0, 3))
        self.points = np.concatenate([self.points, other.points])
        return self

    def __add__(self, other):
        out = FakeCloud(self._rec, self.points.copy(), self.colors.copy())
        out += other
        return out

    def voxel_down_sample(self, voxel_size):
        self._rec.log("voxel_down_sample", voxel_size=float(voxel_size))
        return self


class FakeMesh:
    def __init__(self, rec, nv=12):
        self._rec = rec
        self.vertices = np.zeros((nv, 3))

    def compute_vertex_normals(self):
        self._rec.log("compute_vertex_normals")
        return self

    def sample_points_uniformly(self, number_of_points=100):
        self._rec.log("sample_points_uniformly", number_of_points=int(number_of_points))
        n = int(number_of_points)
        k = np.arange(n, dtype=np.float64)
        pts = np.stack([np.cos(k), np.sin(k), -0.1 + 0.6 * k / max(n - 1, 1)], axis=1)
        cols = np.stack([k % 7 / 7.0, k % 5 / 5.0, k % 3 / 3.0], axis=1)
        return FakeCloud(self._rec, pts, cols)


class FakeVolume:
    def __init__(self, rec, **kw):
        self._rec = rec
        rec.log("ScalableTSDFVolume", voxel_length=float(kw["voxel_length"]), sdf_trunc=float(kw["sdf_trunc"]),
                color_type=str(kw.get("color_type")))

    def integrate(self, rgbd, intrinsic, extrinsic):
        self._rec.log("integrate", color=self._rec.rel(rgbd.color.path), depth=self._rec.rel(rgbd.depth.path),
                      extrinsic=np.asarray(extrinsic, np.float64).tolist())

    def extract_triangle_mesh(self):
        self._rec.log("extract_triangle_mesh")
        return FakeMesh(self._rec)


def _read_ply_points(path):
    """Minimal reader for the ASCII PLY files the fixture generator writes (x y z per vertex)."""
    with open(path) as f:
        lines = f.read().splitlines()
    n = int(next(l.split()[2] for l in lines if l.startswith("element vertex")))
    start = lines.index("end_header") + 1
    return np.array([[float(v) for v in l.split()[:3]] for l in lines[start:start + n]], np.float64)


def cloud_digest(points, colors, full_max=4000):
    """Exact fingerprint of a written cloud: count, sha256 of the float64 bytes, and the full arrays when small."""
    import hashlib

    P = np.ascontiguousarray(np.asarray(points, np.float64))
    Cc = np.ascontiguousarray(np.asarray(colors, np.float64))
    d = {"n": int(P.shape[0]), "points_sha256": hashlib.sha256(P.tobytes()).hexdigest(),
         "colors_sha256": hashlib.sha256(Cc.tobytes()).hexdigest()}
    if P.shape[0] <= full_max:
        d["points"], d["colors"] = P.tolist(), Cc.tolist()
    return d


def make_open3d(rec: Recorder):
    o3d = types.ModuleType("open3d")
    camera = types.ModuleType("open3d.camera")
    io = types.ModuleType("open3d.io")
    geometry = types.ModuleType("open3d.geometry")
    pipelines = types.ModuleType("open3d.pipelines")
    integration = types.ModuleType("open3d.pipelines.integration")
    utility = types.ModuleType("open3d.utility")
    visualization = types.ModuleType("open3d.visualization")

    def PinholeCameraIntrinsic(*args):
        rec.log("PinholeCameraIntrinsic", args=[float(a) for a in args])
        return ("intrinsic", tuple(args))

    camera.PinholeCameraIntrinsic = PinholeCameraIntrinsic

    def read_image(path):
        rec.log("read_image", path=rec.rel(path))
        if not os.path.exists(path):
            raise RuntimeError(f"[Open3D ERROR] Read image failed: {path}")
        return FakeImage(path)

    def write_point_cloud(path, pcd, *a, **k):
        rec.log("write_point_cloud", path=rec.rel(path), **cloud_digest(pcd.points, pcd.colors))
        return True

    def write_triangle_mesh(path, mesh, *a, **k):
        rec.log("write_triangle_mesh", path=rec.rel(path))
        return True

    def read_point_cloud(path, *a, **k):
        rec.log("read_point_cloud", path=rec.rel(path))
        return FakeCloud(rec, _read_ply_points(path))

    def read_triangle_mesh(path, *a, **k):
        rec.log("read_triangle_mesh", path=rec.rel(path))
        return FakeMesh(rec)

    io.read_image, io.write_point_cloud, io.write_triangle_mesh = read_image, write_point_cloud, write_triangle_mesh
    io.read_point_cloud, io.read_triangle_mesh = read_point_cloud, read_triangle_mesh

    class RGBDImage:
        @staticmethod
        def create_from_color_and_depth(color, depth, depth_scale=1000.0, depth_trunc=3.0,
                                        convert_rgb_to_intensity=True):
            rec.log("create_from_color_and_depth", color=rec.rel(color.path), depth=rec.rel(depth.path),
                    depth_scale=float(depth_scale), depth_trunc=float(depth_trunc),
                    convert_rgb_to_intensity=bool(convert_rgb_to_intensity))
            return FakeRGBD(color, depth)

    class PointCloud(FakeCloud):
        def __init__(self):
            super().__init__(rec)

        @staticmethod
        def create_from_rgbd_image(rgbd, intrinsic, *a, **k):
            rec.log("create_from_rgbd_image", color=rec.rel(rgbd.color.path))
            return FakeCloud(rec, np.zeros((4, 3)))

    class TriangleMesh:
        @staticmethod
        def create_coordinate_frame(size=1.0, *a, **k):
            return FakeMesh(rec)

    geometry.RGBDImage, geometry.PointCloud, geometry.TriangleMesh = RGBDImage, PointCloud, TriangleMesh

    class TSDFVolumeColorType:
        NoColor, RGB8, Gray32 = "NoColor", "RGB8", "Gray32"

    integration.ScalableTSDFVolume = lambda **kw: FakeVolume(rec, **kw)
    integration.TSDFVolumeColorType = TSDFVolumeColorType
    pipelines.integration = integration
    utility.Vector3dVector = lambda a: np.asarray(a, np.float64)
    visualization.draw_geometries = lambda geoms, *a, **k: rec.log("draw_geometries")
    o3d.camera, o3d.io, o3d.geometry, o3d.pipelines = camera, io, geometry, pipelines
    o3d.utility, o3d.visualization = utility, visualization
    return o3d


def make_cv2():
    """cv2.imread(path, IMREAD_GRAYSCALE) backed by PIL (OpenCV is absent in this image)."""
    cv2 = types.ModuleType("cv2")
    cv2.IMREAD_GRAYSCALE = 0

    def imread(path, flag=1):
        from PIL import Image

        if not os.path.exists(path):
            return None
        with Image.open(path) as im:
            return np.array(im.convert("L"), dtype=np.uint8)

    cv2.imread = imread
    return cv2


CORE_CALLS = {"PinholeCameraIntrinsic", "ScalableTSDFVolume", "read_image", "create_from_color_and_depth",
              "integrate", "extract_triangle_mesh", "compute_vertex_normals", "sample_points_uniformly",
              "write_point_cloud", "write_triangle_mesh", "read_point_cloud", "read_triangle_mesh",
              "paint_uniform_color"}


def core(calls):
    return [c for c in calls if c["call"] in CORE_CALLS]
