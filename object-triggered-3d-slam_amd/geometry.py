"""open3d.geometry counterparts backed by HBM-resident tensors and the HIP kernels of libotslam_hip.so.

Image, RGBDImage, PointCloud and TriangleMesh keep each array wherever it was last produced (host numpy or
device tensor) and move it on demand: kernel outputs stay in HBM until Python reads `.points` etc., so a
chain like create_from_rgbd_image -> voxel_down_sample -> remove_statistical_outlier never leaves the GPU.
Every compute method calls the C ABI; none has a CPU implementation.
"""
from __future__ import annotations

import ctypes as C
import importlib

import numpy as np

from . import _device as D
from . import _lib as L
from . import streams as _streams
from .utility import DoubleVector, Vector3dVector, Vector3iVector


class _Arr:
    """An (N, k) array living on the host (numpy) and/or the device (torch)."""

    __slots__ = ("_h", "_d", "_viewed", "_ready", "_launch")

    def __init__(self, host=None, dev=None, ready=None, launch=None):
        self._h, self._d = host, dev
        self._viewed = False  # a writable host view was handed out: the host copy is authoritative
        self._ready = ready   # torch.cuda.Event: the device data is complete once it fires (written on another stream)
        self._launch = launch  # deferred producer: queues the kernels that write _d, returns their completion event

    def _start(self, after=None):
        """Queue a deferred producer (once); from then on _ready is its completion event.  after(stream): called with
        the producer's stream before its kernels are queued (an extra dependency)."""
        if self._launch is not None:
            fn, self._launch = self._launch, None
            self._ready = fn(after)

    def ready_event(self):
        """The event the device data waits on (None: complete in stream order), the deferred producer queued first."""
        self._start()
        return self._ready

    def _join(self):
        """Make the current stream wait for the producer of the device data (once)."""
        self._start()
        if self._ready is not None:
            D.torch.cuda.current_stream().wait_event(self._ready)
            self._ready = None

    @staticmethod
    def wrap(a, dtype, cols):
        if a is None:
            return None
        if isinstance(a, _Arr):
            return a
        if isinstance(a, (Vector3dVector, Vector3iVector)):
            a = np.asarray(a)
        if D.is_tensor(a):
            return _Arr(dev=a.reshape(-1, cols).contiguous())
        arr = np.array(a, dtype=dtype, copy=True, order="C")  # assignment copies, as Open3D's does
        if arr.size == 0:
            arr = arr.reshape(0, cols)
        return _Arr(host=arr)

    def host(self):
        if self._h is None:
            self._join()
            self._h = D.to_host(self._d)
        return self._h

    def host_view(self):
        """The host array for a writable view handed to the caller (Open3D's vectors are views of the one copy).
        From now on the host copy is authoritative: every later GPU use uploads it again, so edits made through
        any view taken earlier are seen; reads alone (len(mesh.vertices)) cost one download."""
        h = self.host()
        self._viewed = True
        return h

    def dev(self):
        self._join()
        if self._d is None:
            self._d = D.to_device(self._h)
        elif self._viewed:  # refresh IN PLACE: pointers handed out earlier (queued kernels, job tables) stay valid
            h = np.ascontiguousarray(self._h)
            if tuple(h.shape) != tuple(self._d.shape):
                self._d = D.to_device(h)
            else:
                self._d.copy_(D.to_device(h))
        return self._d

    def copy(self):
        self._join()
        if self._viewed or self._d is None:
            return _Arr(host=self.host().copy())
        return _Arr(dev=self._d.clone())

    def __len__(self):
        return (self._h if self._h is not None else self._d).shape[0]


def _n(a):
    return 0 if a is None else len(a)


# --------------------------------------------------------------------------------------------- Image
class Image:
    """open3d.geometry.Image: uint8 HxW / HxWx3, uint16 HxW (depth, mm) or float32 HxW."""

    def __init__(self, data=None):
        if data is None:
            self._host, self._dev = np.zeros((0, 0), np.uint8), None
        elif isinstance(data, Image):
            self._host, self._dev = data._host, data._dev
        elif D.is_tensor(data):
            self._host, self._dev = None, data.contiguous()
        else:
            self._host, self._dev = np.ascontiguousarray(np.asarray(data)), None

    def _shape(self):
        return tuple(self._host.shape if self._host is not None else self._dev.shape)

    @property
    def height(self):
        return self._shape()[0]

    @property
    def width(self):
        return self._shape()[1] if len(self._shape()) > 1 else 0

    @property
    def num_of_channels(self):
        s = self._shape()
        return s[2] if len(s) == 3 else 1

    @property
    def dtype(self):
        if self._host is not None:
            return self._host.dtype
        return np.dtype(str(self._dev.dtype).replace("torch.", ""))

    def host(self):
        if self._host is None:
            self._host = D.to_host(self._dev)
        return self._host

    def dev(self):
        if self._dev is None:
            self._dev = D.to_device(self._host)
        return self._dev

    def __array__(self, dtype=None, copy=None):
        h = self.host()
        return h if dtype is None else h.astype(dtype)

    def is_empty(self):
        return self.height == 0 or self.width == 0

    def __repr__(self):
        return f"Image of size {self.width}x{self.height}, with {self.num_of_channels} channels."


class RGBDImage:
    """open3d.geometry.RGBDImage.  Keeps the raw uint16 depth next to the converted float depth so the
    volume can take the fused (u16 -> float -> integrate) path."""

    def __init__(self, color=None, depth=None):
        self.color = color if color is not None else Image()
        self.depth = depth if depth is not None else Image()
        self._raw_depth = None  # (device u16 tensor, depth_scale, depth_trunc)

    @staticmethod
    def create_from_color_and_depth(color, depth, depth_scale=1000.0, depth_trunc=3.0,
                                    convert_rgb_to_intensity=True):
        """RGBDImageFactory CreateFromColorAndDepth (reconstruct_rgbd_filter.py:98-103) — depth converted by
        the ot_depth_to_float kernel: f = (float)u16 / scale, 0 if f >= trunc."""
        color = color if isinstance(color, Image) else Image(color)
        depth = depth if isinstance(depth, Image) else Image(depth)
        if color.height != depth.height or color.width != depth.width:
            raise RuntimeError("[CreateFromColorAndDepth] Unsupported image format.")
        out = RGBDImage()
        if depth.dtype == np.uint16:
            d16 = depth.dev()
            df = D.empty((depth.height, depth.width), "float32")
            L.call("ot_depth_to_float", D.ptr(d16), D.ptr(df), d16.numel(), float(depth_scale), float(depth_trunc),
                   D.stream_ptr())
            out._raw_depth = (d16, float(depth_scale), float(depth_trunc))
        elif depth.dtype == np.float32:
            d = depth.dev()
            df = d.clone()
            scale = float(depth_scale)
            df = df / scale if scale != 1.0 else df
            df = df.masked_fill(df >= depth_trunc, 0.0)
        else:
            raise RuntimeError("[CreateFromColorAndDepth] Unsupported image format.")
        out.depth = Image(df)
        if convert_rgb_to_intensity:
            c = color.dev()
            if c.ndim == 3 and c.shape[2] == 3:
                import torch

                cf = c.to(torch.float32)
                gray = (0.2990 * cf[..., 0] + 0.5870 * cf[..., 1] + 0.1140 * cf[..., 2]) / 255.0
                out.color = Image(gray.to(torch.float32).contiguous())
            else:
                out.color = Image(c)
        else:
            out.color = color
        return out

    def __repr__(self):
        return f"RGBDImage of size\nColor image : {self.color.width}x{self.color.height}\nDepth image : {self.depth.width}x{self.depth.height}"


# ---------------------------------------------------------------------------------------- PointCloud
class PointCloud:
    """open3d.geometry.PointCloud with points/colors/normals as float64 (N, 3)."""

    def __init__(self, points=None):
        self._xyz = _Arr.wrap(points, np.float64, 3) if points is not None else _Arr(host=np.zeros((0, 3)))
        self._rgb = None
        self._nrm = None

    # --- attribute access (host views) ---
    @property
    def points(self):
        return Vector3dVector._view(self._xyz.host_view())

    @points.setter
    def points(self, v):
        self._xyz = _Arr.wrap(v, np.float64, 3)

    @property
    def colors(self):
        return Vector3dVector._view(self._rgb.host_view() if self._rgb is not None else np.zeros((0, 3)))

    @colors.setter
    def colors(self, v):
        a = _Arr.wrap(v, np.float64, 3)
        self._rgb = a if a is not None and len(a) > 0 else None

    @property
    def normals(self):
        return Vector3dVector._view(self._nrm.host_view() if self._nrm is not None else np.zeros((0, 3)))

    @normals.setter
    def normals(self, v):
        a = _Arr.wrap(v, np.float64, 3)
        self._nrm = a if a is not None and len(a) > 0 else None

    def has_points(self):
        return len(self._xyz) > 0

    def has_colors(self):
        return self._rgb is not None and len(self._rgb) > 0

    def has_normals(self):
        return self._nrm is not None and len(self._nrm) > 0

    def is_empty(self):
        return not self.has_points()

    def __len__(self):
        return len(self._xyz)

    def __repr__(self):
        return f"PointCloud with {len(self._xyz)} points."

    def clear(self):
        self._xyz, self._rgb, self._nrm = _Arr(host=np.zeros((0, 3))), None, None
        return self

    def get_min_bound(self):
        return self._xyz.host().min(axis=0) if self.has_points() else np.zeros(3)

    def get_max_bound(self):
        return self._xyz.host().max(axis=0) if self.has_points() else np.zeros(3)

    def paint_uniform_color(self, color):
        """PointCloud::PaintUniformColor (hybrid_map.py:59,88)."""
        c = np.clip(np.asarray(color, dtype=np.float64).reshape(1, 3), 0.0, 1.0)
        self._rgb = _Arr(host=np.ascontiguousarray(np.repeat(c, len(self._xyz), axis=0)))
        return self

    # --- concatenation (PointCloud::operator+=, hybrid_map.py:91,115) ---
    def __iadd__(self, other):
        if not other.has_points():
            return self
        had_points = self.has_points()
        cat = _cat_host if (self._xyz._d is None or other._xyz._d is None) else _cat_dev
        nrm = cat(self._nrm, other._nrm) if ((not had_points or self.has_normals()) and other.has_normals()) else None
        rgb = cat(self._rgb, other._rgb) if ((not had_points or self.has_colors()) and other.has_colors()) else None
        self._xyz = cat(self._xyz if had_points else None, other._xyz)
        self._rgb, self._nrm = rgb, nrm
        return self

    def __add__(self, other):
        out = PointCloud()
        cp = lambda a: a.copy() if a is not None else None  # a new cloud never shares arrays with an operand
        out._xyz, out._rgb, out._nrm = cp(self._xyz), cp(self._rgb), cp(self._nrm)
        out += other
        return out

    # --- factories ---
    @staticmethod
    def create_from_rgbd_image(image, intrinsic, extrinsic=None, project_valid_depth_only=True):
        """PointCloudFactory CreateFromRGBDImage (check_one_frame.py:27): HIP unprojection + stable
        compaction (ot_unproject), row-major point order, colour / 255."""
        if image.color.num_of_channels != 3 or image.color.dtype != np.uint8:
            raise RuntimeError("[CreatePointCloudFromRGBDImage] Unsupported image format.")
        return _unproject(image.depth, image.color, intrinsic, extrinsic, 1)

    @staticmethod
    def create_from_depth_image(depth, intrinsic, extrinsic=None, depth_scale=1000.0, depth_trunc=1000.0,
                                stride=1, project_valid_depth_only=True):
        depth = depth if isinstance(depth, Image) else Image(depth)
        if depth.dtype == np.uint16:
            d16 = depth.dev()
            df = D.empty((depth.height, depth.width), "float32")
            L.call("ot_depth_to_float", D.ptr(d16), D.ptr(df), d16.numel(), float(depth_scale), float(depth_trunc),
                   D.stream_ptr())
            depth = Image(df)
        return _unproject(depth, None, intrinsic, extrinsic, int(stride))

    # --- filters ---
    def voxel_down_sample(self, voxel_size):
        """PointCloud::VoxelDownSample (check_one_frame.py:28) — ot_voxel_down_sample.  Voxels come out
        sorted by integer key (Open3D: hash order)."""
        if voxel_size <= 0.0:
            raise RuntimeError("[VoxelDownSample] voxel_size <= 0.")
        n = len(self._xyz)
        out = PointCloud()
        if n == 0:
            return out
        xyz = self._xyz.dev()
        rgb = self._rgb.dev() if self.has_colors() else None
        nrm = self._nrm.dev() if self.has_normals() else None
        oxyz = D.empty((n, 3), "float64")
        orgb = D.empty((n, 3), "float64") if rgb is not None else None
        onrm = D.empty((n, 3), "float64") if nrm is not None else None
        k = C.c_int64(0)
        L.call("ot_voxel_down_sample", D.ptr(xyz), D.ptr(rgb), D.ptr(nrm), n, float(voxel_size), D.ptr(oxyz),
               D.ptr(orgb), D.ptr(onrm), None, C.byref(k), D.stream_ptr())
        k = k.value
        out._xyz = _Arr(dev=oxyz[:k])
        out._rgb = _Arr(dev=orgb[:k]) if orgb is not None else None
        out._nrm = _Arr(dev=onrm[:k]) if onrm is not None else None
        return out

    def remove_statistical_outlier(self, nb_neighbors, std_ratio, print_progress=False):
        """PointCloud::RemoveStatisticalOutliers — ot_remove_statistical_outlier (grid kNN on the GPU)."""
        if nb_neighbors < 1 or std_ratio <= 0:
            raise RuntimeError("[RemoveStatisticalOutliers] Illegal input parameters, the number of neighbors "
                               "and standard deviation ratio must be positive.")
        n = len(self._xyz)
        if n == 0:
            return PointCloud(), []
        idx = D.empty((n,), "int64")
        k = C.c_int64(0)
        L.call("ot_remove_statistical_outlier", D.ptr(self._xyz.dev()), n, int(nb_neighbors), float(std_ratio),
               D.ptr(idx), None, C.byref(k), D.stream_ptr())
        idx = idx[:k.value]
        return self._select_dev(idx), D.to_host(idx).tolist()

    def remove_radius_outlier(self, nb_points, radius, print_progress=False):
        """PointCloud::RemoveRadiusOutliers — ot_remove_radius_outlier."""
        if nb_points < 1 or radius <= 0:
            raise RuntimeError("[RemoveRadiusOutliers] Illegal input parameters, number of points and radius "
                               "must be positive")
        n = len(self._xyz)
        if n == 0:
            return PointCloud(), []
        idx = D.empty((n,), "int64")
        k = C.c_int64(0)
        L.call("ot_remove_radius_outlier", D.ptr(self._xyz.dev()), n, int(nb_points), float(radius), D.ptr(idx),
               C.byref(k), D.stream_ptr())
        idx = idx[:k.value]
        return self._select_dev(idx), D.to_host(idx).tolist()

    def compute_point_cloud_distance(self, target):
        """PointCloud::ComputePointCloudDistance (eval_cone.py:99,103) — ot_compute_point_cloud_distance.
        Per point of self: distance to the nearest point of `target` (float64); 0.0 when target is empty."""
        n, m = len(self._xyz), len(target._xyz)
        if n == 0:
            return DoubleVector()
        out = D.empty((n,), "float64")
        L.call("ot_compute_point_cloud_distance", D.ptr(self._xyz.dev()), n,
               D.ptr(target._xyz.dev()) if m else None, m, D.ptr(out), D.stream_ptr())
        return DoubleVector(D.to_host(out))

    def _select_dev(self, idx):
        out = PointCloud()
        m = int(idx.shape[0])

        def g(a):
            o = D.empty((m, 3), "float64")
            if m:
                L.call("ot_gather_rows3", D.ptr(a.dev()), D.ptr(idx), m, D.ptr(o), D.stream_ptr())
            return _Arr(dev=o)

        out._xyz = g(self._xyz)
        out._rgb = g(self._rgb) if self.has_colors() else None
        out._nrm = g(self._nrm) if self.has_normals() else None
        return out

    def select_by_index(self, indices, invert=False):
        n = len(self._xyz)
        idx = np.asarray(indices, dtype=np.int64)
        if invert:
            mask = np.ones(n, bool)
            mask[idx] = False
            idx = np.nonzero(mask)[0]
        out = PointCloud()
        out._xyz = _Arr(host=self._xyz.host()[idx])
        out._rgb = _Arr(host=self._rgb.host()[idx]) if self.has_colors() else None
        out._nrm = _Arr(host=self._nrm.host()[idx]) if self.has_normals() else None
        return out

    def filter_min_z(self, z_min):
        """Stable Z-mask compaction on the GPU (reconstruct_rgbd_filter.py:126-132 as one kernel chain);
        normals are dropped like the reference's rebuilt cloud."""
        n = len(self._xyz)
        out = PointCloud()
        if n == 0:
            return out
        xyz = self._xyz.dev()
        rgb = self._rgb.dev() if self.has_colors() else None
        oxyz = D.empty((n, 3), "float64")
        orgb = D.empty((n, 3), "float64") if rgb is not None else None
        k = C.c_int64(0)
        L.call("ot_filter_min_z", D.ptr(xyz), D.ptr(rgb), n, float(z_min), D.ptr(oxyz), D.ptr(orgb), C.byref(k),
               D.stream_ptr())
        out._xyz = _Arr(dev=oxyz[:k.value])
        out._rgb = _Arr(dev=orgb[:k.value]) if orgb is not None else None
        return out


def _cat_host(a, b):
    if a is None:
        return _Arr(host=b.host().copy())
    return _Arr(host=np.concatenate([a.host(), b.host()], axis=0))


def _cat_dev(a, b):
    import torch

    if a is None:
        return b.copy()
    return _Arr(dev=torch.cat([a.dev(), b.dev()], dim=0))


def _unproject(depth_img, color_img, intrinsic, extrinsic, stride):
    if depth_img.dtype != np.float32:
        raise RuntimeError("[CreatePointCloudFromRGBDImage] Unsupported image format.")
    depth = depth_img.dev()
    color = color_img.dev() if color_img is not None else None
    h, w = depth.shape[0], depth.shape[1]
    if intrinsic.width != w or intrinsic.height != h:
        # Open3D indexes with the image size and the intrinsic's fx/fy/cx/cy; keep the image size
        pass
    intr = L.ot_intrinsics(w, h, intrinsic.fx, intrinsic.fy, intrinsic.cx, intrinsic.cy)
    ext = np.ascontiguousarray(np.eye(4) if extrinsic is None else np.asarray(extrinsic, np.float64))
    cap = ((h + stride - 1) // stride) * ((w + stride - 1) // stride)
    xyz = D.empty((cap, 3), "float64")
    rgb = D.empty((cap, 3), "float64") if color is not None else None
    n = C.c_int64(0)
    L.call("ot_unproject", D.ptr(depth), D.ptr(color), C.byref(intr), ext.ctypes.data_as(C.c_void_p), stride,
           D.ptr(xyz), D.ptr(rgb), cap, C.byref(n), D.stream_ptr())
    pcd = PointCloud()
    pcd._xyz = _Arr(dev=xyz[:n.value])
    pcd._rgb = _Arr(dev=rgb[:n.value]) if rgb is not None else None
    return pcd


# -------------------------------------------------------------------------------------- TriangleMesh
class TriangleMesh:
    """open3d.geometry.TriangleMesh: vertices f64 (V,3), triangles i32 (T,3), vertex colors / normals."""

    def __init__(self, vertices=None, triangles=None):
        self._v = _Arr.wrap(vertices, np.float64, 3) if vertices is not None else _Arr(host=np.zeros((0, 3)))
        self._t = _Arr.wrap(triangles, np.int32, 3) if triangles is not None else _Arr(
            host=np.zeros((0, 3), np.int32))
        self._vc = None
        self._vn = None

        self._mc = None  # (volume handle, extraction serial) of a mesh fresh out of extract_triangle_mesh
    @property
    def vertices(self):
        self._settle()
        return Vector3dVector._view(self._v.host_view())

    @vertices.setter
    def vertices(self, v):
        self._v = _Arr.wrap(v, np.float64, 3)
        self._mc = None

    @property
    def triangles(self):
        self._settle()
        return Vector3iVector._view(self._t.host_view())

    @triangles.setter
    def triangles(self, t):
        self._t = _Arr.wrap(t, np.int32, 3)
        self._mc = None

    @property
    def vertex_colors(self):
        return Vector3dVector._view(self._vc.host_view() if self._vc is not None else np.zeros((0, 3)))

    @vertex_colors.setter
    def vertex_colors(self, v):
        a = _Arr.wrap(v, np.float64, 3)
        self._vc = a if a is not None and len(a) > 0 else None

    @property
    def vertex_normals(self):
        return Vector3dVector._view(self._vn.host_view() if self._vn is not None else np.zeros((0, 3)))

    @vertex_normals.setter
    def vertex_normals(self, v):
        a = _Arr.wrap(v, np.float64, 3)
        self._vn = a if a is not None and len(a) > 0 else None

    def has_vertices(self):
        return len(self._v) > 0

    def has_triangles(self):
        return len(self._t) > 0

    def has_vertex_colors(self):
        return self._vc is not None and len(self._vc) > 0

    def has_vertex_normals(self):
        return self._vn is not None and len(self._vn) > 0

    def is_empty(self):
        return not self.has_vertices()

    def __repr__(self):
        return f"TriangleMesh with {len(self._v)} points and {len(self._t)} triangles."

    def _settle(self):
        """Deferred vertex normals read V and T on the device: queue them, and order the current stream after them,
        before a writable view of either array is handed out (its edits reach the device copy in place)."""
        if self._vn is not None and self._vn._launch is not None:
            self._vn._join()

    def compute_vertex_normals(self, normalized=True):
        """TriangleMesh::ComputeVertexNormals (reconstruct_rgbd_filter.py:113).  A mesh fresh out of
        extract_triangle_mesh (arrays not reassigned or viewed for writing since) takes the marching-cubes walk of its
        volume (ot_tsdf_mesh_vertex_normals: each vertex's <= 4 cubes in triangle order); any other mesh, or a volume
        changed since, the generic corner sort (ot_mesh_compute_vertex_normals).  Both give the same bits."""
        nv, nt = len(self._v), len(self._t)
        if nv == 0:
            return self
        out = D.empty((nv, 3), "float64")
        mc = getattr(self, "_mc", None)
        vol = mc[0]() if mc is not None else None
        fresh = vol is not None and not self._v._viewed and not self._t._viewed
        if fresh:  # the very arrays the extraction wrote, unmodified since (no view, no in-place device edit)
            V, T = self._v.dev(), self._t.dev()
            fresh = (V.data_ptr(), V._version, T.data_ptr(), T._version) == tuple(mc[2:6])
        if fresh and getattr(vol, "_h", None) is not None:
            # Deferred: the marching-cubes walk is queued on a side stream at the latest when the normals are read, or
            # by the next sampling once its area chains are queued (sample_points_min_z: the walk then runs beside the
            # chains' single-wave walks instead of contending with their wide first passes).  Any reader of the
            # normals waits for them (_Arr ready event; sample_points_uniformly passes it to
            # ot_mesh_sample_points_uniformly_after).
            torch = D.torch
            cur = torch.cuda.current_stream()
            vref, serial = mc[0], mc[1]
            made = torch.cuda.Event()  # the arrays are complete here: the launch waits for this point of `cur` only,
            made.record(cur)           # not for the sampling queued on `cur` after it

            def launch(after=None):
                v = vref()
                side = _streams.side_stream(cur)
                side.wait_event(made)
                if after is not None:
                    after(side)
                st = L.OT_ERR_INVALID_ARGUMENT
                if v is not None and getattr(v, "_h", None) is not None:
                    st = L.load().ot_tsdf_mesh_vertex_normals(v._h, serial, D.ptr(V), nv, D.ptr(T), nt, D.ptr(out),
                                                              C.c_void_p(side.cuda_stream))
                if st != L.OT_OK:  # the volume changed or went away since the extraction: the generic corner sort
                    L.call("ot_mesh_compute_vertex_normals", D.ptr(V), nv, D.ptr(T), nt, D.ptr(out),
                           C.c_void_p(side.cuda_stream))
                for t in (V, T, out):  # allocated on the caller's stream, used on the side stream
                    t.record_stream(side)
                done = torch.cuda.Event()
                done.record(side)
                return done

            self._vn = _Arr(dev=out, launch=launch)
            return self
        L.call("ot_mesh_compute_vertex_normals", D.ptr(self._v.dev()), nv, D.ptr(self._t.dev()), nt, D.ptr(out),
               D.stream_ptr())
        self._vn = _Arr(dev=out)
        return self

    def get_surface_area(self):
        """TriangleMesh::GetSurfaceArea: the float64 sum of the triangle areas in index order (the first serial
        chain of SamplePointsUniformly, reconstruct_rgbd_filter.py:123) — ot_mesh_get_surface_area."""
        out = C.c_double(0.0)
        nt = len(self._t)
        L.call("ot_mesh_get_surface_area", D.ptr(self._v.dev()) if nt else None, len(self._v),
               D.ptr(self._t.dev()) if nt else None, nt, C.byref(out), D.stream_ptr())
        return out.value

    def sample_points_uniformly(self, number_of_points=100, use_triangle_normal=False, seed=0):
        """TriangleMesh::SamplePointsUniformly (reconstruct_rgbd_filter.py:123) with a seeded counter RNG."""
        if number_of_points <= 0:
            raise RuntimeError("[SamplePointsUniformly] number_of_points <= 0")
        if len(self._t) == 0:
            raise RuntimeError("[SamplePointsUniformly] Input mesh has no triangles.")
        if use_triangle_normal:  # the reference never asks for it (reconstruct_rgbd_filter.py:123)
            raise NotImplementedError("[SamplePointsUniformly] use_triangle_normal=True is not implemented by this "
                                      "build (interpolated vertex normals only)")
        n = int(number_of_points)
        P = D.empty((n, 3), "float64")
        PN = D.empty((n, 3), "float64") if self.has_vertex_normals() else None
        PC = D.empty((n, 3), "float64") if self.has_vertex_colors() else None
        # normals still in flight on the side stream (compute_vertex_normals of a fresh mesh): the C side waits for
        # them after the area chains, right before the emission that interpolates them
        ready = self._vn.ready_event() if (PN is not None and not self._vn._viewed and self._vn._d is not None) else None
        VN = (self._vn._d if ready is not None else self._vn.dev()) if PN is not None else None
        job = (L.ot_mesh_sample_job * 1)(L.ot_mesh_sample_job(
            D.ptr(self._v.dev()), D.ptr(VN), D.ptr(self._vc.dev()) if PC is not None else None, len(self._v),
            D.ptr(self._t.dev()), len(self._t), D.ptr(P), D.ptr(PN), D.ptr(PC)))
        L.call("ot_mesh_sample_points_uniformly_after", C.cast(job, C.c_void_p), 1, n,
               C.c_uint64(int(seed) & 0xFFFFFFFFFFFFFFFF), C.c_void_p(ready.cuda_event) if ready is not None else None,
               D.stream_ptr())
        if ready is not None:
            self._vn._ready = None  # the caller's stream has waited for it (inside the call)
        pcd = PointCloud()
        pcd._xyz = _Arr(dev=P)
        pcd._nrm = _Arr(dev=PN) if PN is not None else None
        pcd._rgb = _Arr(dev=PC) if PC is not None else None
        return pcd

    def sample_points_min_z(self, number_of_points, z_min, seed=0):
        """reconstruct_rgbd_filter.py:123-132 fused (not an Open3D API): sample_points_uniformly(number_of_points)
        with this seed, then the rows with z >= z_min, points and colours only (the reference rebuilds its cloud from
        those two) -- the same cloud as sample_points_uniformly(...).filter_min_z(z_min), in one pass over the
        samples (ot_mesh_sample_points_min_z).  Vertex normals are not read, so any still in flight are not waited for."""
        return TriangleMesh.sample_points_min_z_batch([self], number_of_points, z_min, seed)[0]

    @staticmethod
    def sample_points_min_z_batch(meshes, number_of_points, z_min, seed=0):
        """sample_points_min_z for several meshes in one call: their area-CDF chains run side by side."""
        if number_of_points <= 0:
            raise RuntimeError("[SamplePointsUniformly] number_of_points <= 0")
        n = int(number_of_points)
        jobs = (L.ot_mesh_sample_job * max(len(meshes), 1))()
        outs = []
        for j, m in enumerate(meshes):
            if len(m._t) == 0:
                raise RuntimeError("[SamplePointsUniformly] Input mesh has no triangles.")
            P = D.empty((n, 3), "float64")
            PC = D.empty((n, 3), "float64") if m.has_vertex_colors() else None
            jobs[j] = L.ot_mesh_sample_job(
                D.ptr(m._v.dev()), None, D.ptr(m._vc.dev()) if PC is not None else None, len(m._v), D.ptr(m._t.dev()),
                len(m._t), D.ptr(P), None, D.ptr(PC))
            outs.append((P, PC))
        kept = (C.c_int64 * max(len(meshes), 1))()
        if meshes:
            # deferred vertex normals of these meshes are queued once the sampling is (the sampling does not read the
            # normals): its chains' first passes are then dispatched ahead of them
            pend = [m._vn for m in meshes if m._vn is not None and m._vn._launch is not None]
            args = (C.cast(jobs, C.c_void_p), len(meshes), n, C.c_uint64(int(seed) & 0xFFFFFFFFFFFFFFFF), float(z_min))
            if pend:
                L.call("ot_mesh_sample_points_min_z_async", *args, D.stream_ptr())
                try:
                    for a in pend:
                        a._start()
                finally:
                    L.call("ot_mesh_sample_points_min_z_wait", len(meshes), kept)
            else:
                L.call("ot_mesh_sample_points_min_z", *args, kept, D.stream_ptr())
        clouds = []
        for j, (P, PC) in enumerate(outs):
            pcd = PointCloud()
            pcd._xyz = _Arr(dev=P[:kept[j]])
            pcd._rgb = _Arr(dev=PC[:kept[j]]) if PC is not None else None
            clouds.append(pcd)
        return clouds

    @staticmethod
    def sample_points_uniformly_batch(meshes, number_of_points=100, seed=0):
        """sample_points_uniformly for several meshes in one call (not an Open3D API): the same clouds as one
        call per mesh, with the meshes' serial area-CDF chains running side by side on the GPU."""
        if number_of_points <= 0:
            raise RuntimeError("[SamplePointsUniformly] number_of_points <= 0")
        n = int(number_of_points)
        jobs = (L.ot_mesh_sample_job * max(len(meshes), 1))()
        outs = []
        for j, m in enumerate(meshes):
            if len(m._t) == 0:
                raise RuntimeError("[SamplePointsUniformly] Input mesh has no triangles.")
            P = D.empty((n, 3), "float64")
            PN = D.empty((n, 3), "float64") if m.has_vertex_normals() else None
            PC = D.empty((n, 3), "float64") if m.has_vertex_colors() else None
            jobs[j] = L.ot_mesh_sample_job(
                D.ptr(m._v.dev()), D.ptr(m._vn.dev()) if PN is not None else None,
                D.ptr(m._vc.dev()) if PC is not None else None, len(m._v), D.ptr(m._t.dev()), len(m._t), D.ptr(P),
                D.ptr(PN), D.ptr(PC))
            outs.append((P, PN, PC))
        if meshes:
            L.call("ot_mesh_sample_points_uniformly_batch", C.cast(jobs, C.c_void_p), len(meshes), n,
                   C.c_uint64(int(seed) & 0xFFFFFFFFFFFFFFFF), D.stream_ptr())
        clouds = []
        for P, PN, PC in outs:
            pcd = PointCloud()
            pcd._xyz = _Arr(dev=P)
            pcd._nrm = _Arr(dev=PN) if PN is not None else None
            pcd._rgb = _Arr(dev=PC) if PC is not None else None
            clouds.append(pcd)
        return clouds

    @staticmethod
    def create_coordinate_frame(size=1.0, origin=(0.0, 0.0, 0.0)):
        o = np.asarray(origin, np.float64)
        V = np.stack([o, o + [size, 0, 0], o + [0, size, 0], o + [0, 0, size]])
        m = TriangleMesh(V, np.array([[0, 1, 2], [0, 2, 3], [0, 3, 1]], np.int32))
        return m
