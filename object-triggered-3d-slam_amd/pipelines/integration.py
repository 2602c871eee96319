"""open3d.pipelines.integration counterparts: ScalableTSDFVolume on the GPU block hash (tsdf.hip).

Call surface = reconstruct_rgbd_filter.py:81-85 (constructor), :105 (integrate), :112 (extract_triangle_mesh).
"""
from __future__ import annotations

import ctypes as C
import enum
import weakref

import numpy as np

from .. import _device as D
from .. import _lib as L
from .. import streams as _streams
from ..geometry import PointCloud, RGBDImage, TriangleMesh, _Arr


class TSDFVolumeColorType(enum.IntEnum):
    NoColor = 0
    RGB8 = 1
    Gray32 = 2


class ScalableTSDFVolume:
    """pipelines.integration.ScalableTSDFVolume(voxel_length, sdf_trunc, color_type=NoColor,
    volume_unit_resolution=16, depth_sampling_stride=4).

    Like Open3D's, the volume is unbounded: its block pool grows when a batch needs more units (records copied,
    keys rehashed, the batch's dropped units integrated again from its staged frames: the same volume bit for bit).
    Extra keyword arguments (not in Open3D): `max_units` (initial block-pool capacity in HBM), `batch_frames`
    (frames queued per fused integration launch, default and max 64; 1 = integrate immediately; results are
    bit-identical for any value: a batch applies its frames to each voxel in call order) and `color_precision`
    (64, the default: the running colour mean in float64 with exact division, Open3D's TSDFVoxel::color_ --
    bit-exact colours; 32: float32 state with one reciprocal per update, |rel| <= 1e-4, faster)."""

    def __init__(self, voxel_length, sdf_trunc, color_type=TSDFVolumeColorType.NoColor, volume_unit_resolution=16,
                 depth_sampling_stride=4, max_units=0, batch_frames=None, color_precision=64):
        D.require_gpu()
        ct = int(color_type)
        if ct == TSDFVolumeColorType.Gray32:
            raise NotImplementedError("[ScalableTSDFVolume] TSDFVolumeColorType.Gray32 is not implemented by this build "
                                      "(the reference uses RGB8: reconstruct_rgbd_filter.py:81-85)")
        self.voxel_length = float(voxel_length)
        self.sdf_trunc = float(sdf_trunc)
        self.color_type = TSDFVolumeColorType(ct)
        self.volume_unit_resolution = int(volume_unit_resolution)
        self.depth_sampling_stride = int(depth_sampling_stride)
        h = C.c_void_p()
        L.call("ot_tsdf_create", self.voxel_length, self.sdf_trunc, ct, self.volume_unit_resolution,
               self.depth_sampling_stride, int(max_units), C.byref(h))
        self._h = h
        self._keep = []  # frames queued for a batched launch stay referenced until the C side integrates them
        self._batch = 32
        if batch_frames is not None:
            self.set_batch(batch_frames)
        L.call("ot_tsdf_set_color_precision", self._h, int(color_precision))
        bits = C.c_int32(0)
        L.call("ot_tsdf_get_color_precision", self._h, C.byref(bits))
        self.color_precision = bits.value  # NoColor volumes keep no colour state (32: zero float planes)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                L.load().ot_tsdf_destroy(h)
            except Exception:
                pass
            self._h = None

    def set_frontend_overlap(self, mode):
        """Double-buffered batch front end (ot_tsdf_set_frontend_overlap): 1 on, 0 off, -1 (default) on for sharded
        volumes only (with their split front end it is the faster at 2, 4 and 8 ranks).
        Batch k+1's staging / touch run beside batch k's integrate; results are identical in every mode.  Queued
        frames are integrated first, on the facade's stream (the C call refuses a volume with queued frames)."""
        self.flush()
        L.call("ot_tsdf_set_frontend_overlap", self._h, int(mode))

    def set_batch(self, frames):
        L.call("ot_tsdf_set_batch", self._h, int(frames))
        self._batch = int(frames)

    def _queued(self, item):
        """Keep a queued frame's device images alive while the C side holds it.  Each tensor is recorded on the
        current (launch) stream, so the caching allocator cannot hand its memory to another stream before the
        kernels that read it have run, whichever stream allocated it."""
        s = D.torch.cuda.current_stream()
        for t in item:
            if t is not None:
                t.record_stream(s)
        self._keep.append(item)

    def _release(self):
        """Drop the references of the frames the C side has consumed (enqueued on their stream): all but the
        ot_tsdf_pending_frames() newest."""
        n = C.c_int32(0)
        L.call("ot_tsdf_pending_frames", self._h, C.byref(n))
        done = len(self._keep) - n.value
        if done > 0:
            del self._keep[:done]

    def reset(self):
        """ScalableTSDFVolume::Reset, ordered on the current stream (no device-wide synchronisation)."""
        L.call("ot_tsdf_reset_async", self._h, D.stream_ptr())
        self._keep.clear()

    def integrate(self, image: RGBDImage, intrinsic, extrinsic):
        """ScalableTSDFVolume::Integrate.  Raw-uint16 RGBD images take the fused path."""
        ext = np.ascontiguousarray(np.asarray(extrinsic, dtype=np.float64).reshape(4, 4))
        rgb8 = self.color_type == TSDFVolumeColorType.RGB8
        color = image.color
        if rgb8 and (color.num_of_channels != 3 or color.dtype != np.uint8):
            raise RuntimeError("[ScalableTSDFVolume::Integrate] Unsupported image format.")
        depth = image.depth
        if depth.dtype != np.float32 or depth.width != intrinsic.width or depth.height != intrinsic.height:
            raise RuntimeError("[ScalableTSDFVolume::Integrate] Unsupported image format.")
        if rgb8 and (color.width != intrinsic.width or color.height != intrinsic.height):
            raise RuntimeError("[ScalableTSDFVolume::Integrate] Unsupported image format.")
        intr = L.intrinsics_struct(intrinsic)
        cdev = color.dev() if rgb8 else None
        raw = getattr(image, "_raw_depth", None)
        if raw is not None:
            d16, scale, trunc = raw
            self._queued((d16, cdev))
            L.call("ot_tsdf_integrate_u16", self._h, D.ptr(d16), D.ptr(cdev), C.byref(intr),
                   ext.ctypes.data, scale, trunc, D.stream_ptr())  # int address: data_as costs ~2 us a call
            self._release()
        else:
            ddev = depth.dev()
            self._queued((ddev, cdev))
            L.call("ot_tsdf_integrate", self._h, D.ptr(ddev), D.ptr(cdev), C.byref(intr),
                   ext.ctypes.data, D.stream_ptr())
            self._release()

    def flush(self):
        L.call("ot_tsdf_flush", self._h, D.stream_ptr())
        self._keep.clear()

    # ---- readers (each flushes queued frames first) ----
    def num_units(self):
        n = C.c_int64(0)
        L.call("ot_tsdf_num_units", self._h, C.byref(n), D.stream_ptr())
        self._keep.clear()
        return n.value

    def counters(self):
        """(voxel_updates, unit_integrations) since create/reset."""
        u, k = C.c_int64(0), C.c_int64(0)
        L.call("ot_tsdf_counters", self._h, C.byref(u), C.byref(k), D.stream_ptr())
        self._keep.clear()
        return u.value, k.value

    def export_units(self, color_dtype=None):
        """All units sorted by key: keys (U,3) int32, tsdf/weight (U,4096) f32, color (U,4096,3) (voxels in Open3D
        IndexOf order x*256 + y*16 + z).  Colour comes out as float64 for a colour-precision-64 volume (exact) and
        float32 otherwise, unless color_dtype ("float32" / "float64") asks for another."""
        n = self.num_units()
        keys = D.empty((n, 3), "int32")
        tsdf = D.empty((n, 4096), "float32")
        weight = D.empty((n, 4096), "float32")
        cdt = color_dtype or ("float64" if self.color_precision == 64 else "float32")
        color = D.empty((n, 4096, 3), cdt)
        L.call("ot_tsdf_export_units", self._h, n, D.ptr(keys), D.ptr(tsdf), D.ptr(weight),
               D.ptr(color) if cdt == "float32" else None, D.stream_ptr())
        if cdt == "float64":
            if self.color_precision == 64:
                L.call("ot_tsdf_export_color64", self._h, n, D.ptr(color), D.stream_ptr())
            else:
                c32 = D.empty((n, 4096, 3), "float32")
                L.call("ot_tsdf_export_units", self._h, n, None, None, None, D.ptr(c32), D.stream_ptr())
                color.copy_(c32)
        return keys, tsdf, weight, color

    def import_units(self, keys, tsdf, weight, color=None):
        """Insert units in export_units' layout (device tensors or arrays); the inverse of export_units."""
        keys = D.to_device(keys, "int32")
        n = int(keys.shape[0])
        tsdf = D.to_device(tsdf, "float32")
        weight = D.to_device(weight, "float32")
        c64 = self.color_precision == 64
        color = D.to_device(color, "float64" if c64 else "float32") if color is not None else None
        if tuple(tsdf.shape[-1:]) != (4096,) or tsdf.shape[0] != n or weight.shape[0] != n or (
                color is not None and color.shape[0] != n):
            raise RuntimeError("[ScalableTSDFVolume] import_units: shapes do not match export_units")
        L.call("ot_tsdf_import_units_color64" if c64 else "ot_tsdf_import_units", self._h, n, D.ptr(keys),
               D.ptr(tsdf), D.ptr(weight), D.ptr(color), D.stream_ptr())

    def set_shard(self, rank, world):
        """Keep only the units owned by `rank` of `world` (spatial sharding of one object)."""
        L.call("ot_tsdf_set_shard", self._h, int(rank), int(world))

    def set_shard_sector(self, rank, world, centre=(0.0, 0.0)):
        """Keep only the units in azimuth sector `rank` of `world` around the scan centre (x, y) in metres
        (ot_tsdf_set_shard_sector): a ring scan's rank then stages only the image tiles its units project to."""
        L.call("ot_tsdf_set_shard_sector", self._h, int(rank), int(world), float(centre[0]), float(centre[1]))

    def set_shard_block(self, log2_units):
        """Ownership granularity of a sharded volume (ot_tsdf_set_shard_block): 2^log2_units units per axis."""
        L.call("ot_tsdf_set_shard_block", self._h, int(log2_units))

    def border_destinations(self, keys):
        """Per border-row key (export_border's keys), the int64 bitmask of the other ranks whose units read it."""
        keys = D.to_device(keys, "int32")
        out = D.empty((int(keys.shape[0]),), "int64")
        L.call("ot_tsdf_border_destinations", self._h, int(keys.shape[0]), D.ptr(keys), D.ptr(out), D.stream_ptr())
        return out

    def export_border(self):
        """This shard's border (ot_tsdf_export_border): per own unit keys (U,3) int32, tsdf/weight (U,721) f32,
        colour (U,721,3) in the volume's colour precision -- the low-face voxels that neighbouring units' marching
        cubes read (halo units imported earlier are not exported)."""
        n = self.num_units()
        keys = D.empty((n, 3), "int32")
        tsdf = D.empty((n, 721), "float32")
        weight = D.empty((n, 721), "float32")
        color = D.empty((n, 721, 3), "float64" if self.color_precision == 64 else "float32")
        if self.color_type != TSDFVolumeColorType.RGB8:
            color.zero_()  # NoColor: the C side writes no colour rows
        m = C.c_int64(0)
        L.call("ot_tsdf_export_border", self._h, n, D.ptr(keys), D.ptr(tsdf), D.ptr(weight), D.ptr(color),
               C.byref(m), D.stream_ptr())
        m = m.value
        return keys[:m], tsdf[:m], weight[:m], color[:m]

    def import_border(self, keys, tsdf, weight, color=None):
        """Other shards' border rows (export_border's layout): the ones this shard's marching cubes needs become
        halo units; the rest are skipped."""
        keys = D.to_device(keys, "int32")
        n = int(keys.shape[0])
        tsdf = D.to_device(tsdf, "float32")
        weight = D.to_device(weight, "float32")
        c64 = self.color_precision == 64
        color = D.to_device(color, "float64" if c64 else "float32") if color is not None else None
        if tuple(tsdf.shape[-1:]) != (721,) or tsdf.shape[0] != n or weight.shape[0] != n or (
                color is not None and color.shape[0] != n):
            raise RuntimeError("[ScalableTSDFVolume] import_border: shapes do not match export_border")
        L.call("ot_tsdf_import_border", self._h, n, D.ptr(keys), D.ptr(tsdf), D.ptr(weight), D.ptr(color),
               D.stream_ptr())

    def extract_mesh_and_sample_min_z(self, number_of_points, z_min, seed=0, vertex_normals=True):
        """reconstruct_rgbd_filter.py:112-132 in one host call (not an Open3D API): extract_triangle_mesh() ->
        compute_vertex_normals() -> sample_points_uniformly(number_of_points) -> the rows with z >= z_min, points and
        colours (the cloud TriangleMesh.sample_points_min_z returns).  Returns (mesh, cloud); cloud is None for an
        empty mesh (the reference skips it, :115-117).  The marching-cubes totals go straight to the sampler's first
        launch inside ot_tsdf_extract_sample_min_z (no Python between them); the vertex normals run beside the sampling
        on a side stream and a reader of mesh.vertex_normals waits for them.  The first extraction of a volume (no
        capacity guess yet) or a capacity miss takes the separate calls -- the same bits."""
        if number_of_points <= 0:
            raise RuntimeError("[SamplePointsUniformly] number_of_points <= 0")
        cv, ct = getattr(self, "_mesh_cap", (0, 0))
        if not (cv and ct):
            return self._extract_then_sample(number_of_points, z_min, seed, vertex_normals)
        torch = D.torch
        rgb = self.color_type == TSDFVolumeColorType.RGB8
        n = int(number_of_points)
        V = D.empty((cv, 3), "float64")
        VC = D.empty((cv, 3), "float64") if rgb else None
        T = D.empty((ct, 3), "int32")
        N = D.empty((cv, 3), "float64") if vertex_normals else None
        P = D.empty((n, 3), "float64")
        PC = D.empty((n, 3), "float64") if rgb else None
        cur = torch.cuda.current_stream()
        side = _streams.side_stream(cur) if vertex_normals else None
        nv, nt, kept = C.c_int64(0), C.c_int64(0), C.c_int64(0)
        st = L.load().ot_tsdf_extract_sample_min_z(
            self._h, D.ptr(V), D.ptr(VC), D.ptr(T), cv, ct, D.ptr(N), C.c_void_p(side.cuda_stream) if side else None,
            n, C.c_uint64(int(seed) & 0xFFFFFFFFFFFFFFFF), float(z_min), D.ptr(P), D.ptr(PC), C.byref(nv),
            C.byref(nt), C.byref(kept), D.stream_ptr())
        self._keep.clear()
        if st == L.OT_ERR_CAPACITY and (nv.value or nt.value):  # the mesh outgrew the guess: the separate calls
            self._mesh_cap = (nv.value + nv.value // 8 + 1024, nt.value + nt.value // 8 + 1024)
            return self._extract_then_sample(number_of_points, z_min, seed, vertex_normals)
        if st != L.OT_OK:
            raise L.OTError(L.load().ot_last_error().decode())
        self._mesh_cap = (nv.value + nv.value // 8 + 1024, nt.value + nt.value // 8 + 1024)
        mesh = TriangleMesh()
        mesh._v = _Arr(dev=V[:nv.value])
        mesh._t = _Arr(dev=T[:nt.value])
        if VC is not None:
            mesh._vc = _Arr(dev=VC[:nv.value])
        if nv.value == 0:
            return mesh, None
        if nt.value == 0:  # vertices but no triangles (marching cubes cannot emit this): Open3D's sampler raises
            raise RuntimeError("[SamplePointsUniformly] Input mesh has no triangles.")
        if N is not None:
            for t in (V, T, N):  # allocated on the caller's stream, used on the side stream
                t.record_stream(side)
            # one event per volume, re-recorded by each call: a reader of an older mesh's normals then waits for a
            # later point of the same in-order side stream (never too early), and no event is created per call
            done = getattr(self, "_normals_done", None)
            if done is None:
                done = self._normals_done = torch.cuda.Event()
            done.record(side)
            mesh._vn = _Arr(dev=N[:nv.value], ready=done)
        pcd = PointCloud()
        pcd._xyz = _Arr(dev=P[:kept.value])
        pcd._rgb = _Arr(dev=PC[:kept.value]) if PC is not None else None
        return mesh, pcd

    def _extract_then_sample(self, number_of_points, z_min, seed, vertex_normals):
        mesh = self.extract_triangle_mesh()
        if vertex_normals:
            mesh.compute_vertex_normals()
        if not mesh.has_vertices():
            return mesh, None
        return mesh, mesh.sample_points_min_z(number_of_points, z_min, seed)

    def extract_triangle_mesh(self, with_keys=False):
        """ScalableTSDFVolume::ExtractTriangleMesh — GPU marching cubes (mc.hip).  with_keys: also return the merge
        keys (vertex (U,4) int32 = owner unit key + edge bit, triangle (T,3) int32 = its cube's unit key) that
        distributed.merge_shard_meshes uses."""
        nv, nt = C.c_int64(0), C.c_int64(0)
        rgb = self.color_type == TSDFVolumeColorType.RGB8
        cv, ct = getattr(self, "_mesh_cap", (0, 0))
        if cv and ct:
            # sized from this volume's last extraction: the emission straight into the mesh arrays is queued before
            # the totals come back (the GPU does not wait for the host); too small -> emitted again below
            V = D.empty((cv, 3), "float64")
            VC = D.empty((cv, 3), "float64") if rgb else None
            T = D.empty((ct, 3), "int32")
            try:
                L.call("ot_tsdf_extract_triangle_mesh_into", self._h, D.ptr(V), D.ptr(VC), D.ptr(T), cv, ct,
                       C.byref(nv), C.byref(nt), D.stream_ptr())
                fits = True
            except L.OTError:
                if nv.value == 0 and nt.value == 0:  # not a capacity miss: the extraction itself failed
                    raise
                fits = False
        else:
            # count, then emit straight into the mesh's own arrays (no copy out of the volume's buffers)
            L.call("ot_tsdf_extract_triangle_mesh_count", self._h, C.byref(nv), C.byref(nt), D.stream_ptr())
            fits = False
        self._keep.clear()
        if fits:
            V, T = V[:nv.value], T[:nt.value]
            VC = VC[:nv.value] if VC is not None else None
        else:
            V = D.empty((nv.value, 3), "float64")
            VC = D.empty((nv.value, 3), "float64") if rgb else None
            T = D.empty((nt.value, 3), "int32")
            L.call("ot_tsdf_emit_triangle_mesh", self._h, D.ptr(V), D.ptr(VC), D.ptr(T), D.stream_ptr())
        self._mesh_cap = (nv.value + nv.value // 8 + 1024, nt.value + nt.value // 8 + 1024)
        mesh = TriangleMesh()
        mesh._v = _Arr(dev=V)
        mesh._t = _Arr(dev=T)
        serial = C.c_int64(-1)
        L.call("ot_tsdf_mesh_serial", self._h, C.byref(serial))
        # normals via the marching-cubes structure kept with this volume (weakly referenced: the mesh outlives it)
        # the device arrays' identity and torch version counters are recorded too: an in-place edit of V or T (same
        # pointer, same counts) bumps the version and sends compute_vertex_normals to the generic path
        mesh._mc = (weakref.ref(self), serial.value, V.data_ptr(), V._version, T.data_ptr(), T._version) \
            if serial.value >= 0 else None
        if VC is not None:
            mesh._vc = _Arr(dev=VC)
        if not with_keys:
            return mesh
        vk = D.empty((nv.value, 4), "int32")
        tk = D.empty((nt.value, 3), "int32")
        L.call("ot_tsdf_fetch_mesh_keys", self._h, D.ptr(vk), D.ptr(tk), D.stream_ptr())
        return mesh, vk, tk
