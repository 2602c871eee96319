"""GPU parity: marching cubes, vertex normals, uniform sampling and the Z-filter tail of reconstruct_object.

Bit-exact vs the oracle (canonical order): vertex and triangle counts, triangle index lists, vertex
positions; vertex normals; seeded sampled points.  Colours: rel <= 1e-4 (f32 colour state on the GPU).
"""
import numpy as np
import pytest

from conftest import assert_bitwise, ref_intr

pytestmark = pytest.mark.gpu


def _volumes(pkg, O, synth, depth, color, ext, voxel):
    integ = pkg.pipelines.integration
    intr_t = ref_intr(synth)
    intr = pkg.camera.PinholeCameraIntrinsic(*intr_t)
    vol = integ.ScalableTSDFVolume(voxel_length=voxel, sdf_trunc=0.04, color_type=integ.TSDFVolumeColorType.RGB8)
    ref = O.TSDF(voxel, 0.04, 1, 4)
    for k in range(depth.shape[0]):
        rgbd = pkg.geometry.RGBDImage.create_from_color_and_depth(
            pkg.geometry.Image(color[k]), pkg.geometry.Image(depth[k]), depth_scale=1000.0, depth_trunc=3.0,
            convert_rgb_to_intensity=False)
        vol.integrate(rgbd, intr, ext[k])
        ref.integrate(O.depth_to_float(depth[k], 1000.0, 3.0), color[k], intr_t, ext[k])
    return vol, ref


@pytest.fixture(scope="module")
def meshes(pkg, O, synth, seq16, gpu):
    depth, color, ext = seq16
    vol, ref = _volumes(pkg, O, synth, depth, color, ext, 0.01)
    mesh = vol.extract_triangle_mesh()
    V, VC, T = ref.extract_triangle_mesh()
    return mesh, (V, VC, T)


def test_marching_cubes_bitexact(meshes):
    mesh, (V, VC, T) = meshes
    assert V.shape[0] > 10000
    assert len(mesh.vertices) == V.shape[0] and len(mesh.triangles) == T.shape[0]
    assert_bitwise(np.asarray(mesh.triangles), T, "triangles")
    assert_bitwise(np.asarray(mesh.vertices), V, "vertices")
    assert_bitwise(np.asarray(mesh.vertex_colors), VC, "vertex colours (float64 colour state)")


def test_marching_cubes_5mm(pkg, O, synth, seq16):
    depth, color, ext = seq16
    vol, ref = _volumes(pkg, O, synth, depth[:2], color[:2], ext[:2], 0.005)
    mesh = vol.extract_triangle_mesh()
    V, VC, T = ref.extract_triangle_mesh()
    assert_bitwise(np.asarray(mesh.triangles), T, "triangles 5mm")
    assert_bitwise(np.asarray(mesh.vertices), V, "vertices 5mm")


def test_extraction_phases_c_abi(pkg, O, synth, seq16):
    """The facade's count + emit (straight into the mesh arrays) and the one-call ot_tsdf_extract_triangle_mesh +
    ot_tsdf_fetch_triangle_mesh give the same bits; after a count, fetch emits again; emitting after the volume changed
    fails, and so do merge keys before any emission."""
    import ctypes as C

    import torch

    L = pkg._lib
    lib = L.load()
    depth, color, ext = seq16
    vol, ref = _volumes(pkg, O, synth, depth[:3], color[:3], ext[:3], 0.01)
    V, VC, T = ref.extract_triangle_mesh()
    mesh = vol.extract_triangle_mesh()
    assert_bitwise(np.asarray(mesh.vertices), V, "count + emit vertices")
    assert_bitwise(np.asarray(mesh.triangles), T, "count + emit triangles")
    assert_bitwise(np.asarray(mesh.vertex_colors), VC, "count + emit colours")
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    nv, nt = C.c_int64(0), C.c_int64(0)

    def fetch():
        dv = torch.empty((nv.value, 3), dtype=torch.float64, device="cuda")
        dc = torch.empty((nv.value, 3), dtype=torch.float64, device="cuda")
        dt = torch.empty((nt.value, 3), dtype=torch.int32, device="cuda")
        assert lib.ot_tsdf_fetch_triangle_mesh(vol._h, C.c_void_p(dv.data_ptr()), C.c_void_p(dc.data_ptr()),
                                               C.c_void_p(dt.data_ptr()), s) == 0, lib.ot_last_error()
        torch.cuda.synchronize()
        return dv.cpu().numpy(), dc.cpu().numpy(), dt.cpu().numpy()

    # one-call extraction (the volume's own buffers), then fetch copies
    assert lib.ot_tsdf_extract_triangle_mesh(vol._h, C.byref(nv), C.byref(nt), s) == 0
    dv, dc, dt = fetch()
    assert_bitwise(dv, V, "one-call vertices")
    assert_bitwise(dt, T, "one-call triangles")
    assert_bitwise(dc, VC, "one-call colours")
    # count only: keys refuse until an emission, fetch emits from the kept structure
    assert lib.ot_tsdf_extract_triangle_mesh_count(vol._h, C.byref(nv), C.byref(nt), s) == 0
    vk = torch.empty((nv.value, 4), dtype=torch.int32, device="cuda")
    tk = torch.empty((nt.value, 3), dtype=torch.int32, device="cuda")
    assert lib.ot_tsdf_fetch_mesh_keys(vol._h, C.c_void_p(vk.data_ptr()), C.c_void_p(tk.data_ptr()), s) != 0
    dv, dc, dt = fetch()
    assert_bitwise(dv, V, "count + fetch vertices")
    assert_bitwise(dt, T, "count + fetch triangles")
    assert lib.ot_tsdf_fetch_mesh_keys(vol._h, C.c_void_p(vk.data_ptr()), C.c_void_p(tk.data_ptr()), s) == 0
    # the volume changes: emission from the stale structure is refused
    rgbd = pkg.geometry.RGBDImage.create_from_color_and_depth(
        pkg.geometry.Image(color[3]), pkg.geometry.Image(depth[3]), depth_scale=1000.0, depth_trunc=3.0,
        convert_rgb_to_intensity=False)
    vol.integrate(rgbd, pkg.camera.PinholeCameraIntrinsic(*ref_intr(synth)), ext[3])
    vol.flush()
    dv = torch.empty((nv.value, 3), dtype=torch.float64, device="cuda")
    dt = torch.empty((nt.value, 3), dtype=torch.int32, device="cuda")
    assert lib.ot_tsdf_emit_triangle_mesh(vol._h, C.c_void_p(dv.data_ptr()), None, C.c_void_p(dt.data_ptr()),
                                          s) != 0
    assert "changed" in lib.ot_last_error().decode()


def test_extraction_into_guessed_capacity(pkg, O, synth, seq16):
    """ot_tsdf_extract_triangle_mesh_into (the facade's path from a volume's second extraction on: emission queued
    before the totals are read back): a capacity that fits gives the oracle's mesh; one that does not reports
    OT_ERR_CAPACITY with the totals and the facade emits again -- both through the facade (same volume extracted, then
    grown by more frames and extracted again) and through the C ABI directly."""
    import ctypes as C

    import torch

    L = pkg._lib
    lib = L.load()
    depth, color, ext = seq16
    integ = pkg.pipelines.integration
    intr_t = ref_intr(synth)
    intr = pkg.camera.PinholeCameraIntrinsic(*intr_t)
    vol = integ.ScalableTSDFVolume(voxel_length=0.01, sdf_trunc=0.04, color_type=integ.TSDFVolumeColorType.RGB8)
    ref = O.TSDF(0.01, 0.04, 1, 4)
    nf = depth.shape[0]
    for k in range(nf):
        rgbd = pkg.geometry.RGBDImage.create_from_color_and_depth(
            pkg.geometry.Image(color[k]), pkg.geometry.Image(depth[k]), depth_scale=1000.0, depth_trunc=3.0,
            convert_rgb_to_intensity=False)
        vol.integrate(rgbd, intr, ext[k])
        ref.integrate(O.depth_to_float(depth[k], 1000.0, 3.0), color[k], intr_t, ext[k])
        if k in (0, 1, nf - 1):  # 0: count + emit; then guesses from the previous mesh (too small: emitted again)
            mesh = vol.extract_triangle_mesh()
            V, VC, T = ref.extract_triangle_mesh()
            assert_bitwise(np.asarray(mesh.vertices), V, f"vertices after {k + 1} frames")
            assert_bitwise(np.asarray(mesh.triangles), T, f"triangles after {k + 1} frames")
            assert_bitwise(np.asarray(mesh.vertex_colors), VC, f"colours after {k + 1} frames")
            mesh.compute_vertex_normals()
            assert_bitwise(np.asarray(mesh.vertex_normals), O.vertex_normals(V, T), f"normals after {k + 1} frames")
    mesh = vol.extract_triangle_mesh()  # unchanged volume: the guess fits
    assert_bitwise(np.asarray(mesh.vertices), V, "second extraction of an unchanged volume")
    s = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    nv, nt = C.c_int64(0), C.c_int64(0)
    small_v, small_t = V.shape[0] // 2, T.shape[0] // 2
    dv = torch.empty((small_v, 3), dtype=torch.float64, device="cuda")
    dt = torch.empty((small_t, 3), dtype=torch.int32, device="cuda")
    st = lib.ot_tsdf_extract_triangle_mesh_into(vol._h, C.c_void_p(dv.data_ptr()), None, C.c_void_p(dt.data_ptr()),
                                                small_v, small_t, C.byref(nv), C.byref(nt), s)
    assert st == L.OT_ERR_CAPACITY and (nv.value, nt.value) == (V.shape[0], T.shape[0])
    dv = torch.empty((nv.value, 3), dtype=torch.float64, device="cuda")
    dt = torch.empty((nt.value, 3), dtype=torch.int32, device="cuda")
    assert lib.ot_tsdf_emit_triangle_mesh(vol._h, C.c_void_p(dv.data_ptr()), None, C.c_void_p(dt.data_ptr()), s) == 0
    torch.cuda.synchronize()
    assert_bitwise(dv.cpu().numpy(), V, "emitted after a capacity miss")
    assert_bitwise(dt.cpu().numpy(), T, "triangles emitted after a capacity miss")


def test_empty_volume_mesh(pkg, gpu):
    integ = pkg.pipelines.integration
    vol = integ.ScalableTSDFVolume(voxel_length=0.01, sdf_trunc=0.04, color_type=integ.TSDFVolumeColorType.RGB8)
    mesh = vol.extract_triangle_mesh()
    assert len(mesh.vertices) == 0 and len(mesh.triangles) == 0


def test_vertex_normals_bitexact(O, meshes):
    mesh, (V, VC, T) = meshes
    mesh.compute_vertex_normals()
    assert_bitwise(np.asarray(mesh.vertex_normals), O.vertex_normals(V, T), "vertex normals")


def test_sampling_bitexact(O, meshes):
    mesh, (V, VC, T) = meshes
    mesh.compute_vertex_normals()
    N = O.vertex_normals(V, T)
    for n_pts, seed in ((100000, 0), (15000, 42)):
        pcd = mesh.sample_points_uniformly(number_of_points=n_pts, seed=seed)
        P, PN, PC = O.sample_points_uniformly(V, T, n_pts, seed, VN=N, VC=VC)
        assert_bitwise(np.asarray(pcd.points), P, "sampled points")
        assert_bitwise(np.asarray(pcd.normals), PN, "sampled normals")
        assert_bitwise(np.asarray(pcd.colors), PC, "sampled colours")


def test_z_filter_tail(O, meshes):
    """reconstruct_rgbd_filter.py:123-132: sample 100k, keep z >= 0.03 (points and colours)."""
    mesh, (V, VC, T) = meshes
    pcd = mesh.sample_points_uniformly(number_of_points=100000, seed=3)
    out = pcd.filter_min_z(0.03)
    P, _, PC = O.sample_points_uniformly(V, T, 100000, 3, VC=VC)
    rx, _ = O.filter_min_z(P, PC, 0.03)
    assert_bitwise(np.asarray(out.points), rx, "filtered points")
    assert 0 < len(out.points) < 100000
    assert not out.has_normals()


@pytest.mark.parametrize("z_min", [0.03, -np.inf, np.inf, 0.0])
def test_sample_min_z_fused(pkg, O, synth, seq16, meshes, z_min):
    """TriangleMesh.sample_points_min_z (ot_mesh_sample_points_min_z: sampling and Z mask in one pass) = the two steps
    (sample_points_uniformly(...).filter_min_z) = the oracle, for one mesh and for meshes of different sizes in one
    batch; -inf keeps every sample (the last tile partial: 100003 points), +inf none."""
    mesh, (V, VC, T) = meshes
    n = 100003
    out = mesh.sample_points_min_z(n, z_min, seed=3)
    two = mesh.sample_points_uniformly(number_of_points=n, seed=3).filter_min_z(z_min)
    P, _, PC = O.sample_points_uniformly(V, T, n, 3, VC=VC)
    rx, rc = O.filter_min_z(P, PC, z_min)
    assert_bitwise(np.asarray(out.points), rx, "fused points vs oracle")
    assert_bitwise(np.asarray(out.colors), rc, "fused colours vs oracle")
    assert_bitwise(np.asarray(out.points), np.asarray(two.points), "fused vs two steps")
    assert not out.has_normals()
    if z_min == -np.inf:
        assert len(out.points) == n
    if z_min == np.inf:
        assert len(out.points) == 0
    depth, color, ext = seq16
    vol2, _ = _volumes(pkg, O, synth, depth[:1], color[:1], ext[:1], 0.02)
    mesh2 = vol2.extract_triangle_mesh()
    batch = pkg.geometry.TriangleMesh.sample_points_min_z_batch([mesh2, mesh, mesh2], 5000, z_min, seed=9)
    for m, c in zip([mesh2, mesh, mesh2], batch):
        one = m.sample_points_uniformly(number_of_points=5000, seed=9).filter_min_z(z_min)
        assert_bitwise(np.asarray(c.points), np.asarray(one.points), "fused batch vs two steps")
        assert_bitwise(np.asarray(c.colors), np.asarray(one.colors), "fused batch colours")


def test_sample_min_z_with_normals_in_flight(pkg, O, synth, seq16):
    """The fused sampler on a fresh mesh whose vertex normals are still running on the side stream: it does not read
    them (no wait), and the normals stay correct for a later reader."""
    depth, color, ext = seq16
    vol, ref = _volumes(pkg, O, synth, depth[:4], color[:4], ext[:4], 0.01)
    mesh = vol.extract_triangle_mesh()
    V, VC, T = ref.extract_triangle_mesh()
    mesh.compute_vertex_normals()
    out = mesh.sample_points_min_z(100000, 0.03, seed=1)
    P, _, PC = O.sample_points_uniformly(V, T, 100000, 1, VC=VC)
    rx, _ = O.filter_min_z(P, PC, 0.03)
    assert_bitwise(np.asarray(out.points), rx, "fused points")
    assert_bitwise(np.asarray(mesh.vertex_normals), O.vertex_normals(V, T), "normals after the fused sampler")


def test_deferred_normals_queued_by_the_sampler(pkg, O, synth, seq16):
    """compute_vertex_normals of a fresh mesh is deferred: the fused sampler queues it once its own chains are queued
    (ot_mesh_sample_points_min_z_async / _wait) and the normals equal the oracle's.  A mesh whose volume changes
    between compute_vertex_normals and the launch takes the generic corner sort on its own arrays (same bits)."""
    depth, color, ext = seq16
    vol, ref = _volumes(pkg, O, synth, depth[:3], color[:3], ext[:3], 0.01)
    V, VC, T = ref.extract_triangle_mesh()
    rN = O.vertex_normals(V, T)
    mesh = vol.extract_triangle_mesh()
    mesh.compute_vertex_normals()
    assert mesh._vn._launch is not None  # deferred
    out = mesh.sample_points_min_z(100000, 0.03, seed=2)
    assert mesh._vn._launch is None  # queued by the sampler
    P, _, PC = O.sample_points_uniformly(V, T, 100000, 2, VC=VC)
    rx, _ = O.filter_min_z(P, PC, 0.03)
    assert_bitwise(np.asarray(out.points), rx, "fused points (normals deferred)")
    assert_bitwise(np.asarray(mesh.vertex_normals), rN, "deferred normals queued by the sampler")
    mesh2 = vol.extract_triangle_mesh()
    mesh2.compute_vertex_normals()
    rgbd = pkg.geometry.RGBDImage.create_from_color_and_depth(
        pkg.geometry.Image(color[3]), pkg.geometry.Image(depth[3]), convert_rgb_to_intensity=False)
    vol.integrate(rgbd, pkg.camera.PinholeCameraIntrinsic(*ref_intr(synth)), ext[3])
    vol.flush()
    assert_bitwise(np.asarray(mesh2.vertex_normals), rN, "deferred normals after the volume changed")
    # a writable view of the vertices queues the deferred normals first (they read V on the device)
    mesh3 = vol.extract_triangle_mesh()
    mesh3.compute_vertex_normals()
    Vv = np.asarray(mesh3.vertices)
    assert mesh3._vn._launch is None
    assert_bitwise(np.asarray(mesh3.vertex_normals), O.vertex_normals(Vv, np.asarray(mesh3.triangles)),
                   "deferred normals queued by a vertices view")


def test_deferred_normals_vs_later_volume_work(pkg, O, synth, seq16):
    """the deferred vertex normals run on a side stream and read the volume's marching-cubes structure
    (cubes, neighbour tables, triangle bases, vertex keys / owners).  The sampler starts them; the same volume then
    integrates another frame, is extracted again (its structure rewritten) and reset, all on the caller's stream
    before anyone reads the first mesh's normals.  That work waits for the normals (the volume's normals event), so
    the first mesh's normals still equal the oracle's for ITS vertices and triangles."""
    depth, color, ext = seq16
    vol, ref = _volumes(pkg, O, synth, depth[:3], color[:3], ext[:3], 0.005)
    V, VC, T = ref.extract_triangle_mesh()
    rN = O.vertex_normals(V, T)
    mesh = vol.extract_triangle_mesh()
    mesh.compute_vertex_normals()
    mesh.sample_points_min_z(100000, 0.03, seed=3)  # queues the normals on the side stream
    rgbd = pkg.geometry.RGBDImage.create_from_color_and_depth(
        pkg.geometry.Image(color[3]), pkg.geometry.Image(depth[3]), convert_rgb_to_intensity=False)
    vol.integrate(rgbd, pkg.camera.PinholeCameraIntrinsic(*ref_intr(synth)), ext[3])
    mesh2 = vol.extract_triangle_mesh()  # rewrites the structure the first mesh's normals walk
    mesh2.compute_vertex_normals()
    mesh2.sample_points_min_z(1000, 0.03)
    vol.reset()
    assert_bitwise(np.asarray(mesh.vertex_normals), rN, "first mesh's normals after later work on the volume")


def test_fused_extract_sample_min_z(pkg, O, synth, seq16):
    """ScalableTSDFVolume.extract_mesh_and_sample_min_z (ot_tsdf_extract_sample_min_z: marching cubes, the fused
    sampler and the vertex normals in one host call) gives the oracle's mesh, normals and Z-masked cloud -- on the
    volume's first extraction (the separate calls), on a later one (the fused C entry), and on a capacity miss."""
    depth, color, ext = seq16
    intr = pkg.camera.PinholeCameraIntrinsic(*ref_intr(synth))
    vol, ref = _volumes(pkg, O, synth, depth[:2], color[:2], ext[:2], 0.005)

    def check(tag, seed):
        mesh, cloud = vol.extract_mesh_and_sample_min_z(100000, 0.03, seed=seed)
        V, VC, T = ref.extract_triangle_mesh()
        assert_bitwise(np.asarray(mesh.vertices), V, f"vertices ({tag})")
        assert_bitwise(np.asarray(mesh.vertex_colors), VC, f"vertex colours ({tag})")
        assert_bitwise(np.asarray(mesh.triangles), T, f"triangles ({tag})")
        P, _, PC = O.sample_points_uniformly(V, T, 100000, seed, VC=VC)
        rx, rc = O.filter_min_z(P, PC, 0.03)
        assert_bitwise(np.asarray(cloud.points), rx, f"fused cloud points ({tag})")
        assert_bitwise(np.asarray(cloud.colors), rc, f"fused cloud colours ({tag})")
        assert_bitwise(np.asarray(mesh.vertex_normals), O.vertex_normals(V, T), f"normals ({tag})")

    def more(k):
        rgbd = pkg.geometry.RGBDImage.create_from_color_and_depth(
            pkg.geometry.Image(color[k]), pkg.geometry.Image(depth[k]), convert_rgb_to_intensity=False)
        vol.integrate(rgbd, intr, ext[k])
        ref.integrate(O.depth_to_float(depth[k], 1000.0, 3.0), color[k], ref_intr(synth), ext[k])

    check("first extraction: separate calls", 4)
    more(2)
    check("fused C entry", 5)
    more(3)
    vol._mesh_cap = (64, 64)  # a guess far too small: the capacity miss takes the separate calls
    check("capacity miss", 6)
    empty = pkg.pipelines.integration.ScalableTSDFVolume(voxel_length=0.005, sdf_trunc=0.04,
                                                         color_type=pkg.pipelines.integration.TSDFVolumeColorType.RGB8)
    empty._mesh_cap = (1024, 1024)
    mesh, cloud = empty.extract_mesh_and_sample_min_z(1000, 0.03)
    assert cloud is None and not mesh.has_vertices()


@pytest.mark.parametrize("fork,normals_at", [(0, 0), (0, 2), (1, 1)])
def test_fused_call_schedules_bitexact(pkg, O, synth, seq16, gpu, fork, normals_at):
    """The scheduling knobs of the fused call change no bit: the marching-cubes emission as one launch (default) or as
    two kernels on two streams (otx_mc_emit_fork), and the vertex normals started right after the emission, beside the
    area-sum walk (default) or beside the CDF walk (otx_normals_at) -- each against the oracle, twice on one volume."""
    L = pkg._lib
    depth, color, ext = seq16
    vol, ref = _volumes(pkg, O, synth, depth[:3], color[:3], ext[:3], 0.005)
    V, VC, T = ref.extract_triangle_mesh()
    P, _, PC = O.sample_points_uniformly(V, T, 50000, 9, VC=VC)
    rx, rc = O.filter_min_z(P, PC, 0.03)
    VN = O.vertex_normals(V, T)
    vol.extract_mesh_and_sample_min_z(50000, 0.03, seed=9)  # the first extraction (separate calls) sets the guess
    L.call("otx_mc_emit_fork", fork)
    L.call("otx_normals_at", normals_at)
    try:
        for rep in range(2):
            mesh, cloud = vol.extract_mesh_and_sample_min_z(50000, 0.03, seed=9)
            tag = f"fork {fork}, normals at {normals_at}, pass {rep}"
            assert_bitwise(np.asarray(mesh.vertices), V, f"vertices ({tag})")
            assert_bitwise(np.asarray(mesh.vertex_colors), VC, f"vertex colours ({tag})")
            assert_bitwise(np.asarray(mesh.triangles), T, f"triangles ({tag})")
            assert_bitwise(np.asarray(cloud.points), rx, f"cloud points ({tag})")
            assert_bitwise(np.asarray(cloud.colors), rc, f"cloud colours ({tag})")
            assert_bitwise(np.asarray(mesh.vertex_normals), VN, f"normals ({tag})")
    finally:
        L.call("otx_mc_emit_fork", 0)
        L.call("otx_normals_at", 1)


def test_sampling_batch_matches_single(pkg, O, synth, seq16, meshes):
    """TriangleMesh.sample_points_uniformly_batch: the per-mesh clouds equal the single-mesh calls (and the oracle)
    for meshes of different sizes sampled together."""
    mesh, (V, VC, T) = meshes
    mesh.compute_vertex_normals()
    depth, color, ext = seq16
    vol2, _ = _volumes(pkg, O, synth, depth[:1], color[:1], ext[:1], 0.02)
    mesh2 = vol2.extract_triangle_mesh()
    clouds = pkg.geometry.TriangleMesh.sample_points_uniformly_batch([mesh, mesh2, mesh], number_of_points=20000,
                                                                     seed=5)
    for m, c in zip([mesh, mesh2, mesh], clouds):
        one = m.sample_points_uniformly(number_of_points=20000, seed=5)
        assert_bitwise(np.asarray(c.points), np.asarray(one.points), "batched vs single sampling")
        if m.has_vertex_normals():
            assert_bitwise(np.asarray(c.normals), np.asarray(one.normals), "batched normals")
    P, _, _ = O.sample_points_uniformly(V, T, 20000, 5, VN=O.vertex_normals(V, T), VC=VC)
    assert_bitwise(np.asarray(clouds[0].points), P, "batched vs oracle")


@pytest.mark.parametrize("voxel", [0.01, 0.005])
def test_vertex_normals_mc_walk_bitexact(pkg, O, synth, seq16, gpu, voxel):
    """compute_vertex_normals on a mesh fresh out of extract_triangle_mesh takes the marching-cubes walk
    (ot_tsdf_mesh_vertex_normals: each vertex's <= 4 cubes in triangle order, no corner sort); bit-exact vs the oracle
    and vs the generic corner-sort kernel on the same arrays.  Once the volume changes, the walk refuses and the
    facade falls back to the generic kernel (same bits)."""
    import ctypes as C

    import torch

    L = pkg._lib
    depth, color, ext = seq16
    vol, ref = _volumes(pkg, O, synth, depth, color, ext, voxel)
    mesh = vol.extract_triangle_mesh()
    assert mesh._mc is not None
    nv, nt = len(mesh._v), len(mesh._t)
    V, T = mesh._v.dev(), mesh._t.dev()
    walk = torch.empty((nv, 3), dtype=torch.float64, device="cuda")
    st = L.load().ot_tsdf_mesh_vertex_normals(vol._h, mesh._mc[1], C.c_void_p(V.data_ptr()), nv,
                                              C.c_void_p(T.data_ptr()), nt, C.c_void_p(walk.data_ptr()), None)
    assert st == 0, L.load().ot_last_error()
    generic = torch.empty_like(walk)
    L.call("ot_mesh_compute_vertex_normals", C.c_void_p(V.data_ptr()), nv, C.c_void_p(T.data_ptr()), nt,
           C.c_void_p(generic.data_ptr()), None)
    rV, _, rT = ref.extract_triangle_mesh()
    rN = O.vertex_normals(rV, rT)
    assert_bitwise(walk.cpu().numpy(), rN, "vertex normals (marching-cubes walk)")
    assert_bitwise(generic.cpu().numpy(), rN, "vertex normals (corner sort)")
    mesh.compute_vertex_normals()  # the facade's choice: the walk
    assert_bitwise(np.asarray(mesh.vertex_normals), rN, "facade vertex normals")
    # the volume changes: the walk refuses, the facade falls back
    rgbd = pkg.geometry.RGBDImage.create_from_color_and_depth(
        pkg.geometry.Image(color[0]), pkg.geometry.Image(depth[0]), convert_rgb_to_intensity=False)
    vol.integrate(rgbd, pkg.camera.PinholeCameraIntrinsic(*ref_intr(synth)), ext[0])
    vol.flush()
    st = L.load().ot_tsdf_mesh_vertex_normals(vol._h, mesh._mc[1], C.c_void_p(V.data_ptr()), nv,
                                              C.c_void_p(T.data_ptr()), nt, C.c_void_p(walk.data_ptr()), None)
    assert st != 0
    stale = pkg.geometry.TriangleMesh()
    stale._v, stale._t, stale._mc = mesh._v, mesh._t, mesh._mc
    stale.compute_vertex_normals()
    assert_bitwise(np.asarray(stale.vertex_normals), rN, "fallback vertex normals")


def test_vertex_normals_after_in_place_edit(pkg, O, synth, seq16, gpu):
    """an in-place device edit of the triangle array (same pointer, same counts) must not take the
    marching-cubes walk, whose triangle ids come from the stored structure: the facade sees the tensor's version bump
    and takes the corner sort, which equals the oracle's normals of the EDITED mesh."""
    depth, color, ext = seq16
    vol, ref = _volumes(pkg, O, synth, depth, color, ext, 0.01)
    mesh = vol.extract_triangle_mesh()
    T = mesh._t.dev()
    nt = T.shape[0]
    assert nt > 10
    T[: nt // 2] = T[: nt // 2].flip(1).clone()  # reverse the winding of half the triangles, in place
    mesh.compute_vertex_normals()
    V = np.asarray(mesh.vertices)
    rN = O.vertex_normals(V, T.cpu().numpy())
    assert_bitwise(np.asarray(mesh.vertex_normals), rN, "vertex normals after an in-place triangle edit")


def test_vertex_normals_mc_walk_sharded(pkg, O, synth, seq16, gpu):
    """A spatially sharded volume's partial mesh (own cubes only; halo units supply neighbours): the walk equals the
    corner sort on the same partial mesh."""
    import ctypes as C
    import importlib

    import torch

    L = pkg._lib
    D = importlib.import_module(pkg.__name__ + ".distributed")
    integ = pkg.pipelines.integration
    depth, color, ext = seq16
    intr = pkg.camera.PinholeCameraIntrinsic(*ref_intr(synth))
    shards = []
    for r in range(3):
        v = integ.ScalableTSDFVolume(voxel_length=0.01, sdf_trunc=0.04, color_type=integ.TSDFVolumeColorType.RGB8)
        v.set_shard(r, 3)
        for k in range(depth.shape[0]):
            v.integrate(pkg.geometry.RGBDImage.create_from_color_and_depth(
                pkg.geometry.Image(color[k]), pkg.geometry.Image(depth[k]), convert_rgb_to_intensity=False), intr, ext[k])
        shards.append(v)
    rows = torch.cat([D.pack_border(*v.export_border()) for v in shards])
    for v in shards:
        v.import_border(*D.unpack_border(rows))
        mesh = v.extract_triangle_mesh()
        nv, nt = len(mesh._v), len(mesh._t)
        assert nv > 1000
        walk = torch.empty((nv, 3), dtype=torch.float64, device="cuda")
        generic = torch.empty_like(walk)
        Vp, Tp = C.c_void_p(mesh._v.dev().data_ptr()), C.c_void_p(mesh._t.dev().data_ptr())
        L.call("ot_tsdf_mesh_vertex_normals", v._h, mesh._mc[1], Vp, nv, Tp, nt, C.c_void_p(walk.data_ptr()), None)
        L.call("ot_mesh_compute_vertex_normals", Vp, nv, Tp, nt, C.c_void_p(generic.data_ptr()), None)
        assert_bitwise(walk.cpu().numpy(), generic.cpu().numpy(), "sharded partial mesh normals")
