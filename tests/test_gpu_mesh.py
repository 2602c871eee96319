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
