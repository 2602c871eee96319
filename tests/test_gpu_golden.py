"""The HIP path against the committed golden vectors (tests/golden/golden_small.npz, CPU-restatement outputs on
stored 80x60 synthetic inputs): depth conversion, unprojection, voxel downsample (keys, averages), SOR (kept
indices, mean distances), ROR, TSDF (unit keys, tsdf and weight bytes, counters), marching cubes, normals,
surface area and seeded sampling -- arrays compared bit for bit, large outputs through SHA-256 digests."""
import ctypes as C
import os
import sys

import numpy as np
import pytest
import torch

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import gen_golden as G  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def golden():
    return np.load(G.OUT, allow_pickle=False)


def _rgbd(pkg, depth, color, trunc):
    return pkg.geometry.RGBDImage.create_from_color_and_depth(
        pkg.geometry.Image(color), pkg.geometry.Image(depth), depth_scale=1000.0, depth_trunc=trunc,
        convert_rgb_to_intensity=False)


def test_golden_image_and_filters(pkg, gpu, golden):
    L = pkg._lib
    depth, color, ext = golden["in_depth"], golden["in_color"], golden["in_ext"]
    intr = pkg.camera.PinholeCameraIntrinsic(*G.INTR)
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    d16 = torch.from_numpy(depth[0].view(np.int16)).cuda().view(torch.uint16).contiguous()
    df = torch.empty(depth[0].shape, dtype=torch.float32, device="cuda")
    L.call("ot_depth_to_float", C.c_void_p(d16.data_ptr()), C.c_void_p(df.data_ptr()), d16.numel(), 1000.0, 3.0,
           stream)
    assert np.array_equal(df.cpu().numpy(), golden["depth_f"])
    pcd = pkg.geometry.PointCloud.create_from_rgbd_image(_rgbd(pkg, depth[0], color[0], 5.0), intr)
    assert np.array_equal(np.asarray(pcd.points), golden["unproject_xyz"])
    assert np.array_equal(np.asarray(pcd.colors), golden["unproject_rgb"])
    posed = pkg.geometry.PointCloud.create_from_rgbd_image(_rgbd(pkg, depth[1], color[1], 5.0), intr, ext[1])
    xp = np.asarray(posed.points)
    assert xp.shape[0] == int(golden["posed_count"]) and G.digest(xp) == str(golden["posed_digest"])
    ds = posed.voxel_down_sample(0.03)
    assert G.digest(np.asarray(ds.points)) == str(golden["voxel_xyz_digest"])
    assert G.digest(np.asarray(ds.colors)) == str(golden["voxel_rgb_digest"])
    # voxel keys through the C ABI's optional key output
    dx = torch.from_numpy(xp).cuda()
    K = C.c_int64(0)
    n = xp.shape[0]
    vx, vc = (torch.empty((n, 3), dtype=torch.float64, device="cuda") for _ in range(2))
    keys = torch.empty((n, 3), dtype=torch.int32, device="cuda")
    L.call("ot_voxel_down_sample", C.c_void_p(dx.data_ptr()), None, None, n, 0.03, C.c_void_p(vx.data_ptr()), None,
           None, C.c_void_p(keys.data_ptr()), C.byref(K), stream)
    assert np.array_equal(keys[:K.value].cpu().numpy(), golden["voxel_keys"])
    _, sor = ds.remove_statistical_outlier(10, 2.0)
    assert np.array_equal(np.asarray(sor), golden["sor_idx"])
    idx = torch.empty((K.value,), dtype=torch.int64, device="cuda")
    avg = torch.empty((K.value,), dtype=torch.float64, device="cuda")
    kk = C.c_int64(0)
    L.call("ot_remove_statistical_outlier", C.c_void_p(vx.data_ptr()), K.value, 10, 2.0, C.c_void_p(idx.data_ptr()),
           C.c_void_p(avg.data_ptr()), C.byref(kk), stream)
    assert G.digest(avg.cpu().numpy()) == str(golden["sor_avg_digest"])
    _, ror = ds.remove_radius_outlier(4, 0.08)
    assert np.array_equal(np.asarray(ror), golden["ror_idx"])


def test_golden_tsdf_mesh_sampling(pkg, gpu, golden):
    depth, color, ext = golden["in_depth"], golden["in_color"], golden["in_ext"]
    integ = pkg.pipelines.integration
    intr = pkg.camera.PinholeCameraIntrinsic(*G.INTR)
    vol = integ.ScalableTSDFVolume(voxel_length=G.VOXEL, sdf_trunc=G.TRUNC, color_type=integ.TSDFVolumeColorType.RGB8)
    for k in range(depth.shape[0]):
        vol.integrate(_rgbd(pkg, depth[k], color[k], 3.0), intr, ext[k])
    keys, tsdf, weight, _ = (t.cpu().numpy() for t in vol.export_units())
    assert np.array_equal(keys, golden["tsdf_keys"])
    assert G.digest(tsdf) == str(golden["tsdf_digest"]) and G.digest(weight) == str(golden["weight_digest"])
    assert vol.counters() == (int(golden["tsdf_updates"]), int(golden["tsdf_unit_integrations"]))
    mesh = vol.extract_triangle_mesh()
    V, T = np.asarray(mesh.vertices), np.asarray(mesh.triangles)
    assert [V.shape[0], T.shape[0]] == golden["mesh_counts"].tolist()
    assert G.digest(V) == str(golden["mesh_v_digest"]) and G.digest(T) == str(golden["mesh_t_digest"])
    mesh.compute_vertex_normals()
    assert G.digest(np.asarray(mesh.vertex_normals)) == str(golden["normals_digest"])
    assert mesh.get_surface_area() == float(golden["surface_area"])
    pcd = mesh.sample_points_uniformly(number_of_points=3000, seed=7)
    assert G.digest(np.asarray(pcd.points)) == str(golden["sample_digest"])
    assert G.digest(np.asarray(pcd.normals)) == str(golden["sample_normals_digest"])
