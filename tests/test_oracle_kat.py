"""Pin the CPU oracle with analytic known-answer tests (the reference has no tests or fixtures: SURVEY.md §4).

Each KAT recomputes the expected value with an independent numpy formulation of the same IEEE operations, or
against a closed form.
"""
import numpy as np
import pytest

from conftest import assert_bitwise


def test_depth_to_float_kat(O):
    d = np.array([0, 1, 1000, 2999, 3000, 3001, 65535], np.uint16)
    out = O.depth_to_float(d, 1000.0, 3.0)
    exp = d.astype(np.float32) / np.float32(1000.0)
    exp[exp.astype(np.float64) >= 3.0] = 0
    assert_bitwise(out, exp, "depth_to_float")
    assert out[2] == np.float32(1.0) and out[4] == 0.0 and out[3] == np.float32(2.999)


def test_inverse4_kat(O, synth):
    # analytic expectations carry no sign of zero (the cofactors give -0.0): value-exact here, not bitwise
    np.testing.assert_array_equal(O.inverse4(np.eye(4)), np.eye(4), "inverse(I)")
    np.testing.assert_array_equal(O.inverse4(synth.T_FIX), synth.T_FIX.T, "inverse(T_fix) = T_fix^T (permutation)")
    rng = np.random.default_rng(0)
    for _ in range(20):
        A = rng.standard_normal((4, 4)) + 4 * np.eye(4)
        np.testing.assert_allclose(O.inverse4(A), np.linalg.inv(A), rtol=1e-12, atol=1e-13)
    T = synth.camera_pose(synth.Scene(), 3, 16)
    np.testing.assert_allclose(O.inverse4(T) @ T, np.eye(4), atol=1e-14)


def test_multiplier_kat(O):
    w, h, fx, fy, cx, cy = 64, 48, 50.0, 55.0, 31.5, 23.5
    m = O.depth_multiplier(w, h, fx, fy, cx, cy)
    xx = (np.arange(w, dtype=np.float32) - np.float32(cx)) * (np.float32(1.0) / np.float32(fx))
    yy = (np.arange(h, dtype=np.float32) - np.float32(cy)) * (np.float32(1.0) / np.float32(fy))
    exp = np.sqrt((xx[None, :] * xx[None, :] + yy[:, None] * yy[:, None]) + np.float32(1.0)).astype(np.float32)
    assert_bitwise(m, exp, "multiplier")


def test_unproject_plane_kat(O):
    """Fronto-parallel plane at 1.5 m, identity extrinsic: x = (j-cx)*z/fx, y = (i-cy)*z/fy, z, row-major."""
    w, h, fx, fy, cx, cy = 40, 30, 35.0, 36.0, 19.5, 14.5
    depth = np.full((h, w), 1.5, np.float32)
    depth[3, 7] = 0.0  # a hole
    color = np.arange(h * w * 3, dtype=np.uint32).reshape(h, w, 3).astype(np.uint8)
    xyz, rgb = O.unproject(depth, color, (w, h, fx, fy, cx, cy))
    ii, jj = np.nonzero(depth > 0)
    z = depth[ii, jj].astype(np.float64)
    exp = np.stack([(jj - cx) * z / fx, (ii - cy) * z / fy, z], axis=1)
    assert xyz.shape[0] == h * w - 1
    assert_bitwise(xyz, exp, "unprojected plane")
    assert_bitwise(rgb, color[ii, jj].astype(np.float64) / 255.0, "colors")


def test_voxel_down_sample_lattice_kat(O):
    g = np.arange(10) * 0.01 + 0.0025
    P = np.stack(np.meshgrid(g, g, g, indexing="ij"), -1).reshape(-1, 3)
    C = np.tile([[0.2, 0.4, 0.6]], (P.shape[0], 1))
    v, c, k, _ = O.voxel_down_sample(P, C, 0.02)
    # vmin = min - 0.01 = -0.0075 -> points fall 2 per axis per voxel, except the first voxel holds 1 per axis
    assert v.shape[0] == 6 ** 3
    counts = {}
    for p in P:
        key = tuple(np.floor((p - (P.min(0) - 0.01)) / 0.02).astype(int))
        counts[key] = counts.get(key, 0) + 1
    assert sorted(counts) == [tuple(x) for x in k]
    np.testing.assert_allclose(c, 0.2 * np.array([1, 2, 3])[None, :] * np.ones_like(c), rtol=1e-15)
    with pytest.raises(RuntimeError):
        O.voxel_down_sample(P, C, 0.0)


def test_tsdf_single_wall_kat(O):
    """One frame of a fronto-parallel wall at 1.0 m, identity extrinsic, 1 cm voxels: every observed voxel
    has weight 1 and tsdf = min(1, (d - zc) * m / trunc) in float32 with Open3D's operation order."""
    w, h, fx, fy, cx, cy = 64, 48, 60.0, 60.0, 31.5, 23.5
    depth = np.full((h, w), 1.0, np.float32)
    color = np.full((h, w, 3), 100, np.uint8)
    vol = O.TSDF(0.01, 0.04, 1, 4)
    vol.integrate(depth, color, (w, h, fx, fy, cx, cy), np.eye(4))
    keys, tsdf, weight, col = vol.export()
    assert keys.shape[0] > 0
    obs = weight > 0
    assert set(np.unique(weight)) <= {0.0, 1.0}
    # recompute a voxel on the optical axis: unit containing (0, 0, 1.0)
    for kk, ts in zip(keys, tsdf):
        if tuple(kk) != (0, 0, 6):  # 1.0 m / 0.16 m = 6.25 -> unit 6 holds z in [0.96, 1.12)
            continue
        vl = np.float32(0.01)
        half = vl * np.float32(0.5)
        oz = np.float32(6 * 0.16)
        for z in range(16):
            # x = y = 0 column: pc = (half + 0 + 0, ..., half + oz) then += vl per z step
            pz = np.float32(half + oz)
            for _ in range(z):
                pz = np.float32(pz + vl)
            u = int(np.float32(np.float32(np.float32(half) * np.float32(fx)) / pz + np.float32(cx)) + np.float32(0.5))
            v = u if False else int(np.float32(np.float32(np.float32(half) * np.float32(fy)) / pz + np.float32(cy)) + np.float32(0.5))
            xx = (np.float32(u) - np.float32(cx)) * (np.float32(1) / np.float32(fx))
            yy = (np.float32(v) - np.float32(cy)) * (np.float32(1) / np.float32(fy))
            m = np.sqrt(np.float32(xx * xx + yy * yy) + np.float32(1))
            sdf = np.float32((np.float32(1.0) - pz) * m)
            if sdf > -np.float32(0.04):
                exp = min(np.float32(1.0), np.float32(sdf * (np.float32(1) / np.float32(0.04))))
                assert ts[z] == exp, (z, ts[z], exp)
            else:
                assert ts[z] == 0.0
        break
    else:
        raise AssertionError("unit (0,0,6) not allocated")
    np.testing.assert_allclose(col[obs], 100.0)


def test_tsdf_repeat_frames_weight(O):
    w, h, fx, fy, cx, cy = 64, 48, 60.0, 60.0, 31.5, 23.5
    depth = np.full((h, w), 1.0, np.float32)
    color = np.full((h, w, 3), 50, np.uint8)
    vol = O.TSDF(0.01, 0.04, 1, 4)
    for _ in range(5):
        vol.integrate(depth, color, (w, h, fx, fy, cx, cy), np.eye(4))
    _, tsdf, weight, col = vol.export()
    assert set(np.unique(weight)) <= {0.0, 5.0}
    one = O.TSDF(0.01, 0.04, 1, 4)
    one.integrate(depth, color, (w, h, fx, fy, cx, cy), np.eye(4))
    _, t1, _, _ = one.export()
    np.testing.assert_allclose(tsdf, t1, rtol=0, atol=1e-6)
    np.testing.assert_allclose(col[weight > 0], 50.0, rtol=1e-12)


def test_mesh_of_wall_lies_on_wall(O):
    w, h, fx, fy, cx, cy = 96, 72, 80.0, 80.0, 47.5, 35.5
    depth = np.full((h, w), 1.2, np.float32)
    color = np.full((h, w, 3), 200, np.uint8)
    vol = O.TSDF(0.01, 0.04, 1, 4)
    for _ in range(2):
        vol.integrate(depth, color, (w, h, fx, fy, cx, cy), np.eye(4))
    V, VC, T = vol.extract_triangle_mesh()
    assert V.shape[0] > 100 and T.shape[0] > 100
    # near the optical axis the zero crossing is at z = 1.2 / m(u,v) ~ 1.2
    axis = (np.abs(V[:, 0]) < 0.05) & (np.abs(V[:, 1]) < 0.05)
    assert axis.any()
    np.testing.assert_allclose(V[axis, 2], 1.2, atol=2e-3)
    np.testing.assert_allclose(VC, 200.0 / 255.0, rtol=1e-12)
    assert T.min() >= 0 and T.max() < V.shape[0]


def _brute_knn_mean(P, k):
    d2 = ((P[:, None, :] - P[None, :, :]) ** 2).sum(-1)
    d2.sort(axis=1)
    return np.sqrt(d2[:, :k]).mean(axis=1)


def test_sor_ror_vs_bruteforce(O):
    rng = np.random.default_rng(3)
    P = rng.uniform(0, 1, size=(1500, 3))
    P[:20] = rng.uniform(3, 4, size=(20, 3))  # outliers
    idx, avg = O.remove_statistical_outlier(P, 10, 1.0)
    np.testing.assert_allclose(avg, _brute_knn_mean(P, 10), rtol=1e-12)
    assert not set(range(20)) & set(idx.tolist())
    d2 = ((P[:, None, :] - P[None, :, :]) ** 2).sum(-1)
    for nb, r in ((3, 0.08), (8, 0.12)):
        ridx = O.remove_radius_outlier(P, nb, r)
        assert_bitwise(ridx, np.nonzero((d2 < r * r).sum(1) > nb)[0], "ROR kept")
    with pytest.raises(RuntimeError):
        O.remove_statistical_outlier(P, 0, 1.0)
    with pytest.raises(RuntimeError):
        O.remove_radius_outlier(P, 1, 0.0)


def test_sampling_kat(O):
    V = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [1, 1, 0]], np.float64)
    T = np.array([[0, 1, 2], [1, 3, 2]], np.int32)
    P, _, _ = O.sample_points_uniformly(V, T, 1000, seed=7)
    assert P.shape == (1000, 3)
    assert (P[:, 2] == 0).all() and (P[:, :2] >= 0).all() and (P[:, :2] <= 1).all()
    P2, _, _ = O.sample_points_uniformly(V, T, 1000, seed=7)
    assert_bitwise(P, P2, "seeded sampling")
    # equal areas -> 500 points per triangle; first 500 in triangle 0 (x + y <= 1)
    assert (P[:500].sum(1) <= 1 + 1e-12).all()


def test_occupancy_kat(O):
    img = np.full((4, 5), 254, np.uint8)
    img[0, 1] = 0
    img[3, 4] = 99
    img[2, 2] = 100  # not occupied (threshold is strict)
    pts = O.occupancy_to_points(img, 100, 0.05, -1.0, -2.0)
    exp = np.array([[-1.0 + 1 * 0.05, -2.0 + 3 * 0.05, 0.0], [-1.0 + 4 * 0.05, -2.0 + 0 * 0.05, 0.0]])
    assert_bitwise(pts, exp, "occupancy points")


def test_point_cloud_distance_kat(O):
    """Oracle 1-NN distance == numpy brute force; empty target -> zeros (Open3D: no neighbour found)."""
    rng = np.random.default_rng(5)
    a, b = rng.normal(size=(300, 3)), rng.normal(size=(200, 3))
    d = O.point_cloud_distance(a, b)
    diff = a[:, None, :] - b[None, :, :]
    ref = np.sqrt(((diff[..., 0] * diff[..., 0] + diff[..., 1] * diff[..., 1]) + diff[..., 2] * diff[..., 2]).min(1))
    assert np.array_equal(d, ref)
    assert not np.any(O.point_cloud_distance(a, np.zeros((0, 3))))


def test_smart_paste_kat(O):
    """2d_selective_merge.py:58-69 on a hand-checked grid: only values outside [200, 210] are pasted."""
    base = np.full((3, 4), 7, np.uint8)
    over = np.array([[0, 200, 205, 210], [211, 254, 199, 100], [1, 2, 3, 4]], np.uint8)
    out = O.smart_paste(base, over, 0, 0, 4, 2)
    assert out.tolist() == [[0, 7, 7, 7], [211, 254, 199, 100], [7, 7, 7, 7]]
    assert np.array_equal(O.smart_paste(base, over, 2, 0, 3, 1), base)  # rectangle leaves the image


def test_scan_diff_and_grid_kat(O):
    """Identical scans flag nothing; a return 1 m beyond the wall is 'new' and its wall beam 'gone'; the grid
    publishes a cell only after its evidence exceeds time_threshold."""
    n = 90
    amin, ainc = np.float32(-np.pi / 4), np.float32(np.pi / 2 / 90)
    virt = np.full((1, n), 3.0, np.float32)
    pose = np.array([[0, 0, 0, 0, 0, 0, 1.0]])
    nf, gf, _, _ = O.scan_diff(virt, virt, float(amin), float(ainc), 10.0, float(amin), float(ainc), 0.5, 20, pose, 0.1)
    assert nf.sum() == 0 and gf.sum() == 0
    real = virt.copy()
    real[0, 45] = 4.0
    nf, gf, nk, gk = O.scan_diff(real, virt, float(amin), float(ainc), 10.0, float(amin), float(ainc), 0.5, 20, pose,
                                 0.1)
    assert nf[0].nonzero()[0].tolist() == [45] and gf.sum() == 0
    a = amin + np.float32(45) * ainc
    assert nk[0, 45].tolist() == [int(np.float64(np.float32(4.0) * np.float32(np.cos(a))) / 0.1),
                                  int(np.float64(np.float32(4.0) * np.float32(np.sin(a))) / 0.1)]
    keys = np.repeat(nk, 3, axis=0)
    flags = np.repeat(nf, 3, axis=0)
    assert len(O.change_grid_run(keys[:1], flags[:1], [1.0], 2.0, 0.5, 0.1)) == 0   # 1.0 <= 2.0
    assert len(O.change_grid_run(keys, flags, [1.0, 1.0, 1.0], 2.0, 0.5, 0.1)) == 1  # capped 3.0 > 2.0


def test_virtual_scan_kat(O):
    """A wall 1 m east of the robot on a 0.1 m grid: the eastward beam stops at the first step whose cell is the wall."""
    g = np.zeros((20, 20), np.int8)
    g[:, 15] = 100  # cells x in [1.5, 1.6) with origin 0
    r = O.virtual_scan(g, 0.1, 0.0, 0.0, 4, 0.0, float(np.float32(np.pi / 2)), 10.0, np.array([[0.55, 1.05, 0.0]]))
    d = 0.0
    while True:
        d += np.float64(np.float32(0.1))
        if int((0.55 + d - 0.0) / np.float64(np.float32(0.1))) >= 15:
            break
    assert r[0, 0] == np.float32(d)
    assert np.isinf(r[0, 2])  # westward beam leaves the map


def test_oracle_surface_area_is_index_order_sum(O):
    """oro_mesh_surface_area (Open3D GetSurfaceArea) == numpy areas summed strictly left to right."""
    rng = np.random.default_rng(11)
    V = rng.random((400, 3))
    T = rng.integers(0, 400, (5000, 3)).astype(np.int32)
    x = V[T[:, 0]] - V[T[:, 1]]
    y = V[T[:, 0]] - V[T[:, 2]]
    c = np.stack([x[:, 1] * y[:, 2] - x[:, 2] * y[:, 1], x[:, 2] * y[:, 0] - x[:, 0] * y[:, 2],
                  x[:, 0] * y[:, 1] - x[:, 1] * y[:, 0]], 1)
    a = 0.5 * np.sqrt((c[:, 0] * c[:, 0] + c[:, 1] * c[:, 1]) + c[:, 2] * c[:, 2])
    assert O.surface_area(V, T) == np.cumsum(a)[-1]
