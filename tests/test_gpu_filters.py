"""GPU parity: voxel_down_sample, remove_statistical_outlier, remove_radius_outlier, Z-mask, occupancy points.

Bit-exact: voxel key set, per-voxel averaged xyz/colour (sums in index order), ROR kept indices, Z-mask
compaction, occupancy points, SOR mean kNN distances and kept indices.  The SOR cloud mean and squared-deviation
sum are Open3D's sequential float64 accumulations (exact chains on the GPU): test_sor_threshold_exact puts points
exactly ON the threshold, where any other summation order moves the kept set.
"""
import ctypes as C

import numpy as np
import pytest
import torch

from conftest import assert_bitwise, ref_intr

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def frame_cloud(pkg, O, synth, seq16, gpu):
    depth, color, ext = seq16
    intr_t = ref_intr(synth)
    df = O.depth_to_float(depth[0], 1000.0, 5.0)
    xyz, rgb = O.unproject(df, color[0], intr_t, ext[0])
    return xyz, rgb


def _pcd(pkg, xyz, rgb=None):
    p = pkg.geometry.PointCloud()
    p.points = pkg.utility.Vector3dVector(xyz)
    if rgb is not None:
        p.colors = pkg.utility.Vector3dVector(rgb)
    return p


@pytest.mark.parametrize("vs", [0.005, 0.01, 0.037])
def test_voxel_down_sample_bitexact(pkg, O, frame_cloud, vs):
    xyz, rgb = frame_cloud
    ds = _pcd(pkg, xyz, rgb).voxel_down_sample(vs)
    rv, rc, rk, _ = O.voxel_down_sample(xyz, rgb, vs)
    assert len(ds.points) == rv.shape[0]
    assert_bitwise(np.asarray(ds.points), rv, "voxel averages")
    assert_bitwise(np.asarray(ds.colors), rc, "voxel colours")


def test_voxel_down_sample_keys_and_edges(pkg, O, gpu):
    L = pkg._lib
    rng = np.random.default_rng(5)
    xyz = rng.uniform(-3, 3, size=(20000, 3))
    xyz[:100] = xyz[100:200]  # duplicates
    d = torch.from_numpy(xyz).cuda()
    ox = torch.empty_like(d)
    ok = torch.empty((xyz.shape[0], 3), dtype=torch.int32, device="cuda")
    n = C.c_int64(0)
    L.call("ot_voxel_down_sample", C.c_void_p(d.data_ptr()), None, None, xyz.shape[0], 0.05,
           C.c_void_p(ox.data_ptr()), None, None, C.c_void_p(ok.data_ptr()), C.byref(n), None)
    rv, _, rk, _ = O.voxel_down_sample(xyz, None, 0.05)
    assert n.value == rv.shape[0]
    assert_bitwise(ok[:n.value].cpu().numpy(), rk, "voxel keys")
    assert_bitwise(ox[:n.value].cpu().numpy(), rv, "voxel averages")
    # single point, empty, invalid size
    one = _pcd(pkg, xyz[:1]).voxel_down_sample(0.1)
    assert_bitwise(np.asarray(one.points), xyz[:1], "single point")
    assert len(_pcd(pkg, np.zeros((0, 3))).voxel_down_sample(0.1).points) == 0
    with pytest.raises(RuntimeError, match="voxel_size"):
        _pcd(pkg, xyz).voxel_down_sample(0.0)


def test_ror_bitexact(pkg, O, frame_cloud):
    xyz, rgb = frame_cloud
    ds = O.voxel_down_sample(xyz, rgb, 0.01)[0]
    for nb, r in ((16, 0.05), (4, 0.02)):
        out, idx = _pcd(pkg, ds).remove_radius_outlier(nb, r)
        ridx = O.remove_radius_outlier(ds, nb, r)
        assert_bitwise(np.asarray(idx, np.int64), ridx, f"ROR({nb},{r}) kept")
        assert_bitwise(np.asarray(out.points), ds[ridx], "ROR points")


@pytest.mark.parametrize("k,ratio", [(20, 2.0), (8, 1.0), (48, 0.5)])
def test_sor_bitexact(pkg, O, frame_cloud, k, ratio):
    xyz, rgb = frame_cloud
    ds = O.voxel_down_sample(xyz, rgb, 0.01)[0]
    rng = np.random.default_rng(1)
    ds = np.concatenate([ds, rng.uniform(-2, 2, size=(50, 3))])  # isolated outliers
    L = pkg._lib
    d = torch.from_numpy(ds).cuda()
    idx = torch.empty(ds.shape[0], dtype=torch.int64, device="cuda")
    avg = torch.empty(ds.shape[0], dtype=torch.float64, device="cuda")
    n = C.c_int64(0)
    L.call("ot_remove_statistical_outlier", C.c_void_p(d.data_ptr()), ds.shape[0], k, ratio,
           C.c_void_p(idx.data_ptr()), C.c_void_p(avg.data_ptr()), C.byref(n), None)
    ridx, ravg = O.remove_statistical_outlier(ds, k, ratio)
    assert_bitwise(avg.cpu().numpy(), ravg, "SOR mean kNN distance")
    assert_bitwise(idx[:n.value].cpu().numpy(), ridx, "SOR kept indices")
    assert not set(range(ds.shape[0] - 50, ds.shape[0])) <= set(ridx.tolist())


@pytest.mark.parametrize("k", [20, 64])
def test_sor_sparse_tail(pkg, O, frame_cloud, k):
    """Stage 3 of the SOR kNN (one wave per query, rings split over the lanes, lists merged per ring): points whose
    k-th neighbour lies beyond their 5x5x5 cell block -- isolated points at geometric distances (5 cm .. 20 m) from
    the surface, clusters of fewer than k points, a far sparse line; k = 64 also merges 64-entry lists."""
    xyz, rgb = frame_cloud
    ds = O.voxel_down_sample(xyz, rgb, 0.01)[0]
    rng = np.random.default_rng(7)
    c = ds.mean(0)
    dirs = rng.normal(size=(300, 3))
    dirs /= np.linalg.norm(dirs, axis=1, keepdims=True)
    iso = c + dirs * np.geomspace(0.05, 20.0, 300)[:, None]
    clusters = [c + rng.uniform(-3, 3, 3) + rng.normal(scale=0.01, size=(m, 3)) for m in rng.integers(2, 16, 30)]
    line = c + np.array([5.0, 0.0, 0.0]) + np.linspace(0.0, 1.0, 40)[:, None] * np.array([0.0, 0.0, 1.0])
    pts = np.ascontiguousarray(np.concatenate([ds, iso] + clusters + [line]))
    idx, avg = _sor_gpu(pkg, pts, k, 1.0)
    ridx, ravg = O.remove_statistical_outlier(pts, k, 1.0)
    assert_bitwise(avg, ravg, f"SOR({k}) mean kNN distance, sparse tail")
    assert_bitwise(idx, ridx, f"SOR({k}) kept indices, sparse tail")


def _sor_gpu(pkg, pts, k, ratio):
    L = pkg._lib
    d = torch.from_numpy(np.ascontiguousarray(pts)).cuda()
    idx = torch.empty(pts.shape[0], dtype=torch.int64, device="cuda")
    avg = torch.empty(pts.shape[0], dtype=torch.float64, device="cuda")
    n = C.c_int64(0)
    L.call("ot_remove_statistical_outlier", C.c_void_p(d.data_ptr()), pts.shape[0], k, ratio,
           C.c_void_p(idx.data_ptr()), C.c_void_p(avg.data_ptr()), C.byref(n), None)
    return idx[:n.value].cpu().numpy(), avg.cpu().numpy()


def _seq_stats(avg):
    """RemoveStatisticalOutliers' cloud statistics in Open3D's order (std::accumulate / std::inner_product)."""
    valid = int((avg >= 0).sum())
    s = 0.0
    for a in avg.tolist():
        s = s + a if a > 0 else s
    mean = s / valid
    q = 0.0
    for a in avg.tolist():
        q = q + ((a - mean) * (a - mean) if a > 0 else 0.0)
    return mean, float(np.sqrt(q / (valid - 1)))


def test_sor_threshold_exact(pkg, O, gpu):
    """Points exactly ON the threshold: k = 2 on isolated pairs makes every mean kNN distance an exact dyadic
    s_j / 2; std_ratio is solved so that mean + ratio * std == one pair's distance bit for bit.  That pair must be
    dropped (strict <) and the pairs one step below kept.  The values span 2^20 in magnitude, so a pairwise or tree
    summation gives a different mean / std than Open3D's sequential one (asserted) — only the exact sequential
    chains reproduce the kept set."""
    for seed in range(64):
        rng = np.random.default_rng(seed)
        m = 12 ** 3  # pairs on a 12^3 lattice of spacing 10 (the partner is every point's only close neighbour)
        s = rng.integers(1, 1 << 20, size=m).astype(np.float64) * 2.0 ** -24
        p0 = np.stack(np.meshgrid(*([np.arange(12, dtype=np.float64) * 10.0] * 3), indexing="ij"), -1).reshape(-1, 3)
        p1 = p0 + np.stack([s, np.zeros(m), np.zeros(m)], 1)
        pts = np.stack([p0, p1], 1).reshape(-1, 3)
        avg = np.repeat(s / 2.0, 2)
        mean, sd = _seq_stats(avg)
        if np.sum(avg) / avg.size == mean and np.sqrt(np.sum((avg - mean) ** 2) / (avg.size - 1)) == sd:
            continue  # pairwise summation happens to agree: not adversarial
        t = float(np.quantile(avg, 0.9, method="higher"))
        r = (t - mean) / sd
        for _ in range(4000):
            thr = mean + r * sd
            if thr == t:
                break
            r = np.nextafter(r, np.inf if thr < t else -np.inf)
        if mean + r * sd != t:
            continue
        ridx, ravg = O.remove_statistical_outlier(pts, 2, float(r))
        assert_bitwise(ravg, avg, "oracle mean distances of the pair cloud")
        gidx, gavg = _sor_gpu(pkg, pts, 2, float(r))
        assert_bitwise(gavg, avg, "SOR mean distances (pairs)")
        on = np.nonzero(avg == t)[0]
        assert on.size >= 2 and not set(on.tolist()) & set(ridx.tolist()), "points on the threshold are dropped"
        assert_bitwise(gidx, ridx, "SOR kept indices at the exact threshold")
        return
    pytest.fail("no adversarial configuration found")


def test_sor_coincident_points(pkg, O, frame_cloud):
    """More than k coincident points: their mean kNN distance is 0 — counted in `valid` but not summed (Open3D's
    valid_distances vs the accumulate's avg > 0 lambda); they are never kept."""
    xyz, rgb = frame_cloud
    ds = O.voxel_down_sample(xyz, rgb, 0.01)[0]
    dup = np.concatenate([ds, np.repeat(ds[:1], 30, 0), np.repeat(ds[500:501], 25, 0)])
    for k, ratio in ((20, 2.0), (8, 0.7)):
        ridx, ravg = O.remove_statistical_outlier(dup, k, ratio)
        gidx, gavg = _sor_gpu(pkg, dup, k, ratio)
        assert (ravg == 0).sum() >= 55
        assert_bitwise(gavg, ravg, f"SOR mean distances with coincident points (k={k})")
        assert_bitwise(gidx, ridx, f"SOR kept with coincident points (k={k})")


def test_sor_small_and_errors(pkg, O, gpu):
    pts = np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [0, 0, 5.0]])
    out, idx = _pcd(pkg, pts).remove_statistical_outlier(10, 1.0)  # k > n: every point sees all 4
    ridx, _ = O.remove_statistical_outlier(pts, 10, 1.0)
    assert idx == ridx.tolist()
    with pytest.raises(RuntimeError, match="Illegal input"):
        _pcd(pkg, pts).remove_statistical_outlier(0, 1.0)
    with pytest.raises(RuntimeError, match="Illegal input"):
        _pcd(pkg, pts).remove_radius_outlier(2, -1.0)
    e, ei = _pcd(pkg, np.zeros((0, 3))).remove_statistical_outlier(5, 1.0)
    assert len(e.points) == 0 and ei == []


def test_filter_min_z_bitexact(pkg, O, frame_cloud):
    xyz, rgb = frame_cloud
    out = _pcd(pkg, xyz, rgb).filter_min_z(0.03)
    rx, rc = O.filter_min_z(xyz, rgb, 0.03)
    assert_bitwise(np.asarray(out.points), rx, "z-mask xyz")
    assert_bitwise(np.asarray(out.colors), rc, "z-mask rgb")
    mask = xyz[:, 2] >= 0.03  # reconstruct_rgbd_filter.py:128
    assert_bitwise(rx, xyz[mask], "numpy boolean mask")


def test_occupancy_points_bitexact(pkg, O, gpu):
    rng = np.random.default_rng(2)
    img = rng.integers(0, 256, size=(333, 517), dtype=np.uint8)
    L = pkg._lib
    d = torch.from_numpy(img).cuda()
    out = torch.empty((img.size, 3), dtype=torch.float64, device="cuda")
    n = C.c_int64(0)
    L.call("ot_occupancy_to_points", C.c_void_p(d.data_ptr()), img.shape[0], img.shape[1], 100, 0.05, -12.5, -7.25,
           C.c_void_p(out.data_ptr()), C.byref(n), None)
    ref = O.occupancy_to_points(img, 100, 0.05, -12.5, -7.25)
    assert_bitwise(out[:n.value].cpu().numpy(), ref, "occupancy points")


@pytest.fixture(scope="module")
def hd_voxels(O, synth, gpu):
    """configs[2] shape: one 1280x720 frame, unprojected (depth_trunc 5 m) and 5 mm voxel-downsampled."""
    depth, color, ext = synth.make_sequence(n_frames=16, intr=synth.REF_INTRINSICS_1280, frames=[5])
    df = O.depth_to_float(depth[0], 1000.0, 5.0)
    xyz, rgb = O.unproject(df, color[0], synth.REF_INTRINSICS_1280, ext[0])
    return O.voxel_down_sample(xyz, rgb, 0.005)[0]


@pytest.mark.parametrize("netfill", [1, 0])
def test_sor_bench_scale_bitexact(pkg, O, hd_voxels, netfill):
    """The bench's SOR(20, 2.0) on ~270k voxels: mean kNN distances and kept indices bit-exact -- with stage 1's list
    filled by the sorting network (the default) and by sequential insertion (otx_sor_netfill(0))."""
    ds = hd_voxels
    L = pkg._lib
    L.call("otx_sor_netfill", netfill)
    d = torch.from_numpy(ds).cuda()
    idx = torch.empty(ds.shape[0], dtype=torch.int64, device="cuda")
    avg = torch.empty(ds.shape[0], dtype=torch.float64, device="cuda")
    n = C.c_int64(0)
    L.call("ot_remove_statistical_outlier", C.c_void_p(d.data_ptr()), ds.shape[0], 20, 2.0,
           C.c_void_p(idx.data_ptr()), C.c_void_p(avg.data_ptr()), C.byref(n), None)
    L.call("otx_sor_netfill", 1)
    ridx, ravg = O.remove_statistical_outlier(ds, 20, 2.0)
    assert_bitwise(avg.cpu().numpy(), ravg, "SOR mean kNN distance (bench scale)")
    assert_bitwise(idx[:n.value].cpu().numpy(), ridx, "SOR kept indices (bench scale)")


def test_ror_bench_scale_bitexact(pkg, O, hd_voxels):
    ds = hd_voxels
    out, idx = _pcd(pkg, ds).remove_radius_outlier(16, 0.02)
    ridx = O.remove_radius_outlier(ds, 16, 0.02)
    assert_bitwise(np.asarray(idx, np.int64), ridx, "ROR kept (bench scale)")


def test_concurrent_streams_match_serial(pkg, O, synth, seq16, gpu):
    """Different host threads on their own HIP streams (per-thread scratch) give the serial results bit for bit:
    voxel_down_sample -> remove_statistical_outlier -> remove_radius_outlier on 4 clouds, 4 threads at once."""
    from concurrent.futures import ThreadPoolExecutor

    depth, color, ext = seq16
    intr_t = ref_intr(synth)
    clouds = [O.unproject(O.depth_to_float(depth[f], 1000.0, 5.0), color[f], intr_t, ext[f]) for f in range(4)]

    def chain(xyz, rgb):
        ds = _pcd(pkg, xyz, rgb).voxel_down_sample(0.005)
        _, sor = ds.remove_statistical_outlier(20, 2.0)
        _, ror = ds.remove_radius_outlier(16, 0.02)
        return np.asarray(ds.points), np.asarray(sor), np.asarray(ror)

    serial = [chain(*c) for c in clouds]

    def threaded(i):
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            out = [chain(*clouds[i]) for _ in range(3)]
            s.synchronize()
        return out

    with ThreadPoolExecutor(max_workers=4) as ex:
        results = list(ex.map(threaded, range(4)))
    for i in range(4):
        for rep in results[i]:
            for got, exp, what in zip(rep, serial[i], ("voxels", "SOR kept", "ROR kept")):
                assert_bitwise(got, exp, f"concurrent {what} (cloud {i})")
