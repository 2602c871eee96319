"""GPU parity: change detection against a saved map (configs[4]).

* smart_paste (2d_selective_merge.py:58-69): bit-exact grids vs the numpy restatement, including rectangles
  partly outside the image (unchanged) and values at the edges of the unknown band (200, 210 stay unknown).
* scan diff (diff_node.cpp:103-160): per-beam new / gone flags and map cells identical to the oracle's literal
  restatement (float beam geometry, double map transform, C++ truncation), with NaN / inf returns.
* evidence grid (diff_node.cpp:163-222): published added / removed clouds identical after a sequence of scans.
* voxel-key diff of clouds: added / removed lattice keys identical to the numpy set difference.
"""
import numpy as np
import pytest

from conftest import assert_bitwise

pytestmark = pytest.mark.gpu


def test_smart_paste_bitexact(pkg, synth, O, gpu):
    cd = pkg.change_detection
    old, new = synth.occupancy_pair(512, 640, seed=3)
    for rect in ((0, 0, 640, 512), (100, 50, 300, 200), (600, 500, 100, 100), (-1, 0, 10, 10), (5, 7, 1, 1)):
        base = old.copy()
        out = cd.smart_paste(base, new, *rect)
        assert out is base
        assert_bitwise(base, O.smart_paste(old, new, *rect), f"smart_paste {rect}")
    merged, n = cd.merge_maps(old, new)
    ref = O.smart_paste(old, new, 0, 0, 640, 512)
    assert_bitwise(merged, ref, "merge_maps")
    assert n == int((ref != old).sum())
    band = np.array([[199, 200, 205, 210, 211]], np.uint8)
    b = np.zeros_like(band)
    cd.smart_paste(b, band, 0, 0, 5, 1)
    assert b.tolist() == [[199, 0, 0, 0, 211]]


@pytest.fixture(scope="module")
def scans(synth):
    return synth.laser_scan_batch(n_scans=48, n_beams=720, seed=4)


def test_scan_diff_flags_bitexact(pkg, O, scans, gpu):
    real, virt, poses, dts, amin, ainc, rmax = scans
    det = pkg.change_detection.ChangeDetector()
    meta = pkg.change_detection.LaserScan(None, amin, ainc, rmax)
    fn, fg, kn, kg = det.flag_beams(real, virt, meta, meta, poses)
    rn, rg, rkn, rkg = O.scan_diff(real, virt, amin, ainc, rmax, amin, ainc, 0.5, 20, poses, 0.1)
    assert fn.sum() > 100 and fg.sum() > 100  # the added boxes and the removed pillar are seen
    assert_bitwise(fn, rn, "new flags")
    assert_bitwise(fg, rg, "gone flags")
    assert_bitwise(kn, rkn, "new cells")
    assert_bitwise(kg, rkg, "gone cells")


def test_change_grid_published_clouds(pkg, O, scans, gpu):
    real, virt, poses, dts, amin, ainc, rmax = scans
    det = pkg.change_detection.ChangeDetector(time_threshold=0.25, decay_rate=0.5)
    meta = pkg.change_detection.LaserScan(None, amin, ainc, rmax)
    added, removed = det.process(real[:30], virt[:30], meta, meta, poses[:30], dts[:30])
    for b in range(30, 48):  # then scan by scan, as the node's callback
        added, removed = det.scan_callback(pkg.change_detection.LaserScan(real[b], amin, ainc, rmax),
                                           pkg.change_detection.LaserScan(virt[b], amin, ainc, rmax), poses[b], dts[b])
    rn, rg, rkn, rkg = O.scan_diff(real, virt, amin, ainc, rmax, amin, ainc, 0.5, 20, poses, 0.1)
    assert_bitwise(added, O.change_grid_run(rkn, rn, dts, 0.25, 0.5, 0.1), "added cloud")
    assert_bitwise(removed, O.change_grid_run(rkg, rg, dts, 0.25, 0.5, 0.1), "removed cloud")
    assert len(added) > 0 and len(removed) > 0


def test_voxel_key_diff_bitexact(pkg, O, seq16, synth, gpu):
    depth, color, ext = seq16
    intr = synth.REF_INTRINSICS_640
    a = O.unproject(O.depth_to_float(depth[0], 1000.0, 5.0), color[0], intr, ext[0])[0]
    b = O.unproject(O.depth_to_float(depth[1], 1000.0, 5.0), color[1], intr, ext[1])[0]
    origin = np.minimum(a.min(0), b.min(0)) - 0.025
    added, removed = pkg.change_detection.voxel_key_diff(a, b, 0.05, origin)
    ra, rr = O.voxel_key_diff(a, b, 0.05, origin)
    assert len(ra) > 0 and len(rr) > 0
    assert_bitwise(added, ra, "added keys")
    assert_bitwise(removed, rr, "removed keys")
    same_a, same_r = pkg.change_detection.voxel_key_diff(a, a, 0.05, origin)
    assert len(same_a) == 0 and len(same_r) == 0
    e_a, e_r = pkg.change_detection.voxel_key_diff(np.zeros((0, 3)), b, 0.05, origin)
    assert len(e_a) == 0
    assert_bitwise(e_r, rr_all(O, b, origin), "removed keys vs empty cloud")


def rr_all(O, b, origin):
    return O.voxel_key_diff(np.zeros((0, 3)), b, 0.05, origin)[1]


def test_virtual_scan_bitexact(pkg, synth, O, gpu):
    """virtual_scan_node.cpp:245-292: ray-marched ranges from the saved occupancy grid, bit-exact vs the oracle's
    literal restatement, for a batch of robot poses (1440 beams, 10 m range as the node's LiDAR)."""
    cd = pkg.change_detection
    grid, res, origin = synth.room_occupancy(0.05)
    rng = np.random.default_rng(8)
    poses = np.stack([rng.uniform(-4, 4, 24), rng.uniform(-3, 3, 24), rng.uniform(-np.pi, np.pi, 24)], 1)
    tmpl = cd.LaserScan(np.zeros(1440, np.float32), 0.0, float(np.float32(6.28 / 1440)), 10.0)
    got = cd.virtual_scan(grid, res, origin, tmpl, poses)
    ref = O.virtual_scan(grid, res, origin[0], origin[1], 1440, 0.0, float(np.float32(6.28 / 1440)), 10.0, poses)
    assert np.isfinite(ref).mean() > 0.9
    assert_bitwise(got, ref, "virtual scan ranges")
    # robot outside the map: every ray leaves the grid at once
    off = cd.virtual_scan(grid, res, origin, tmpl, [[50.0, 50.0, 0.0]])
    assert np.isinf(off).all()


def test_voxel_key_diff_multi_matches_single(pkg, synth, gpu):
    """voxel_key_diff_multi over several objects == one voxel_key_diff per object (object column + cells)."""
    cd = pkg.change_detection
    new = [synth.object_cloud(i, n_points=20000) for i in range(6)]
    old = [synth.object_cloud(i, n_points=20000, moved=True) for i in range(6)]
    new[4] = np.zeros((0, 3))  # an object missing from the new scan: everything removed
    origin = (-1.0, -1.0, -1.0)
    added, removed = cd.voxel_key_diff_multi(new, old, 0.02, origin)
    ra, rr = [], []
    for j in range(6):
        a, r = cd.voxel_key_diff(new[j], old[j], 0.02, origin)
        ra.append(np.concatenate([np.full((len(a), 1), j, np.int32), a], 1))
        rr.append(np.concatenate([np.full((len(r), 1), j, np.int32), r], 1))
    assert_bitwise(added, np.concatenate(ra), "multi added")
    assert_bitwise(removed, np.concatenate(rr), "multi removed")
    assert (removed[:, 0] == 4).sum() > 0 and (added[:, 0] == 4).sum() == 0
