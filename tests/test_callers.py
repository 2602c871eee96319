"""Caller parity (CPU): this repo's restated callers (object-triggered-3d-slam_amd/reconstruct.py) make the same
Open3D-API call sequence, with the same arguments, frame order, extrinsic matrices (bitwise), error/skip
behaviour and written Z-filtered clouds (sha256 of the float64 bytes), as the reference scripts themselves.
The expected logs in tests/golden/caller_fixture.json were captured by EXECUTING the reference scripts against
the same recording stub (tests/golden/gen_caller_fixture.py)."""
import importlib
import json
import os
import sys

import numpy as np
import pytest

from conftest import PKG, ROOT

sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import dataset  # noqa: E402
import recorder  # noqa: E402

FIXTURE = json.load(open(os.path.join(ROOT, "tests", "golden", "caller_fixture.json")))["calls"]


@pytest.fixture(scope="module")
def R():
    return importlib.import_module(PKG + ".reconstruct")


def _split(calls):
    intr = [c["args"] for c in calls if c["call"] == "PinholeCameraIntrinsic"]
    rest = [c for c in recorder.core(calls) if c["call"] != "PinholeCameraIntrinsic"]
    return intr, rest


def _run(tmp_path, fn):
    root = str(tmp_path)
    dataset.write_scan_dataset(root)
    rec = recorder.Recorder(root)
    stub = recorder.make_open3d(rec)
    try:
        fn(root, stub)
    except Exception as exc:
        rec.log("exception", type=type(exc).__name__)
    return rec.calls


def _check(ours, name):
    ref_intr, ref_rest = _split(FIXTURE[name])
    our_intr, our_rest = _split(ours)
    assert set(map(tuple, our_intr)) == set(map(tuple, ref_intr))
    assert [c["call"] for c in our_rest] == [c["call"] for c in ref_rest]
    for a, b in zip(our_rest, ref_rest):
        assert a == b, f"{name}: {a['call']} differs"
    ref_exc = [c for c in FIXTURE[name] if c["call"] == "exception"]
    assert [c for c in ours if c["call"] == "exception"] == ref_exc


def test_reconstruct_rgbd_filter(R, tmp_path):
    calls = _run(tmp_path, lambda root, o3d: R.run_all(R.ScanConfig(base_dir=root), o3d=o3d, output="points"))
    _check(calls, "reconstruct_rgbd_filter")
    order = [c["color"] for c in calls if c["call"] == "integrate"]
    assert order[:4] == ["color/Object_0_1.jpg", "color/Object_0_10.jpg", "color/Object_0_11.jpg",
                         "color/Object_0_2.jpg"]  # lexical, not numeric (reconstruct_rgbd_filter.py:68-70)


def test_reconstruct_rgbd_mesh(R, tmp_path):
    calls = _run(tmp_path, lambda root, o3d: R.run_all(R.ScanConfig(base_dir=root), o3d=o3d, output="mesh"))
    _check(calls, "reconstruct_rgbd")
    assert calls[-1] == {"call": "exception", "type": "IndexError"}  # no try/except in reconstruct_rgbd.py


def test_reconstruct_range(R, tmp_path):
    calls = _run(tmp_path, lambda root, o3d: R.reconstruct_range("object_0", 1, 16, R.ScanConfig(base_dir=root),
                                                                 file_prefix="Object_0", o3d=o3d))
    _check(calls, "multi_reconstruct_rgbd_filter")
    order = [c["color"] for c in calls if c["call"] == "integrate"]
    assert order == [f"color/Object_0_{i}.jpg" for i in range(1, 12)]  # numeric order, 12..16 missing


def test_reconstruct_gt(R, tmp_path):
    calls = _run(tmp_path, lambda root, o3d: R.reconstruct_gt(R.ScanConfig(base_dir=root), o3d=o3d))
    _check(calls, "reconstruct_rgbd_gt")


def test_check_one_frame(R, tmp_path):
    """check_one_frame.py's recorded sequence (intrinsic, two image reads, depth_trunc 5.0 RGBD,
    create_from_rgbd_image, voxel_down_sample(0.01), draw_geometries) made by the restated caller, call for call and
    argument for argument."""
    calls = _run(tmp_path, lambda root, o3d: R.check_one_frame(root, o3d=o3d))
    _check(calls, "check_one_frame")
    assert [c["call"] for c in calls][-2:] == ["voxel_down_sample", "draw_geometries"]


def test_extrinsics_are_inverse_of_pose_times_tfix(R, tmp_path):
    calls = _run(tmp_path, lambda root, o3d: R.run_all(R.ScanConfig(base_dir=root), o3d=o3d))
    first = next(c for c in calls if c["call"] == "integrate")
    pose = np.loadtxt(os.path.join(str(tmp_path), "poses", "Object_0_1.txt"))
    T_fix = np.array([[0, -1, 0, 0], [0, 0, -1, 0], [1, 0, 0, 0], [0, 0, 0, 1]], dtype=float)
    assert np.array_equal(np.array(first["extrinsic"]), np.linalg.inv(pose @ T_fix))


def test_hybrid_map_fixture_shape():
    """The reference's create_map_cloud + merge, recorded on the map dataset: map points first (row-major
    occupied pixels), then the objects in sorted file order; pinned bitwise in tests/test_gpu_hybrid.py."""
    calls = FIXTURE["hybrid_map"]
    w = next(c for c in calls if c["call"] == "write_point_cloud")
    reads = [c["path"] for c in calls if c["call"] == "read_point_cloud"]
    assert reads == ["objects/Object_0.ply", "objects/Object_1.ply"]
    assert w["n"] == len(w["points"]) > 12
