"""End-to-end drop-in path on the GPU: the restated reference caller (reconstruct_object, the body of
reconstruct_rgbd_filter.py) reads a dataset written in the reference's on-disk layout, runs every stage on the
MI355X facade and writes the Z-filtered PLY; the same decoded inputs through the CPU oracle give the same
points bit for bit.  Also the single-rank RCCL merge driver (configs[3]/[4] code path)."""
import importlib
import os
import socket

import numpy as np
import pytest

from conftest import PKG, assert_bitwise

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def scan_dir(tmp_path_factory, synth):
    root = str(tmp_path_factory.mktemp("scan"))
    for obj in (0, 1):
        scene = synth.object_scene(obj) if obj else synth.Scene()
        n = 10
        depth, color, _ = synth.make_sequence(scene, n_frames=n)
        synth.write_dataset(root, f"Object_{obj}", depth, color, synth.ros_poses(scene, n))
    return root


def _oracle_object(O, synth, root, label, cfg):
    import glob

    from PIL import Image

    pick = lambda d, e: sorted(glob.glob(os.path.join(root, d, f"{label}_*.{e}")))
    intr_t = synth.REF_INTRINSICS_640
    vol = O.TSDF(cfg.voxel_length, cfg.sdf_trunc, 1, 4)
    for c, d, p in zip(pick("color", "jpg"), pick("depth", "png"), pick("poses", "txt")):
        color = np.array(Image.open(c).convert("RGB"), np.uint8)
        depth = np.array(Image.open(d), np.uint16)
        ext = np.linalg.inv(np.loadtxt(p) @ synth.T_FIX)
        vol.integrate(O.depth_to_float(depth, 1000.0, 3.0), color, intr_t, ext)
    V, VC, T = vol.extract_triangle_mesh()
    P, _, PC = O.sample_points_uniformly(V, T, cfg.n_samples, 0, VC=VC)
    return O.filter_min_z(P, PC, cfg.z_filter)


def test_reconstruct_object_end_to_end(pkg, O, synth, gpu, scan_dir):
    R = importlib.import_module(PKG + ".reconstruct")
    cfg = R.ScanConfig(base_dir=scan_dir)
    assert R.get_unique_object_names(cfg) == ["Object_0", "Object_1"]
    out = R.reconstruct_object("Object_0", cfg)
    assert out.endswith("Object_0.ply")
    got = pkg.io.read_point_cloud(out)
    rx, rc = _oracle_object(O, synth, scan_dir, "Object_0", cfg)
    assert 1000 < len(got.points) < cfg.n_samples
    assert_bitwise(np.asarray(got.points), rx, "reconstructed points (PLY float64)")
    c8 = np.asarray(got.colors) * 255.0  # float64 colour state: the PLY's uchar colours equal the oracle's exactly
    assert np.array_equal(c8, np.round(np.clip(rc, 0, 1) * 255.0))


def test_merge_driver_single_rank(pkg, O, synth, gpu, scan_dir, tmp_path):
    import torch
    import torch.distributed as dist

    D = importlib.import_module(PKG + ".distributed")
    R = importlib.import_module(PKG + ".reconstruct")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        cfg = R.ScanConfig(base_dir=scan_dir)
        pts = D.reconstruct_and_merge(cfg, save_path=str(tmp_path / "merged.ply"), streams=1)
        pts2 = D.reconstruct_and_merge(cfg, streams=2)  # objects on two concurrent host threads / streams
    finally:
        dist.destroy_process_group()
    parts = [_oracle_object(O, synth, scan_dir, lab, cfg)[0] for lab in ("Object_0", "Object_1")]
    assert_bitwise(pts, np.concatenate(parts), "merged object clouds (sorted object order)")
    assert_bitwise(pts2, pts, "merged object clouds, 2 concurrent streams")
