"""GPU parity at the benchmark's full size (BASELINE.json configs[1]): the 256-frame 640x480 synthetic scan bench.py
times, integrated at 5 mm through the same C-ABI entry point (ot_tsdf_integrate_u16, 64-frame fused batches by default), is
bit-exact against the CPU oracle on every unit key, voxel weight and tsdf value, and the exact voxel-update /
unit-integration counters agree (they are the `roofline` accounting's inputs).  Colours: bit-exact in float64 with
colour precision 64 (Open3D's TSDFVoxel::color_), within 1e-4 with the float32 headline setting.
The oracle takes ~5-10 s with OpenMP here."""
import ctypes as C

import numpy as np
import pytest
import torch

from conftest import assert_bitwise

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def scan(synth):
    return synth.make_sequence(synth.Scene(seed=0), n_frames=256, intr=synth.REF_INTRINSICS_640)


@pytest.fixture(scope="module")
def oracle_volume(O, synth, scan):
    depth, color, ext = scan
    ref = O.TSDF(0.005, 0.04, 1, 4)
    for k in range(256):
        ref.integrate(O.depth_to_float(depth[k], 1000.0, 3.0), color[k], synth.REF_INTRINSICS_640, ext[k])
    return ref.export(), ref.total_updates(), ref.unit_integrations()


@pytest.mark.parametrize("bits", [32, 64, None])
def test_bench_workload_bitexact(pkg, synth, scan, oracle_volume, gpu, bits):
    """bits None: the C ABI default (no set_color_precision call) -- colour precision 64, as the facade."""
    L = pkg._lib
    lib = L.load()
    intr_t = synth.REF_INTRINSICS_640
    W, H = intr_t[0], intr_t[1]
    depth, color, ext = scan
    d16 = torch.from_numpy(depth.view(np.int16)).cuda().view(torch.uint16).contiguous()
    col = torch.from_numpy(color).cuda().contiguous()
    ext = np.ascontiguousarray(ext, dtype=np.float64)
    intr = L.ot_intrinsics(W, H, *intr_t[2:])
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    vol = C.c_void_p()
    L.call("ot_tsdf_create", 0.005, 0.04, L.OT_COLOR_RGB8, 16, 4, 0, C.byref(vol))
    try:
        if bits is not None:
            L.call("ot_tsdf_set_color_precision", vol, bits)
        got = C.c_int32(0)
        L.call("ot_tsdf_get_color_precision", vol, C.byref(got))
        assert got.value == (bits or 64)
        bits = got.value
        npx = W * H
        for k in range(256):
            st = lib.ot_tsdf_integrate_u16(vol, C.c_void_p(d16.data_ptr() + k * npx * 2),
                                           C.c_void_p(col.data_ptr() + k * npx * 3), C.byref(intr),
                                           ext[k].ctypes.data_as(C.c_void_p), 1000.0, 3.0, stream)
            assert st == 0, lib.ot_last_error()
        nu = C.c_int64(0)
        L.call("ot_tsdf_num_units", vol, C.byref(nu), stream)
        keys = torch.empty((nu.value, 3), dtype=torch.int32, device="cuda")
        tsdf = torch.empty((nu.value, 4096), dtype=torch.float32, device="cuda")
        weight = torch.empty((nu.value, 4096), dtype=torch.float32, device="cuda")
        colr = torch.empty((nu.value, 4096, 3), dtype=torch.float32 if bits == 32 else torch.float64, device="cuda")
        L.call("ot_tsdf_export_units", vol, nu.value, C.c_void_p(keys.data_ptr()), C.c_void_p(tsdf.data_ptr()),
               C.c_void_p(weight.data_ptr()), C.c_void_p(colr.data_ptr()) if bits == 32 else None, stream)
        if bits == 64:
            L.call("ot_tsdf_export_color64", vol, nu.value, C.c_void_p(colr.data_ptr()), stream)
        with pytest.raises(RuntimeError, match="capacity"):  # outputs sized from an older unit count
            L.call("ot_tsdf_export_units", vol, nu.value - 1, None, None, None, None, stream)
        upd, units = C.c_int64(0), C.c_int64(0)
        L.call("ot_tsdf_counters", vol, C.byref(upd), C.byref(units), stream)
    finally:
        L.call("ot_tsdf_destroy", vol)
    (rk, rt, rw, rc), r_upd, r_units = oracle_volume
    assert nu.value == rk.shape[0] > 5000
    assert_bitwise(keys.cpu().numpy(), rk, "unit keys (bench workload)")
    assert_bitwise(weight.cpu().numpy(), rw, "voxel weights (bench workload)")
    assert_bitwise(tsdf.cpu().numpy(), rt, "voxel tsdf (bench workload)")
    if bits == 64:
        assert_bitwise(colr.cpu().numpy(), rc, "float64 voxel colours (bench workload)")
    else:
        np.testing.assert_allclose(colr.cpu().numpy(), rc, rtol=1e-4, atol=1e-4 * 255)
    assert upd.value == r_upd
    assert units.value == r_units


def _export64(L, vol, stream):
    nu = C.c_int64(0)
    L.call("ot_tsdf_num_units", vol, C.byref(nu), stream)
    keys = torch.empty((nu.value, 3), dtype=torch.int32, device="cuda")
    tsdf = torch.empty((nu.value, 4096), dtype=torch.float32, device="cuda")
    weight = torch.empty((nu.value, 4096), dtype=torch.float32, device="cuda")
    colr = torch.empty((nu.value, 4096, 3), dtype=torch.float64, device="cuda")
    L.call("ot_tsdf_export_units", vol, nu.value, C.c_void_p(keys.data_ptr()), C.c_void_p(tsdf.data_ptr()),
           C.c_void_p(weight.data_ptr()), None, stream)
    L.call("ot_tsdf_export_color64", vol, nu.value, C.c_void_p(colr.data_ptr()), stream)
    upd, units = C.c_int64(0), C.c_int64(0)
    L.call("ot_tsdf_counters", vol, C.byref(upd), C.byref(units), stream)
    return keys.cpu().numpy(), tsdf.cpu().numpy(), weight.cpu().numpy(), colr.cpu().numpy(), upd.value, units.value


def test_bench_step_after_reset_bitexact(pkg, synth, scan, oracle_volume, gpu):
    """VERDICT r3 'next' 1: the state bench.py times.  Its step() is reset_async + 256 x integrate_u16 + flush into ONE
    volume whose pool still holds the previous step's voxels (fresh units start from zero in registers, not from a
    zeroed pool).  Three steps back to back, exactly as bench.py's step(); the volume after the third is bitwise the
    oracle's (keys, tsdf, weight, float64 colour) and the per-step counters are the oracle's."""
    L = pkg._lib
    lib = L.load()
    intr_t = synth.REF_INTRINSICS_640
    W, H = intr_t[0], intr_t[1]
    depth, color, ext = scan
    d16 = torch.from_numpy(depth.view(np.int16)).cuda().view(torch.uint16).contiguous()
    col = torch.from_numpy(color).cuda().contiguous()
    ext = np.ascontiguousarray(ext, dtype=np.float64)
    intr = L.ot_intrinsics(W, H, *intr_t[2:])
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    npx = W * H
    vol = C.c_void_p()
    L.call("ot_tsdf_create", 0.005, 0.04, L.OT_COLOR_RGB8, 16, 4, 0, C.byref(vol))
    (rk, rt, rw, rc), r_upd, r_units = oracle_volume
    try:
        L.call("ot_tsdf_set_color_precision", vol, 64)

        def step():  # bench.py main().step()
            L.call("ot_tsdf_reset_async", vol, stream)
            for k in range(256):
                st = lib.ot_tsdf_integrate_u16(vol, C.c_void_p(d16.data_ptr() + k * npx * 2),
                                               C.c_void_p(col.data_ptr() + k * npx * 3), C.byref(intr),
                                               ext[k].ctypes.data_as(C.c_void_p), 1000.0, 3.0, stream)
                assert st == 0, lib.ot_last_error()
            L.call("ot_tsdf_flush", vol, stream)

        for s in range(3):
            step()
            keys, tsdf, weight, colr, upd, units = _export64(L, vol, stream)
            assert upd == r_upd and units == r_units, f"counters after step {s}"
            if s == 0:
                continue  # the first step integrates into a new pool (test_bench_workload_bitexact's state)
            assert_bitwise(keys, rk, f"unit keys after reset (step {s})")
            assert_bitwise(weight, rw, f"voxel weights after reset (step {s})")
            assert_bitwise(tsdf, rt, f"voxel tsdf after reset (step {s})")
            assert_bitwise(colr, rc, f"float64 voxel colours after reset (step {s})")
    finally:
        L.call("ot_tsdf_destroy", vol)


def test_reset_then_other_scan_bitexact(pkg, O, synth, gpu):
    """Reset between two DIFFERENT scans: the second volume's units land on pool records the first scan filled (unit
    ids are reissued from 0), and nothing of the first scan may leak into it (keys, tsdf, weight, float64 colour)."""
    L = pkg._lib
    intr_t = synth.REF_INTRINSICS_640
    integ = pkg.pipelines.integration
    intr = pkg.camera.PinholeCameraIntrinsic(*intr_t)
    vol = integ.ScalableTSDFVolume(voxel_length=0.005, sdf_trunc=0.04, color_type=integ.TSDFVolumeColorType.RGB8)
    a = synth.make_sequence(synth.object_scene(1), n_frames=64, frames=range(0, 64, 4))
    b = synth.make_sequence(synth.object_scene(2), n_frames=64, frames=range(1, 64, 5))

    def integrate(seq):
        depth, color, ext = seq
        for k in range(depth.shape[0]):
            rgbd = pkg.geometry.RGBDImage.create_from_color_and_depth(
                pkg.geometry.Image(color[k]), pkg.geometry.Image(depth[k]), depth_scale=1000.0, depth_trunc=3.0,
                convert_rgb_to_intensity=False)
            vol.integrate(rgbd, intr, ext[k])

    integrate(a)
    vol.reset()
    integrate(b)
    ref = O.TSDF(0.005, 0.04, 1, 4)
    for k in range(b[0].shape[0]):
        ref.integrate(O.depth_to_float(b[0][k], 1000.0, 3.0), b[1][k], intr_t, b[2][k])
    keys, tsdf, weight, colr = (t.cpu().numpy() for t in vol.export_units())
    rk, rt, rw, rc = ref.export()
    assert_bitwise(keys, rk, "unit keys (second scan after reset)")
    assert_bitwise(weight, rw, "weights (second scan after reset)")
    assert_bitwise(tsdf, rt, "tsdf (second scan after reset)")
    assert_bitwise(colr, rc, "float64 colours (second scan after reset)")
