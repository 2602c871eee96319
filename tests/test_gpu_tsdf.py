"""GPU parity: depth conversion, multiplier, unprojection and ScalableTSDFVolume integration vs the CPU oracle.

Bit-exact: depth float image, multiplier image, unprojected point count/order/xyz (identity and posed
extrinsic), TSDF unit key set, per-voxel weight and tsdf.  Colour (f32 running mean on the GPU vs f64 in
Open3D/oracle): |rel| <= 1e-4 (SURVEY.md §8(c) parity contract).
"""
import ctypes as C

import numpy as np
import pytest
import torch

from conftest import assert_bitwise, ref_intr

pytestmark = pytest.mark.gpu


def _integration(pkg):
    return pkg.pipelines.integration


def test_depth_to_float_bitexact(pkg, O, gpu, seq16):
    depth = seq16[0][0]
    for trunc in (3.0, 5.0):
        img = pkg.geometry.Image(depth)
        rgbd = pkg.geometry.RGBDImage.create_from_color_and_depth(
            pkg.geometry.Image(seq16[1][0]), img, depth_scale=1000.0, depth_trunc=trunc,
            convert_rgb_to_intensity=False)
        assert_bitwise(np.asarray(rgbd.depth), O.depth_to_float(depth, 1000.0, trunc), "depth float")


def test_depth_to_float_edge_values(pkg, O, gpu):
    d = np.array([[0, 1, 2999, 3000, 3001, 65535, 4999, 5000, 7, 13, 2, 3]], np.uint16)
    img = pkg.geometry.Image(d)
    rgbd = pkg.geometry.RGBDImage.create_from_color_and_depth(
        pkg.geometry.Image(np.zeros((1, 12, 3), np.uint8)), img, depth_scale=1000.0, depth_trunc=3.0,
        convert_rgb_to_intensity=False)
    assert_bitwise(np.asarray(rgbd.depth), O.depth_to_float(d, 1000.0, 3.0), "depth edge values")


def test_multiplier_bitexact(pkg, O, gpu, synth):
    L = pkg._lib
    for intr_t in (synth.REF_INTRINSICS_640, synth.REF_INTRINSICS_1280):
        w, h = intr_t[0], intr_t[1]
        out = torch.empty((h, w), dtype=torch.float32, device="cuda")
        intr = L.ot_intrinsics(*intr_t)
        L.call("ot_depth_multiplier", C.byref(intr), C.c_void_p(out.data_ptr()), None)
        torch.cuda.synchronize()
        assert_bitwise(out.cpu().numpy(), O.depth_multiplier(*intr_t), "multiplier")


@pytest.mark.parametrize("posed", [False, True])
def test_unproject_bitexact(pkg, O, gpu, synth, seq16, posed):
    depth, color, ext = seq16
    intr_t = ref_intr(synth)
    intr = pkg.camera.PinholeCameraIntrinsic(*intr_t)
    rgbd = pkg.geometry.RGBDImage.create_from_color_and_depth(
        pkg.geometry.Image(color[1]), pkg.geometry.Image(depth[1]), depth_scale=1000.0, depth_trunc=5.0,
        convert_rgb_to_intensity=False)
    e = ext[1] if posed else None
    pcd = pkg.geometry.PointCloud.create_from_rgbd_image(rgbd, intr, *( [e] if posed else []))
    rx, rc = O.unproject(O.depth_to_float(depth[1], 1000.0, 5.0), color[1], intr_t, e)
    assert len(pcd.points) == rx.shape[0] > 100000
    assert_bitwise(np.asarray(pcd.points), rx, "unprojected xyz")
    assert_bitwise(np.asarray(pcd.colors), rc, "unprojected rgb")


def test_unproject_and_voxel_odd_resolution(pkg, O, gpu, synth):
    """321x243 frame (odd sizes, off-centre principal point): unprojection order and values, then the voxel
    downsample, bit-exact."""
    intr_t = (321, 243, 283.1, 283.4, 161.7, 120.2)
    depth, color, ext = synth.make_sequence(n_frames=8, frames=[3], intr=intr_t)
    intr = pkg.camera.PinholeCameraIntrinsic(*intr_t)
    rgbd = pkg.geometry.RGBDImage.create_from_color_and_depth(
        pkg.geometry.Image(color[0]), pkg.geometry.Image(depth[0]), depth_scale=1000.0, depth_trunc=5.0,
        convert_rgb_to_intensity=False)
    pcd = pkg.geometry.PointCloud.create_from_rgbd_image(rgbd, intr, ext[0])
    rx, rc = O.unproject(O.depth_to_float(depth[0], 1000.0, 5.0), color[0], intr_t, ext[0])
    assert len(pcd.points) == rx.shape[0] > 20000
    assert_bitwise(np.asarray(pcd.points), rx, "unprojected xyz (odd size)")
    ds = pcd.voxel_down_sample(0.005)
    rv, rvc, _, _ = O.voxel_down_sample(rx, rc, 0.005)
    assert_bitwise(np.asarray(ds.points), rv, "voxel averages (odd size)")


def test_unproject_stride_and_empty(pkg, O, gpu, synth, seq16):
    depth = seq16[0][2]
    intr_t = ref_intr(synth)
    intr = pkg.camera.PinholeCameraIntrinsic(*intr_t)
    pcd = pkg.geometry.PointCloud.create_from_depth_image(pkg.geometry.Image(depth), intr, seq16[2][2],
                                                          depth_scale=1000.0, depth_trunc=3.0, stride=4)
    rx, _ = O.unproject(O.depth_to_float(depth, 1000.0, 3.0), None, intr_t, seq16[2][2], stride=4)
    assert_bitwise(np.asarray(pcd.points), rx, "stride-4 xyz")
    empty = pkg.geometry.PointCloud.create_from_depth_image(pkg.geometry.Image(np.zeros_like(depth)), intr)
    assert len(empty.points) == 0


def _run_pair(pkg, O, synth, depth, color, ext, voxel, batch=None, trunc=3.0, float_path=False, intr_t=None,
              color_precision=64):
    integ = _integration(pkg)
    intr_t = intr_t or ref_intr(synth)
    intr = pkg.camera.PinholeCameraIntrinsic(*intr_t)
    vol = integ.ScalableTSDFVolume(voxel_length=voxel, sdf_trunc=0.04, color_type=integ.TSDFVolumeColorType.RGB8,
                                   batch_frames=batch, color_precision=color_precision)
    ref = O.TSDF(voxel, 0.04, 1, 4)
    for k in range(depth.shape[0]):
        rgbd = pkg.geometry.RGBDImage.create_from_color_and_depth(
            pkg.geometry.Image(color[k]), pkg.geometry.Image(depth[k]), depth_scale=1000.0, depth_trunc=trunc,
            convert_rgb_to_intensity=False)
        if float_path:
            rgbd._raw_depth = None  # force the float-depth entry point (ot_tsdf_integrate)
        vol.integrate(rgbd, intr, ext[k])
        ref.integrate(O.depth_to_float(depth[k], 1000.0, trunc), color[k], intr_t, ext[k])
    return vol, ref


def _compare_volumes(vol, ref):
    keys, tsdf, weight, col = (t.cpu().numpy() for t in vol.export_units())
    rk, rt, rw, rc = ref.export()
    assert_bitwise(keys, rk, "unit keys")
    assert_bitwise(weight, rw, "voxel weights")
    assert_bitwise(tsdf, rt, "voxel tsdf")
    if vol.color_precision == 64:  # Open3D's float64 colour state: bit-exact
        assert_bitwise(col, rc, "voxel colours (float64)")
    else:  # float32 state with one reciprocal per update
        np.testing.assert_allclose(col, rc, rtol=1e-4, atol=1e-4 * 255)
    upd, units = vol.counters()
    assert upd == ref.total_updates()
    assert units == ref.unit_integrations()
    return keys.shape[0]


def test_unit_order_rank_sort_matches_radix(pkg, O, gpu, synth, seq16):
    """Unit order: the one-launch rank sort (unit keys packed in <= 20 bits, every volume here) and the radix sort it
    replaces give the same order -- both volumes export the oracle's sorted unit keys and the same mesh, bit for bit."""
    L = pkg._lib
    depth, color, ext = seq16
    out = []
    for radix in (1, 0):
        L.call("otx_unit_sort_radix", radix)
        try:
            vol, ref = _run_pair(pkg, O, synth, depth, color, ext, 0.005)
            assert _compare_volumes(vol, ref) > 300
            m = vol.extract_triangle_mesh()
            out.append((np.asarray(m.vertices).copy(), np.asarray(m.vertex_colors).copy(),
                        np.asarray(m.triangles).copy()))
        finally:
            L.call("otx_unit_sort_radix", 0)
    for a, b, what in zip(out[0], out[1], ("vertices", "vertex colours", "triangles")):
        assert a.shape[0] > 1000
        assert_bitwise(b, a, what + " (rank sort vs radix sort)")


@pytest.mark.parametrize("voxel", [0.01, 0.005])
@pytest.mark.parametrize("batch", [1, 3, None])
def test_tsdf_integrate_bitexact(pkg, O, gpu, synth, seq16, voxel, batch):
    depth, color, ext = seq16
    vol, ref = _run_pair(pkg, O, synth, depth, color, ext, voxel, batch=batch)
    n = _compare_volumes(vol, ref)
    assert n > 300


@pytest.mark.parametrize("fine,depth", [(0, -1), (1, 1), (1, 2), (1, 3)])
def test_integrate_granularity_bitexact(pkg, O, gpu, synth, fine, depth):
    """Both slice granularities of k_batch_integrate (4 voxels per lane along z, 16 waves per unit; or 2, 32 waves --
    taken for batches with few units) forced for every batch, the fine one at every frame-pipeline depth (round 6:
    frame f + KT's taps and f + KT - 1's colour gathers issued before frame f's update): 40 frames at 5 mm in 16-frame
    batches (and a 3-frame batch: shorter than the pipeline), bitwise vs the oracle (keys, tsdf, weight, float64
    colour, counters)."""
    L = pkg._lib
    depth_img, color, ext = synth.make_sequence(synth.Scene(seed=5), n_frames=80, frames=range(0, 80, 2))
    L.call("otx_integrate_fine", fine)
    L.call("otx_integrate_depth", depth)
    try:
        vol, ref = _run_pair(pkg, O, synth, depth_img, color, ext, 0.005, batch=16)
        assert _compare_volumes(vol, ref) > 1000
        vol, ref = _run_pair(pkg, O, synth, depth_img[:7], color[:7], ext[:7], 0.005, batch=3)
        assert _compare_volumes(vol, ref) > 100
    finally:
        L.call("otx_integrate_fine", -1)
        L.call("otx_integrate_depth", -1)


@pytest.mark.parametrize("blocks,tf", [(0, 2), (7, 2), (-1, 4), (-1, 3), (-1, 8)])
def test_touch_staging_forms_bitexact(pkg, O, gpu, synth, blocks, tf):
    """The batch touch's staging by separate staging-only workgroups (-1: two per touch tile, the default; 7: a
    count that does not divide the frame) and by the touch workgroups themselves (0): 40 frames at 5 mm in 16-frame
    batches and the odd 321x243 camera (per-pixel staging tail), bitwise vs the oracle; with 4 frames per touch
    workgroup (the default 2, and 3 -- a ragged last group -- 4 and 8)."""
    L = pkg._lib
    L.call("otx_touch_stage_blocks", blocks)
    L.call("otx_touch_frames", tf)
    try:
        depth, color, ext = synth.make_sequence(synth.Scene(seed=5), n_frames=80, frames=range(0, 80, 2))
        vol, ref = _run_pair(pkg, O, synth, depth, color, ext, 0.005, batch=16)
        assert _compare_volumes(vol, ref) > 1000
        intr_t = (321, 243, 283.1, 283.4, 161.7, 120.2)
        depth, color, ext = synth.make_sequence(n_frames=12, frames=[0, 2, 5, 9], intr=intr_t)
        vol, ref = _run_pair(pkg, O, synth, depth, color, ext, 0.01, batch=None, intr_t=intr_t)
        assert _compare_volumes(vol, ref) > 100
    finally:
        L.call("otx_touch_stage_blocks", -1)
        L.call("otx_touch_frames", 2)


@pytest.mark.parametrize("batch,defer,fine", [(16, 0, -1), (1, 0, -1), (16, 1, -1), (1, 1, -1), (16, 1, 1), (16, 1, 0)])
def test_split_frontend_bitexact(pkg, O, gpu, synth, seq16, batch, defer, fine):
    """The split front end (round 6: touch without staging, the batch units' footprint tiles marked, only those tiles
    staged) forced on an unsharded volume, where every visible tile must be marked: 40 frames at 5 mm, the odd
    321x243 camera (partial 32x16 tiles, quads straddling rows) and the float-depth path, bitwise vs the oracle;
    with the deferred integrate too (each batch's integrate launched with the next batch's touch, k_integrate_touch,
    the last one by the reader's flush), its integrate in coarse or fine slices (by the batch's unit count, or forced:
    k_integrate_touch_fine)."""
    L = pkg._lib
    L.call("otx_split_frontend", 1)
    L.call("otx_defer_integrate", defer)
    L.call("otx_integrate_fine", fine)
    try:
        depth, color, ext = synth.make_sequence(synth.Scene(seed=5), n_frames=80, frames=range(0, 80, 2))
        vol, ref = _run_pair(pkg, O, synth, depth, color, ext, 0.005, batch=batch)
        assert _compare_volumes(vol, ref) > 1000
        intr_t = (321, 243, 283.1, 283.4, 161.7, 120.2)
        depth, color, ext = synth.make_sequence(n_frames=12, frames=[0, 2, 5, 9], intr=intr_t)
        vol, ref = _run_pair(pkg, O, synth, depth, color, ext, 0.01, batch=batch, intr_t=intr_t)
        assert _compare_volumes(vol, ref) > 100
        # width a multiple of 4 but not of 32: the staging kernel's quad path with a narrower last tile column
        intr_t = (324, 242, 283.1, 283.4, 161.7, 120.2)
        depth, color, ext = synth.make_sequence(n_frames=12, frames=[0, 2, 5, 9], intr=intr_t)
        vol, ref = _run_pair(pkg, O, synth, depth, color, ext, 0.01, batch=batch, intr_t=intr_t)
        assert _compare_volumes(vol, ref) > 100
        depth, color, ext = seq16
        vol, ref = _run_pair(pkg, O, synth, depth, color, ext, 0.01, float_path=True)
        _compare_volumes(vol, ref)
    finally:
        L.call("otx_split_frontend", -1)
        L.call("otx_defer_integrate", -1)
        L.call("otx_integrate_fine", -1)


@pytest.mark.parametrize("batch", [1, None])
def test_tsdf_odd_resolution(pkg, O, gpu, synth, batch):
    """A 321x243 camera (width not a multiple of 4: the staging kernel's per-pixel path; odd sample grid at
    stride 4) with an off-centre principal point: bit-exact like the reference resolution."""
    intr_t = (321, 243, 283.1, 283.4, 161.7, 120.2)
    depth, color, ext = synth.make_sequence(n_frames=12, frames=[0, 2, 5, 9], intr=intr_t)
    vol, ref = _run_pair(pkg, O, synth, depth, color, ext, 0.01, batch=batch, intr_t=intr_t)
    assert _compare_volumes(vol, ref) > 100


def test_tsdf_float_path_batched(pkg, O, gpu, synth, seq16):
    depth, color, ext = seq16
    vol, ref = _run_pair(pkg, O, synth, depth, color, ext, 0.01, float_path=True)
    _compare_volumes(vol, ref)


@pytest.mark.parametrize("batch", [None, 32])
def test_tsdf_many_batches_5mm(pkg, O, gpu, synth, batch):
    """70 frames of a 70-frame ring at 5 mm: one 64-frame batch (the default) and a 6-frame one, or two 32-frame
    batches and a 6-frame one; full 360 deg coverage."""
    depth, color, ext = synth.make_sequence(n_frames=70)
    vol, ref = _run_pair(pkg, O, synth, depth, color, ext, 0.005, batch=batch)
    n = _compare_volumes(vol, ref)
    assert n > 3000


@pytest.mark.parametrize("bits", [64, 32])
def test_ieee_division_kernel_after_import(pkg, O, gpu, synth, bits):
    """after import_units the weights are arbitrary state, so the host launches the IEEE-division
    integrate (k_batch_integrate<C64, false>) instead of the reciprocal-table one.  Volume A integrates the first
    12 frames and exports; volume B imports A's units and integrates the next 12 frames in 5-frame batches; B must
    equal the oracle that integrated all 24 frames (tsdf / weight / keys bitwise; colour bitwise at precision 64)."""
    integ = _integration(pkg)
    intr_t = ref_intr(synth)
    intr = pkg.camera.PinholeCameraIntrinsic(*intr_t)
    depth, color, ext = synth.make_sequence(synth.Scene(seed=4), n_frames=48, frames=range(0, 48, 2))
    ref = O.TSDF(0.01, 0.04, 1, 4)

    def feed(vol, ks):
        for k in ks:
            rgbd = pkg.geometry.RGBDImage.create_from_color_and_depth(
                pkg.geometry.Image(color[k]), pkg.geometry.Image(depth[k]), depth_scale=1000.0, depth_trunc=3.0,
                convert_rgb_to_intensity=False)
            vol.integrate(rgbd, intr, ext[k])
            ref.integrate(O.depth_to_float(depth[k], 1000.0, 3.0), color[k], intr_t, ext[k])

    a = integ.ScalableTSDFVolume(voxel_length=0.01, sdf_trunc=0.04, color_type=integ.TSDFVolumeColorType.RGB8,
                                 color_precision=bits)
    feed(a, range(12))
    keys, tsdf, weight, col = a.export_units()
    b = integ.ScalableTSDFVolume(voxel_length=0.01, sdf_trunc=0.04, color_type=integ.TSDFVolumeColorType.RGB8,
                                 color_precision=bits, batch_frames=5)
    b.import_units(keys, tsdf, weight, col)
    feed(b, range(12, 24))
    bk, bt, bw, bc = (t.cpu().numpy() for t in b.export_units())
    rk, rt, rw, rc = ref.export()
    assert_bitwise(bk, rk, "unit keys (import + IEEE kernel)")
    assert_bitwise(bw, rw, "voxel weights (import + IEEE kernel)")
    assert_bitwise(bt, rt, "voxel tsdf (import + IEEE kernel)")
    if bits == 64:
        assert_bitwise(bc, rc, "float64 colours (import + IEEE kernel)")
    else:
        np.testing.assert_allclose(bc, rc, rtol=1e-4, atol=1e-4 * 255)


@pytest.mark.parametrize("bits", [64, 32])
def test_long_scan_crosses_reciprocal_table(pkg, O, gpu, synth, bits):
    """the reciprocal-table integrate serves weights below RCP_N = 2048; once frames since reset + the
    batch reach it the host switches to the IEEE-division kernel.  2,200 frames (a 16-frame 80x60 ring cycled), so
    weights run past 2048 and the scan crosses the switch part-way; bitwise vs the oracle at the end."""
    L = pkg._lib
    lib = L.load()
    intr_t = (80, 60, 70.7, 70.7, 40.5, 30.5)
    depth, color, ext = synth.make_sequence(synth.Scene(seed=6), n_frames=16, intr=intr_t)
    ext = np.ascontiguousarray(ext, dtype=np.float64)
    n_total = 2200
    d16 = torch.from_numpy(depth.view(np.int16)).cuda().view(torch.uint16).contiguous()
    col = torch.from_numpy(color).cuda().contiguous()
    W, H = intr_t[0], intr_t[1]
    intr = L.ot_intrinsics(W, H, *intr_t[2:])
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    vol = C.c_void_p()
    L.call("ot_tsdf_create", 0.02, 0.08, L.OT_COLOR_RGB8, 16, 4, 0, C.byref(vol))
    ref = O.TSDF(0.02, 0.08, 1, 4)
    dfs = [O.depth_to_float(depth[k], 1000.0, 3.0) for k in range(16)]
    try:
        L.call("ot_tsdf_set_color_precision", vol, bits)
        for i in range(n_total):
            k = i % 16
            st = lib.ot_tsdf_integrate_u16(vol, C.c_void_p(d16.data_ptr() + k * W * H * 2),
                                           C.c_void_p(col.data_ptr() + k * W * H * 3), C.byref(intr),
                                           ext[k].ctypes.data_as(C.c_void_p), 1000.0, 3.0, stream)
            assert st == 0, lib.ot_last_error()
            ref.integrate(dfs[k], color[k], intr_t, ext[k])
        nu = C.c_int64(0)
        L.call("ot_tsdf_num_units", vol, C.byref(nu), stream)
        n = nu.value
        keys = torch.empty((n, 3), dtype=torch.int32, device="cuda")
        tsdf = torch.empty((n, 4096), dtype=torch.float32, device="cuda")
        weight = torch.empty((n, 4096), dtype=torch.float32, device="cuda")
        colr = torch.empty((n, 4096, 3), dtype=torch.float64 if bits == 64 else torch.float32, device="cuda")
        L.call("ot_tsdf_export_units", vol, n, C.c_void_p(keys.data_ptr()), C.c_void_p(tsdf.data_ptr()),
               C.c_void_p(weight.data_ptr()), C.c_void_p(colr.data_ptr()) if bits == 32 else None, stream)
        if bits == 64:
            L.call("ot_tsdf_export_color64", vol, n, C.c_void_p(colr.data_ptr()), stream)
    finally:
        L.call("ot_tsdf_destroy", vol)
    rk, rt, rw, rc = ref.export()
    assert rw.max() > 2048, "the scan must drive weights past the reciprocal table"
    assert_bitwise(keys.cpu().numpy(), rk, "unit keys (long scan)")
    assert_bitwise(weight.cpu().numpy(), rw, "voxel weights (long scan)")
    assert_bitwise(tsdf.cpu().numpy(), rt, "voxel tsdf (long scan)")
    if bits == 64:
        assert_bitwise(colr.cpu().numpy(), rc, "float64 colours (long scan)")
    else:
        np.testing.assert_allclose(colr.cpu().numpy(), rc, rtol=1e-4, atol=1e-4 * 255)


def test_tsdf_lexical_order_matters(pkg, O, gpu, synth, seq16):
    """Running averages depend on frame order: the GPU must apply frames in call order."""
    depth, color, ext = seq16
    vol, ref = _run_pair(pkg, O, synth, depth[::-1].copy(), color[::-1].copy(), ext[::-1].copy(), 0.01)
    _compare_volumes(vol, ref)


def test_tsdf_reset_and_empty_frame(pkg, O, gpu, synth, seq16):
    depth, color, ext = seq16
    integ = _integration(pkg)
    intr = pkg.camera.PinholeCameraIntrinsic(*ref_intr(synth))
    vol = integ.ScalableTSDFVolume(voxel_length=0.01, sdf_trunc=0.04, color_type=integ.TSDFVolumeColorType.RGB8)
    zero = pkg.geometry.RGBDImage.create_from_color_and_depth(
        pkg.geometry.Image(color[0]), pkg.geometry.Image(np.zeros_like(depth[0])), convert_rgb_to_intensity=False)
    vol.integrate(zero, intr, ext[0])
    assert vol.num_units() == 0
    rgbd = pkg.geometry.RGBDImage.create_from_color_and_depth(
        pkg.geometry.Image(color[0]), pkg.geometry.Image(depth[0]), convert_rgb_to_intensity=False)
    vol.integrate(rgbd, intr, ext[0])
    assert vol.num_units() > 0
    vol.reset()
    assert vol.num_units() == 0


def test_tsdf_unsupported_format(pkg, gpu, synth, seq16):
    depth, color, ext = seq16
    integ = _integration(pkg)
    intr = pkg.camera.PinholeCameraIntrinsic(*ref_intr(synth))
    vol = integ.ScalableTSDFVolume(voxel_length=0.01, sdf_trunc=0.04, color_type=integ.TSDFVolumeColorType.RGB8)
    gray = pkg.geometry.RGBDImage.create_from_color_and_depth(
        pkg.geometry.Image(color[0]), pkg.geometry.Image(depth[0]), convert_rgb_to_intensity=True)
    with pytest.raises(RuntimeError, match="Unsupported image format"):
        vol.integrate(gray, intr, ext[0])
    small = pkg.camera.PinholeCameraIntrinsic(320, 240, 300.0, 300.0, 160.0, 120.0)
    rgbd = pkg.geometry.RGBDImage.create_from_color_and_depth(
        pkg.geometry.Image(color[0]), pkg.geometry.Image(depth[0]), convert_rgb_to_intensity=False)
    with pytest.raises(RuntimeError, match="Unsupported image format"):
        vol.integrate(rgbd, small, ext[0])


@pytest.mark.parametrize("batch", [1, None])
def test_tsdf_pool_grows(pkg, O, gpu, synth, batch):
    """Open3D's ScalableTSDFVolume is unbounded.  A volume created with room for 64 units integrates the
    configs[1] scan's first 16 frames at 5 mm (hundreds of units: the first batch alone overflows the pool and the
    hash) -- frame by frame (every flush a 1-frame batch) and as one 16-frame batch.  The pool grows and the dropped
    units are integrated again from the staged frames: keys, tsdf, weight, float64 colour and the update counters
    bitwise equal to the oracle's, and no error at any call."""
    integ = _integration(pkg)
    intr_t = ref_intr(synth)
    intr = pkg.camera.PinholeCameraIntrinsic(*intr_t)
    depth, color, ext = synth.make_sequence(synth.Scene(seed=0), n_frames=256, frames=range(16), intr=intr_t)
    vol = integ.ScalableTSDFVolume(voxel_length=0.005, sdf_trunc=0.04, color_type=integ.TSDFVolumeColorType.RGB8,
                                   max_units=64, batch_frames=batch)
    ref = O.TSDF(0.005, 0.04, 1, 4)
    for k in range(depth.shape[0]):
        rgbd = pkg.geometry.RGBDImage.create_from_color_and_depth(
            pkg.geometry.Image(color[k]), pkg.geometry.Image(depth[k]), depth_scale=1000.0, depth_trunc=3.0,
            convert_rgb_to_intensity=False)
        vol.integrate(rgbd, intr, ext[k])
        ref.integrate(O.depth_to_float(depth[k], 1000.0, 3.0), color[k], intr_t, ext[k])
    assert _compare_volumes(vol, ref) > 600
    m, (V, VC, T) = vol.extract_triangle_mesh(), ref.extract_triangle_mesh()
    assert_bitwise(np.asarray(m.vertices), V, "mesh vertices after pool growth")
    assert_bitwise(np.asarray(m.triangles), T, "mesh triangles after pool growth")


@pytest.mark.parametrize("batch,max_units", [(8, 0), (1, 0), (16, 64)])
def test_frontend_overlap_bitexact(pkg, O, gpu, synth, batch, max_units):
    """The double-buffered front end (batch k+1's staging / touch / units on the caller's stream beside batch k's
    integrate on the volume's integrate stream; off by default) forced on for an unsharded volume:
    70 frames in batches of 8 (9 batches, both staging sets reused), frame by frame, and with a 64-unit pool that
    grows mid-scan (replay from the batch's own set) -- bitwise equal to the oracle, counters included."""
    integ = _integration(pkg)
    intr_t = ref_intr(synth)
    intr = pkg.camera.PinholeCameraIntrinsic(*intr_t)
    depth, color, ext = synth.make_sequence(synth.Scene(seed=2), n_frames=70, frames=range(0, 70, 2 if batch == 1 else 1))
    vol = integ.ScalableTSDFVolume(voxel_length=0.005, sdf_trunc=0.04, color_type=integ.TSDFVolumeColorType.RGB8,
                                   batch_frames=batch, max_units=max_units)
    vol.set_frontend_overlap(1)
    ref = O.TSDF(0.005, 0.04, 1, 4)
    for k in range(depth.shape[0]):
        rgbd = pkg.geometry.RGBDImage.create_from_color_and_depth(
            pkg.geometry.Image(color[k]), pkg.geometry.Image(depth[k]), depth_scale=1000.0, depth_trunc=3.0,
            convert_rgb_to_intensity=False)
        vol.integrate(rgbd, intr, ext[k])
        ref.integrate(O.depth_to_float(depth[k], 1000.0, 3.0), color[k], intr_t, ext[k])
    assert _compare_volumes(vol, ref) > 1000
    vol.reset()  # a reset after overlapped batches, then one more pass bit-exact again
    ref2 = O.TSDF(0.005, 0.04, 1, 4)
    for k in range(0, depth.shape[0], 3):
        rgbd = pkg.geometry.RGBDImage.create_from_color_and_depth(
            pkg.geometry.Image(color[k]), pkg.geometry.Image(depth[k]), depth_scale=1000.0, depth_trunc=3.0,
            convert_rgb_to_intensity=False)
        vol.integrate(rgbd, intr, ext[k])
        ref2.integrate(O.depth_to_float(depth[k], 1000.0, 3.0), color[k], intr_t, ext[k])
    _compare_volumes(vol, ref2)


def test_tsdf_pool_grows_on_import(pkg, gpu, synth, seq16):
    """import_units into a 64-unit volume makes room first (the rows are counted before the import kernel)."""
    integ = _integration(pkg)
    intr = pkg.camera.PinholeCameraIntrinsic(*ref_intr(synth))
    depth, color, ext = seq16
    a = integ.ScalableTSDFVolume(voxel_length=0.005, sdf_trunc=0.04, color_type=integ.TSDFVolumeColorType.RGB8)
    for k in range(depth.shape[0]):
        a.integrate(pkg.geometry.RGBDImage.create_from_color_and_depth(
            pkg.geometry.Image(color[k]), pkg.geometry.Image(depth[k]), convert_rgb_to_intensity=False), intr, ext[k])
    rows = [t.cpu().numpy() for t in a.export_units()]
    assert rows[0].shape[0] > 300
    b = integ.ScalableTSDFVolume(voxel_length=0.005, sdf_trunc=0.04, color_type=integ.TSDFVolumeColorType.RGB8,
                                 max_units=64)
    b.import_units(*a.export_units())
    for x, y, what in zip((t.cpu().numpy() for t in b.export_units()), rows, ("keys", "tsdf", "weight", "colour")):
        assert_bitwise(x, y, f"imported {what} after pool growth")


@pytest.mark.parametrize("batch", [1, 32])
def test_float32_colour_mode(pkg, O, synth, seq16, gpu, batch):
    """colour precision 32 (the labelled secondary bench leg): tsdf / weight still bit-exact, colour within
    1e-4; both the per-frame (batch 1) and the fused kernel."""
    depth, color, ext = seq16
    vol, ref = _run_pair(pkg, O, synth, depth, color, ext, 0.01, batch=batch, color_precision=32)
    _compare_volumes(vol, ref)
    with pytest.raises(RuntimeError, match="colour precision"):  # float64 colours into a float32 volume
        pkg._lib.call("ot_tsdf_import_units_color64", vol._h, 0, None, None, None, None, None)


def test_nocolor_volume_default_precision(pkg, O, gpu, synth, seq16):
    """NoColor volumes keep no colour state whatever the requested precision (the facade asks for 64): float32
    records with zero colour planes, exports / imports at either dtype, tsdf and weight bit-exact vs the oracle."""
    depth, color, ext = seq16
    integ = _integration(pkg)
    intr_t = ref_intr(synth)
    intr = pkg.camera.PinholeCameraIntrinsic(*intr_t)
    vol = integ.ScalableTSDFVolume(voxel_length=0.01, sdf_trunc=0.04)
    assert vol.color_precision == 32
    ref = O.TSDF(0.01, 0.04, 0, 4)
    for k in range(depth.shape[0]):
        rgbd = pkg.geometry.RGBDImage.create_from_color_and_depth(
            pkg.geometry.Image(color[k]), pkg.geometry.Image(depth[k]), convert_rgb_to_intensity=False)
        vol.integrate(rgbd, intr, ext[k])
        ref.integrate(O.depth_to_float(depth[k], 1000.0, 3.0), None, intr_t, ext[k])
    keys, tsdf, weight, col = (t.cpu().numpy() for t in vol.export_units(color_dtype="float64"))
    rk, rt, rw, _ = ref.export()
    assert_bitwise(keys, rk, "NoColor unit keys")
    assert_bitwise(tsdf, rt, "NoColor tsdf")
    assert_bitwise(weight, rw, "NoColor weight")
    assert not col.any()
    kb, tb, wb, cb = vol.export_border()
    assert not cb.cpu().numpy().any()
    twin = integ.ScalableTSDFVolume(voxel_length=0.01, sdf_trunc=0.04)
    twin.import_units(*vol.export_units())
    assert_bitwise(twin.export_units()[1].cpu().numpy(), rt, "NoColor import / export round trip")


def test_frame_lifetime_across_streams(pkg, O, gpu, synth):
    """frames allocated on one stream and integrated on another, their Python references dropped
    right after the call.  The facade records the launch stream on every queued tensor and releases a frame only
    once the C side has consumed it (ot_tsdf_pending_frames), so the caching allocator cannot recycle a frame's
    memory (here: overwritten by garbage allocated on the producer stream) before its batch runs: bit-exact."""
    import torch

    depth, color, ext = synth.make_sequence(n_frames=24)
    integ = _integration(pkg)
    intr_t = ref_intr(synth)
    intr = pkg.camera.PinholeCameraIntrinsic(*intr_t)
    vol = integ.ScalableTSDFVolume(voxel_length=0.01, sdf_trunc=0.04, color_type=integ.TSDFVolumeColorType.RGB8,
                                   batch_frames=8)
    ref = O.TSDF(0.01, 0.04, 1, 4)
    producer, consumer = torch.cuda.Stream(), torch.cuda.Stream()
    for k in range(depth.shape[0]):
        with torch.cuda.stream(producer):
            d16 = torch.from_numpy(depth[k].view(np.int16)).cuda().view(torch.uint16)
            col = torch.from_numpy(color[k]).cuda()
        producer.synchronize()
        with torch.cuda.stream(consumer):
            rgbd = pkg.geometry.RGBDImage.create_from_color_and_depth(
                pkg.geometry.Image(col), pkg.geometry.Image(d16), convert_rgb_to_intensity=False)
            vol.integrate(rgbd, intr, ext[k])
        del rgbd, d16, col
        with torch.cuda.stream(producer):  # garbage into whatever memory the allocator hands out now
            junk = torch.full((480 * 640 * 3,), 255, dtype=torch.uint8, device="cuda")
            junk2 = torch.full((480 * 640,), 7, dtype=torch.int16, device="cuda")
            del junk, junk2
        ref.integrate(O.depth_to_float(depth[k], 1000.0, 3.0), color[k], intr_t, ext[k])
        if k % 8 != 7:
            assert len(vol._keep) >= 1  # queued frames stay referenced until their batch is enqueued
    with torch.cuda.stream(consumer):
        _compare_volumes(vol, ref)
