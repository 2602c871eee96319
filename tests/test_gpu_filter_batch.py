"""GPU parity of the configs[2] filter chain (BASELINE.json configs[2]: 1280x720, unproject -> voxel_down_sample(0.005)
-> remove_statistical_outlier(20, 2.0)), per frame as Open3D would run it (check_one_frame.py:22-28 + SURVEY A.7).

* the per-call HIP chain on one full 1280x720 frame vs the CPU oracle (bit-exact voxels, mean kNN distances, kept);
* the batched device-resident chain (ot_rgbd_filter_run) on several distinct full-size frames vs the oracle, and vs
  the per-call HIP chain, including an empty frame and ragged frame sizes;
* the Open3D-shaped facade (filters.RGBDFilterBatch.frame) returns what remove_statistical_outlier returns.
"""
import ctypes as C
import os

import numpy as np
import pytest
import torch

from conftest import assert_bitwise

pytestmark = pytest.mark.gpu


def _oracle_chain(O, depth, color, ext, intr_t, trunc=5.0, vs=0.005, k=20, ratio=2.0, scale=1000.0, batch=True):
    """The oracle's per-frame chain.  batch=True: the voxel cloud in the batched chain's canonical order (cell-major
    keys, oracle.cell_major_order; Open3D's own order is hash-map order), the SOR run on that order (its cloud
    statistics sum in cloud order); batch=False: voxel_down_sample's key order, as the per-call facade."""
    xyz, rgb = O.unproject(O.depth_to_float(depth, scale, trunc), color, intr_t, ext)
    v, vc, keys, _ = O.voxel_down_sample(xyz, rgb, vs)
    if batch:
        perm = O.cell_major_order(keys, O.batch_cell_shift(k))
        v, vc = v[perm], vc[perm]
    idx, avg = O.remove_statistical_outlier(v, k, ratio)
    return xyz.shape[0], v, vc, avg, idx


@pytest.fixture(scope="module")
def hd_frames(synth):
    """3 distinct frames of a 512-frame 1280x720 ring stream (frames 0, 171, 342)."""
    return synth.make_sequence(synth.Scene(seed=0), n_frames=512, intr=synth.REF_INTRINSICS_1280, frames=[0, 171, 342])


@pytest.fixture(scope="module")
def hd_oracle(O, synth, hd_frames):
    depth, color, ext = hd_frames
    return [_oracle_chain(O, depth[f], color[f], ext[f], synth.REF_INTRINSICS_1280) for f in range(depth.shape[0])]


def test_hd_chain_per_call_bitexact(pkg, O, synth, hd_frames, gpu):
    """VERDICT r1 'Next' 1: the HIP unproject -> voxel -> SOR chain on one full 1280x720 frame, Open3D-shaped calls."""
    depth, color, ext = hd_frames
    hd_oracle = [_oracle_chain(O, depth[0], color[0], ext[0], synth.REF_INTRINSICS_1280, batch=False)]
    intr = pkg.camera.PinholeCameraIntrinsic(*synth.REF_INTRINSICS_1280)
    rgbd = pkg.geometry.RGBDImage.create_from_color_and_depth(
        pkg.geometry.Image(color[0]), pkg.geometry.Image(depth[0]), depth_scale=1000.0, depth_trunc=5.0,
        convert_rgb_to_intensity=False)
    pcd = pkg.geometry.PointCloud.create_from_rgbd_image(rgbd, intr, ext[0])
    down = pcd.voxel_down_sample(0.005)
    kept, ind = down.remove_statistical_outlier(20, 2.0)
    P, v, vc, avg, idx = hd_oracle[0]
    assert len(pcd.points) == P
    assert_bitwise(np.asarray(down.points), v, "voxel averages (1280x720)")
    assert_bitwise(np.asarray(down.colors), vc, "voxel colours (1280x720)")
    assert_bitwise(np.asarray(ind, np.int64), idx, "SOR kept indices (1280x720)")
    assert_bitwise(np.asarray(kept.points), v[idx], "kept points (1280x720)")
    assert_bitwise(np.asarray(kept.colors), vc[idx], "kept colours (1280x720)")


def _run_batch(pkg, intr_t, depth, color, ext, max_frames=None, trunc=5.0):
    flt = pkg.filters.RGBDFilterBatch(pkg.camera.PinholeCameraIntrinsic(*intr_t), max_frames=max_frames or depth.shape[0],
                                      depth_trunc=trunc)
    return flt.run(depth, color, ext)


def test_hd_batch_bitexact(pkg, synth, hd_frames, hd_oracle, gpu):
    depth, color, ext = hd_frames
    flt = _run_batch(pkg, synth.REF_INTRINSICS_1280, depth, color, ext)
    assert flt.points == sum(o[0] for o in hd_oracle)
    for f, (P, v, vc, avg, idx) in enumerate(hd_oracle):
        assert flt.point_offsets[f + 1] - flt.point_offsets[f] == P
        down, davg = flt.voxel_cloud(f)
        assert_bitwise(np.asarray(down.points), v, f"batch voxel averages (frame {f})")
        assert_bitwise(np.asarray(down.colors), vc, f"batch voxel colours (frame {f})")
        assert_bitwise(davg, avg, f"batch mean kNN distances (frame {f})")
        kept, ind = flt.frame(f)
        assert_bitwise(np.asarray(ind, np.int64), idx, f"batch SOR kept indices (frame {f})")
        assert_bitwise(np.asarray(kept.points), v[idx], f"batch kept points (frame {f})")
        assert_bitwise(np.asarray(kept.colors), vc[idx], f"batch kept colours (frame {f})")


@pytest.mark.parametrize("F", [64, 32])
def test_bench_batch_shape_bitexact(pkg, O, synth, gpu, F):
    """VERDICT r3 'next' 1: configs[2] exactly as bench.py times it -- one F-frame batch (frames 256..) of the bench's
    512-frame 1280x720 stream through ot_rgbd_filter_run on handles created as FilterStream creates them, two batches in
    flight on two host threads x worker streams (thread-local scratch, as the bench's 3 workers).  At F = 64 every
    frame of the batch, at F = 32 four (first, last, two inside), vs the oracle chain (voxels, colours, mean kNN distances, kept indices); the frame
    tags, segment table and key widths at F full frames are the bench's (F = 64: bench.py's default since late round 4,
    the segmented sort's 64-segment limit; 32: the earlier default)."""
    import threading

    L = pkg._lib
    intr_t = synth.REF_INTRINSICS_1280
    W, H = intr_t[0], intr_t[1]
    npx = W * H
    depth, color, ext = synth.make_sequence(synth.Scene(seed=0), n_frames=512, intr=intr_t, frames=range(256, 256 + F))
    d16 = torch.from_numpy(depth.view(np.int16)).cuda().view(torch.uint16).contiguous()
    col = torch.from_numpy(color).cuda().contiguous()
    exts = np.ascontiguousarray(ext, dtype=np.float64).reshape(F, 16)
    intr = L.ot_intrinsics(W, H, *intr_t[2:])
    import importlib

    streams = importlib.import_module(pkg.__name__ + ".streams").worker_streams(2)
    handles = []
    for _ in range(2):
        h = C.c_void_p()
        L.call("ot_rgbd_filter_create", C.byref(intr), F, 1000.0, 5.0, 0.005, 20, 2.0, C.byref(h))
        handles.append(h)
    errors = []

    def worker(t):
        try:
            with torch.cuda.stream(streams[t]):
                L.call("ot_rgbd_filter_run", handles[t], F, C.c_void_p(d16.data_ptr()), C.c_void_p(col.data_ptr()),
                       exts.ctypes.data_as(C.c_void_p), C.c_void_p(streams[t].cuda_stream))
                streams[t].synchronize()
        except Exception as e:  # surfaced below
            errors.append(e)

    try:
        ths = [threading.Thread(target=worker, args=(t,)) for t in range(2)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        assert not errors, errors
        torch.cuda.synchronize()
        # the bench's shape (F = 64): every frame of the batch vs the oracle; the earlier 32: four frames
        picks = list(range(F)) if F == 64 else [0, 9, F - 10, F - 1]
        from concurrent.futures import ThreadPoolExecutor

        with ThreadPoolExecutor(max_workers=min(16, os.cpu_count() or 4)) as ex:  # the oracle's C calls drop the GIL
            ref = dict(zip(picks, ex.map(lambda f: _oracle_chain(O, depth[f], color[f], ext[f], intr_t), picks)))
        for t in range(2):
            n = F + 1
            po, vo, ko = (np.zeros(n, np.int64) for _ in range(3))
            P, K, KK = C.c_int64(0), C.c_int64(0), C.c_int64(0)
            L.call("ot_rgbd_filter_sizes", handles[t], C.byref(P), C.byref(K), C.byref(KK),
                   po.ctypes.data_as(C.c_void_p), vo.ctypes.data_as(C.c_void_p), ko.ctypes.data_as(C.c_void_p))
            assert P.value > F * 500000, "bench-sized frames"
            for f in picks:
                Pf, v, vc, avg, idx = ref[f]
                assert po[f + 1] - po[f] == Pf
                nv, nk = int(vo[f + 1] - vo[f]), int(ko[f + 1] - ko[f])
                vx = torch.empty((nv, 3), dtype=torch.float64, device="cuda")
                vcol = torch.empty((nv, 3), dtype=torch.float64, device="cuda")
                vavg = torch.empty((nv,), dtype=torch.float64, device="cuda")
                kx = torch.empty((nk, 3), dtype=torch.float64, device="cuda")
                kc = torch.empty((nk, 3), dtype=torch.float64, device="cuda")
                ki = torch.empty((nk,), dtype=torch.int64, device="cuda")
                s_ = C.c_void_p(torch.cuda.current_stream().cuda_stream)
                L.call("ot_rgbd_filter_copy", handles[t], f, C.c_void_p(kx.data_ptr()), C.c_void_p(kc.data_ptr()),
                       C.c_void_p(ki.data_ptr()), C.c_void_p(vx.data_ptr()), C.c_void_p(vcol.data_ptr()),
                       C.c_void_p(vavg.data_ptr()), s_)
                tag = f"bench batch, handle {t}, frame {f}"
                assert_bitwise(vx.cpu().numpy(), v, f"voxel averages ({tag})")
                assert_bitwise(vcol.cpu().numpy(), vc, f"voxel colours ({tag})")
                assert_bitwise(vavg.cpu().numpy(), avg, f"mean kNN distances ({tag})")
                assert_bitwise(ki.cpu().numpy(), idx, f"kept indices ({tag})")
                assert_bitwise(kx.cpu().numpy(), v[idx], f"kept points ({tag})")
                assert_bitwise(kc.cpu().numpy(), vc[idx], f"kept colours ({tag})")
    finally:
        for h in handles:
            L.call("ot_rgbd_filter_destroy", h)


def test_batch_matches_per_call_ragged(pkg, O, synth, gpu):
    """640x480 frames incl. an all-invalid frame (empty cloud) and one truncated by depth_trunc: the batch equals
    the per-frame Open3D-shaped calls, frame by frame; the batch buffers are reused by a second, smaller run."""
    intr_t = synth.REF_INTRINSICS_640
    depth, color, ext = synth.make_sequence(synth.Scene(seed=3), n_frames=64, frames=[1, 9, 17, 40, 63])
    depth = depth.copy()
    depth[2] = 0                        # no valid pixel
    depth[3][depth[3] > 1500] = 4000    # beyond depth_trunc (3 m) -> invalid
    intr = pkg.camera.PinholeCameraIntrinsic(*intr_t)
    flt = _run_batch(pkg, intr_t, depth, color, ext, max_frames=8, trunc=3.0)
    for f in range(depth.shape[0]):
        rgbd = pkg.geometry.RGBDImage.create_from_color_and_depth(
            pkg.geometry.Image(color[f]), pkg.geometry.Image(depth[f]), depth_scale=1000.0, depth_trunc=3.0,
            convert_rgb_to_intensity=False)
        down = pkg.geometry.PointCloud.create_from_rgbd_image(rgbd, intr, ext[f]).voxel_down_sample(0.005)
        P, v, vc, avg, idx = _oracle_chain(O, depth[f], color[f], ext[f], intr_t, trunc=3.0)
        bdown, _ = flt.voxel_cloud(f)
        bkept, bind = flt.frame(f)
        # the same voxels as the per-call chain (as a set: the batch emits them in cell-major order) ...
        dp = np.asarray(down.points).reshape(-1, 3)
        bp = np.asarray(bdown.points).reshape(-1, 3)
        assert_bitwise(bp[np.lexsort(bp.T[::-1])], dp[np.lexsort(dp.T[::-1])], f"ragged voxel set (frame {f})")
        # ... and in that order exactly the oracle chain's
        assert_bitwise(bp, v.reshape(-1, 3), f"ragged voxels (frame {f})")
        assert bind == idx.tolist(), f"ragged kept indices (frame {f})"
        assert_bitwise(np.asarray(bkept.points).reshape(-1, 3), v.reshape(-1, 3)[idx], f"ragged kept (frame {f})")
    assert flt.voxel_offsets[3] == flt.voxel_offsets[2]  # the empty frame
    # a second run on 2 frames reuses the handle
    flt.run(depth[:2], color[:2], ext[:2])
    assert flt.n_frames == 2 and flt.kept_offsets[2] == flt.kept


def test_batch_wide_keys_match_per_call(pkg, O, synth, gpu):
    """A 0.4 mm voxel makes the voxel key wider than 32 bits: the batch takes its 64-bit-key path (frame in the
    key) and must still equal the per-frame calls."""
    intr_t = synth.REF_INTRINSICS_640
    depth, color, ext = synth.make_sequence(synth.Scene(seed=5), n_frames=16, frames=[2, 11])
    flt = pkg.filters.RGBDFilterBatch(pkg.camera.PinholeCameraIntrinsic(*intr_t), max_frames=2, depth_trunc=5.0,
                                      voxel_size=0.0004).run(depth, color, ext)
    for f in range(2):
        P, v, vc, avg, idx = _oracle_chain(O, depth[f], color[f], ext[f], intr_t, vs=0.0004)
        bdown, davg = flt.voxel_cloud(f)
        bkept, bind = flt.frame(f)
        assert_bitwise(np.asarray(bdown.points), v, f"wide-key voxels (frame {f})")
        assert_bitwise(davg, avg, f"wide-key mean kNN distances (frame {f})")
        assert bind == idx.tolist(), f"wide-key kept indices (frame {f})"


def test_batch_sparse_tail(pkg, O, synth, gpu):
    """SOR stages 2-3 inside the batched chain (frame in the grid key): speckle pixels at far depths become isolated
    voxels whose k-th neighbour lies many cells away (one wave per query, rings and the whole-frame scan bounded by
    their own frame), and a frame of 12 valid pixels has fewer points than k."""
    intr_t = synth.REF_INTRINSICS_640
    depth, color, ext = synth.make_sequence(synth.Scene(seed=11), n_frames=32, frames=[3, 14, 27])
    depth = depth.copy()
    rng = np.random.default_rng(4)
    for f in (0, 1):
        iy, ix = rng.integers(0, 480, 300), rng.integers(0, 640, 300)
        depth[f][iy, ix] = rng.integers(300, 2999, 300).astype(np.uint16)   # speckles at any depth
    keep = np.zeros_like(depth[2])
    iy, ix = rng.integers(0, 480, 12), rng.integers(0, 640, 12)
    keep[iy, ix] = depth[2][iy, ix]
    depth[2] = keep                                                          # 12 valid pixels (< k = 20)
    flt = _run_batch(pkg, intr_t, depth, color, ext, max_frames=3, trunc=3.0)
    for f in range(3):
        P, v, vc, avg, idx = _oracle_chain(O, depth[f], color[f], ext[f], intr_t, trunc=3.0)
        down, davg = flt.voxel_cloud(f)
        assert_bitwise(np.asarray(down.points), v, f"sparse-tail voxels (frame {f})")
        assert_bitwise(davg, avg, f"sparse-tail mean kNN distances (frame {f})")
        _, ind = flt.frame(f)
        assert_bitwise(np.asarray(ind, np.int64), idx, f"sparse-tail kept indices (frame {f})")


@pytest.mark.parametrize("scale", [5000.0, 1234.5])
def test_batch_odd_scale_and_intrinsics(pkg, O, synth, scale, gpu):
    """Depth scales other than 1000 and intrinsics with non-half principal points and fx != fy: the batch's
    reciprocal-product divisions (depth / scale in float32, (c - cx) z / fx, colour / 255, sum / count in float64)
    must still give the IEEE quotients, frame by frame against the oracle chain."""
    intr_t = (640, 480, 517.31, 516.07, 318.71, 243.29)
    depth, color, ext = synth.make_sequence(synth.Scene(seed=7), n_frames=32, frames=[4, 19])
    flt = pkg.filters.RGBDFilterBatch(pkg.camera.PinholeCameraIntrinsic(*intr_t), max_frames=2, depth_scale=scale,
                                      depth_trunc=3.0, voxel_size=0.004).run(depth, color, ext)
    for f in range(2):
        P, v, vc, avg, idx = _oracle_chain(O, depth[f], color[f], ext[f], intr_t, trunc=3.0, vs=0.004, scale=scale)
        assert flt.point_offsets[f + 1] - flt.point_offsets[f] == P
        down, davg = flt.voxel_cloud(f)
        assert_bitwise(np.asarray(down.points), v, f"scale {scale} voxel averages (frame {f})")
        assert_bitwise(np.asarray(down.colors), vc, f"scale {scale} voxel colours (frame {f})")
        assert_bitwise(davg, avg, f"scale {scale} mean kNN distances (frame {f})")
        _, ind = flt.frame(f)
        assert_bitwise(np.asarray(ind, np.int64), idx, f"scale {scale} kept indices (frame {f})")


def test_batch_errors(pkg, synth, gpu):
    intr = pkg.camera.PinholeCameraIntrinsic(*synth.REF_INTRINSICS_640)
    with pytest.raises(RuntimeError, match="voxel_size"):
        pkg.filters.RGBDFilterBatch(intr, voxel_size=0.0)
    with pytest.raises(RuntimeError, match="Illegal input"):
        pkg.filters.RGBDFilterBatch(intr, nb_neighbors=0)
    flt = pkg.filters.RGBDFilterBatch(intr, max_frames=2)
    d = np.zeros((3, 480, 640), np.uint16)
    c = np.zeros((3, 480, 640, 3), np.uint8)
    with pytest.raises(RuntimeError):
        flt.run(d, c, np.stack([np.eye(4)] * 3))           # more frames than max_frames
    with pytest.raises(RuntimeError, match="Unsupported image format"):
        flt.run(d[:1, :100], c[:1, :100], np.eye(4)[None])  # wrong image size


def test_batch_tiny_images_many_frames(pkg, O, synth, gpu):
    """a 32x32 intrinsic (one pixel tile per frame) with 256 frames per run: the per-run tile / frame
    tables (frame bounds, key widths, point and voxel offsets) grow with the frame count, not with the image, and
    must fit their allocation.  Every frame vs the oracle chain."""
    intr_t = (32, 32, 28.3, 28.3, 15.5, 15.5)  # the reference's hfov at 32 px
    depth, color, ext = synth.make_sequence(synth.Scene(seed=2), n_frames=256, intr=intr_t)
    flt = _run_batch(pkg, intr_t, depth, color, ext, max_frames=256, trunc=5.0)
    for f in range(0, 256, 5):
        P, v, vc, avg, idx = _oracle_chain(O, depth[f], color[f], ext[f], intr_t)
        assert flt.point_offsets[f + 1] - flt.point_offsets[f] == P
        down, davg = flt.voxel_cloud(f)
        assert_bitwise(np.asarray(down.points).reshape(-1, 3), v.reshape(-1, 3), f"tiny-image voxels (frame {f})")
        assert_bitwise(davg, avg, f"tiny-image mean kNN distances (frame {f})")
        _, ind = flt.frame(f)
        assert_bitwise(np.asarray(ind, np.int64), idx, f"tiny-image kept indices (frame {f})")


def test_batch_far_clusters(pkg, O, synth, gpu):
    """SOR at its limits: a 4-voxel cluster 3.5 m behind a 30x30-pixel patch needs neighbours beyond every bounded
    box (the whole-frame scan of stage 3), a frame of one cluster stretched along the viewing axis (identity pose: long
    z columns of cells), and a frame of a single pixel (k > points)."""
    intr_t = synth.REF_INTRINSICS_640
    depth = np.zeros((3, 480, 640), np.uint16)
    depth[0, 200:230, 300:330] = 1000
    depth[0, 0:2, 0:2] = 4500
    rng = np.random.default_rng(9)
    depth[1, 100:160, 200:260] = rng.integers(800, 1400, (60, 60)).astype(np.uint16)  # a noisy slab in depth
    depth[2, 240, 320] = 2000
    color = rng.integers(0, 256, (3, 480, 640, 3)).astype(np.uint8)
    ext = np.stack([np.eye(4)] * 3)
    flt = _run_batch(pkg, intr_t, depth, color, ext, max_frames=3, trunc=5.0)
    for f in range(3):
        P, v, vc, avg, idx = _oracle_chain(O, depth[f], color[f], ext[f], intr_t)
        down, davg = flt.voxel_cloud(f)
        assert_bitwise(np.asarray(down.points).reshape(-1, 3), v.reshape(-1, 3), f"far-cluster voxels (frame {f})")
        assert_bitwise(davg, avg, f"far-cluster mean kNN distances (frame {f})")
        _, ind = flt.frame(f)
        assert_bitwise(np.asarray(ind, np.int64), idx, f"far-cluster kept indices (frame {f})")
