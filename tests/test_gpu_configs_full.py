"""Full-size oracle parity of BASELINE.json configs[3] and configs[4] -- the workloads bench.py times as `objects` and
`hybrid_map`, through exactly the calls the bench makes.

configs[3] (reconstruct_rgbd_filter.py:81-132,154-155): 8 object scans x 64 640x480 frames, per object integrate at
5 mm (colour precision 64, the facade and C-ABI default) -> extract_triangle_mesh -> compute_vertex_normals ->
sample_points_uniformly(100000) -> z >= 0.03 mask (fused and batched over the objects, as bench.py runs it, and the
two-step form beside it), then the merge in sorted object order (distributed.merge_object_clouds; one process: local
concatenation).  Every object's mesh (vertices,
triangles, colours, normals), its filtered cloud (points and colours) and the merged cloud are bit-exact against the
CPU oracle, and the batched sampler equals the oracle's single-mesh sampler per object.

configs[4] (hybrid_map.py:25-60,62-96,115; 2d_selective_merge.py:58-69): a 1024 x 1024 occupancy grid @ 5 cm (saved +
new) and 32 object clouds with their saved versions: smart_paste of the whole new grid onto the saved one, the
occupied-cell cloud of the merged grid, the 2 cm voxel-key diff of every object against its saved version
(ot_voxel_key_diff_multi), and the hybrid cloud (map cloud first, then the objects in order) -- bit-exact against
the numpy / C restatements."""
import ctypes as C
import importlib

import numpy as np
import pytest

from conftest import PKG, assert_bitwise

pytestmark = pytest.mark.gpu

N_OBJECTS, N_FRAMES, VOXEL, TRUNC, N_SAMPLES, Z_MIN = 8, 64, 0.005, 0.04, 100000, 0.03


@pytest.fixture(scope="module")
def obj_scans(synth):
    """The 8 synthetic object scans bench.py renders (object_scene(i), 64-frame rings), rendered by a spawned
    process pool (fresh interpreters: this process has already initialised the GPU)."""
    import multiprocessing as mp
    from concurrent.futures import ProcessPoolExecutor

    with ProcessPoolExecutor(max_workers=N_OBJECTS, mp_context=mp.get_context("spawn")) as ex:
        jobs = [(synth.object_scene(i), N_FRAMES, synth.REF_INTRINSICS_640, None) for i in range(N_OBJECTS)]
        return list(ex.map(synth.render_frames, jobs))


@pytest.fixture(scope="module")
def obj_oracle(O, synth, obj_scans):
    out = []
    for depth, color, ext in obj_scans:
        vol = O.TSDF(VOXEL, TRUNC, 1, 4)
        for k in range(depth.shape[0]):
            vol.integrate(O.depth_to_float(depth[k], 1000.0, 3.0), color[k], synth.REF_INTRINSICS_640, ext[k])
        V, VC, T = vol.extract_triangle_mesh()
        VN = O.vertex_normals(V, T)
        P, PN, PC = O.sample_points_uniformly(V, T, N_SAMPLES, 0, VN=VN, VC=VC)
        fx, fc = O.filter_min_z(P, PC, Z_MIN)
        out.append({"V": V, "VC": VC, "T": T, "VN": VN, "P": fx, "PC": fc})
    return out


def test_configs3_objects_full_size_bitexact(pkg, synth, obj_scans, obj_oracle, gpu):
    import torch

    L = pkg._lib
    lib = L.load()
    D = importlib.import_module(PKG + ".distributed")
    integ = pkg.pipelines.integration
    intr_t = synth.REF_INTRINSICS_640
    W, H = intr_t[0], intr_t[1]
    npx = W * H
    intr = L.ot_intrinsics(W, H, *intr_t[2:])
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    meshes = []
    for depth, color, ext in obj_scans:  # bench.objects_pipeline.reconstruct, one object after the other
        d16 = torch.from_numpy(depth.view(np.int16)).cuda().view(torch.uint16).contiguous()
        col = torch.from_numpy(color).cuda().contiguous()
        ext = np.ascontiguousarray(ext, dtype=np.float64)
        vol = integ.ScalableTSDFVolume(voxel_length=VOXEL, sdf_trunc=TRUNC,
                                       color_type=integ.TSDFVolumeColorType.RGB8)
        assert vol.color_precision == 64
        st = lib.ot_tsdf_integrate_u16_frames(vol._h, ext.shape[0], C.c_void_p(d16.data_ptr()),
                                              C.c_void_p(col.data_ptr()), C.byref(intr),
                                              ext.ctypes.data_as(C.c_void_p), 1000.0, 3.0, stream)
        assert st == 0, lib.ot_last_error()
        mesh = vol.extract_triangle_mesh()
        mesh.compute_vertex_normals()
        meshes.append(mesh)
        del vol
    # the bench's tail: sampling and Z mask fused, all objects in one call, then one collective merge (capacity in-band)
    filtered = pkg.geometry.TriangleMesh.sample_points_min_z_batch(meshes, N_SAMPLES, Z_MIN)
    merged = D.merge_object_clouds([f._xyz.dev() for f in filtered], capacity=N_OBJECTS * N_SAMPLES)
    # and the reference's two steps (sample, then mask) on the batched sampler: the same clouds
    two = [p.filter_min_z(Z_MIN) for p in
           pkg.geometry.TriangleMesh.sample_points_uniformly_batch(meshes, number_of_points=N_SAMPLES)]
    for f, t in zip(filtered, two):
        assert_bitwise(np.asarray(f.points), np.asarray(t.points), "fused vs two-step z-masked samples")
    for j, (m, f, ref) in enumerate(zip(meshes, filtered, obj_oracle)):
        assert len(ref["T"]) > 10000, f"object {j}: degenerate oracle mesh"
        assert_bitwise(np.asarray(m.vertices), ref["V"], f"object {j} mesh vertices")
        assert_bitwise(np.asarray(m.triangles), ref["T"], f"object {j} mesh triangles")
        assert_bitwise(np.asarray(m.vertex_colors), ref["VC"], f"object {j} vertex colours")
        assert_bitwise(np.asarray(m.vertex_normals), ref["VN"], f"object {j} vertex normals")
        assert 0 < len(ref["P"]) < N_SAMPLES
        assert_bitwise(np.asarray(f.points), ref["P"], f"object {j} z-masked samples")
        assert_bitwise(np.asarray(f.colors), ref["PC"], f"object {j} z-masked sample colours")
    assert_bitwise(merged.cpu().numpy(), np.concatenate([r["P"] for r in obj_oracle]),
                   "merged object clouds (sorted object order)")


def test_configs4_hybrid_full_size_bitexact(pkg, O, synth, gpu):
    import torch

    L = pkg._lib
    CD = pkg.change_detection
    D = importlib.import_module(PKG + ".distributed")
    n_obj = 32
    objs = [synth.object_cloud(i) for i in range(n_obj)]
    saved = [synth.object_cloud(i, moved=True) for i in range(n_obj)]
    old_map, new_map = synth.occupancy_pair(1024, 1024, seed=0)
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    # exactly bench.hybrid_fusion's calls
    cat_new = torch.from_numpy(np.concatenate(objs)).cuda().contiguous()
    cat_old = torch.from_numpy(np.concatenate(saved)).cuda().contiguous()
    off_new = np.concatenate([[0], np.cumsum([len(o) for o in objs])]).astype(np.int64)
    off_old = np.concatenate([[0], np.cumsum([len(o) for o in saved])]).astype(np.int64)
    keys_a = torch.empty((int(off_new[-1]) + 1, 4), dtype=torch.int32, device="cuda")
    keys_r = torch.empty((int(off_old[-1]) + 1, 4), dtype=torch.int32, device="cuda")
    origin = (C.c_double * 3)(-1.0, -1.0, -1.0)
    na, nr = C.c_int64(0), C.c_int64(0)
    L.call("ot_voxel_key_diff_multi", C.c_void_p(cat_new.data_ptr()), off_new.ctypes.data_as(C.c_void_p),
           C.c_void_p(cat_old.data_ptr()), off_old.ctypes.data_as(C.c_void_p), n_obj, 0.02, origin,
           C.c_void_p(keys_a.data_ptr()), C.byref(na), C.c_void_p(keys_r.data_ptr()), C.byref(nr), stream)
    d_base = torch.from_numpy(old_map).cuda().contiguous()
    d_new = torch.from_numpy(new_map).cuda().contiguous()
    ch, nq = C.c_int64(0), C.c_int64(0)
    L.call("ot_grid_smart_paste", C.c_void_p(d_base.data_ptr()), C.c_void_p(d_new.data_ptr()), 1024, 1024, 0, 0,
           1024, 1024, CD.UNKNOWN_PIXEL, CD.PASTE_THRESHOLD, C.byref(ch), stream)
    occ = torch.empty((1024 * 1024, 3), dtype=torch.float64, device="cuda")
    L.call("ot_occupancy_to_points", C.c_void_p(d_base.data_ptr()), 1024, 1024, 100, 0.05, -25.6, -25.6,
           C.c_void_p(occ.data_ptr()), C.byref(nq), stream)
    merged = torch.cat([occ[:nq.value], D.merge_object_clouds([torch.from_numpy(o).cuda() for o in objs])], 0)
    torch.cuda.synchronize()
    # oracle
    ref_grid = O.smart_paste(old_map, new_map, 0, 0, 1024, 1024, CD.UNKNOWN_PIXEL, CD.PASTE_THRESHOLD)
    assert_bitwise(d_base.cpu().numpy(), ref_grid, "smart_paste 1024x1024 grid")
    assert ch.value == int((ref_grid != old_map).sum()) > 10000
    ref_occ = O.occupancy_to_points(ref_grid, 100, 0.05, -25.6, -25.6)
    assert nq.value == len(ref_occ) > 1000
    assert_bitwise(occ[:nq.value].cpu().numpy(), ref_occ, "occupied-cell cloud")
    ra, rr = [], []
    for j in range(n_obj):
        a, r = O.voxel_key_diff(objs[j], saved[j], 0.02, np.array([-1.0, -1.0, -1.0]))
        ra.append(np.concatenate([np.full((len(a), 1), j, np.int32), a], 1))
        rr.append(np.concatenate([np.full((len(r), 1), j, np.int32), r], 1))
    ra, rr = np.concatenate(ra), np.concatenate(rr)
    assert len(ra) > 1000 and len(rr) > 1000
    assert_bitwise(keys_a[:na.value].cpu().numpy(), ra, "added voxel keys, 32 objects")
    assert_bitwise(keys_r[:nr.value].cpu().numpy(), rr, "removed voxel keys, 32 objects")
    assert_bitwise(merged.cpu().numpy(), np.concatenate([ref_occ] + objs), "hybrid cloud (map first, then objects)")
