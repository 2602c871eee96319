"""Spatial sharding of one object's volume: `world` volumes, each keeping only the units with
owner(key) == rank, integrate the same frames.  The union of their exported units equals one unsharded volume bit
for bit (keys, tsdf, weight and colour: every voxel sees the same frames in the same order), the update counters
add up, and importing all shards into one volume gives the unsharded volume's marching-cubes mesh exactly."""
import importlib

import numpy as np
import pytest

from conftest import assert_bitwise, ref_intr

pytestmark = pytest.mark.gpu


def _integrate(pkg, seq, voxel, shard=None, overlap=None):
    depth, color, ext = seq
    integ = pkg.pipelines.integration
    intr = pkg.camera.PinholeCameraIntrinsic(*ref_intr(importlib.import_module(pkg.__name__ + ".synth")))
    vol = integ.ScalableTSDFVolume(voxel_length=voxel, sdf_trunc=0.04, color_type=integ.TSDFVolumeColorType.RGB8)
    if shard is not None:
        _set_shard(vol, shard)
    if overlap is not None:
        vol.set_frontend_overlap(overlap)
    for k in range(depth.shape[0]):
        rgbd = pkg.geometry.RGBDImage.create_from_color_and_depth(
            pkg.geometry.Image(color[k]), pkg.geometry.Image(depth[k]), depth_scale=1000.0, depth_trunc=3.0,
            convert_rgb_to_intensity=False)
        vol.integrate(rgbd, intr, ext[k])
    return vol


def _set_shard(vol, shard):
    """(rank, world): hashed ownership blocks; (rank, world, cx, cy): azimuth sectors around (cx, cy) (round 6)"""
    if len(shard) == 4:
        vol.set_shard_sector(shard[0], shard[1], shard[2:])
    else:
        vol.set_shard(*shard)


def _host(t):
    return t.cpu().numpy()


@pytest.mark.parametrize("voxel,world,overlap,sector", [(0.01, 3, None, None), (0.005, 8, 1, None),
                                                        (0.005, 8, None, (0.0, 0.0)), (0.01, 3, None, (0.13, -0.2)),
                                                        (0.005, 4, None, (0.0, 0.0)), (0.005, 8, 1, (0.0, 0.0))])
def test_shard_union_bitexact(pkg, seq16, gpu, voxel, world, overlap, sector):
    """hashed blocks and azimuth sectors (split front end: the touch stages nothing, only the tiles the rank's units
    project to are staged), centred and off-centre; at 8 ranks also with the double-buffered front end (the split
    front end on the caller's stream beside the previous batch's integrate on the volume's integrate stream)"""
    full = _integrate(pkg, seq16, voxel)
    fk, ft, fw, fc = (_host(a) for a in full.export_units())
    parts = [_integrate(pkg, seq16, voxel, (r, world) + tuple(sector or ()), overlap) for r in range(world)]
    exports = [[_host(a) for a in v.export_units()] for v in parts]
    counts = [e[0].shape[0] for e in exports]
    assert sum(counts) == fk.shape[0] and min(counts) > (0.5 if sector is None or sector == (0.0, 0.0) else 0.2) * \
        fk.shape[0] / world
    keys = np.concatenate([e[0] for e in exports])
    order = np.lexsort((keys[:, 2], keys[:, 1], keys[:, 0]))
    assert_bitwise(keys[order], fk, "shard union keys")
    assert_bitwise(np.concatenate([e[1] for e in exports])[order], ft, "shard union tsdf")
    assert_bitwise(np.concatenate([e[2] for e in exports])[order], fw, "shard union weight")
    assert_bitwise(np.concatenate([e[3] for e in exports])[order], fc, "shard union colour")
    upd = [v.counters() for v in parts]
    assert sum(u for u, _ in upd) == full.counters()[0]
    assert sum(k for _, k in upd) == full.counters()[1]


def test_shard_import_mesh_bitexact(pkg, seq16, gpu):
    integ = pkg.pipelines.integration
    full = _integrate(pkg, seq16, 0.01)
    m0 = full.extract_triangle_mesh()
    merged = integ.ScalableTSDFVolume(voxel_length=0.01, sdf_trunc=0.04, color_type=integ.TSDFVolumeColorType.RGB8)
    for r in range(4):
        merged.import_units(*_integrate(pkg, seq16, 0.01, (r, 4)).export_units())
    assert merged.num_units() == full.num_units()
    m1 = merged.extract_triangle_mesh()
    assert_bitwise(np.asarray(m1.vertices), np.asarray(m0.vertices), "merged-shard mesh vertices")
    assert_bitwise(np.asarray(m1.triangles), np.asarray(m0.triangles), "merged-shard mesh triangles")
    assert_bitwise(np.asarray(m1.vertex_colors), np.asarray(m0.vertex_colors), "merged-shard mesh colours")


@pytest.mark.parametrize("world,precision,sector", [(3, 64, None), (8, 32, None), (8, 64, (0.0, 0.0))])
def test_shard_border_halo_mesh_bitexact(pkg, seq16, gpu, world, precision, sector):
    """SURVEY §8(e) border halo: every shard imports the other shards' border rows (721 low-face voxels per unit)
    it needs, extracts only its own units' cubes, and the partial meshes merge (distributed.merge_shard_meshes)
    into the unsharded mesh bit for bit -- without moving whole units."""
    integ = pkg.pipelines.integration
    D = importlib.import_module(pkg.__name__ + ".distributed")

    def make(shard=None):
        v = _integrate_p(pkg, seq16, 0.01, shard, precision)
        return v

    full = make()
    m0 = full.extract_triangle_mesh()
    shards = [make((r, world) + tuple(sector or ())) for r in range(world)]
    rows = [D.pack_border(*v.export_border()) for v in shards]
    import torch

    allrows = torch.cat(rows)
    unit_bytes = full.num_units() * (3 + 4096 * (2 + (6 if precision == 64 else 3))) * 4
    assert allrows.numel() * 4 < unit_bytes / 5  # border layers only
    parts = []
    for v in shards:
        v.import_border(*D.unpack_border(allrows))
        mesh, vk, tk = v.extract_triangle_mesh(with_keys=True)
        parts.append((mesh._v.dev(), mesh._vc.dev(), mesh._t.dev(), vk, tk))
    V, VC, T = D.merge_shard_meshes(parts)
    assert_bitwise(V.cpu().numpy(), np.asarray(m0.vertices), "halo-merged mesh vertices")
    assert_bitwise(VC.cpu().numpy(), np.asarray(m0.vertex_colors), "halo-merged mesh colours")
    assert_bitwise(T.cpu().numpy(), np.asarray(m0.triangles), "halo-merged mesh triangles")
    # every shard emitted only its own cubes: the triangle counts add up
    assert sum(p[2].shape[0] for p in parts) == np.asarray(m0.triangles).shape[0]


def _integrate_p(pkg, seq, voxel, shard, precision):
    depth, color, ext = seq
    integ = pkg.pipelines.integration
    intr = pkg.camera.PinholeCameraIntrinsic(*ref_intr(importlib.import_module(pkg.__name__ + ".synth")))
    vol = integ.ScalableTSDFVolume(voxel_length=voxel, sdf_trunc=0.04, color_type=integ.TSDFVolumeColorType.RGB8,
                                   color_precision=precision)
    if shard is not None:
        _set_shard(vol, shard)
    for k in range(depth.shape[0]):
        rgbd = pkg.geometry.RGBDImage.create_from_color_and_depth(
            pkg.geometry.Image(color[k]), pkg.geometry.Image(depth[k]), depth_scale=1000.0, depth_trunc=3.0,
            convert_rgb_to_intensity=False)
        vol.integrate(rgbd, intr, ext[k])
    return vol


def test_shard_argument_errors(pkg, seq16, gpu):
    integ = pkg.pipelines.integration
    vol = _integrate(pkg, (seq16[0][:2], seq16[1][:2], seq16[2][:2]), 0.01)
    vol.num_units()
    with pytest.raises(RuntimeError, match="before the first integrate"):
        vol.set_shard(0, 2)
    fresh = integ.ScalableTSDFVolume(voxel_length=0.01, sdf_trunc=0.04)
    with pytest.raises(RuntimeError, match="rank < world"):
        fresh.set_shard(2, 2)
    fresh.set_shard(0, 1)  # world 1: no sharding
    with pytest.raises(RuntimeError, match="finite centre"):
        fresh.set_shard_sector(0, 2, (float("nan"), 0.0))
    with pytest.raises(RuntimeError, match="before the first integrate"):
        vol.set_shard_sector(0, 2)


@pytest.mark.parametrize("sector", [None, (0.0, 0.0)])
def test_split_frontend_pool_growth_bitexact(pkg, O, gpu, synth, sector):
    """The split front end with a 64-unit pool: the first batch overflows, the pool grows and the dropped units are
    integrated again from the staged frames (the replay touch reads each stride sample's staged pixel, which the
    split touch writes; the dropped units' tiles were staged by the first pass).  Union of 4 shards == the oracle."""
    integ = pkg.pipelines.integration
    intr_t = ref_intr(synth)
    intr = pkg.camera.PinholeCameraIntrinsic(*intr_t)
    depth, color, ext = synth.make_sequence(synth.Scene(seed=0), n_frames=256, frames=range(0, 64, 4), intr=intr_t)
    ref = O.TSDF(0.005, 0.04, 1, 4)
    for k in range(depth.shape[0]):
        ref.integrate(O.depth_to_float(depth[k], 1000.0, 3.0), color[k], intr_t, ext[k])
    rk, rt, rw, rc = ref.export()[:4]
    world = 4
    exports = []
    for r in range(world):
        vol = integ.ScalableTSDFVolume(voxel_length=0.005, sdf_trunc=0.04, color_type=integ.TSDFVolumeColorType.RGB8,
                                       max_units=64, batch_frames=16)
        _set_shard(vol, (r, world) + tuple(sector or ()))
        for k in range(depth.shape[0]):
            vol.integrate(pkg.geometry.RGBDImage.create_from_color_and_depth(
                pkg.geometry.Image(color[k]), pkg.geometry.Image(depth[k]), depth_scale=1000.0, depth_trunc=3.0,
                convert_rgb_to_intensity=False), intr, ext[k])
        exports.append([_host(a) for a in vol.export_units()])
    keys = np.concatenate([e[0] for e in exports])
    order = np.lexsort((keys[:, 2], keys[:, 1], keys[:, 0]))
    assert keys.shape[0] > 4 * 64
    assert_bitwise(keys[order], rk, "split-front-end union keys after growth")
    assert_bitwise(np.concatenate([e[1] for e in exports])[order], rt, "union tsdf")
    assert_bitwise(np.concatenate([e[2] for e in exports])[order], rw, "union weight")
    assert_bitwise(np.concatenate([e[3] for e in exports])[order], rc, "union colour")


def test_border_api_errors(pkg, seq16, gpu):
    """export_border capacity and import_border shape checks; an unsharded volume exports every unit and imports
    nothing from rows it owns."""
    import ctypes as C

    import torch

    L = pkg._lib
    vol = _integrate_p(pkg, (seq16[0][:2], seq16[1][:2], seq16[2][:2]), 0.01, None, 32)
    n = vol.num_units()
    keys, tsdf, weight, color = vol.export_border()
    assert keys.shape[0] == n and tsdf.shape == (n, 721) and color.shape == (n, 721, 3)
    small = torch.empty((1, 3), dtype=torch.int32, device="cuda")
    t1 = torch.empty((1, 721), dtype=torch.float32, device="cuda")
    m = C.c_int64(0)
    with pytest.raises(RuntimeError, match="capacity"):
        L.call("ot_tsdf_export_border", vol._h, 1, C.c_void_p(small.data_ptr()), C.c_void_p(t1.data_ptr()),
               C.c_void_p(t1.data_ptr()), None, C.byref(m), None)
    with pytest.raises(RuntimeError, match="import_border"):
        vol.import_border(keys, tsdf[:, :100], weight, color)
    before = vol.num_units()
    vol.import_border(keys, tsdf, weight, color)  # every row is owned here (unsharded): nothing is imported
    assert vol.num_units() == before


def test_assemble_after_halo_extraction_bitexact(pkg, seq16, gpu):
    """after a shard imported halo units (import_border) and extracted its mesh, export_units and
    num_units still cover only its own units, so assembling the shards' exports in one volume (what
    distributed.assemble_sharded_volume does over ranks) gives the unsharded volume and mesh bit for bit -- no
    duplicate keys, no zero halo copy overwriting the owner's data."""
    integ = pkg.pipelines.integration
    D = importlib.import_module(pkg.__name__ + ".distributed")
    world = 3
    full = _integrate_p(pkg, seq16, 0.01, None, 64)
    fk, ft, fw, fc = (_host(a) for a in full.export_units())
    m0 = full.extract_triangle_mesh()
    shards = [_integrate_p(pkg, seq16, 0.01, (r, world), 64) for r in range(world)]
    own = [v.num_units() for v in shards]
    import torch

    allrows = torch.cat([D.pack_border(*v.export_border()) for v in shards])
    for v in shards:
        v.import_border(*D.unpack_border(allrows))
        v.extract_triangle_mesh()
    assert [v.num_units() for v in shards] == own  # halo units are not counted
    merged = integ.ScalableTSDFVolume(voxel_length=0.01, sdf_trunc=0.04, color_type=integ.TSDFVolumeColorType.RGB8)
    exports = [v.export_units() for v in shards]
    assert sum(int(e[0].shape[0]) for e in exports) == fk.shape[0]
    for e in exports:
        merged.import_units(*e)
    mk, mt, mw, mc = (_host(a) for a in merged.export_units())
    assert_bitwise(mk, fk, "assembled keys")
    assert_bitwise(mt, ft, "assembled tsdf")
    assert_bitwise(mw, fw, "assembled weight")
    assert_bitwise(mc, fc, "assembled colour")
    m1 = merged.extract_triangle_mesh()
    assert_bitwise(np.asarray(m1.vertices), np.asarray(m0.vertices), "assembled mesh vertices")
    assert_bitwise(np.asarray(m1.vertex_colors), np.asarray(m0.vertex_colors), "assembled mesh colours")


def _halo_worker(rank, world, port, q, sector=None):
    import os
    import sys

    import torch
    import torch.distributed as dist

    from conftest import PKG, ROOT

    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pkg = importlib.import_module(PKG)
        synth = importlib.import_module(PKG + ".synth")
        D = importlib.import_module(PKG + ".distributed")
        seq = synth.make_sequence(n_frames=16, frames=[0, 3, 7, 12])
        print(f"[halo rank {rank}] integrating", flush=True)
        vol = _integrate_p(pkg, seq, 0.005, (rank, world) + tuple(sector or ()), 64)
        keys, _, _, _ = vol.export_border()
        print(f"[halo rank {rank}] extracting", flush=True)
        mesh, got = D.extract_sharded_mesh(vol)
        print(f"[halo rank {rank}] extracted", flush=True)
        n_rows = torch.tensor([[int(keys.shape[0])]], dtype=torch.int64)
        counts = D.all_gather_rows(n_rows).flatten().tolist()
        row_bytes = (3 + 721 * 8) * 4  # pack_border row, float64 colour
        allgather = (sum(counts) - counts[rank]) * row_bytes  # what the all-gather of every border row delivered
        q.put((rank, mesh._v.dev().cpu().numpy(), mesh._t.dev().cpu().numpy(), mesh._vc.dev().cpu().numpy(), got,
               allgather))
        dist.barrier()
    except BaseException as e:  # report it: the parent fails at once instead of waiting out its queue timeout
        q.put((rank, f"{type(e).__name__}: {e}"))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,sector", [(2, None), (3, None), (4, (0.0, 0.0))])
def test_halo_exchange_ranks_bitexact(pkg, seq16, gpu, world, sector):
    """`world` ranks (gloo, sharing this GPU) each integrate one object's frames into their shard
    (ownership by blocks of units; at 4 ranks by azimuth sectors, with the deferred integrate), exchange border rows
    only with the ranks owning a -x/-y/-z neighbour (distributed.exchange_rows: all_to_all), extract and merge: every
    rank's mesh equals the unsharded mesh bit for bit, and each rank receives at most half the border bytes an
    all-gather of every row delivers.  At 4 sector ranks a rank can receive a single border row (round 6: its
    float64 colours sat at an odd int32 offset, which unpack_border now copies out)."""
    import socket

    import torch.multiprocessing as mp

    full = _integrate_p(pkg, seq16, 0.005, None, 64)
    m0 = full.extract_triangle_mesh()
    V0, T0, C0 = (np.asarray(a) for a in (m0.vertices, m0.triangles, m0.vertex_colors))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_halo_worker, args=(r, world, port, q, sector)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        r, *rest = q.get(timeout=240)
        assert len(rest) > 1, f"rank {r} failed: {rest[0]}"
        out[r] = rest
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(world):
        V, T, VC, got, allgather = out[r]
        assert_bitwise(V, V0, f"rank {r} merged vertices")
        assert_bitwise(T, T0, f"rank {r} merged triangles")
        assert_bitwise(VC, C0, f"rank {r} merged colours")
        assert got <= 0.5 * allgather, f"rank {r}: {got} border bytes received vs {allgather} by all-gather"


def test_deferred_integrate_sync_reset(pkg, gpu, synth):
    """A sector shard of 4 ranks runs the deferred integrate (batch k's integrate launched with batch k + 1's touch):
    ot_tsdf_reset (the synchronous C reset) with a batch still deferred drops it with the old contents, and the
    volume then integrates a new scan exactly as a fresh volume does (keys, tsdf, weight, float64 colour bitwise)."""
    integ = pkg.pipelines.integration
    intr = pkg.camera.PinholeCameraIntrinsic(*ref_intr(synth))
    depth, color, ext = synth.make_sequence(synth.Scene(seed=3), n_frames=80, frames=range(0, 80, 4))

    def make():
        v = integ.ScalableTSDFVolume(voxel_length=0.005, sdf_trunc=0.04, color_type=integ.TSDFVolumeColorType.RGB8,
                                     batch_frames=4)
        v.set_shard_sector(0, 4, (0.0, 0.0))
        return v

    def feed(v, ks):
        for k in ks:
            v.integrate(pkg.geometry.RGBDImage.create_from_color_and_depth(
                pkg.geometry.Image(color[k]), pkg.geometry.Image(depth[k]), depth_scale=1000.0, depth_trunc=3.0,
                convert_rgb_to_intensity=False), intr, ext[k])

    a = make()
    feed(a, range(12))  # three 4-frame batches: the third one's integrate is still deferred
    import torch

    torch.cuda.synchronize()
    pkg._lib.call("ot_tsdf_reset", a._h)
    a._keep.clear()
    feed(a, range(12, 20))
    b = make()
    feed(b, range(12, 20))
    for x, y, what in zip(a.export_units(), b.export_units(), ("keys", "tsdf", "weight", "colour")):
        assert_bitwise(_host(x), _host(y), f"after a synchronous reset: {what}")
