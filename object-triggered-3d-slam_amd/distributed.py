"""Multi-GPU execution: independent object scans sharded over ranks, one RCCL all-gather for the hybrid-map merge.

The reference reconstructs objects one after another in a Python loop (reconstruct_rgbd_filter.py:154-155) and
later concatenates their clouds behind the occupancy-grid cloud (hybrid_map.py:62-96, :115).  Objects share no
state, so here each rank (one process per GPU, torch.distributed over RCCL/xGMI) takes a CONTIGUOUS chunk of
the sorted object list; concatenating the per-rank results in rank order therefore reproduces the reference's
sorted-file order exactly.  The only data-path collective is the final all-gather of the filtered clouds
(merge_object_clouds), float64 rows so the merge is bit-exact, in one of two forms chosen by the padded size:
  * all_gather_rows_capped: ONE all_gather_into_tensor of [capacity + 1, 3] rows per rank with the row count
    in-band (no count exchange, no host read between collectives) -- while world * (capacity + 1) * 24 B stays
    under CAPPED_MAX_BYTES;
  * all_gather_rows: an all_gather of the int64 counts, one host read, then an all_gather of [max count, 3] rows --
    when padding to the common bound would move more (configs[3] at 8 ranks: 100k-row bound per object against
    ~6.7k real rows, DESIGN.md §6 models both over xGMI).
Every rank trims the padding; rank 0 prepends the map cloud and writes the PLY.
Works unchanged on gloo (CPU tensors) for the world-size-2 CPU tests.
"""
from __future__ import annotations

import os

import numpy as np


def shard(items, rank, world):
    """Contiguous chunk `rank` of `items` (sorted order preserved across ranks)."""
    n = len(items)
    lo = (n * rank) // world
    hi = (n * (rank + 1)) // world
    return list(items[lo:hi])


def all_gather_rows(local, group=None):
    """Concatenate every rank's (n_r, k) tensor in rank order on every rank.  `local` lives on the backend's
    device (HIP tensor for nccl/RCCL, CPU for gloo)."""
    import torch
    import torch.distributed as dist

    if not dist.is_initialized():  # single process: nothing to exchange
        return local
    if dist.get_backend(group) == "gloo" and local.is_cuda:  # gloo collectives run through host memory
        return all_gather_rows(local.cpu(), group).to(local.device)
    world = dist.get_world_size(group)
    k = local.shape[1]
    counts = torch.zeros(world, dtype=torch.int64, device=local.device)
    mine = torch.tensor([local.shape[0]], dtype=torch.int64, device=local.device)
    dist.all_gather_into_tensor(counts, mine, group=group)
    counts_h = counts.cpu().tolist()
    m = max(counts_h) if counts_h else 0
    if m == 0:
        return local.new_zeros((0, k))
    pad = local.new_zeros((m, k))
    pad[: local.shape[0]] = local
    out = local.new_empty((world * m, k))
    dist.all_gather_into_tensor(out, pad, group=group)
    return torch.cat([out[r * m: r * m + c] for r, c in enumerate(counts_h)], dim=0)


UNIT_WORDS = 3 + 4096 * 5  # packed unit row: key int3 | tsdf f32 | weight f32 | colour f32 x3 (bit patterns)
UNIT_WORDS_C64 = 3 + 4096 * 8  # the same with float64 colours (colour precision 64)


def pack_units(keys, tsdf, weight, color):
    """export_units' arrays -> one int32 row per unit (float fields carried as raw bits, so the exchange is exact)."""
    import torch

    n = keys.shape[0]
    parts = [keys.reshape(n, 3).to(torch.int32), tsdf.reshape(n, 4096).view(torch.int32),
             weight.reshape(n, 4096).view(torch.int32), color.reshape(n, 4096 * 3).view(torch.int32)]
    return torch.cat(parts, 1)


def unpack_units(rows):
    """Inverse of pack_units; the row width tells float32 from float64 colours."""
    import torch

    n = rows.shape[0]
    f = rows[:, 3:].contiguous().view(torch.float32)
    # a fresh buffer: .contiguous() would keep a one-row (or empty) slice at its odd int32 offset / stride
    c = rows[:, 3 + 8192:].clone(memory_format=torch.contiguous_format)
    c = c.view(torch.float64) if rows.shape[1] == UNIT_WORDS_C64 else c.view(torch.float32)
    return rows[:, :3].contiguous(), f[:, :4096].contiguous(), f[:, 4096:8192].contiguous(), c.view(n, 4096, 3)


def assemble_sharded_volume(volume, group=None):
    """Spatial sharding of one object: every rank integrated the same frames into a volume created
    with set_shard(rank, world); this all-gathers the ranks' units (one RCCL all-gather of packed unit rows) and
    imports them into one fresh volume on every rank, bit-identical to an unsharded volume -- the input of
    extract_triangle_mesh, which needs neighbouring units across shard borders."""
    from .pipelines.integration import ScalableTSDFVolume

    rows = all_gather_rows(pack_units(*volume.export_units()), group)
    merged = ScalableTSDFVolume(volume.voxel_length, volume.sdf_trunc, color_type=volume.color_type,
                                volume_unit_resolution=volume.volume_unit_resolution,
                                depth_sampling_stride=volume.depth_sampling_stride,
                                max_units=max(32768, int(rows.shape[0])), color_precision=volume.color_precision)
    merged.import_units(*unpack_units(rows))
    return merged


BORDER_VOX = 721  # low-face voxels per unit (tsdf.h)


def pack_border(keys, tsdf, weight, color):
    """export_border's arrays -> one int32 row per unit (floats as raw bits: the exchange is exact)."""
    import torch

    n = keys.shape[0]
    return torch.cat([keys.reshape(n, 3).to(torch.int32), tsdf.reshape(n, BORDER_VOX).view(torch.int32),
                      weight.reshape(n, BORDER_VOX).view(torch.int32),
                      color.reshape(n, BORDER_VOX * 3).contiguous().view(torch.int32)], 1)


def unpack_border(rows):
    """Inverse of pack_border; the row width tells float32 from float64 colours."""
    import torch

    n = rows.shape[0]
    f = rows[:, 3:3 + 2 * BORDER_VOX].contiguous().view(torch.float32)
    # a fresh buffer: .contiguous() would keep a one-row (or empty) slice at its odd int32 offset / stride
    c = rows[:, 3 + 2 * BORDER_VOX:].clone(memory_format=torch.contiguous_format)
    c = c.view(torch.float64) if rows.shape[1] == 3 + BORDER_VOX * 8 else c.view(torch.float32)
    return (rows[:, :3].contiguous(), f[:, :BORDER_VOX].contiguous(), f[:, BORDER_VOX:].contiguous(),
            c.reshape(n, BORDER_VOX, 3))


def merge_shard_meshes(parts):
    """Shards' marching-cubes outputs -> the unsharded volume's mesh, bit for bit.  parts: per shard
    (V (n,3) f64, VC (n,3) f64 or None, T (m,3) int32, vertex keys (n,4) int32, triangle unit keys (m,3) int32).
    A vertex is identified by its edge (owner unit key, edge bit): shards that both reference an edge computed it
    from the same voxels with the same expression, so duplicates are identical and one is kept.  Vertices come out
    in the canonical order (unit key, local voxel, axis), triangles in (unit key, voxel, table order) -- every
    unit's triangles come from its one owner, already in that order."""
    import torch

    V = torch.cat([p[0] for p in parts])
    VC = torch.cat([p[1] for p in parts]) if parts[0][1] is not None else None
    vk = torch.cat([p[3] for p in parts]).to(torch.int64)
    tk = torch.cat([p[4] for p in parts]).to(torch.int64)
    # unit ordinals over every key that appears (lexicographic = the volume's packed-key order)
    units, inv = torch.unique(torch.cat([vk[:, :3], tk]), dim=0, sorted=True, return_inverse=True)
    vo, to = inv[:vk.shape[0]], inv[vk.shape[0]:]
    ekey = vo * (4096 * 3) + vk[:, 3]  # (unit ordinal, edge bit): the canonical vertex order
    uniq, vmap = torch.unique(ekey, sorted=True, return_inverse=True)
    first = torch.full((uniq.shape[0],), ekey.shape[0], dtype=torch.int64, device=ekey.device)
    first.scatter_reduce_(0, vmap, torch.arange(ekey.shape[0], device=ekey.device), reduce="amin")
    Vm = V[first]
    VCm = VC[first] if VC is not None else None
    # triangles: shard-local vertex ids -> merged ids; units in key order, each unit's block kept as emitted
    offs, tris = 0, []
    for p in parts:
        tris.append(vmap[offs + p[2].to(torch.int64)])
        offs += p[0].shape[0]
    Tm = torch.cat(tris)
    order = torch.sort(to, stable=True).indices
    return Vm, VCm, Tm[order].to(torch.int32)


def exchange_rows(rows, dest_mask, group=None):
    """Send each row to the ranks whose bit is set in its dest_mask (int64 bitmask per row) and return the rows this
    rank receives, grouped by source rank (one all_to_all of counts, one all_to_all of rows: RCCL on nccl, through host
    memory on gloo).  Single process: nothing to exchange."""
    import torch
    import torch.distributed as dist

    if not dist.is_initialized():
        return rows[:0]
    if dist.get_backend(group) == "gloo" and rows.is_cuda:  # gloo collectives run through host memory
        return exchange_rows(rows.cpu(), dest_mask.cpu(), group).to(rows.device)
    world = dist.get_world_size(group)
    idx = [torch.nonzero((dest_mask >> r) & 1).flatten() for r in range(world)]
    send = torch.cat([rows[i] for i in idx]) if rows.shape[0] else rows
    splits = torch.tensor([int(i.numel()) for i in idx], dtype=torch.int64, device=rows.device)
    rsplits = torch.empty_like(splits)
    dist.all_to_all_single(rsplits, splits, group=group)
    rs = rsplits.cpu().tolist()
    out = rows.new_empty((sum(rs), rows.shape[1]))
    dist.all_to_all_single(out, send.contiguous(), output_split_sizes=rs, input_split_sizes=splits.cpu().tolist(),
                           group=group)
    return out


def extract_sharded_mesh(volume, group=None):
    """Marching cubes of ONE object whose volume is spatially sharded over the ranks (ot_tsdf_set_shard), with a
    border halo instead of whole units: every rank sends its border rows (721 low-face voxels per unit,
    ~1/5.7 of a unit) only to the ranks owning one of the unit's -x/-y/-z neighbours (ot_tsdf_border_destinations;
    ownership is by blocks of units, so most neighbours are local), imports the ones its own units' cubes read (halo
    units), extracts the own units' cubes, and the partial meshes are all-gathered and merged (merge_shard_meshes)
    into the unsharded volume's mesh on every rank.  Returns (TriangleMesh, bytes of border rows this rank
    received)."""
    import torch

    from .geometry import TriangleMesh, _Arr

    keys, tsdf, weight, color = volume.export_border()
    rows = pack_border(keys, tsdf, weight, color)
    allrows = exchange_rows(rows, volume.border_destinations(keys), group)
    volume.import_border(*unpack_border(allrows))
    mesh, vk, tk = volume.extract_triangle_mesh(with_keys=True)
    V = mesh._v.dev()
    VC = mesh._vc.dev() if mesh._vc is not None else torch.zeros_like(V)
    T = mesh._t.dev()
    vrows = torch.cat([V.view(torch.int32), VC.view(torch.int32), vk], 1)  # 6 + 6 + 4 int32 per vertex
    trows = torch.cat([T, tk], 1)
    av = all_gather_rows(vrows, group)
    at = all_gather_rows(trows, group)
    nv = all_gather_rows(torch.tensor([[V.shape[0], T.shape[0]]], dtype=torch.int64, device=V.device), group)
    parts, ov, ot = [], 0, 0
    for r in range(nv.shape[0]):
        a, b = int(nv[r, 0]), int(nv[r, 1])
        vr, tr = av[ov:ov + a], at[ot:ot + b]
        parts.append((vr[:, :6].contiguous().view(torch.float64), vr[:, 6:12].contiguous().view(torch.float64),
                      tr[:, :3].contiguous(), vr[:, 12:].contiguous(), tr[:, 3:].contiguous()))
        ov, ot = ov + a, ot + b
    Vm, VCm, Tm = merge_shard_meshes(parts)
    out = TriangleMesh()
    out._v = _Arr(dev=Vm)
    out._t = _Arr(dev=Tm)
    if mesh._vc is not None:
        out._vc = _Arr(dev=VCm)
    return out, int(allrows.numel()) * 4


def all_gather_rows_capped(local, capacity, group=None):
    """all_gather_rows in ONE collective when every rank knows a common bound on the rows (capacity): each rank sends
    [capacity + 1, k] float64 rows -- row 0 carries its row count in-band (exact below 2^53), the rest its rows
    zero-padded -- so there is no separate count exchange and no host read between two collectives; one read of the
    world's counts afterwards trims the padding.  A rank above the bound raises (the bound is the caller's contract:
    no rank could otherwise learn that another one fell back)."""
    import torch
    import torch.distributed as dist

    if not dist.is_initialized():
        return local
    if dist.get_backend(group) == "gloo" and local.is_cuda:  # gloo collectives run through host memory
        return all_gather_rows_capped(local.cpu(), capacity, group).to(local.device)
    world = dist.get_world_size(group)
    n, k = int(local.shape[0]), int(local.shape[1])
    cap = int(capacity)
    if n > cap:
        raise ValueError(f"all_gather_rows_capped: {n} rows exceed the capacity {cap}")
    buf = local.new_zeros((cap + 1, k), dtype=torch.float64)
    buf[0, 0] = float(n)
    buf[1:n + 1] = local
    out = local.new_empty((world * (cap + 1), k), dtype=torch.float64)
    dist.all_gather_into_tensor(out, buf, group=group)
    out = out.view(world, cap + 1, k)
    counts = out[:, 0, 0].cpu().tolist()
    return torch.cat([out[r, 1:int(c) + 1] for r, c in enumerate(counts)], dim=0)


def merge_object_clouds(local_clouds, group=None, capacity=None):
    """Rank-ordered concatenation of this rank's object clouds with everyone else's (points only: colours are
    repainted uniformly by the hybrid map, hybrid_map.py:88).  capacity: a bound on any rank's total rows that every
    rank knows (objects per rank x samples per object): then one collective with the counts in-band
    (all_gather_rows_capped) instead of a count exchange, a host read and a second collective."""
    import torch

    dev = local_clouds[0].device if local_clouds else None
    if dev is None:
        import torch.distributed as dist

        dev = torch.device("cuda", torch.cuda.current_device()) if (not dist.is_initialized() or
                                                                   dist.get_backend(group) == "nccl") else \
            torch.device("cpu")
    local = torch.cat(local_clouds, 0) if local_clouds else torch.zeros((0, 3), dtype=torch.float64, device=dev)
    if capacity is not None and capped_fits(capacity, 3, group):
        return all_gather_rows_capped(local.to(torch.float64), capacity, group)
    return all_gather_rows(local.to(torch.float64), group)


# ONE padded collective only while the padded gather stays small: every rank receives world x (capacity + 1)
# rows, so at 8 ranks x 100k-row bounds (19 MB) the padding costs ~0.17 ms over xGMI against ~0.05 ms for a count
# exchange + host read + a tight gather of the real ~6.7k rows per object
CAPPED_MAX_BYTES = 4 << 20


def capped_fits(capacity, k, group=None):
    """whether all_gather_rows_capped's padded gather (world x (capacity + 1) x k float64) is under CAPPED_MAX_BYTES"""
    import torch.distributed as dist

    world = dist.get_world_size(group) if dist.is_initialized() else 1
    return world * (int(capacity) + 1) * int(k) * 8 <= CAPPED_MAX_BYTES


def reconstruct_and_merge(cfg, yaml_file=None, pgm_file=None, save_path=None, objects=None, o3d=None, streams=2):
    """configs[3]/[4] driver: every rank reconstructs its shard of the objects on its own GPU (integrate ->
    extract -> normals -> sample 100k -> Z mask, reconstruct_rgbd_filter.py:60-141), then the filtered clouds
    are all-gathered; rank 0 builds and writes the hybrid map (map cloud first, then objects in sorted order).
    `streams` objects of a rank are reconstructed concurrently (host threads, each with its own HIP stream:
    one object's file decoding and mesh kernels overlap another's integration); the clouds keep sorted order.
    Returns the merged point array on rank 0 (None elsewhere)."""
    import importlib

    import torch
    import torch.distributed as dist

    pkg = __package__
    R = importlib.import_module(pkg + ".reconstruct")
    o3d = o3d or importlib.import_module(pkg)
    rank, world = dist.get_rank(), dist.get_world_size()
    labels = R.get_unique_object_names(cfg) if objects is None else sorted(objects)
    mine = shard(labels, rank, world)
    T = max(1, min(int(streams), len(mine)))
    if T == 1:
        results = [_reconstruct_points(R, cfg, label, o3d) for label in mine]
    else:
        from concurrent.futures import ThreadPoolExecutor

        streams_ = importlib.import_module(pkg + ".streams").worker_streams(T)

        def work(t):
            s = streams_[t]
            out = {}
            with torch.cuda.stream(s):
                for j in range(t, len(mine), T):
                    out[j] = _reconstruct_points(R, cfg, mine[j], o3d)
                s.synchronize()
            return out

        done = {}
        with ThreadPoolExecutor(max_workers=T) as ex:
            for part in ex.map(work, range(T)):
                done.update(part)
        results = [done[j] for j in range(len(mine))]
    clouds = [pts for pts in results if pts is not None]
    # every rank's objects: ceil(len(labels) / world) at most, each <= n_samples points after the Z mask
    cap = ((len(labels) + world - 1) // world) * int(cfg.n_samples)
    merged = merge_object_clouds(clouds, capacity=cap)
    if rank != 0:
        return None
    objs = o3d.geometry.PointCloud()
    objs.points = merged
    if len(objs.points):
        objs.paint_uniform_color([1.0, 0.0, 0.0])
    out = objs
    if yaml_file and pgm_file:
        hm = importlib.import_module(pkg + ".hybrid_map")
        map_pcd = hm.create_map_cloud(yaml_file, pgm_file, o3d)
        if map_pcd is not None:
            out = map_pcd + objs if len(objs.points) else map_pcd
    if save_path:
        os.makedirs(os.path.dirname(os.path.abspath(save_path)), exist_ok=True)
        o3d.io.write_point_cloud(save_path, out)
    return np.asarray(out.points)


def _reconstruct_points(R, cfg, label, o3d):
    """In-memory variant of reconstruct_object(output="points") returning the filtered points as a device
    tensor (no PLY round trip: the reference's float64 PLY write/read is lossless)."""
    colors, depths, poses = R._frame_lists(cfg, label)
    if not colors:
        return None
    intrinsic = R._intrinsic(o3d, cfg)
    volume = R._new_volume(o3d, cfg)
    for i in range(len(colors)):
        try:
            R._integrate_frame(o3d, cfg, volume, intrinsic, colors, depths, poses, i)
        except Exception:
            pass
    fused = getattr(volume, "extract_mesh_and_sample_min_z", None)
    if fused is not None:  # extract, normals, sample_points_uniformly + the Z mask (:112-132) in one host call
        _mesh, cloud = fused(cfg.n_samples, cfg.z_filter, cfg.sample_seed)
        return None if cloud is None else cloud._xyz.dev()
    mesh = volume.extract_triangle_mesh()
    mesh.compute_vertex_normals()
    if R._mesh_empty(mesh):  # reference: len(mesh.vertices) == 0, without a writable host view
        return None
    return mesh.sample_points_min_z(cfg.n_samples, cfg.z_filter, cfg.sample_seed)._xyz.dev()
