"""Multi-rank logic on CPU (gloo, world_size 2): object sharding keeps sorted order across ranks, and the
padded all-gather merge reproduces the rank-ordered concatenation bit for bit (ragged and empty ranks)."""
import importlib
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG, ROOT


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, sizes, q):
    import sys

    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    D = importlib.import_module(PKG + ".distributed")
    rng = np.random.default_rng(rank)
    clouds = [torch.from_numpy(rng.standard_normal((n, 3))) for n in sizes[rank]]
    merged = D.merge_object_clouds(clouds)
    capped = D.merge_object_clouds(clouds, capacity=max(sum(ns) for ns in sizes) + 1)  # one collective, counts in-band
    q.put((rank, merged.numpy(), capped.numpy()))
    dist.barrier()
    dist.destroy_process_group()


def _expected(sizes):
    parts = []
    for r, ns in enumerate(sizes):
        rng = np.random.default_rng(r)
        parts += [rng.standard_normal((n, 3)) for n in ns]
    return np.concatenate(parts) if parts else np.zeros((0, 3))


@pytest.mark.parametrize("sizes", [[[5, 3], [7]], [[0], [4, 1]], [[], [2]]])
def test_all_gather_merge_gloo(sizes):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, sizes, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(2):
        r, merged, capped = q.get(timeout=120)
        out[r] = (merged, capped)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    exp = _expected(sizes)
    for r in range(2):
        assert np.array_equal(out[r][0], exp)
        assert np.array_equal(out[r][1], exp)


def test_shard_contiguous_sorted():
    D = importlib.import_module(PKG + ".distributed")
    labels = [f"Object_{i}" for i in range(11)]
    for world in (1, 2, 3, 4, 8):
        parts = [D.shard(labels, r, world) for r in range(world)]
        assert sum(parts, []) == labels
        assert max(map(len, parts)) - min(map(len, parts)) <= 1


def _unit_worker(rank, world, port, sizes, q):
    import sys

    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    D = importlib.import_module(PKG + ".distributed")
    k, t, w, c = _fake_units(rank, sizes[rank])
    rows = D.all_gather_rows(D.pack_units(k, t, w, c))
    q.put((rank, [a.numpy() for a in D.unpack_units(rows)]))
    dist.barrier()
    dist.destroy_process_group()


def _fake_units(seed, n):
    rng = np.random.default_rng(seed + 100)
    keys = torch.from_numpy(rng.integers(-500, 500, (n, 3)).astype(np.int32))
    bits = rng.integers(0, 2 ** 32, (n, 4096 * 5), dtype=np.uint64).astype(np.uint32).view(np.float32)
    f = torch.from_numpy(bits.copy())  # arbitrary bit patterns (NaN payloads, -0, denormals) must survive
    return keys, f[:, :4096].contiguous(), f[:, 4096:8192].contiguous(), f[:, 8192:].contiguous().view(n, 4096, 3)


@pytest.mark.parametrize("sizes", [[3, 5], [0, 2]])
def test_sharded_unit_exchange_gloo(sizes):
    """assemble_sharded_volume's exchange: packed unit rows all-gathered over 2 ranks unpack to the rank-ordered
    concatenation of every field, bit for bit."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_unit_worker, args=(r, 2, port, sizes, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    exp = [np.concatenate([_fake_units(r, sizes[r])[i].numpy() for r in range(2)]) for i in range(4)]
    for r in range(2):
        for got, e in zip(out[r], exp):
            assert got.shape == e.shape and np.array_equal(got.view(np.uint32) if got.dtype == np.float32 else got,
                                                           e.view(np.uint32) if e.dtype == np.float32 else e)


def test_merge_shard_meshes_cpu():
    """distributed.merge_shard_meshes on a synthetic canonical mesh split by unit ownership (CPU tensors): shared
    vertices appear in several shards and are kept once, vertices and triangles come out in canonical order."""
    import importlib

    import torch

    D = importlib.import_module("object-triggered-3d-slam_amd.distributed")
    g = torch.Generator().manual_seed(0)
    units = torch.tensor([[-1, 0, 2], [0, 0, 0], [0, 0, 1], [0, 1, 0], [1, -2, 0], [1, 0, 0]], dtype=torch.int64)
    # canonical vertices: sorted (unit, bit) keys
    vu = torch.randint(0, units.shape[0], (400,), generator=g)
    vb = torch.randint(0, 4096 * 3, (400,), generator=g)
    key = torch.unique(vu * 12288 + vb)
    vu, vb = key // 12288, key % 12288
    n = key.shape[0]
    V = torch.randn(n, 3, dtype=torch.float64, generator=g)
    VC = torch.rand(n, 3, dtype=torch.float64, generator=g)
    vk = torch.cat([units[vu], vb[:, None]], 1).to(torch.int32)
    # triangles grouped by unit (canonical), each referencing random vertices
    tu = torch.sort(torch.randint(0, units.shape[0], (300,), generator=g)).values
    T = torch.randint(0, n, (300, 3), generator=g).to(torch.int32)
    used = torch.unique(T.flatten().long())
    keep = torch.zeros(n, dtype=torch.bool)
    keep[used] = True
    # reference: only referenced vertices survive (MC emits exactly the referenced edges)
    remap = torch.full((n,), -1, dtype=torch.int64)
    remap[used] = torch.arange(used.shape[0])
    Vr, VCr, Tr = V[used], VC[used], remap[T.long()].to(torch.int32)
    parts = []
    for shard in range(3):
        mine = (tu % 3) == shard
        Ts = T[mine].long()
        loc = torch.unique(Ts.flatten())
        lmap = torch.full((n,), -1, dtype=torch.int64)
        lmap[loc] = torch.arange(loc.shape[0])
        parts.append((V[loc], VC[loc], lmap[Ts].to(torch.int32), vk[loc], units[tu[mine]].to(torch.int32)))
    Vm, VCm, Tm = D.merge_shard_meshes(parts)
    assert torch.equal(Vm, Vr) and torch.equal(VCm, VCr) and torch.equal(Tm, Tr)


@pytest.mark.parametrize("n", [0, 1, 2])
@pytest.mark.parametrize("wide", [False, True])
def test_pack_unpack_rows_small(n, wide):
    """pack/unpack of unit and border rows with 0, 1 and 2 rows, float32 and float64 colours, arbitrary bit
    patterns: a one-row slice counts as contiguous at its odd int32 column offset, so the float64 colours must be
    copied out before the dtype view (round 6: a 4-rank halo exchange delivered exactly one row)."""
    D = importlib.import_module(PKG + ".distributed")
    rng = np.random.default_rng(n)
    cdt = np.uint64 if wide else np.uint32

    def bits(shape, dt):
        return torch.from_numpy(rng.integers(0, 2 ** 63, shape, dtype=np.uint64).astype(dt).view(
            np.float64 if dt == np.uint64 else np.float32).copy())

    keys = torch.from_numpy(rng.integers(-500, 500, (n, 3)).astype(np.int32))
    for vox, pack, unpack in ((4096, D.pack_units, D.unpack_units), (D.BORDER_VOX, D.pack_border, D.unpack_border)):
        t, w, c = bits((n, vox), np.uint32), bits((n, vox), np.uint32), bits((n, vox, 3), cdt)
        k2, t2, w2, c2 = unpack(pack(keys, t, w, c))
        assert torch.equal(k2, keys) and c2.dtype == c.dtype and c2.shape == c.shape
        for x, y in ((t2, t), (w2, w), (c2, c)):
            assert np.array_equal(x.numpy().view(np.uint8), y.numpy().view(np.uint8))
