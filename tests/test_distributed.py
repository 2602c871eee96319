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
    q.put((rank, merged.numpy()))
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
    out = dict(q.get(timeout=120) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    exp = _expected(sizes)
    for r in range(2):
        assert np.array_equal(out[r], exp)


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
