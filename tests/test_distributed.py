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
