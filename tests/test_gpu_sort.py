"""GPU parity of the library's stable LSD radix sort (sort.hip: upsweep, scan, one decoupled-look-back scatter per
8-bit digit), which orders volume units, marching-cubes edges, voxel keys and every neighbour grid.  Oracle:
numpy's stable argsort of key & (2^end_bit - 1) -- the sort ignores bits at and above end_bit and keeps input
order among equal keys.  Sizes straddle the 2048-item tile; bit widths cover 1..64; duplicates test stability."""
import ctypes as C

import numpy as np
import pytest
import torch

from conftest import assert_bitwise

pytestmark = pytest.mark.gpu


def _sort(pkg, keys, end_bit):
    L = pkg._lib
    n = keys.shape[0]
    kin = torch.from_numpy(keys.view(np.int64)).cuda()
    vin = torch.arange(n, dtype=torch.int32, device="cuda")
    kout = torch.empty_like(kin)
    vout = torch.empty_like(vin)
    L.call("otx_sort_pairs_u64_u32", C.c_void_p(kin.data_ptr()), C.c_void_p(kout.data_ptr()),
           C.c_void_p(vin.data_ptr()), C.c_void_p(vout.data_ptr()), n, end_bit,
           C.c_void_p(torch.cuda.current_stream().cuda_stream))
    return kout.cpu().numpy().view(np.uint64), vout.cpu().numpy().view(np.uint32)


@pytest.mark.parametrize("n,end_bit,hi", [
    (1, 8, 4), (100, 8, 256), (2047, 13, 1 << 13), (2048, 16, 50), (2049, 30, 1 << 30), (100003, 30, 1 << 30),
    (1 << 20, 51, 1 << 51), (3000017, 24, 1 << 24), (250000, 64, None), (77777, 1, 2), (500000, 40, 1000),
    # 9-bit digits where they save a pass (18, 27, 36 bits)
    (2049, 18, 1 << 18), (100003, 27, 1 << 27), (500000, 36, 1 << 36),
])
def test_sort_stable_bitexact(pkg, gpu, n, end_bit, hi):
    rng = np.random.default_rng(n + end_bit)
    if hi is None:
        keys = rng.integers(0, 2 ** 63, n, dtype=np.uint64) * np.uint64(2) + rng.integers(0, 2, n, dtype=np.uint64)
    else:
        keys = rng.integers(0, hi, n, dtype=np.uint64)
    mask = np.uint64((1 << end_bit) - 1) if end_bit < 64 else np.uint64(0xFFFFFFFFFFFFFFFF)
    if end_bit < 64:  # junk above end_bit must be ignored
        junk = rng.integers(0, 2 ** 63, n, dtype=np.uint64) & ~mask
        keys = (keys & mask) | junk
    order = np.argsort(keys & mask, kind="stable")
    k, v = _sort(pkg, keys, end_bit)
    assert_bitwise(v, order.astype(np.uint32), f"sort order n={n} bits={end_bit}")
    assert_bitwise(k, keys[order], f"sorted keys n={n} bits={end_bit}")


def test_sort_presorted_and_reversed(pkg, gpu):
    n = 300000
    for keys in (np.arange(n, dtype=np.uint64), np.arange(n, dtype=np.uint64)[::-1].copy(),
                 np.zeros(n, dtype=np.uint64)):
        k, v = _sort(pkg, keys, 20)
        order = np.argsort(keys, kind="stable")
        assert_bitwise(v, order.astype(np.uint32), "sort order (structured input)")


@pytest.mark.parametrize("sizes,end_bit", [
    ([0, 1, 2047, 2048, 2049, 0, 5], 12), ([812746, 810001, 0, 799999], 28), ([100000] * 33, 32), ([3] * 64, 2),
    # 9-bit digits (3 passes for 25..27 bits, 2 for 17..18): the configs[2] voxel keys
    ([812746, 810001, 0, 799999], 27), ([0, 1, 4095, 4096, 4097, 0, 5], 25), ([100000] * 33, 18),
    # 28..30-bit keys (the cell-major configs[2] keys of 1280x720 frames)
    ([0, 1, 4095, 4096, 4097, 0, 5], 29), ([480000] * 32, 30), ([3] * 64, 28),
])
def test_segmented_sort_bitexact(pkg, gpu, sizes, end_bit):
    """sort_segments_u32_u32 (the batched configs[2] voxel sort): every segment sorted stably on its own, nothing
    crosses a boundary; vs numpy's stable argsort per segment."""
    L = pkg._lib
    rng = np.random.default_rng(sum(sizes) + end_bit)
    n = int(sum(sizes))
    seg = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    keys = rng.integers(0, 1 << end_bit, max(n, 1), dtype=np.uint64).astype(np.uint32)[:n]
    keys[: n // 3] = keys[: n // 3] % 7  # duplicates: stability
    kin = torch.from_numpy(keys.view(np.int32)).cuda()
    vin = torch.arange(n, dtype=torch.int32, device="cuda")
    kout = torch.empty_like(kin)
    vout = torch.empty_like(vin)
    L.call("otx_sort_segments_u32_u32", C.c_void_p(kin.data_ptr()), C.c_void_p(kout.data_ptr()),
           C.c_void_p(vin.data_ptr()), C.c_void_p(vout.data_ptr()), seg.ctypes.data_as(C.c_void_p), len(sizes),
           end_bit, C.c_void_p(torch.cuda.current_stream().cuda_stream))
    order = np.concatenate([seg[s] + np.argsort(keys[seg[s]:seg[s + 1]], kind="stable") for s in range(len(sizes))])
    assert_bitwise(vout.cpu().numpy().view(np.uint32), order.astype(np.uint32), "segmented sort order")
    assert_bitwise(kout.cpu().numpy().view(np.uint32), keys[order], "segmented sorted keys")
