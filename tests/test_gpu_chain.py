"""GPU parity of the float64 running sums inside SamplePointsUniformly (Open3D GetSurfaceArea and the area CDF,
reconstruct_rgbd_filter.py:123 / Appendix A.8).  The GPU computes them with the binade-wise integer prefix scan
(mesh_ops.hip, k_chain_*); the oracle here is the strict left-to-right loop: numpy.cumsum (a sequential
np.add.accumulate, x_t + s_{t-1}) for every prefix, its last element for the sum.  Bit-exact on inputs built to hit
every escape path: leading zeros, ties (x / ulp(s) = k + 1/2 on every step), wide dynamic ranges, binade
crossings at chunk and wave-group boundaries, NaN / inf, values past the fast path's exponent range."""
import ctypes as C

import numpy as np
import pytest
import torch

from conftest import assert_bitwise

pytestmark = pytest.mark.gpu


def _chain(pkg, x, cdf):
    L = pkg._lib
    d = torch.from_numpy(np.ascontiguousarray(x, np.float64)).cuda()
    out = torch.empty(d.shape[0] if cdf else 1, dtype=torch.float64, device="cuda")
    L.call("otx_serial_chain_f64", C.c_void_p(d.data_ptr()), d.shape[0], int(cdf), C.c_void_p(out.data_ptr()), None,
           C.c_void_p(torch.cuda.current_stream().cuda_stream))
    return out.cpu().numpy()


def _cases():
    rng = np.random.default_rng(7)
    tie = np.concatenate([[1.0], (2 * rng.integers(0, 1 << 10, 50000) + 1) * 2.0 ** -53])  # every add a tie
    half = np.concatenate([[1.0], rng.integers(0, 1 << 12, 70000) * 2.0 ** -53])  # ties on odd values
    lz = np.concatenate([np.zeros(1000), rng.random(300001)])
    zint = rng.random(200000)
    zint[rng.random(200000) < 0.3] = 0.0
    wide = np.exp(rng.normal(0.0, 6.0, 250000))  # ~17 binades either side
    grow = np.exp(np.linspace(-700, 600, 40000))  # past 1e300: fast path ends, serial from there
    nan = rng.random(100000)
    nan[54321] = np.nan
    inf = rng.random(70000)
    inf[40000] = np.inf
    desc = np.sort(rng.random(120000) ** 8)[::-1].copy()
    mesh_like = rng.gamma(2.0, 1e-5, 1 << 20)
    return {
        "uniform_1M": rng.random(1000003), "tiny_1": np.array([0.3]), "n_257": rng.random(257),
        "group_edge": rng.random(256 * 64 + 1), "ties_all": tie, "ties_half": half, "leading_zeros": lz,
        "zeros_mixed": zint, "wide_range": wide, "past_1e300": grow, "nan": nan, "inf": inf,
        "descending": desc, "mesh_like": mesh_like, "cdf_like": mesh_like / mesh_like.sum(),
    }


@pytest.mark.parametrize("name", list(_cases().keys()))
def test_chain_bitexact(pkg, gpu, name):
    x = _cases()[name]
    ref = np.cumsum(x)
    got = _chain(pkg, x, True)
    if np.isnan(ref).any():
        assert np.array_equal(np.isnan(got), np.isnan(ref))
        m = ~np.isnan(ref)
        assert_bitwise(got[m], ref[m], f"chain prefix {name}")
    else:
        assert_bitwise(got, ref, f"chain prefix {name}")
    s = _chain(pkg, x, False)[0]
    assert (np.isnan(s) and np.isnan(ref[-1])) or s.view(np.uint64) == ref[-1:].view(np.uint64)[0], name


def test_surface_area_bitexact(pkg, O, synth, gpu):
    rng = np.random.default_rng(3)
    V = rng.random((5000, 3)) * 0.3
    T = rng.integers(0, 5000, (300000, 3)).astype(np.int32)
    T[:7] = 0  # degenerate triangles: exact zero areas first
    mesh = pkg.geometry.TriangleMesh(pkg.utility.Vector3dVector(V), pkg.utility.Vector3iVector(T))
    a = mesh.get_surface_area()
    assert np.float64(a).view(np.uint64) == np.float64(O.surface_area(V, T)).view(np.uint64)
    empty = pkg.geometry.TriangleMesh()
    assert empty.get_surface_area() == 0.0
