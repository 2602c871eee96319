"""GPU parity: PointCloud.compute_point_cloud_distance (eval_cone.py:99,103 — accuracy / completeness).

Bit-exact against the oracle's exhaustive float64 1-NN minimum on the same inputs: clouds from a synthetic frame
(surface-like), the same cloud displaced far outside the target's bounding box (ring-expansion + exhaustive
fallback paths), queries in empty cells inside the box, and the empty cases (Open3D: 0.0 when no neighbour)."""
import numpy as np
import pytest

from conftest import assert_bitwise, ref_intr

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def clouds(O, synth, seq16, gpu):
    depth, color, ext = seq16
    intr = ref_intr(synth)
    a = O.unproject(O.depth_to_float(depth[0], 1000.0, 5.0), color[0], intr, ext[0])[0]
    b = O.unproject(O.depth_to_float(depth[1], 1000.0, 5.0), color[1], intr, ext[1])[0]
    a = O.voxel_down_sample(a, None, 0.02)[0]
    b = O.voxel_down_sample(b, None, 0.01)[0]
    return a, b


def _pcd(pkg, xyz):
    p = pkg.geometry.PointCloud()
    p.points = pkg.utility.Vector3dVector(xyz)
    return p


def test_nn_distance_bitexact(pkg, O, clouds):
    a, b = clouds
    d = np.asarray(_pcd(pkg, a).compute_point_cloud_distance(_pcd(pkg, b)))
    assert_bitwise(d, O.point_cloud_distance(a, b), "map -> target distances")
    d2 = np.asarray(_pcd(pkg, b).compute_point_cloud_distance(_pcd(pkg, a)))
    assert_bitwise(d2, O.point_cloud_distance(b, a), "target -> map distances")
    # accuracy / completeness as the eval script computes them
    assert np.mean(d) * 100 == np.mean(O.point_cloud_distance(a, b)) * 100


def test_nn_distance_far_and_sparse_queries(pkg, O, clouds):
    a, b = clouds
    rng = np.random.default_rng(3)
    far = np.concatenate([a[:500] + np.array([3.0, -2.0, 1.5]),            # outside the target's box
                          rng.uniform(b.min(0), b.max(0), size=(2000, 3)),  # inside the box, mostly empty cells
                          rng.uniform(-50, 50, size=(20, 3))])              # very far: exhaustive fallback
    d = np.asarray(_pcd(pkg, far).compute_point_cloud_distance(_pcd(pkg, b)))
    assert_bitwise(d, O.point_cloud_distance(far, b), "far / sparse query distances")


def test_nn_distance_self_and_empty(pkg, O, clouds):
    a, _ = clouds
    assert not np.any(np.asarray(_pcd(pkg, a).compute_point_cloud_distance(_pcd(pkg, a))))
    z = np.asarray(_pcd(pkg, a[:10]).compute_point_cloud_distance(_pcd(pkg, np.zeros((0, 3)))))
    assert z.shape == (10,) and not np.any(z)
    assert len(_pcd(pkg, np.zeros((0, 3))).compute_point_cloud_distance(_pcd(pkg, a))) == 0
    one = np.asarray(_pcd(pkg, a[:64]).compute_point_cloud_distance(_pcd(pkg, a[100:101])))
    assert_bitwise(one, O.point_cloud_distance(a[:64], a[100:101]), "single-point target")
