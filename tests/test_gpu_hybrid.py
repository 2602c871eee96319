"""GPU parity of the hybrid-map builder (fusion/hybrid_map.py) against the golden output captured by running
the reference script itself (tests/golden/caller_fixture.json, hybrid_map): the occupancy-grid points come from
the ot_occupancy_to_points kernel, the merge order and colours from the restated caller — bit-exact."""
import importlib
import json
import os
import sys

import numpy as np
import pytest

from conftest import PKG, ROOT, assert_bitwise

sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import dataset  # noqa: E402

pytestmark = pytest.mark.gpu


def test_hybrid_map_bitexact(pkg, gpu, tmp_path):
    hm = importlib.import_module(PKG + ".hybrid_map")
    root = str(tmp_path)
    dataset.write_map_dataset(root)
    out = os.path.join(root, "out", "hybrid_map_selective.ply")
    merged = hm.build_hybrid_map(os.path.join(root, "map", "map_selective.yaml"),
                                 os.path.join(root, "map", "map_selective.pgm"), os.path.join(root, "objects"), out)
    ref = next(c for c in json.load(open(os.path.join(ROOT, "tests", "golden", "caller_fixture.json")))["calls"]
               ["hybrid_map"] if c["call"] == "write_point_cloud")
    assert_bitwise(np.asarray(merged.points), np.array(ref["points"]), "hybrid map points")
    assert_bitwise(np.asarray(merged.colors), np.array(ref["colors"]), "hybrid map colours")
    back = pkg.io.read_point_cloud(out)
    assert_bitwise(np.asarray(back.points), np.array(ref["points"]), "PLY round trip")
