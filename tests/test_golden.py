"""The CPU restatement reproduces the committed golden vectors (tests/golden/golden_small.npz, written by
tests/golden/gen_golden.py): any drift of the oracle between rounds or builds shows up here, on CPU."""
import os
import sys

import numpy as np

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import gen_golden as G  # noqa: E402


def test_oracle_matches_golden_vectors(O):
    g = np.load(G.OUT, allow_pickle=False)
    exp = G.expected(O, g["in_depth"], g["in_color"], g["in_ext"])
    assert set(exp) <= set(g.files)
    for k, v in exp.items():
        ref = g[k]
        if ref.dtype.kind == "U":
            assert str(v) == str(ref), k
        else:
            assert np.asarray(v).dtype == ref.dtype and np.array_equal(np.asarray(v), ref), k
