"""Marching-cubes tables (include/otslam_mc_tables.h): edge sets match the sign configuration, and the
triangulation is watertight and consistently oriented on random closed fields (an error in any of the 256
rows shows up as an unmatched directed edge)."""
import os
import re
from collections import Counter

import numpy as np

from conftest import ROOT

SHIFT = [(0, 0, 0), (1, 0, 0), (1, 1, 0), (0, 1, 0), (0, 0, 1), (1, 0, 1), (1, 1, 1), (0, 1, 1)]
E2V = [(0, 1), (1, 2), (3, 2), (0, 3), (4, 5), (5, 6), (7, 6), (4, 7), (0, 4), (1, 5), (2, 6), (3, 7)]
ESHIFT = [(0, 0, 0, 0), (1, 0, 0, 1), (0, 1, 0, 0), (0, 0, 0, 1), (0, 0, 1, 0), (1, 0, 1, 1), (0, 1, 1, 0),
          (0, 0, 1, 1), (0, 0, 0, 2), (1, 0, 0, 2), (1, 1, 0, 2), (0, 1, 0, 2)]


def _tri_table():
    src = open(os.path.join(ROOT, "include", "otslam_mc_tables.h")).read()
    body = src[src.index("OT_MC_TRI_TABLE"):]
    body = body[body.index("{") + 1:]
    rows = re.findall(r"\{([-\d, ]+)\}", body)
    out = []
    for r in rows:
        v = [int(x) for x in r.split(",") if x.strip()]
        assert v[-1] == -1
        out.append(v[:-1])
    return out


def test_table_shape_and_edges():
    tri = _tri_table()
    assert len(tri) == 256
    for c in range(256):
        assert len(tri[c]) % 3 == 0 and len(tri[c]) <= 15
        cut = {e for e in range(12) if ((c >> E2V[e][0]) & 1) != ((c >> E2V[e][1]) & 1)}
        assert set(tri[c]) == cut, c


def test_watertight_on_random_fields():
    tri = _tri_table()
    rng = np.random.default_rng(0)
    for _ in range(3):
        N = 10
        f = rng.standard_normal((N, N, N))
        f[0], f[-1], f[:, 0], f[:, -1], f[:, :, 0], f[:, :, -1] = 1, 1, 1, 1, 1, 1
        de = Counter()
        for x in range(N - 1):
            for y in range(N - 1):
                for z in range(N - 1):
                    c = sum(1 << i for i, s in enumerate(SHIFT) if f[x + s[0], y + s[1], z + s[2]] < 0)
                    t = tri[c]
                    keys = [(x + ESHIFT[e][0], y + ESHIFT[e][1], z + ESHIFT[e][2], ESHIFT[e][3]) for e in t]
                    for k in range(0, len(t), 3):
                        a, b, cc = keys[k], keys[k + 2], keys[k + 1]  # Open3D winding (0, 2, 1)
                        for u, v in ((a, b), (b, cc), (cc, a)):
                            de[(u, v)] += 1
        assert de
        assert all(de.get((v, u), 0) == n for (u, v), n in de.items())
        assert all(n == 1 for n in de.values())
