"""open3d.utility counterparts: Vector3dVector / Vector3iVector / Vector2iVector / IntVector.

Open3D's vectors are views over std::vector<Eigen::Vector3d>; here they are thin wrappers over a host numpy
array that `np.asarray(...)` returns without a copy (reconstruct_rgbd_filter.py:126-132 relies on that).
Constructing one from caller data copies it, as Open3D does (pybind11 builds a new std::vector); the geometry
getters wrap their own host array without a copy (_view) and drop the device copy, so in-place edits through
np.asarray(pcd.points) reach the next GPU call.
"""
from __future__ import annotations

import numpy as np


class _VecN:
    _dtype = np.float64
    _cols = 3

    def __init__(self, data=None):
        if data is None:
            self._a = np.zeros((0, self._cols), self._dtype)
        else:
            a = np.array(data, dtype=self._dtype, copy=True)
            if a.size == 0:
                a = a.reshape(0, self._cols)
            if a.ndim != 2 or a.shape[1] != self._cols:
                raise RuntimeError(f"{type(self).__name__} expects an (N, {self._cols}) array, got {a.shape}")
            self._a = np.ascontiguousarray(a)

    @classmethod
    def _view(cls, arr):
        """Wrap an existing (N, cols) array without copying (geometry getters)."""
        v = cls.__new__(cls)
        v._a = arr
        return v

    def __array__(self, dtype=None, copy=None):
        return self._a if dtype is None else self._a.astype(dtype)

    def __len__(self):
        return self._a.shape[0]

    def __getitem__(self, i):
        return self._a[i]

    def __setitem__(self, i, v):
        self._a[i] = v

    def __iter__(self):
        return iter(self._a)

    def __repr__(self):
        return f"std::vector<Eigen::Vector{self._cols}{'d' if self._dtype == np.float64 else 'i'}> with {len(self)} elements."


class Vector3dVector(_VecN):
    _dtype = np.float64
    _cols = 3


class Vector3iVector(_VecN):
    _dtype = np.int32
    _cols = 3


class Vector2iVector(_VecN):
    _dtype = np.int32
    _cols = 2


class IntVector(list):
    pass


class DoubleVector(np.ndarray):
    """open3d.utility.DoubleVector: a float64 vector (numpy view; np.mean / np.asarray work unchanged)."""

    def __new__(cls, data=()):
        return np.ascontiguousarray(np.asarray(data, dtype=np.float64).reshape(-1)).view(cls)


class VerbosityLevel:
    Error = 0
    Warning = 1
    Info = 2
    Debug = 3


def set_verbosity_level(level):
    return None
