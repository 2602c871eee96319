"""open3d.camera.PinholeCameraIntrinsic (reconstruct_rgbd_filter.py:29, check_one_frame.py:15)."""
from __future__ import annotations

import numpy as np


class PinholeCameraIntrinsicParameters:
    PrimeSenseDefault = 0
    Kinect2DepthCameraDefault = 1
    Kinect2ColorCameraDefault = 2


class PinholeCameraIntrinsic:
    def __init__(self, width=-1, height=-1, fx=None, fy=None, cx=None, cy=None, intrinsic_matrix=None):
        if isinstance(width, int) and width in (0, 1, 2) and height == -1 and fx is None:
            # PinholeCameraIntrinsic(PinholeCameraIntrinsicParameters.X)
            presets = {0: (640, 480, 525.0, 525.0, 319.5, 239.5),
                       1: (512, 424, 365.456, 365.456, 254.878, 205.395),
                       2: (1920, 1080, 1059.9718, 1059.9718, 975.7193, 545.9533)}
            width, height, fx, fy, cx, cy = presets[width]
        if intrinsic_matrix is not None:
            K = np.asarray(intrinsic_matrix, dtype=np.float64)
            fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
        self.width = int(width)
        self.height = int(height)
        self._K = np.eye(3)
        if fx is not None:
            self.set_intrinsics(self.width, self.height, fx, fy, cx, cy)

    def set_intrinsics(self, width, height, fx, fy, cx, cy):
        self.width, self.height = int(width), int(height)
        self._K = np.array([[fx, 0.0, cx], [0.0, fy, cy], [0.0, 0.0, 1.0]], dtype=np.float64)

    @property
    def intrinsic_matrix(self):
        return self._K.copy()

    @intrinsic_matrix.setter
    def intrinsic_matrix(self, K):
        self._K = np.asarray(K, dtype=np.float64).copy()

    @property
    def fx(self):
        return float(self._K[0, 0])

    @property
    def fy(self):
        return float(self._K[1, 1])

    @property
    def cx(self):
        return float(self._K[0, 2])

    @property
    def cy(self):
        return float(self._K[1, 2])

    def get_focal_length(self):
        return (self.fx, self.fy)

    def get_principal_point(self):
        return (self.cx, self.cy)

    def is_valid(self):
        return self.width > 0 and self.height > 0

    def __repr__(self):
        return f"PinholeCameraIntrinsic with width = {self.width} and height = {self.height}."
