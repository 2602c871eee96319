"""otslam-mi355x — MI355X-native drop-in for the RGB-D reconstruction / voxel-filter path of
TakiRyo/object-triggered-3D-SLAM.

The namespaces mirror the Open3D modules the reference scripts use, so a reference caller
switches with one line:

    o3d = importlib.import_module("object-triggered-3d-slam_amd")   # instead of `import open3d as o3d`

    o3d.camera.PinholeCameraIntrinsic, o3d.io.read_image / read_point_cloud / write_point_cloud / ...,
    o3d.geometry.{Image, RGBDImage, PointCloud, TriangleMesh}, o3d.utility.Vector3dVector,
    o3d.pipelines.integration.{ScalableTSDFVolume, TSDFVolumeColorType}, o3d.visualization.draw_geometries (headless)

Every compute call goes through the C ABI in include/otslam.h (libotslam_hip.so, HIP kernels for gfx950).
"""
from . import camera, change_detection, filters, geometry, io, pipelines, utility, visualization  # noqa: F401
from ._lib import LIB_PATH, OTError  # noqa: F401

__version__ = "0.1.0"


def native_library():
    """Load and return the HIP library handle (raises if it was not built)."""
    from . import _lib

    return _lib.load()
