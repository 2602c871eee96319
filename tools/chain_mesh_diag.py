"""Exact float64 chains (otx_serial_chain_f64) on a real configs[3] object mesh: the sampling's area sum and CDF
chains over the triangle areas of object_scene(0) (64 frames, 5 mm) -- serial-chunk count and time.  Tool only."""
import ctypes as C
import importlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "object-triggered-3d-slam_amd"
synth = importlib.import_module(PKG + ".synth")
depth, color, ext = synth.make_sequence(synth.object_scene(0), n_frames=64)
import torch

pkg = importlib.import_module(PKG)
L = importlib.import_module(PKG + "._lib")
integ = pkg.pipelines.integration
intr = pkg.camera.PinholeCameraIntrinsic(*synth.REF_INTRINSICS_640)
vol = integ.ScalableTSDFVolume(voxel_length=0.005, sdf_trunc=0.04, color_type=integ.TSDFVolumeColorType.RGB8)
for k in range(64):
    vol.integrate(pkg.geometry.RGBDImage.create_from_color_and_depth(
        pkg.geometry.Image(color[k]), pkg.geometry.Image(depth[k]), convert_rgb_to_intensity=False), intr, ext[k])
mesh = vol.extract_triangle_mesh()
V, T = mesh._v.dev(), mesh._t.dev().long()
p0, p1, p2 = V[T[:, 0]], V[T[:, 1]], V[T[:, 2]]
x, y = p0 - p1, p0 - p2
cr = torch.stack([x[:, 1] * y[:, 2] - x[:, 2] * y[:, 1], x[:, 2] * y[:, 0] - x[:, 0] * y[:, 2],
                  x[:, 0] * y[:, 1] - x[:, 1] * y[:, 0]], 1)
areas = (0.5 * torch.sqrt((cr * cr).sum(1))).contiguous()
cases = {"areas": areas, "cdf": (areas / areas.sum()).contiguous()}
s_ = C.c_void_p(torch.cuda.current_stream().cuda_stream)
for name, d in cases.items():
    out = torch.empty_like(d)
    for cdf in (0, 1):
        ser = C.c_int64(0)
        L.call("otx_serial_chain_f64", C.c_void_p(d.data_ptr()), d.shape[0], cdf, C.c_void_p(out.data_ptr()), C.byref(ser), s_)
        ts = []
        for _ in range(7):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            L.call("otx_serial_chain_f64", C.c_void_p(d.data_ptr()), d.shape[0], cdf, C.c_void_p(out.data_ptr()), None, s_)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        print(f"{name:6s} cdf={cdf} n={d.shape[0]} chunks={(d.shape[0] + 255) // 256} serial={ser.value} "
              f"ms={np.median(ts) * 1e3:.3f}", flush=True)
