"""Phase times of one configs[3] object on one stream (integrate 64 frames -> mesh -> normals -> 100k samples ->
z mask), each phase closed by a device synchronisation: where single_object_ms goes.  Tool only."""
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
lib = L.load()
intr_t = synth.REF_INTRINSICS_640
W, H = intr_t[0], intr_t[1]
intr = L.ot_intrinsics(W, H, *intr_t[2:])
npx = W * H
d16 = torch.from_numpy(depth.view(np.int16)).cuda().view(torch.uint16).contiguous()
col = torch.from_numpy(color).cuda().contiguous()
ext = np.ascontiguousarray(ext, dtype=np.float64)
vol = pkg.pipelines.integration.ScalableTSDFVolume(voxel_length=0.005, sdf_trunc=0.04,
                                                   color_type=pkg.pipelines.integration.TSDFVolumeColorType.RGB8)
if len(sys.argv) > 1:
    vol.set_batch(int(sys.argv[1]))  # frames per fused launch
s_ = C.c_void_p(torch.cuda.current_stream().cuda_stream)
dp, cp, ep, intr_ref = d16.data_ptr(), col.data_ptr(), ext.ctypes.data, C.byref(intr)
phases = {}


def mark(name, t0):
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    phases.setdefault(name, []).append((t1 - t0) * 1e3)
    return t1


def one(record):
    t = time.perf_counter()
    vol.reset()
    lib.ot_tsdf_integrate_u16_frames(vol._h, ext.shape[0], dp, cp, intr_ref, ep, 1000.0, 3.0, s_)
    t_calls = time.perf_counter()
    lib.ot_tsdf_flush(vol._h, s_)
    t = mark("integrate (64 calls + flush)", t)
    phases.setdefault("  of which host calls", []).append((t_calls - (t - phases["integrate (64 calls + flush)"][-1] / 1e3)) * 1e3)
    mesh = vol.extract_triangle_mesh()
    t = mark("extract_triangle_mesh", t)
    mesh.compute_vertex_normals()
    t = mark("compute_vertex_normals", t)
    mesh.sample_points_min_z(100000, 0.03)  # sample_points_uniformly + the Z mask in one pass
    mark("sample_points_min_z", t)


for i in range(7):
    one(i >= 2)
for k, v in phases.items():
    print(f"{k:32s} {np.median(v[2:]):8.3f} ms")
print(f"{'total (sum of phases)':32s} {sum(np.median(v[2:]) for k, v in phases.items() if not k.startswith(' ')):8.3f} ms")
