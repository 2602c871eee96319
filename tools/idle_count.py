"""Diagnostic: fraction of (wave, frame) pairs of k_batch_integrate in which no lane updates (needs a library
built with -DOT_COUNT_IDLE, selected through OTSLAM_LIB)."""
import ctypes as C
import importlib
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = "object-triggered-3d-slam_amd"
L = importlib.import_module(PKG + "._lib")
synth = importlib.import_module(PKG + ".synth")
lib = L.load()
for voxel in (0.005, 0.01):
    intr_t = synth.REF_INTRINSICS_640
    W, H = intr_t[0], intr_t[1]
    depth, color, ext = synth.make_sequence(synth.Scene(seed=0), n_frames=256, intr=intr_t)
    d16 = torch.from_numpy(depth.view(np.int16)).cuda().view(torch.uint16).contiguous()
    col = torch.from_numpy(color).cuda().contiguous()
    ext = np.ascontiguousarray(ext, dtype=np.float64)
    intr = L.ot_intrinsics(W, H, *intr_t[2:])
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    vol = C.c_void_p()
    L.call("ot_tsdf_create", voxel, 0.04, L.OT_COLOR_RGB8, 16, 4, 0, C.byref(vol))
    for k in range(256):
        L.call("ot_tsdf_integrate_u16", vol, C.c_void_p(d16.data_ptr() + k * W * H * 2),
               C.c_void_p(col.data_ptr() + k * W * H * 3), C.byref(intr), ext[k].ctypes.data_as(C.c_void_p),
               1000.0, 3.0, stream)
    st = (C.c_uint64 * 4)()
    L.call("otx_tsdf_stats", vol, st)
    print(f"voxel {voxel}: updates {st[0]} unit_int {st[1]} idle wave-frames {st[2]} of {st[3]} "
          f"= {st[2] / max(st[3], 1):.3f}; update fraction of visits {st[0] / (st[1] * 4096):.3f}")
    L.call("ot_tsdf_destroy", vol)
