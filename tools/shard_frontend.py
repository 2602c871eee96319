"""One rank's share of a spatially sharded configs[1] object, alone on the GPU: the volume keeps the
units of rank --rank of --world (ot_tsdf_set_shard) and integrates the 256-frame 640x480 scan, --reps times.  Run
under rocprofv3 --kernel-trace --stats once per world size: the per-launch k_batch_touch / k_batch_units /
k_batch_integrate times are one rank's front end and integrate (VERDICT r3 'next' 6: the sharded front end must
divide).  --world 1 is the unsharded headline volume.  Prints ms per step."""
import argparse
import ctypes as C
import importlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "object-triggered-3d-slam_amd"

ap = argparse.ArgumentParser()
ap.add_argument("--world", type=int, default=1)
ap.add_argument("--rank", type=int, default=0)
ap.add_argument("--reps", type=int, default=20)
a = ap.parse_args()
synth = importlib.import_module(PKG + ".synth")
depth, color, ext = synth.make_sequence_parallel(synth.Scene(seed=0), n_frames=256, intr=synth.REF_INTRINSICS_640)
import torch

L = importlib.import_module(PKG + "._lib")
lib = L.load()
W, H = synth.REF_INTRINSICS_640[:2]
intr = L.ot_intrinsics(W, H, *synth.REF_INTRINSICS_640[2:])
d16 = torch.from_numpy(depth.view(np.int16)).cuda().view(torch.uint16).contiguous()
col = torch.from_numpy(color).cuda().contiguous()
ext = np.ascontiguousarray(ext, dtype=np.float64)
stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
vol = C.c_void_p()
L.call("ot_tsdf_create", 0.005, 0.04, L.OT_COLOR_RGB8, 16, 4, 0, C.byref(vol))
if a.world > 1:
    L.call("ot_tsdf_set_shard", vol, a.rank, a.world)
npx = W * H


def step():
    L.call("ot_tsdf_reset_async", vol, stream)
    for k in range(256):
        if lib.ot_tsdf_integrate_u16(vol, C.c_void_p(d16.data_ptr() + k * npx * 2), C.c_void_p(col.data_ptr() + k * npx * 3),
                                     C.byref(intr), ext[k].ctypes.data_as(C.c_void_p), 1000.0, 3.0, stream):
            raise RuntimeError(lib.ot_last_error().decode())
    L.call("ot_tsdf_flush", vol, stream)


step()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(a.reps):
    step()
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / a.reps
nu = C.c_int64(0)
L.call("ot_tsdf_num_units", vol, C.byref(nu), stream)
print(f"world {a.world} rank {a.rank}: {dt * 1e3:.3f} ms per 256-frame step, {nu.value} units", flush=True)
L.call("ot_tsdf_destroy", vol)
