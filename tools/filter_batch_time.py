"""Time the batched configs[2] chain (ot_rgbd_filter_run) on distinct 1280x720 frames: per-frame ms for a few
batch sizes (and the kernel breakdown when run under rocprofv3 --kernel-trace --stats)."""
import argparse
import ctypes as C
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "object-triggered-3d-slam_amd"

ap = argparse.ArgumentParser()
ap.add_argument("--frames", type=int, default=64)
ap.add_argument("--batches", default="8,16,32,64")
ap.add_argument("--reps", type=int, default=3)
ap.add_argument("--ab-netfill", type=int, default=0, help="alternate otx_sor_netfill(1) / (0) over this many rounds")
ap.add_argument("--ab-hook", default="otx_sor_netfill", help="the 0/1 test hook --ab-netfill alternates")
a = ap.parse_args()
synth = importlib.import_module(PKG + ".synth")
from concurrent.futures import ProcessPoolExecutor
import multiprocessing as mp

intr_t = synth.REF_INTRINSICS_1280
t0 = time.time()
with ProcessPoolExecutor(max_workers=16, mp_context=mp.get_context("fork")) as ex:
    parts = list(ex.map(synth.render_frames, [(synth.Scene(seed=0), 512, intr_t, list(range(i, min(i + 4, a.frames))))
                                               for i in range(0, a.frames, 4)]))
depth = np.concatenate([p[0] for p in parts])
color = np.concatenate([p[1] for p in parts])
ext = np.concatenate([p[2] for p in parts])
print(f"rendered {a.frames} frames in {time.time() - t0:.1f} s", flush=True)
import torch

L = importlib.import_module(PKG + "._lib")
L.load()
d = torch.from_numpy(depth.view(np.int16)).cuda().view(torch.uint16).contiguous()
c = torch.from_numpy(color).cuda().contiguous()
W, H = intr_t[0], intr_t[1]
intr = L.ot_intrinsics(W, H, *intr_t[2:])
stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
npx = W * H
for B in [int(x) for x in a.batches.split(",")]:
    h = C.c_void_p()
    L.call("ot_rgbd_filter_create", C.byref(intr), B, 1000.0, 5.0, 0.005, 20, 2.0, C.byref(h))
    def run_all():
        pts = kept = vox = 0
        for f0 in range(0, a.frames, B):
            n = min(B, a.frames - f0)
            e = np.ascontiguousarray(ext[f0:f0 + n])
            L.call("ot_rgbd_filter_run", h, n, C.c_void_p(d.data_ptr() + f0 * npx * 2), C.c_void_p(c.data_ptr() + f0 * npx * 3),
                   e.ctypes.data_as(C.c_void_p), stream)
            P, K, KK = C.c_int64(), C.c_int64(), C.c_int64()
            L.call("ot_rgbd_filter_sizes", h, C.byref(P), C.byref(K), C.byref(KK), None, None, None)
            pts += P.value
            vox += K.value
            kept += KK.value
        run_all.vox = vox
        return pts, kept
    run_all()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(a.reps):
        pts, kept = run_all()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t1) / a.reps
    print(f"batch {B}: {dt * 1e3 / a.frames:.4f} ms/frame, {pts / dt / 1e6:.1f} Mpoints/s, kept/frame {kept / a.frames:.0f}",
          flush=True)
    for rnd in range(a.ab_netfill):  # A/B of the stage-1 list fill, alternating in one process
        for on in (1, 0):
            L.call(a.ab_hook, on)
            run_all()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            run_all()
            torch.cuda.synchronize()
            print(f"{a.ab_hook} {on}: {(time.perf_counter() - t2) * 1e3 / a.frames:.4f} ms/frame (batch {B}, round {rnd})",
                  flush=True)
    L.call(a.ab_hook, 1)
    nb = (a.frames + B - 1) // B
    # per launch of the batch's kernels (one k_sor_knn per batch): SURVEY 8(d) algorithmic bytes of the SOR kNN =
    # 12 B per input point (the voxel centroids) + 12 B per kept point; read by tools/parse_pmc.py
    print(json.dumps({"filter_batch": B, "frames": a.frames, "voxels_per_launch": run_all.vox / nb,
                      "kept_per_launch": kept / nb,
                      "sor_algorithmic_bytes_per_launch": 12.0 * (run_all.vox + kept) / nb}), flush=True)
    L.call("ot_rgbd_filter_destroy", h)
