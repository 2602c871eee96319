"""One rank's shard of the headline scan vs the shard count (tool): the configs[1] scan (256 frames, 64-frame batches)
into a volume keeping rank r's units of N; per (N, ownership, front end, integrate granularity) the units kept, the step
time (reset + 256 frames in one host call + flush), the integrate kernel's mean time per batch (HIP events,
ot_tsdf_kernel_time) and the front end's (ot_tsdf_frontend_time), max over the ranks asked for.
  --owners blocks,sectors   hashed ownership blocks (ot_tsdf_set_shard) / azimuth sectors (ot_tsdf_set_shard_sector)
  --split -1,0              split front end (-1: the library's choice = split for sharded volumes; 0: fused staging)
  --fine -1                 integrate granularity (otx_integrate_fine: -1 by the batch, 0 coarse, 1 fine)
  --ranks all               every rank of N (else rank 0 only)"""
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--owners", default="blocks,sectors")
    ap.add_argument("--split", default="-1")
    ap.add_argument("--fine", default="-1")
    ap.add_argument("--depth", default="-1", help="fine integrate's frame-pipeline depth KT (otx_integrate_depth)")
    ap.add_argument("--tf", default="2", help="frames per touch workgroup (otx_touch_frames)")
    ap.add_argument("--overlap", default="0", help="double-buffered front end (ot_tsdf_set_frontend_overlap)")
    ap.add_argument("--batch", default="64", help="frames per batch (ot_tsdf_set_batch)")
    ap.add_argument("--defer", default="-1", help="deferred integrate (otx_defer_integrate)")
    ap.add_argument("--ranks", default="all")
    ap.add_argument("--steps", type=int, default=10)
    a = ap.parse_args()
    synth = importlib.import_module(PKG + ".synth")
    depth, color, ext = synth.make_sequence_parallel(synth.Scene(seed=0), n_frames=256, intr=synth.REF_INTRINSICS_640)
    import torch

    L = importlib.import_module(PKG + "._lib")
    lib = L.load()
    bench = importlib.import_module("bench")
    intr = L.ot_intrinsics(*synth.REF_INTRINSICS_640)
    d16 = torch.from_numpy(depth.view(np.int16)).cuda().view(torch.uint16).contiguous()
    col = torch.from_numpy(color).cuda().contiguous()
    ext = np.ascontiguousarray(ext, dtype=np.float64)
    cx, cy = bench.scan_centre_xy(ext)
    s_ = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    for N in [int(x) for x in a.worlds.split(",")]:
        for owner in (a.owners.split(",") if N > 1 else ["unsharded"]):
            for split in [int(x) for x in a.split.split(",")]:
                for fine, depth, tf, ov, bt, df in [(int(x), int(y), int(t), int(o), int(b), int(df)) for x in a.fine.split(",")
                                                for y in a.depth.split(",") for t in a.tf.split(",")
                                                for o in a.overlap.split(",") for b in a.batch.split(",")
                                                for df in a.defer.split(",")]:
                    L.call("otx_defer_integrate", df)
                    L.call("otx_touch_frames", tf)
                    L.call("otx_split_frontend", split)
                    L.call("otx_integrate_fine", fine)
                    L.call("otx_integrate_depth", depth)
                    worst = {"step": 0.0, "int": 0.0, "fe": 0.0, "units": 0}
                    for r in (range(N) if a.ranks == "all" else [0]):
                        vol = C.c_void_p()
                        L.call("ot_tsdf_create", 0.005, 0.04, L.OT_COLOR_RGB8, 16, 4, 0, C.byref(vol))
                        if owner == "blocks":
                            L.call("ot_tsdf_set_shard", vol, r, N)
                        elif owner == "sectors":
                            L.call("ot_tsdf_set_shard_sector", vol, r, N, cx, cy)
                        L.call("ot_tsdf_set_frontend_overlap", vol, ov)
                        L.call("ot_tsdf_set_batch", vol, bt)

                        def step():
                            L.call("ot_tsdf_reset_async", vol, s_)
                            if lib.ot_tsdf_integrate_u16_frames(vol, 256, d16.data_ptr(), col.data_ptr(), C.byref(intr),
                                                                ext.ctypes.data, 1000.0, 3.0, s_):
                                raise RuntimeError(lib.ot_last_error().decode())
                            L.call("ot_tsdf_flush", vol, s_)

                        for _ in range(3):
                            step()
                        torch.cuda.synchronize()
                        t0 = time.perf_counter()
                        for _ in range(a.steps):
                            step()
                        torch.cuda.synchronize()
                        dt = (time.perf_counter() - t0) * 1e3 / a.steps
                        L.call("ot_tsdf_set_profiling", vol, 1)
                        for _ in range(3):
                            step()
                        km, kl, fm, fb = C.c_double(), C.c_int64(), C.c_double(), C.c_int64()
                        L.call("ot_tsdf_kernel_time", vol, C.byref(km), C.byref(kl))
                        L.call("ot_tsdf_frontend_time", vol, C.byref(fm), C.byref(fb))
                        L.call("ot_tsdf_set_profiling", vol, 0)
                        nu = C.c_int64()
                        L.call("ot_tsdf_num_units", vol, C.byref(nu), s_)
                        worst["step"] = max(worst["step"], dt)
                        worst["int"] = max(worst["int"], km.value / max(kl.value, 1) * 1e3)
                        worst["fe"] = max(worst["fe"], fm.value / max(fb.value, 1) * 1e3)
                        worst["units"] = max(worst["units"], nu.value)
                        L.call("ot_tsdf_destroy", vol)
                    print(f"N {N:2d} {owner:9s} split {split:2d} fine {fine:2d} depth {depth:2d} tf {tf} overlap {ov} batch {bt} defer {df}: step {worst['step']:.3f} ms  "
                          f"units max {worst['units']:5d}  integrate {worst['int']:6.1f} us/batch  front end "
                          f"{worst['fe']:6.1f} us/batch", flush=True)
    L.call("otx_integrate_fine", -1)
    L.call("otx_integrate_depth", -1)
    L.call("otx_split_frontend", -1)
    L.call("otx_touch_frames", 2)
    L.call("otx_defer_integrate", -1)


if __name__ == "__main__":
    main()
