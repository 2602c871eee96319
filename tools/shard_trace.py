"""One rank's shard of the headline scan (ot_tsdf_set_shard(rank, N) on the configs[1] 256-frame scan, the bench's
shard_rank_steps step: reset + the scan in one ot_tsdf_integrate_u16_frames call + flush), repeated; run it under
`rocprofv3 --kernel-trace` and report the kernel timeline of the last repetition on both of the volume's streams
(front end on the caller's stream, integrate on the volume's integrate stream when the front end is double-buffered).
Tool only.

  rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 tools/shard_trace.py --world 8 [--owner blocks]
  python3 tools/shard_trace.py --report DIR/run_kernel_trace.csv
"""
import argparse
import ctypes as C
import importlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
PKG = "object-triggered-3d-slam_amd"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--overlap", type=int, default=-1)
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--fine", type=int, default=-1, help="otx_integrate_fine: -1 auto, 0 coarse, 1 fine slices")
    ap.add_argument("--depth", type=int, default=-1, help="otx_integrate_depth: fine slices' frame-pipeline depth")
    ap.add_argument("--owner", default="sectors", help="blocks (ot_tsdf_set_shard) or sectors (set_shard_sector)")
    ap.add_argument("--split", type=int, default=-1, help="otx_split_frontend: -1 library choice, 0 fused, 1 split")
    ap.add_argument("--report")
    a = ap.parse_args()
    if a.report:
        import single_object_trace as T

        T.REPS = a.reps
        T.AFTER_PASSES = 1  # main() runs one more step (one more reset) after the timed repetitions
        T.report(a.report)
        return
    synth = importlib.import_module(PKG + ".synth")
    depth, color, ext = synth.make_sequence_parallel(synth.Scene(seed=0), n_frames=256, intr=synth.REF_INTRINSICS_640)
    import torch

    L = importlib.import_module(PKG + "._lib")
    lib = L.load()
    intr_t = synth.REF_INTRINSICS_640
    intr = L.ot_intrinsics(*intr_t)
    d16 = torch.from_numpy(depth.view(np.int16)).cuda().view(torch.uint16).contiguous()
    col = torch.from_numpy(color).cuda().contiguous()
    ext = np.ascontiguousarray(ext, dtype=np.float64)
    s_ = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    vol = C.c_void_p()
    L.call("ot_tsdf_create", 0.005, 0.04, L.OT_COLOR_RGB8, 16, 4, 0, C.byref(vol))
    if a.world > 1 and a.owner == "blocks":
        L.call("ot_tsdf_set_shard", vol, a.rank, a.world)
    elif a.world > 1:
        bench = importlib.import_module("bench")
        L.call("ot_tsdf_set_shard_sector", vol, a.rank, a.world, *bench.scan_centre_xy(ext))
    L.call("ot_tsdf_set_frontend_overlap", vol, a.overlap)
    L.call("otx_integrate_fine", a.fine)
    L.call("otx_integrate_depth", a.depth)
    L.call("otx_split_frontend", a.split)

    def step():
        L.call("ot_tsdf_reset_async", vol, s_)
        if lib.ot_tsdf_integrate_u16_frames(vol, 256, d16.data_ptr(), col.data_ptr(), C.byref(intr), ext.ctypes.data,
                                            1000.0, 3.0, s_):
            raise RuntimeError(lib.ot_last_error().decode())
        L.call("ot_tsdf_flush", vol, s_)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        step()
    torch.cuda.synchronize()
    print(f"world {a.world} rank {a.rank} owner {a.owner} split {a.split} overlap {a.overlap} fine {a.fine} "
          f"depth {a.depth}: "
          f"{(time.perf_counter() - t0) * 1e3 / a.reps:.4f} ms/step")
    step()  # the report's last repetition ends at this step's reset
    torch.cuda.synchronize()
    L.call("ot_tsdf_destroy", vol)


if __name__ == "__main__":
    main()
