"""Integrate time of one rank's shard vs the shard count (tool): the headline scan (configs[1], 256 frames, 64-frame
batches) into a volume keeping rank 0's units of N, for N = 1 .. 64; per N the units kept, the integrate kernel's mean
time per batch (HIP events, ot_tsdf_kernel_time) and the front end's (ot_tsdf_frontend_time), for both integrate
granularities (otx_integrate_fine 0 / 1), front end not overlapped (so the two do not contend)."""
import ctypes as C
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "object-triggered-3d-slam_amd"


def main():
    synth = importlib.import_module(PKG + ".synth")
    depth, color, ext = synth.make_sequence_parallel(synth.Scene(seed=0), n_frames=256, intr=synth.REF_INTRINSICS_640)
    import torch

    L = importlib.import_module(PKG + "._lib")
    lib = L.load()
    intr = L.ot_intrinsics(*synth.REF_INTRINSICS_640)
    d16 = torch.from_numpy(depth.view(np.int16)).cuda().view(torch.uint16).contiguous()
    col = torch.from_numpy(color).cuda().contiguous()
    ext = np.ascontiguousarray(ext, dtype=np.float64)
    s_ = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    for N in (1, 2, 4, 8, 16, 32, 64):
        for fine in (0, 1):
            vol = C.c_void_p()
            L.call("ot_tsdf_create", 0.005, 0.04, L.OT_COLOR_RGB8, 16, 4, 0, C.byref(vol))
            if N > 1:
                L.call("ot_tsdf_set_shard", vol, 0, N)
            L.call("ot_tsdf_set_frontend_overlap", vol, 0)
            L.call("otx_integrate_fine", fine)

            def step():
                L.call("ot_tsdf_reset_async", vol, s_)
                if lib.ot_tsdf_integrate_u16_frames(vol, 256, d16.data_ptr(), col.data_ptr(), C.byref(intr),
                                                    ext.ctypes.data, 1000.0, 3.0, s_):
                    raise RuntimeError(lib.ot_last_error().decode())
                L.call("ot_tsdf_flush", vol, s_)

            for _ in range(3):
                step()
            L.call("ot_tsdf_set_profiling", vol, 1)
            for _ in range(5):
                step()
            km, kl, fm, fb = C.c_double(), C.c_int64(), C.c_double(), C.c_int64()
            L.call("ot_tsdf_kernel_time", vol, C.byref(km), C.byref(kl))
            L.call("ot_tsdf_frontend_time", vol, C.byref(fm), C.byref(fb))
            L.call("ot_tsdf_set_profiling", vol, 0)
            nu, upd, ui = C.c_int64(), C.c_int64(), C.c_int64()
            L.call("ot_tsdf_num_units", vol, C.byref(nu), s_)
            print(f"N {N:3d} fine {fine}: units {nu.value:5d}  integrate {km.value / max(kl.value, 1) * 1e3:7.1f} us/batch"
                  f"  front end {fm.value / max(fb.value, 1) * 1e3:7.1f} us/batch", flush=True)
            L.call("ot_tsdf_destroy", vol)
    L.call("otx_integrate_fine", -1)


if __name__ == "__main__":
    main()
