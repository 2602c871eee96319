"""A/B of the batch touch's staging forms (tool): the headline scan (configs[1], 256 frames, 64-frame batches), the
unsharded volume and rank 0 of 8 shards, with otx_touch_stage_blocks 0 (every touch workgroup stages a share first) or
N staging-only workgroups per frame group (FORMS, comma-separated; a 640x480 frame at stride 4 has 80 touch tiles, and
-1 is the default, 2 per tile; an optional ':F' sets the frames per touch workgroup, default 2); per form
the front end's mean time per batch (ot_tsdf_frontend_time, HIP events around staging + touch + units) and the step
(reset + 256 frames + flush, HIP events), forms interleaved over rounds so drift hits them alike."""
import ctypes as C
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "object-triggered-3d-slam_amd"
FORMS = tuple(tuple(int(v) for v in (x + ":2").split(":")[:2]) for x in os.environ.get("FORMS", "0,-1:2,-1:4").split(","))


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
    stream = torch.cuda.current_stream()
    s_ = C.c_void_p(stream.cuda_stream)
    res = {}
    for N in (1, 8):
        vol = C.c_void_p()
        L.call("ot_tsdf_create", 0.005, 0.04, L.OT_COLOR_RGB8, 16, 4, 0, C.byref(vol))
        if N > 1:
            L.call("ot_tsdf_set_shard", vol, 0, N)

        def step():
            L.call("ot_tsdf_reset_async", vol, s_)
            if lib.ot_tsdf_integrate_u16_frames(vol, 256, d16.data_ptr(), col.data_ptr(), C.byref(intr),
                                                ext.ctypes.data, 1000.0, 3.0, s_):
                raise RuntimeError(lib.ot_last_error().decode())
            L.call("ot_tsdf_flush", vol, s_)

        for rnd in range(3):
            for form in FORMS:
                L.call("otx_touch_stage_blocks", form[0])
                L.call("otx_touch_frames", form[1])
                for _ in range(2):
                    step()
                L.call("ot_tsdf_set_profiling", vol, 1)
                for _ in range(4):
                    step()
                fm, fb = C.c_double(), C.c_int64()
                L.call("ot_tsdf_frontend_time", vol, C.byref(fm), C.byref(fb))
                L.call("ot_tsdf_set_profiling", vol, 0)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(10):
                    step()
                e1.record(stream)
                torch.cuda.synchronize()
                r = res.setdefault((N, form), {"fe": [], "step": []})
                r["fe"].append(fm.value / max(fb.value, 1) * 1e3)
                r["step"].append(e0.elapsed_time(e1) / 10)
                print(f"round {rnd} N {N} form {form[0]:4d}:{form[1]}: front end {r['fe'][-1]:6.1f} us/batch  step "
                      f"{r['step'][-1]:.4f} ms", flush=True)
        L.call("ot_tsdf_destroy", vol)
    L.call("otx_touch_stage_blocks", -1)
    L.call("otx_touch_frames", 2)
    for (N, form), r in sorted(res.items()):
        print(f"N {N} form {form[0]:4d}:{form[1]}: front end median {np.median(r['fe']):6.1f} us/batch  step median "
              f"{np.median(r['step']):.4f} ms")


if __name__ == "__main__":
    main()
