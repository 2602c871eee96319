"""One configs[3] object end to end on one stream, unsynchronised between phases (exactly bench.py's single_object
leg), repeated: run it under `rocprofv3 --kernel-trace` and feed the trace to `--report` for the kernel timeline of
the last repetition (durations and the idle gaps between kernels).  Tool only.

  rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 tools/single_object_trace.py
  python3 tools/single_object_trace.py --report DIR/run_kernel_trace.csv
  python3 tools/single_object_trace.py --separate     (the facade's separate extract / normals / sample calls)
  python3 tools/single_object_trace.py --normals-at N (A/B: the normals start after the emission (0), beside the
                                                       area-sum walk (1) or the CDF walk (2, default))
  python3 tools/single_object_trace.py --fork         (A/B: the marching-cubes emission as two kernels on two streams)
  python3 tools/single_object_trace.py --no-normals   (diagnostic: the same object without compute_vertex_normals, i.e.
                                                       what the normals' side-stream kernel costs the critical path)
"""
import csv
import ctypes as C
import importlib
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "object-triggered-3d-slam_amd"
REPS = 8
AFTER_PASSES = 6 + 6 + 6 + 1  # volume resets after the timed repetitions (see main)


def report(path):
    rows = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], int(r.get("Stream_Id", 0) or 0)))
    rows.sort()
    # every repetition starts with the volume reset (k_tsdf_clear), and so does every pass of main()'s later loops (6
    # host-timing passes of the timed sequence, 6 of the separate calls, 6 host-breakdown passes of the separate calls,
    # the final statistics pass): the last timed
    # repetition (the path bench.py times) lies between the 20th- and 19th-last clears
    clears = [i for i, r in enumerate(rows) if "k_tsdf_clear" in r[2]]
    after = AFTER_PASSES
    last = rows[clears[-after - 1]:clears[-after]]
    t0 = last[0][0]
    busy = {}
    prev_end = t0
    print(f"{'start_us':>9} {'dur_us':>8} {'gap_us':>8} stream kernel")
    for s, e, name, sid in last:
        gap = (s - prev_end) / 1e3
        print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {gap:8.1f} {sid:6d} {name[:90]}")
        prev_end = max(prev_end, e)
        short = name.split("(")[0][:60]
        busy[short] = busy.get(short, 0.0) + (e - s) / 1e3
    span = (max(r[1] for r in last) - t0) / 1e3
    print(f"span {span:.1f} us over {len(last)} kernels")
    for k, v in sorted(busy.items(), key=lambda kv: -kv[1])[:25]:
        print(f"{v:9.1f} us  {k}")


def main(normals=True):
    synth = importlib.import_module(PKG + ".synth")
    depth, color, ext = synth.make_sequence(synth.object_scene(0), n_frames=64)
    import torch

    pkg = importlib.import_module(PKG)
    L = importlib.import_module(PKG + "._lib")
    lib = L.load()
    if "--hi" in sys.argv:  # A/B: the fused sampler on a greatest-priority stream, as before late round 4
        L.call("otx_sampler_hi_stream", 1)
    if "--normals-at" in sys.argv:  # A/B: where the fused call lets the vertex normals start (0 / 1 / 2)
        L.call("otx_normals_at", int(sys.argv[sys.argv.index("--normals-at") + 1]))
    if "--fork" in sys.argv:  # A/B: the round-4 emission (vertices on the side stream, fork / join by events)
        L.call("otx_mc_emit_fork", 1)
    intr_t = synth.REF_INTRINSICS_640
    W, H = intr_t[0], intr_t[1]
    intr = L.ot_intrinsics(W, H, *intr_t[2:])
    npx = W * H
    d16 = torch.from_numpy(depth.view(np.int16)).cuda().view(torch.uint16).contiguous()
    col = torch.from_numpy(color).cuda().contiguous()
    ext = np.ascontiguousarray(ext, dtype=np.float64)
    vol = pkg.pipelines.integration.ScalableTSDFVolume(voxel_length=0.005, sdf_trunc=0.04,
                                                       color_type=pkg.pipelines.integration.TSDFVolumeColorType.RGB8)
    s_ = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    dp, cp, ep, intr_ref = d16.data_ptr(), col.data_ptr(), ext.ctypes.data, C.byref(intr)

    def one():
        vol.reset()
        lib.ot_tsdf_integrate_u16_frames(vol._h, ext.shape[0], dp, cp, intr_ref, ep, 1000.0, 3.0, s_)
        if normals and "--separate" not in sys.argv:  # bench.py's path: one host call from the totals to the sampler
            return vol.extract_mesh_and_sample_min_z(100000, 0.03)[1]
        mesh = vol.extract_triangle_mesh()
        if normals:
            mesh.compute_vertex_normals()
        return mesh.sample_points_min_z(100000, 0.03)

    ts = []
    for _ in range(REPS):
        torch.cuda.synchronize()
        t = time.perf_counter()
        one()
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t) * 1e3)
    # host side of the timed (fused) sequence: when each call returns, medians over 5 (reset, integrate, fused call,
    # final synchronize)
    fmarks = []
    for _ in range(6):
        torch.cuda.synchronize()
        t = [time.perf_counter()]
        vol.reset()
        t.append(time.perf_counter())
        lib.ot_tsdf_integrate_u16_frames(vol._h, ext.shape[0], dp, cp, intr_ref, ep, 1000.0, 3.0, s_)
        t.append(time.perf_counter())
        if normals and "--separate" not in sys.argv:
            vol.extract_mesh_and_sample_min_z(100000, 0.03)
        t.append(time.perf_counter())
        torch.cuda.synchronize()
        t.append(time.perf_counter())
        fmarks.append(np.diff(np.array(t)) * 1e6)
    med = np.median(np.array(fmarks[1:]), axis=0)
    print("host us per call of the timed sequence (reset, integrate, fused extract+sample, final sync):",
          [round(float(x), 1) for x in med])
    # host side of the separate call sequence: when each call returns (no synchronisation in between), medians over 5
    marks = []
    for _ in range(6):
        torch.cuda.synchronize()
        t = [time.perf_counter()]
        vol.reset()
        lib.ot_tsdf_integrate_u16_frames(vol._h, ext.shape[0], dp, cp, intr_ref, ep, 1000.0, 3.0, s_)
        t.append(time.perf_counter())
        mesh = vol.extract_triangle_mesh()
        t.append(time.perf_counter())
        if normals:
            mesh.compute_vertex_normals()
        t.append(time.perf_counter())
        mesh.sample_points_min_z(100000, 0.03)
        t.append(time.perf_counter())
        torch.cuda.synchronize()
        t.append(time.perf_counter())
        marks.append(np.diff(np.array(t)) * 1e6)
    med = np.median(np.array(marks[1:]), axis=0)
    print("host us per call (integrate, extract, normals, sample, final sync):", [round(float(x), 1) for x in med])
    # the host's work between the extraction's return and the sampling's first launch, piece by piece (the sampler call
    # of TriangleMesh.sample_points_min_z_batch unrolled here)
    D = importlib.import_module(PKG + "._device")
    parts = []
    for _ in range(6):
        torch.cuda.synchronize()
        vol.reset()
        lib.ot_tsdf_integrate_u16_frames(vol._h, ext.shape[0], dp, cp, intr_ref, ep, 1000.0, 3.0, s_)
        mesh = vol.extract_triangle_mesh()
        t = [time.perf_counter()]
        mesh.compute_vertex_normals()
        t.append(time.perf_counter())
        P = D.empty((100000, 3), "float64")
        PC = D.empty((100000, 3), "float64")
        t.append(time.perf_counter())
        jobs = (L.ot_mesh_sample_job * 1)()
        jobs[0] = L.ot_mesh_sample_job(D.ptr(mesh._v.dev()), None, D.ptr(mesh._vc.dev()), len(mesh._v),
                                       D.ptr(mesh._t.dev()), len(mesh._t), D.ptr(P), None, D.ptr(PC))
        kept = (C.c_int64 * 1)()
        t.append(time.perf_counter())
        L.call("ot_mesh_sample_points_min_z_async", C.cast(jobs, C.c_void_p), 1, 100000, C.c_uint64(0), 0.03,
               D.stream_ptr())
        t.append(time.perf_counter())
        if normals:
            mesh._vn._start()
        t.append(time.perf_counter())
        L.call("ot_mesh_sample_points_min_z_wait", 1, kept)
        torch.cuda.synchronize()
        parts.append(np.diff(np.array(t)) * 1e6)
    med = np.median(np.array(parts[1:]), axis=0)
    print("host us after the extraction (normals call, output allocs, job table, sampler enqueue, normals launch):",
          [round(float(x), 1) for x in med])
    print("stream priority range (least, greatest):", torch.cuda.Stream.priority_range())
    print("single object ms (median of last 5)" + ("" if normals else ", WITHOUT normals") +
          (", sampler on the greatest-priority stream" if "--hi" in sys.argv else "") +
          (", two-stream emission" if "--fork" in sys.argv else "") +
          (f", normals at {sys.argv[sys.argv.index('--normals-at') + 1]}" if "--normals-at" in sys.argv else "") + ":", round(float(np.median(ts[3:])), 3), [round(x, 3) for x in ts])
    # the volume's size against configs[1]'s (integrate occupancy): units, voxel updates, unit integrations
    vol.reset()
    lib.ot_tsdf_integrate_u16_frames(vol._h, ext.shape[0], dp, cp, intr_ref, ep, 1000.0, 3.0, s_)
    nu, vu, ui = C.c_int64(0), C.c_int64(0), C.c_int64(0)
    lib.ot_tsdf_num_units(vol._h, C.byref(nu), s_)
    lib.ot_tsdf_counters(vol._h, C.byref(vu), C.byref(ui), s_)
    print(f"units {nu.value}, voxel updates {vu.value} ({vu.value / 64:.0f} per frame), unit integrations {ui.value} "
          f"({ui.value / max(nu.value, 1):.1f} frames per unit)")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--report":
        report(sys.argv[2])
    else:
        main(normals="--no-normals" not in sys.argv)
