"""bench.py — headline benchmark: BASELINE.json configs[1], 256-frame 640x480 TSDF integration, 5 mm voxel.

One step = integrate every frame of one synthetic object scan (256 RGB-D frames, inputs resident in HBM as
uint16 depth + RGB8 colour) into a fresh ScalableTSDFVolume through the C ABI (ot_tsdf_integrate_u16 =
create_from_color_and_depth + integrate, the reference's per-frame calls at reconstruct_rgbd_filter.py:98-105).
Multi-GPU: one process per GPU, each integrates its own object (objects are independent,
reconstruct_rgbd_filter.py:154-155) => weak scaling, no data-path collective; barrier + max-over-ranks
timing.  Prints ONE JSON line on rank 0.

Also reported:
  roofline     — dominant kernel (k_batch_integrate<true>, float64 colour): the measured HBM bytes per launch from
                 rocprofv3 PMC counters (profiles/pmc_traffic.json, used only when its source hash and workload match
                 this build) over its mean device time measured with HIP events on the launch stream (`frac`, physical,
                 <= 1); beside it `frac_effective` = algorithmic bytes per launch (5*W*H + 40*U_f) over
                 the same time (temporal blocking keeps voxel state on chip across a batch, so it may exceed 1) and the
                 VALU / TA / TD busy fractions that bind the kernel;
  cpu_baseline — the CPU oracle (strict-IEEE restatement of Open3D's ScalableTSDFVolume, OpenMP where Open3D
                 places it) on all 256 frames of the same scan, rank 0 only: 1 warm-up, median of 3 passes;
  sustained    — the headline step repeated for >= 12 s after the timed steps (corroborates `value`);
  filtered     — configs[2]: 512 distinct 1280x720 frames through the batched device-resident chain
                 (ot_rgbd_filter_run), Mpoints/s;
  objects / hybrid_map / single_frame / spatial — configs[3], [4], [0] and single-object sharding (N > 1).
"""
from __future__ import annotations

import argparse
import ctypes as C
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
PKG = "object-triggered-3d-slam_amd"

METRIC = "RGB-D frames/sec (640×480, 5mm voxel TSDF) at 1/2/4/8 GPU; Mpoints/s filtered"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s peak
COLL_DEV = "cuda"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--frames", type=int, default=256)
    ap.add_argument("--voxel", type=float, default=0.005)
    ap.add_argument("--sdf-trunc", type=float, default=0.04)
    ap.add_argument("--batch", type=int, default=0, help="frames per fused launch (0 = library default)")
    ap.add_argument("--overlap", type=int, default=-1, choices=(-1, 0, 1),
                    help="headline volume's batch front end double-buffered beside the previous integrate "
                         "(ot_tsdf_set_frontend_overlap; -1 = library default: "
                         "sharded volumes double-buffer at 2-3 ranks and defer the integrate from 4, whole volumes "
                         "neither; 0 off, 1 on)")
    ap.add_argument("--cpu-frames", type=int, default=256, help="frames in the CPU-baseline sample (0 = skip)")
    ap.add_argument("--sustain", type=float, default=12.0,
                    help="seconds of sustained headline steps after the timed ones (0 = skip): >= 12 s so a 5-s busy "
                         "sampler lands in it at least twice")
    ap.add_argument("--color-bits", type=int, default=64, choices=(32, 64),
                    help="headline colour precision: 64 = Open3D's float64 TSDFVoxel::color_ (the C ABI and facade "
                         "default, bit-exact colours); 32 = float32 colour state")
    ap.add_argument("--color32", type=int, default=1,
                    help="also time the headline workload with float32 colour state (a labelled secondary leg)")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    ap.add_argument("--filter-frames", type=int, default=512,
                    help="configs[2] stream length, distinct frames (1280x720 unproject + 5 mm voxel + SOR); 0 = skip")
    ap.add_argument("--filter-batch", type=int, default=64,
                    help="configs[2]: frames per batched chain call (64: 0.120-0.121 vs 0.122-0.124 ms/frame at 32, r04al)")
    ap.add_argument("--objects", type=int, default=8,
                    help="configs[3]: object scans shared by all ranks (full per-object pipeline + RCCL merge); 0 = skip")
    ap.add_argument("--object-frames", type=int, default=64, help="configs[3]: frames per object scan")
    ap.add_argument("--filter-streams", type=int, default=3,
                    help="configs[2]: batches filtered concurrently (host threads x HIP streams)")
    ap.add_argument("--objects-sampling", default="fused", choices=("fused", "batch"),
                    help="configs[3]: per object one host call from the marching-cubes totals to the sampler "
                         "(extract_mesh_and_sample_min_z), or every object's mesh first and one batched sampling call")
    ap.add_argument("--object-streams", type=int, default=2,
                    help="configs[3]: objects reconstructed concurrently per GPU (host threads x HIP streams)")
    ap.add_argument("--spatial", type=int, default=1,
                    help="N > 1: also time one object spatially sharded over the N GPUs (SURVEY 8(e))")
    ap.add_argument("--shard-steps", type=int, default=20,
                    help="N = 1: per-rank step of the headline scan spatially sharded over 2 / 4 / 8 ranks, every rank's "
                         "shard timed on this GPU (0 = skip)")
    ap.add_argument("--hybrid-objects", type=int, default=32,
                    help="configs[4]: object clouds in the hybrid-map fusion + change detection; 0 = skip")
    return ap.parse_args()


def resolve_world(gpus, env):
    """Reconcile --gpus with a launcher's environment.  Returns ("spawn", N) when this process must start N ranks
    itself (no WORLD_SIZE, --gpus N > 1), ("run", world) when it is one rank of `world` (or the only process);
    raises SystemExit when a launcher's WORLD_SIZE disagrees with --gpus."""
    ws = env.get("WORLD_SIZE")
    if ws is None:
        return ("spawn", gpus) if gpus > 1 else ("run", 1)
    if int(ws) != gpus:
        raise SystemExit(f"bench.py: WORLD_SIZE={ws} from the launcher but --gpus {gpus}")
    return "run", int(ws)


def launch_ranks(n, script, argv, env=None):
    """Start n ranks of `script argv` as child processes (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, rendezvous on
    127.0.0.1), before this process touches the GPU; rank 0 prints the JSON line.  If a rank fails the others are
    terminated (they would wait in a collective forever).  Returns the worst exit status."""
    import signal
    import socket
    import subprocess

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    base = dict(os.environ if env is None else env)
    base.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n))
    procs = []
    for r in range(n):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r))
        procs.append(subprocess.Popen([sys.executable, script] + list(argv), env=e))
    rcs = [None] * n
    while any(rc is None for rc in rcs):
        for i, p in enumerate(procs):
            if rcs[i] is None:
                rcs[i] = p.poll()
        if any(rc not in (None, 0) for rc in rcs):
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    p.send_signal(signal.SIGTERM)
            for i, p in enumerate(procs):
                if rcs[i] is None:
                    try:
                        rcs[i] = p.wait(timeout=30)
                    except subprocess.TimeoutExpired:
                        p.kill()
                        rcs[i] = p.wait()
            break
        time.sleep(0.05)
    bad = [rc for rc in rcs if rc != 0]
    return (max(bad, key=abs) if bad else 0), rcs


def main():
    args = parse()
    mode, world = resolve_world(args.gpus, os.environ)
    if mode == "spawn":  # `python bench.py --gpus N` with no launcher: one child process per GPU
        rc, _ = launch_ranks(world, os.path.abspath(__file__), sys.argv[1:])
        sys.exit(rc if 0 <= rc < 256 else 1)
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # configs[3] scans are rendered before this process touches the GPU (the render pool forks workers)
    synth0 = importlib.import_module(PKG + ".synth")
    obj_ids = list(range(args.objects))[(args.objects * rank) // world:(args.objects * (rank + 1)) // world]
    obj_scans = _render_objects(synth0, obj_ids, args.object_frames) if args.objects > 0 else None
    # every scan is rendered by forked workers before this process touches the GPU
    head_scan = synth0.make_sequence_parallel(synth0.Scene(seed=rank), n_frames=args.frames,
                                              intr=synth0.REF_INTRINSICS_640)
    filt_frames = synth0.make_sequence_parallel(synth0.Scene(seed=rank), n_frames=args.filter_frames,
                                                intr=synth0.REF_INTRINSICS_1280) \
        if (args.filter_frames > 0 and rank == 0) else None
    # OT_BENCH_BACKEND=gloo + OT_BENCH_SHARE_GPU=1 rehearse the N-rank path on a one-GPU box (every rank on
    # device 0, collectives through host memory); the driver's runs use RCCL ("nccl"), one GPU per rank.
    backend = os.environ.get("OT_BENCH_BACKEND", "nccl")
    dev_index = 0 if os.environ.get("OT_BENCH_SHARE_GPU") == "1" else local
    if world > 1:
        torch.cuda.set_device(dev_index)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    global COLL_DEV
    COLL_DEV = "cuda" if backend == "nccl" else "cpu"  # device of the small timing / count tensors

    pkg = importlib.import_module(PKG)
    synth = importlib.import_module(PKG + ".synth")
    L = importlib.import_module(PKG + "._lib")
    lib = L.load()
    # the concurrent legs' worker streams, created once and first (distinct hardware queues; streams.py)
    importlib.import_module(PKG + ".streams").worker_streams(max(args.filter_streams, args.object_streams, 1))

    # ---- synthetic object scan for this rank (same geometry, rank-seeded noise) ----
    intr_t = synth.REF_INTRINSICS_640
    W, H = intr_t[0], intr_t[1]
    depth, color, ext = head_scan
    d_depth = torch.from_numpy(depth.view(np.int16)).cuda().view(torch.uint16).contiguous()
    d_color = torch.from_numpy(color).cuda().contiguous()
    ext = np.ascontiguousarray(ext, dtype=np.float64)
    intr = L.ot_intrinsics(W, H, *intr_t[2:])
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)

    vol = C.c_void_p()
    L.call("ot_tsdf_create", args.voxel, args.sdf_trunc, L.OT_COLOR_RGB8, 16, 4, 0, C.byref(vol))
    L.call("ot_tsdf_set_color_precision", vol, args.color_bits)  # 64 is already the default; explicit for the record
    if args.batch > 0:
        L.call("ot_tsdf_set_batch", vol, args.batch)
    L.call("ot_tsdf_set_frontend_overlap", vol, args.overlap)
    frame_bytes = W * H
    dptrs = [C.c_void_p(d_depth.data_ptr() + k * frame_bytes * 2) for k in range(args.frames)]
    cptrs = [C.c_void_p(d_color.data_ptr() + k * frame_bytes * 3) for k in range(args.frames)]
    eptrs = [ext[k].ctypes.data_as(C.c_void_p) for k in range(args.frames)]
    integrate = lib.ot_tsdf_integrate_u16
    pintr = C.byref(intr)

    def step():
        L.call("ot_tsdf_reset_async", vol, stream)  # stream-ordered: no device-wide synchronisation per step
        for k in range(args.frames):
            st = integrate(vol, dptrs[k], cptrs[k], pintr, eptrs[k], 1000.0, 3.0, stream)
            if st:
                raise RuntimeError(lib.ot_last_error().decode())
        L.call("ot_tsdf_flush", vol, stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=COLL_DEV)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # ---- sustained: the same step back to back for >= args.sustain seconds (corroborates value over a long window) ----
    sustained = None
    if args.sustain > 0:
        n_s, t_s = 0, time.perf_counter()
        while time.perf_counter() - t_s < args.sustain:
            step()
            n_s += 1
            if n_s % 8 == 0:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        dt_s = time.perf_counter() - t_s
        sustained = {"steps": n_s, "seconds": round(dt_s, 3), "frames_per_s": round(world * n_s * args.frames / dt_s, 1)}

    # ---- per-step accounting: exact voxel updates (U_f summed over frames) ----
    upd, unit_int = C.c_int64(0), C.c_int64(0)
    L.call("ot_tsdf_counters", vol, C.byref(upd), C.byref(unit_int), stream)
    n_units = C.c_int64(0)
    L.call("ot_tsdf_num_units", vol, C.byref(n_units), stream)

    # ---- roofline: one extra (untimed) step with HIP events around every dominant-kernel launch ----
    L.call("ot_tsdf_set_profiling", vol, 1)
    step()
    kms, klaunch = C.c_double(0.0), C.c_int64(0)
    L.call("ot_tsdf_kernel_time", vol, C.byref(kms), C.byref(klaunch))
    fms, fbatches = C.c_double(0.0), C.c_int64(0)  # each batch's front end (staging + touch + unit headers)
    L.call("ot_tsdf_frontend_time", vol, C.byref(fms), C.byref(fbatches))
    L.call("ot_tsdf_set_profiling", vol, 0)
    # the step's batches (the profiled step began with a reset): units touched per batch and how many were new
    sb, sub, sfresh = C.c_int64(0), C.c_int64(0), C.c_int64(0)
    L.call("ot_tsdf_batch_stats", vol, C.byref(sb), C.byref(sub), C.byref(sfresh))

    frames_total = world * args.frames * args.steps
    value = frames_total / elapsed
    ms_per_step = elapsed * 1e3 / args.steps
    # 40 B per voxel update = read + write of a 20-B record (f32 tsdf, weight, 3 x f32 colour) whatever
    # the layout -- also at colour precision 64, whose record is 32 B (the figure stays the survey's, so the two
    # precisions' fractions compare the same work)
    algo_bytes_step = 5.0 * W * H * args.frames + 40.0 * upd.value
    per_launch_bytes = algo_bytes_step / max(klaunch.value, 1)
    kernel_ms_avg = kms.value / max(klaunch.value, 1)
    achieved = per_launch_bytes / (kernel_ms_avg * 1e-3) / 1e9 if kernel_ms_avg > 0 else 0.0
    kname = "k_batch_integrate<true>" if args.color_bits == 64 else "k_batch_integrate<false>"
    pmc_cfg = {"voxel": args.voxel, "frames": args.frames, "batch": args.batch, "color_bits": args.color_bits}
    traffic, traffic_note = _traffic(args, L, kname, pmc_cfg)
    # `frac` is PHYSICAL: HBM bytes the kernel moved per launch (rocprofv3 PMC FETCH_SIZE x measured
    # correction + WRITE_SIZE, same build and workload) over its launch time.  The algorithmic figure of SURVEY 8(d)
    # counts a voxel's 40-B read + write once per FRAME, but temporal blocking keeps the state on chip across the
    # batch, so it is reported apart as `frac_effective` (it may exceed 1: it counts bytes never moved).
    hbm_achieved = traffic / (kernel_ms_avg * 1e-3) / 1e9 if (traffic and kernel_ms_avg > 0) else None
    roofline = {"bound": "hbm", "achieved": round(hbm_achieved, 1) if hbm_achieved else None, "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(hbm_achieved / HBM_PEAK_GBS, 4) if hbm_achieved else None,
                "traffic": traffic, "traffic_source": traffic_note,
                "achieved_basis": "PMC HBM bytes per launch (traffic) / kernel_ms_avg" if hbm_achieved else
                                  "no same-build PMC entry: physical fraction unmeasured",
                "algorithmic_achieved": round(achieved, 1), "frac_effective": round(achieved / HBM_PEAK_GBS, 4),
                "effective_note": "algorithmic bytes (5*W*H + 40*U_f per frame, SURVEY 8(d)) / kernel time: voxel state "
                                  "stays in registers across the batch, so this counts bytes the kernel never moves",
                "kernel": ("k_integrate" if args.batch == 1 else "k_batch_integrate") +
                          ("<true>" if args.color_bits == 64 else "<false>"),
                "color_bits": args.color_bits,
                "kernel_ms_avg": round(kernel_ms_avg, 5), "launches_per_step": klaunch.value,
                "algorithmic_bytes_per_launch": round(per_launch_bytes),
                "voxel_updates_per_frame": round(upd.value / args.frames)}
    if hbm_achieved:  # kept under the old names too (round-3/4 records)
        roofline["hbm_achieved"] = roofline["achieved"]
        roofline["hbm_frac"] = roofline["frac"]
        roofline["traffic_level"] = ("L2-miss (fabric) bytes: FETCH_SIZE / WRITE_SIZE count the requests that leave "
                                     "the XCD's L2, including those the Infinity Cache (MALL) then serves "
                                     "(MI355X_MICROARCH.md), so the DRAM bytes may be lower and `frac` is an upper "
                                     "bound on the HBM fraction")
    # compulsory bytes per launch: the touched units' state read once (units new in the batch
    # start from zero: not read) and written once, plus the batch's staged frames read once (8-B depth / multiplier +
    # 4-B colour per pixel) -- what a kernel that re-fetched nothing would move
    rec = 4096 * (32 if args.color_bits == 64 else 20)
    if sb.value > 0 and klaunch.value > 0:
        comp = ((2 * sub.value - sfresh.value) * rec + 12.0 * W * H * args.frames) / klaunch.value
        roofline["compulsory_bytes"] = round(comp)
        roofline["compulsory_basis"] = (f"per launch: (2 x {sub.value / sb.value:.0f} touched units - "
                                        f"{sfresh.value / sb.value:.0f} new) x {rec} B records + 12 B x W x H x frames "
                                        "of staged pixels (ot_tsdf_batch_stats over one step)")
        if traffic:
            roofline["traffic_over_compulsory"] = round(traffic / comp, 3)
    ient, _ = _pmc_entry(args, L, kname, pmc_cfg)
    # the ceilings that actually bind this kernel: vector-ALU issue and the vector-memory data path (PMC, same build)
    for key in ("valu_busy_frac", "ta_busy_frac", "td_busy_frac", "tcc_hit_frac"):
        if ient and ient.get(key) is not None:
            roofline[key] = round(ient[key], 4)
    if ient and ient.get("valu_busy_frac") is not None:
        roofline["binding"] = "VALU issue {:.2f} + TD {:.2f} busy (HBM {:.2f})".format(
            ient["valu_busy_frac"], ient.get("td_busy_frac") or 0.0, roofline["frac"] or 0.0)
    roofline["frontend_ms_per_batch"] = round(fms.value / max(fbatches.value, 1), 5)
    if ient:  # raw counters and the correction applied to them (calibrated on 8-B gathers, tools/fetch_calib.hip)
        roofline["traffic_raw"] = {k: ient.get(k) for k in ("raw_fetch_kib", "raw_write_kib", "fetch_correction",
                                                            "fetch_correction_source", "write_correction")}

    # configs[2] stream set up (uploaded, handles + worker threads warmed) before the other legs allocate
    fstream = FilterStream(args, L, synth, torch, filt_frames) if (args.filter_frames > 0 and rank == 0) else None
    color32 = headline_color32(args, L, lib, torch, dist, world, d_depth, d_color, ext, intr, stream, upd.value) \
        if (args.color32 and args.color_bits == 64) else None

    # leg order: OT_BENCH_ORDER may repeat legs and insert "sleep" (5 s idle) for diagnosis; the
    # reported filtered / objects objects are the first run of each, later filtered runs go to filtered_repeat_ms
    order = os.environ.get("OT_BENCH_ORDER", "filtered,objects").split(",")
    filt = objects = None
    filt_repeat = []
    for leg in order:
        if leg == "filtered" and fstream is not None:
            r = fstream.run()
            if filt is None:
                filt = r
            else:
                filt_repeat.append(r["ms_per_frame"])
        if leg == "objects" and args.objects > 0:
            r = objects_pipeline(args, L, lib, synth, torch, dist, rank, world, obj_ids, obj_scans)
            objects = objects or r
        if leg == "sleep":
            time.sleep(5.0)
    if fstream is not None:
        fstream.close()
    if filt is not None and filt_repeat:
        filt["filtered_repeat_ms"] = filt_repeat
    hybrid = hybrid_fusion(args, L, synth, torch, dist, rank, world) if args.hybrid_objects > 0 else None

    spatial = spatial_shard(args, L, lib, synth, torch, dist, rank, world, n_units.value) \
        if (world > 1 and args.spatial) else None
    shard_steps = shard_rank_steps(args, L, lib, torch, d_depth, d_color, ext, intr, stream, ms_per_step) \
        if (world == 1 and args.shard_steps > 0) else None

    cpu = None
    if rank == 0 and args.cpu_frames > 0:
        cpu = cpu_baseline(depth, color, ext, intr_t, args)
    single = single_frame(L, synth, torch, depth, color, ext, intr_t) if (rank == 0 and args.cpu_frames > 0) \
        else None

    out = {"metric": METRIC, "value": round(value, 2), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
           "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None,
           "dtype": "f32 tsdf/weight + f64 colour" if args.color_bits == 64 else "f32 (colour state f32)",
           "data": "synthetic",
           "config": {"workload": "configs[1]: 256-frame 640x480 RGB-D TSDF integration, 5 mm voxel, "
                                  "sdf_trunc 0.04, one object scan per GPU (synthetic box-on-floor ring scan), "
                                  f"colour precision {args.color_bits}" +
                                  (" (Open3D's float64 TSDFVoxel::color_, exact division: bit-exact colours)"
                                   if args.color_bits == 64 else " (float32 colour state, |rel| <= 1e-4)"),
                      "color_precision": args.color_bits,
                      "frames_per_step": args.frames, "width": W, "height": H, "voxel_length": args.voxel,
                      "sdf_trunc": args.sdf_trunc, "volume_units": n_units.value,
                      "unit_integrations_per_step": unit_int.value, "parallelism": f"objects{world}"},
           "roofline": roofline, "cpu_baseline": cpu, "sustained": sustained, "color32": color32,
           "spatial_amdahl": spatial_amdahl(fms.value / max(fbatches.value, 1), kernel_ms_avg, shard_steps),
           "filtered": filt, "objects": objects,
           "hybrid_map": hybrid, "single_frame": single, "spatial": spatial, "source_hash": L.source_hash()}
    if rank == 0:
        print(json.dumps(out), flush=True)
    L.call("ot_tsdf_destroy", vol)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def headline_color32(args, L, lib, torch, dist, world, d_depth, d_color, ext, intr, stream, updates_c64):
    """Secondary leg, labelled: the configs[1] workload with the voxel colour state in float32 (one reciprocal per
    update, |rel| <= 1e-4 against Open3D's float64 colour; tsdf, weight and the update set are bit-identical).  Same
    frames, same timing method (K steps between barrier + synchronize, max over ranks)."""
    vol = C.c_void_p()
    L.call("ot_tsdf_create", args.voxel, args.sdf_trunc, L.OT_COLOR_RGB8, 16, 4, 0, C.byref(vol))
    L.call("ot_tsdf_set_color_precision", vol, 32)
    if args.batch > 0:
        L.call("ot_tsdf_set_batch", vol, args.batch)
    W, H = intr.width, intr.height
    npx = W * H
    integrate, pintr = lib.ot_tsdf_integrate_u16, C.byref(intr)
    dptrs = [C.c_void_p(d_depth.data_ptr() + k * npx * 2) for k in range(args.frames)]
    cptrs = [C.c_void_p(d_color.data_ptr() + k * npx * 3) for k in range(args.frames)]
    eptrs = [ext[k].ctypes.data_as(C.c_void_p) for k in range(args.frames)]

    def step():
        L.call("ot_tsdf_reset_async", vol, stream)
        for k in range(args.frames):
            if integrate(vol, dptrs[k], cptrs[k], pintr, eptrs[k], 1000.0, 3.0, stream):
                raise RuntimeError(lib.ot_last_error().decode())
        L.call("ot_tsdf_flush", vol, stream)

    for _ in range(2):
        step()
    steps = max(1, min(args.steps, 50))
    dt, _ = _timed(torch, dist, world, step, steps)
    upd = C.c_int64(0)
    L.call("ot_tsdf_counters", vol, C.byref(upd), None, stream)
    L.call("ot_tsdf_set_profiling", vol, 1)
    step()
    kms, kl = C.c_double(0.0), C.c_int64(0)
    L.call("ot_tsdf_kernel_time", vol, C.byref(kms), C.byref(kl))
    L.call("ot_tsdf_destroy", vol)
    kavg = kms.value / max(kl.value, 1)
    per_launch = (5.0 * W * H * args.frames + 40.0 * upd.value) / max(kl.value, 1)
    ent, note = _pmc_entry(args, L, "k_batch_integrate<false>", {"voxel": args.voxel, "frames": args.frames,
                                                                 "batch": args.batch, "color_bits": 32})
    roof = {"kernel": "k_batch_integrate<false>", "kernel_ms_avg": round(kavg, 5),
            "frac_effective": round(per_launch / (kavg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if kavg > 0 else None}
    if ent and kavg > 0:
        roof["hbm_frac"] = round(ent["bytes_per_launch"] / (kavg * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
        roof["traffic"] = ent["bytes_per_launch"]
    else:
        roof["traffic_source"] = note
    return {"workload": "configs[1] with colour precision 32 (float32 colour state, one reciprocal per update, "
                        "|rel| <= 1e-4 vs Open3D's float64 colour) -- a faster, narrower variant, not the headline",
            "steps": steps, "frames_per_s": round(world * args.frames / dt, 1), "ms_per_step": round(dt * 1e3, 3),
            "roofline": roof, "voxel_updates_match_headline": upd.value == updates_c64}


def spatial_shard(args, L, lib, synth, torch, dist, rank, world, units_rank0):
    """ONE object's scan (seed 0) on every rank, its volume spatially sharded (ot_tsdf_set_shard:
    rank r keeps the units with owner(key) == r), so N GPUs integrate one object together (strong scaling; at
    N = 1 this is the headline itself).  Timed like the headline (reset + all frames + flush, max over ranks).
    Then marching cubes over the shards with a border halo (distributed.extract_sharded_mesh: all-gather of the
    units' 721 low-face voxels sent to the owners of their -x/-y/-z neighbours only, halo import, own-unit extraction,
    all-gather + merge of the partial meshes) -- timed
    apart as the per-object cost before normals / sampling; assemble_bytes = border rows each rank receives (the
    old whole-unit all-gather's bytes beside it), and the merged mesh must equal rank 0's unsharded mesh."""
    import importlib

    pkg = importlib.import_module(PKG)
    Dm = importlib.import_module(PKG + ".distributed")
    integ = pkg.pipelines.integration
    intr_t = synth.REF_INTRINSICS_640
    W, H = intr_t[0], intr_t[1]
    depth, color, ext = synth.make_sequence(synth.Scene(seed=0), n_frames=args.frames, intr=intr_t)
    d_depth = torch.from_numpy(depth.view(np.int16)).cuda().view(torch.uint16).contiguous()
    d_color = torch.from_numpy(color).cuda().contiguous()
    ext = np.ascontiguousarray(ext, dtype=np.float64)
    intr = L.ot_intrinsics(W, H, *intr_t[2:])
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)

    def make(shard):
        v = integ.ScalableTSDFVolume(voxel_length=args.voxel, sdf_trunc=args.sdf_trunc,
                                     color_type=integ.TSDFVolumeColorType.RGB8)
        if shard:
            v.set_shard_sector(rank, world, scan_centre_xy(ext))
        if args.batch > 0:
            v.set_batch(args.batch)
        return v

    vol = make(True)
    npx = W * H
    dptrs = [C.c_void_p(d_depth.data_ptr() + k * npx * 2) for k in range(args.frames)]
    cptrs = [C.c_void_p(d_color.data_ptr() + k * npx * 3) for k in range(args.frames)]
    eptrs = [ext[k].ctypes.data_as(C.c_void_p) for k in range(args.frames)]
    integrate, pintr = lib.ot_tsdf_integrate_u16, C.byref(intr)

    def step(v=vol):
        L.call("ot_tsdf_reset_async", v._h, stream)
        for k in range(args.frames):
            if integrate(v._h, dptrs[k], cptrs[k], pintr, eptrs[k], 1000.0, 3.0, stream):
                raise RuntimeError(lib.ot_last_error().decode())
        L.call("ot_tsdf_flush", v._h, stream)

    dt, _ = _timed(torch, dist, world, step, args.steps)
    # this rank's per-batch front end (undivided: staging + touch + unit headers) and integrate (divided), one step
    L.call("ot_tsdf_set_profiling", vol._h, 1)
    step()
    fe, fb, ik, il = C.c_double(0.0), C.c_int64(0), C.c_double(0.0), C.c_int64(0)
    L.call("ot_tsdf_frontend_time", vol._h, C.byref(fe), C.byref(fb))
    L.call("ot_tsdf_kernel_time", vol._h, C.byref(ik), C.byref(il))
    L.call("ot_tsdf_set_profiling", vol._h, 0)
    per = torch.tensor([[fe.value / max(fb.value, 1), ik.value / max(il.value, 1)]], dtype=torch.float64,
                       device=COLL_DEV)
    per = Dm.all_gather_rows(per).cpu().numpy()
    nu = vol.num_units()
    cnt = Dm.all_gather_rows(torch.tensor([[nu]], dtype=torch.int64, device=COLL_DEV)).flatten().tolist()
    group = None

    def assemble():
        return Dm.extract_sharded_mesh(vol, group)

    t_asm, (mesh, border_bytes) = _timed(torch, dist, world, assemble, 1)
    whole = sum(cnt) * (3 + 4096 * (2 + 6)) * 4  # the whole-unit all-gather (f64 colour rows) it replaces
    nb = Dm.all_gather_rows(torch.tensor([[int(vol.export_border()[0].shape[0])]], dtype=torch.int64,
                                         device=COLL_DEV)).flatten().tolist()
    allgather_border = (sum(nb) - nb[rank]) * (3 + 721 * 8) * 4  # every rank's border rows to every rank (round 2)
    match = None
    if rank == 0:  # the unsharded volume of the same scan, extracted on rank 0 (untimed)
        ref = make(False)
        step(ref)
        m0 = ref.extract_triangle_mesh()
        match = bool(torch.equal(mesh._v.dev(), m0._v.dev()) and torch.equal(mesh._t.dev(), m0._t.dev()) and
                     torch.equal(mesh._vc.dev(), m0._vc.dev()))
        del ref
    return {"workload": f"configs[1] scan (seed 0) as ONE object spatially sharded over {world} GPU(s): unit owner = "
                        f"the unit centre's azimuth sector (1/{world} of the turn) around the mean camera position "
                        "(tsdf.h unit_owner, ot_tsdf_set_shard_sector), every rank integrates every frame into its own "
                        "units and stages only the image tiles they project to; marching cubes with a border halo "
                        "routed to the owners of the -x/-y/-z neighbours",
            "scaling": "strong", "frames_per_s": round(args.frames * 1.0 / dt, 1), "ms_per_step": round(dt * 1e3, 3),
            "units_per_rank_min": min(cnt), "units_per_rank_max": max(cnt), "assemble_ms": round(t_asm * 1e3, 2),
            "assemble_bytes": border_bytes, "allgather_border_bytes": allgather_border, "whole_unit_bytes": whole,
            "mesh_vertices": int(mesh._v.dev().shape[0]), "mesh_matches_unsharded": match,
            "frontend_ms_per_batch_max": round(float(per[:, 0].max()), 5),
            "integrate_ms_per_batch_max": round(float(per[:, 1].max()), 5),
            "frontend_note": "every rank unprojects every stride sample; staging divides by the tiles its units project "
                             "to (split front end); the integrate divides by units"}


def scan_centre_xy(ext):
    """The centre of a ring scan for sector ownership: the mean camera position (x, y) over the frames (camera centre
    = -R^T t of each world->camera extrinsic).  A reference caller knows it as the ScanObject goal's x, y."""
    e = np.asarray(ext, np.float64).reshape(-1, 4, 4)
    c = -np.einsum("nji,nj->ni", e[:, :3, :3], e[:, :3, 3])
    return float(c[:, 0].mean()), float(c[:, 1].mean())


def shard_rank_steps(args, L, lib, torch, d_depth, d_color, ext, intr, stream, headline_ms, worlds=(1, 2, 4, 8)):
    """SURVEY 8(e) measured on one GPU: the headline step (reset + the 256-frame scan + flush) of a volume that keeps
    only rank r's units, for every rank r of N = 2, 4, 8, under both ownerships: `blocks` (ot_tsdf_set_shard: hashed
    blocks of units) and `sectors` (ot_tsdf_set_shard_sector: azimuth sectors around the scan centre, the product
    choice since round 6) -- both with the library's sharded defaults: the split front end (a sharded volume stages
    only the image tiles its batch's units project to), double-buffered beside the previous batch's integrate.  A rank's step on an N-GPU node is this time (its shard, its front end, nothing shared with the
    other ranks), so the unsharded step (N = 1, the same method) / max over r is the strong-scaling speed-up of one
    object before the halo extraction.  The resident scan goes in with ot_tsdf_integrate_u16_frames (one host call
    per scan, the bits of 256 per-frame calls): at 1/8 of the integrate a rank's GPU step is shorter than 256 ctypes
    round trips."""
    cx, cy = scan_centre_xy(ext[:args.frames])
    integrate_frames, pintr = lib.ot_tsdf_integrate_u16_frames, C.byref(intr)
    dp, cp, ep = d_depth.data_ptr(), d_color.data_ptr(), ext.ctypes.data
    out = {}
    for N in worlds:
        per_mode = {}
        for mode in (("blocks", "sectors") if N > 1 else ("unsharded",)):
            worst, units = 0.0, []
            for r in range(N):
                vol = C.c_void_p()
                L.call("ot_tsdf_create", args.voxel, args.sdf_trunc, L.OT_COLOR_RGB8, 16, 4, 0, C.byref(vol))
                try:
                    L.call("ot_tsdf_set_color_precision", vol, args.color_bits)
                    if mode == "blocks":
                        L.call("ot_tsdf_set_shard", vol, r, N)
                    elif mode == "sectors":
                        L.call("ot_tsdf_set_shard_sector", vol, r, N, cx, cy)

                    def step():
                        L.call("ot_tsdf_reset_async", vol, stream)
                        if integrate_frames(vol, args.frames, dp, cp, pintr, ep, 1000.0, 3.0, stream):
                            raise RuntimeError(lib.ot_last_error().decode())
                        L.call("ot_tsdf_flush", vol, stream)

                    for _ in range(3):
                        step()
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for _ in range(args.shard_steps):
                        step()
                    torch.cuda.synchronize()
                    worst = max(worst, (time.perf_counter() - t0) * 1e3 / args.shard_steps)
                    nu = C.c_int64(0)
                    L.call("ot_tsdf_num_units", vol, C.byref(nu), stream)
                    units.append(nu.value)
                finally:
                    L.call("ot_tsdf_destroy", vol)
            per_mode[mode] = {"rank_step_ms_max": round(worst, 4), "units_per_rank_min_max": [min(units), max(units)]}
        out[str(N)] = per_mode
    base = out["1"]["unsharded"]["rank_step_ms_max"]
    for N, per_mode in out.items():
        for m in per_mode.values():
            if m["rank_step_ms_max"]:
                m["speedup"] = round(base / m["rank_step_ms_max"], 2)
    return {"method": "every rank's shard of the headline scan timed on this GPU (reset + 256 frames in one "
                      f"ot_tsdf_integrate_u16_frames call + flush, {args.shard_steps} steps after 3 warm-up), max over "
                      "ranks; speedup = the unsharded volume's step (N = 1, same method) / that; sectors centred on "
                      f"the mean camera position ({cx:.4f}, {cy:.4f})",
            "headline_ms_per_step": round(headline_ms, 4), "worlds": out}


def spatial_amdahl(frontend_ms, integrate_ms, measured=None):
    """Amdahl bound of ONE object spatially sharded over N GPUs, from this run's per-batch device times
    of the UNSHARDED volume: if every rank repeated the whole front end (staging + touch + unit headers) while the
    integrate divides by the units each rank owns, the speed-up at N would be capped at (F + I) / (F + I / N).  Since
    round 6 a sharded rank's front end is split and stages only the tiles its units project to (sector ownership:
    ~1/N of the pixels of a ring scan), so `measured` (every rank's shard timed) can pass this cap."""
    F, I = frontend_ms, integrate_ms
    if F <= 0 or I <= 0:
        return None
    return {"frontend_ms_per_batch": round(F, 5), "integrate_ms_per_batch": round(I, 5),
            "undivided_fraction": round(F / (F + I), 4),
            "speedup_cap_serial": {str(n): round((F + I) / (F + I / n), 2) for n in (2, 4, 8)},
            "speedup_cap_overlap": {str(n): round((F + I) / max(F, I / n), 2) for n in (2, 4, 8)},
            "measured": measured,
            "note": "one object over N GPUs; caps model a step as F + I/N per batch (front end then integrate) or "
                    "max(F, I/N) (double-buffered front end beside the previous batch's integrate); `measured` times "
                    "every rank's shard; the weak-scaling headline (one object per GPU) is not bounded by this"}


def single_frame(L, synth, torch, depth, color, ext, intr_t, reps=50):
    """configs[0]: one 640x480 RGB-D frame -> create_from_color_and_depth (depth_trunc 5 m) ->
    create_from_rgbd_image -> voxel_down_sample(0.005) (check_one_frame.py:22-28), the reference's own CPU case.
    Reported beside the CPU restatement of the same calls on the same frame (the GPU slice is the parity case)."""
    W, H = intr_t[0], intr_t[1]
    npx = W * H
    d16 = torch.from_numpy(depth[0].view(np.int16)).cuda().view(torch.uint16).contiguous()
    col = torch.from_numpy(color[0]).cuda().contiguous()
    df = torch.empty((H, W), dtype=torch.float32, device="cuda")
    xyz = torch.empty((npx, 3), dtype=torch.float64, device="cuda")
    rgb = torch.empty((npx, 3), dtype=torch.float64, device="cuda")
    vx = torch.empty((npx, 3), dtype=torch.float64, device="cuda")
    vc = torch.empty((npx, 3), dtype=torch.float64, device="cuda")
    intr = L.ot_intrinsics(W, H, *intr_t[2:])
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    ident = np.eye(4)
    P, K = C.c_int64(0), C.c_int64(0)
    ptr = lambda t: C.c_void_p(t.data_ptr())

    def run():
        L.call("ot_depth_to_float", ptr(d16), ptr(df), npx, 1000.0, 5.0, stream)
        L.call("ot_unproject", ptr(df), ptr(col), C.byref(intr), ident.ctypes.data_as(C.c_void_p), 1, ptr(xyz),
               ptr(rgb), npx, C.byref(P), stream)
        L.call("ot_voxel_down_sample", ptr(xyz), ptr(rgb), None, P.value, 0.005, ptr(vx), ptr(vc), None, None,
               C.byref(K), stream)

    run()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    torch.cuda.synchronize()
    gdt = (time.perf_counter() - t0) / reps
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    t1 = time.perf_counter()
    for _ in range(3):
        x, c = O.unproject(O.depth_to_float(depth[0], 1000.0, 5.0), color[0], intr_t, ident)
        v = O.voxel_down_sample(x, c, 0.005)[0]
    cdt = (time.perf_counter() - t1) / 3
    return {"workload": "configs[0]: one 640x480 RGB-D frame, create_from_rgbd_image + voxel_down_sample(0.005) "
                        "(check_one_frame.py:22-28)", "points": P.value, "voxels": K.value,
            "gpu_ms": round(gdt * 1e3, 3), "cpu_ms": round(cdt * 1e3, 3), "cpu_voxels": int(v.shape[0]),
            "cpu_kind": "port (serial, as Open3D's unprojection and voxel downsample)"}


def _timed(torch, dist, world, fn, steps):
    """max-over-ranks seconds per call of fn() (barrier + synchronize on both sides of the timed calls)."""
    fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        out = fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = (time.perf_counter() - t0) / steps
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device=COLL_DEV)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt, out


def _render_objects(synth, ids, n_frames):
    """Synthetic ring scans of object_scene(i) for the given ids (process pool when a rank renders several)."""
    if len(ids) <= 1:
        return [synth.make_sequence(synth.object_scene(i), n_frames=n_frames) for i in ids]
    from concurrent.futures import ProcessPoolExecutor

    import multiprocessing as mp

    with ProcessPoolExecutor(max_workers=min(len(ids), 8), mp_context=mp.get_context("fork")) as ex:
        futs = [ex.submit(synth.make_sequence, synth.object_scene(i), n_frames) for i in ids]
        return [f.result() for f in futs]


def objects_pipeline(args, L, lib, synth, torch, dist, rank, world, ids, scans):
    """configs[3]: --objects independent object scans x --object-frames 640x480 frames, contiguous shards per rank
    (reconstruct_rgbd_filter.py:154-155).  Per object, on device: integrate every frame (5 mm, sdf_trunc 0.04) ->
    extract_triangle_mesh -> compute_vertex_normals -> sample_points_uniformly(100000) -> z >= 0.03 mask
    (reconstruct_rgbd_filter.py:81-132); then the RCCL all-gather merge of the filtered clouds in sorted order
    (distributed.merge_object_clouds).  frames/s = all frames of all objects / max-over-ranks wall time."""
    pkg = importlib.import_module(PKG)
    D = importlib.import_module(PKG + ".distributed")
    intr_t = synth.REF_INTRINSICS_640
    W, H = intr_t[0], intr_t[1]
    intr = L.ot_intrinsics(W, H, *intr_t[2:])
    intr_ref = C.byref(intr)
    dev = []
    for depth, color, ext in scans:
        dev.append((torch.from_numpy(depth.view(np.int16)).cuda().view(torch.uint16).contiguous(),
                    torch.from_numpy(color).cuda().contiguous(), np.ascontiguousarray(ext, dtype=np.float64)))
    vols = [pkg.pipelines.integration.ScalableTSDFVolume(
        voxel_length=args.voxel, sdf_trunc=args.sdf_trunc,
        color_type=pkg.pipelines.integration.TSDFVolumeColorType.RGB8) for _ in dev]
    npx = W * H
    sizes = {}
    # objects are independent: T host threads, each driving its own HIP stream (the library's scratch buffers
    # are per thread), reconstruct them concurrently so one object's mesh kernels overlap another's integration
    from concurrent.futures import ThreadPoolExecutor

    T = max(1, min(args.object_streams, len(dev)))
    streams = importlib.import_module(PKG + ".streams").worker_streams(T)
    pool = ThreadPoolExecutor(max_workers=T)

    def reconstruct(t):
        out = {}
        with torch.cuda.stream(streams[t]):
            stream = C.c_void_p(streams[t].cuda_stream)
            for j in range(t, len(dev), T):
                vol, (d16, col, ext) = vols[j], dev[j]
                vol.reset()
                dp, cp, ep = d16.data_ptr(), col.data_ptr(), ext.ctypes.data  # plain int addresses per call
                # the object's 64 frames in one host call (ot_tsdf_integrate_u16_frames = 64 ot_tsdf_integrate_u16)
                if lib.ot_tsdf_integrate_u16_frames(vol._h, ext.shape[0], dp, cp, intr_ref, ep, 1000.0, 3.0, stream):
                    raise RuntimeError(lib.ot_last_error().decode())
                if fused:  # extract -> normals -> 100k samples + Z mask, one host call
                    out[j] = vol.extract_mesh_and_sample_min_z(100000, 0.03)[1]
                    continue
                mesh = vol.extract_triangle_mesh()
                mesh.compute_vertex_normals()
                out[j] = mesh
            streams[t].synchronize()
        return out

    fused = args.objects_sampling == "fused"

    def run():
        parts = {}
        for r in pool.map(reconstruct, range(T)):
            parts.update(r)
        if fused:
            pcds = [parts[j] for j in range(len(dev))]
        else:  # the objects' 100k-point samplings and Z masks in one call: their area-CDF chains side by side
            pcds = pkg.geometry.TriangleMesh.sample_points_min_z_batch([parts[j] for j in range(len(dev))], 100000,
                                                                      0.03)
        clouds = [p._xyz.dev() for p in pcds]
        # every rank holds <= ceil(objects / N) objects of <= 100k points: one collective with the counts in-band while
        # that padded bound stays small (distributed.CAPPED_MAX_BYTES), else a count exchange and a tight gather
        merged = D.merge_object_clouds(clouds, capacity=((args.objects + world - 1) // world) * 100000)
        sizes["local"] = sum(int(c.shape[0]) for c in clouds)
        return merged

    dt, merged = _timed(torch, dist, world, run, 10)  # ~20 ms per call: 10 calls keep run-to-run noise near 2 %
    pool.shutdown()

    # one object end to end on one stream (integrate -> mesh -> normals -> 100k samples -> z mask): the latency that
    # bounds the objects-over-GPUs time from below (8 objects on 8 GPUs cannot finish faster than one object)
    single = None
    if dev:
        vol, (d16, col, ext) = vols[0], dev[0]
        s_ = C.c_void_p(torch.cuda.current_stream().cuda_stream)

        dp, cp, ep = d16.data_ptr(), col.data_ptr(), ext.ctypes.data

        def one():
            vol.reset()
            if lib.ot_tsdf_integrate_u16_frames(vol._h, ext.shape[0], dp, cp, intr_ref, ep, 1000.0, 3.0, s_):
                raise RuntimeError(lib.ot_last_error().decode())
            if fused:
                return vol.extract_mesh_and_sample_min_z(100000, 0.03)[1]
            mesh = vol.extract_triangle_mesh()
            mesh.compute_vertex_normals()
            return mesh.sample_points_min_z(100000, 0.03)

        one()
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            t1 = time.perf_counter()
            one()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t1)
        single = round(float(np.median(ts)) * 1e3, 3)
    merge = _merge_label(world, ((args.objects + world - 1) // world) * 100000)
    return {"workload": f"configs[3]: {args.objects} object scans x {args.object_frames} 640x480 frames, "
                        f"{args.voxel * 1000:g} mm TSDF -> mesh -> normals -> 100k samples + z mask (one pass) per object "
                        f"({'one host call from the mesh totals to the sampler' if fused else 'batched sampling'}), "
                        f"contiguous object shards over {world} GPU(s) ({T} concurrent streams per GPU), merge: {merge}",
            "frames_per_s": round(args.objects * args.object_frames / dt, 1), "ms": round(dt * 1e3, 3),
            "objects_per_rank": len(ids), "merged_points": int(merged.shape[0]), "merge": merge,
            "single_object_ms": single,
            "single_object_note": "median of 5, object 0 of this rank on one stream, same pipeline, no merge",
            # this run's objects time over one object's latency: the most an objects-over-GPUs run (one object per
            # GPU) can gain over this one, before its merge
            "objects_over_single": round(dt * 1e3 / single, 2) if single else None}


def _merge_label(world, capacity=None):
    """the collectives a merge actually runs at this world size / backend / capacity bound (merge_object_clouds takes
    the padded single collective only while it stays under distributed.CAPPED_MAX_BYTES)"""
    if world == 1:
        return "local concatenation (N=1: no process group, no collective)"
    D = importlib.import_module(PKG + ".distributed")
    lib = "RCCL" if COLL_DEV == "cuda" else "gloo"
    if capacity is not None and D.capped_fits(capacity, 3):
        return f"one {lib} all-gather (counts in-band)" + (" over xGMI" if lib == "RCCL" else "")
    return f"a {lib} all-gather of the row counts, one host read, a {lib} all-gather of the rows"


def hybrid_fusion(args, L, synth, torch, dist, rank, world):
    """configs[4]: hybrid-map fusion with change detection against a saved map.  Inputs resident in HBM: a
    1024x1024 occupancy grid @ 5 cm (saved + new) and --hybrid-objects object clouds (~100k points, sharded over
    ranks) with their saved-map versions.  Timed per fusion: per rank, voxel-key diff (2 cm lattice) of each of
    its objects vs the saved version; rank 0, smart_paste merge of the new grid onto the saved one
    (2d_selective_merge.py) and the occupied-cell cloud (hybrid_map.py:25-60); then the RCCL all-gather of the
    object clouds (hybrid_map.py:62-96, map cloud first)."""
    import ctypes as Cc

    Dm = importlib.import_module(PKG + ".distributed")
    CD = importlib.import_module(PKG + ".change_detection")
    ids = Dm.shard(list(range(args.hybrid_objects)), rank, world)
    objs = [torch.from_numpy(synth.object_cloud(i)).cuda() for i in ids]
    saved = [torch.from_numpy(synth.object_cloud(i, moved=True)).cuda() for i in ids]
    old_map, new_map = synth.occupancy_pair(1024, 1024, seed=0)
    d_old = torch.from_numpy(old_map).cuda()
    d_new = torch.from_numpy(new_map).cuda()
    d_base = torch.empty_like(d_old)
    occ = torch.empty((1024 * 1024, 3), dtype=torch.float64, device="cuda")
    stream = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    origin = (Cc.c_double * 3)(-1.0, -1.0, -1.0)
    stats = {}

    # this rank's object clouds concatenated once (resident input), with host row offsets per object
    empty = torch.zeros((0, 3), dtype=torch.float64, device="cuda")
    cat_new = torch.cat(objs, 0).contiguous() if objs else empty
    cat_old = torch.cat(saved, 0).contiguous() if saved else empty
    off_new = np.concatenate([[0], np.cumsum([int(o.shape[0]) for o in objs])]).astype(np.int64)
    off_old = np.concatenate([[0], np.cumsum([int(o.shape[0]) for o in saved])]).astype(np.int64)
    cap = ((args.hybrid_objects + world - 1) // world) * 100000  # synth.object_cloud: 100k points per object
    keys_a = torch.empty((int(off_new[-1]) + 1, 4), dtype=torch.int32, device="cuda")
    keys_r = torch.empty((int(off_old[-1]) + 1, 4), dtype=torch.int32, device="cuda")

    def run():
        # change detection of every object vs its saved version: one multi-object voxel-key diff
        na, nr = C.c_int64(0), C.c_int64(0)
        if objs:
            L.call("ot_voxel_key_diff_multi", C.c_void_p(cat_new.data_ptr()), off_new.ctypes.data_as(C.c_void_p),
                   C.c_void_p(cat_old.data_ptr()), off_old.ctypes.data_as(C.c_void_p), len(objs), 0.02, origin,
                   C.c_void_p(keys_a.data_ptr()), C.byref(na), C.c_void_p(keys_r.data_ptr()), C.byref(nr), stream)
        added, removed = na.value, nr.value
        nq = C.c_int64(0)
        if rank == 0:
            d_base.copy_(d_old)
            ch = C.c_int64(0)
            L.call("ot_grid_smart_paste", C.c_void_p(d_base.data_ptr()), C.c_void_p(d_new.data_ptr()), 1024, 1024,
                   0, 0, 1024, 1024, CD.UNKNOWN_PIXEL, CD.PASTE_THRESHOLD, C.byref(ch), stream)
            L.call("ot_occupancy_to_points", C.c_void_p(d_base.data_ptr()), 1024, 1024, 100, 0.05, -25.6, -25.6,
                   C.c_void_p(occ.data_ptr()), C.byref(nq), stream)
            stats["changed_cells"] = ch.value
        merged = Dm.merge_object_clouds(objs, capacity=cap)  # counts in-band while the padding is small
        if rank == 0:
            merged = torch.cat([occ[:nq.value], merged], 0)
        stats.update(added=added, removed=removed)
        return merged

    dt, merged = _timed(torch, dist, world, run, 5)
    npts = sum(int(o.shape[0]) for o in objs)
    t = torch.tensor([npts], dtype=torch.int64, device=COLL_DEV)
    if world > 1:
        dist.all_reduce(t)
    return {"workload": f"configs[4]: 1024x1024 occupancy grid @ 5 cm + {args.hybrid_objects} object clouds, "
                        "change detection vs the saved map (smart_paste grid merge + 2 cm voxel-key diff per object), "
                        f"hybrid cloud assembled over {world} GPU(s), merge: {_merge_label(world, cap)}",
            "ms": round(dt * 1e3, 3), "mpoints_per_s": round(int(t.item()) / dt / 1e6, 2),
            "merged_points": int(merged.shape[0]) if rank == 0 else None,
            "changed_grid_cells": stats.get("changed_cells"), "added_keys_rank0": stats.get("added"),
            "removed_keys_rank0": stats.get("removed")}


class FilterStream:
    """configs[2]: a 1280x720 RGB-D stream of --filter-frames DISTINCT frames (rendered before GPU init, resident in
    HBM: 512 x 4.6 MB), per frame create_from_color_and_depth(depth_trunc 5 m) -> create_from_rgbd_image ->
    voxel_down_sample(0.005) -> remove_statistical_outlier(20, 2.0) -> select_by_index (check_one_frame.py:22-28 +
    SURVEY A.7), through the batched device-resident chain ot_rgbd_filter_run: --filter-batch frames per call,
    --filter-streams calls in flight (one host thread + HIP stream + handle each).  Mpoints/s counts valid input
    points per second.  The CPU oracle runs the same chain on 2 of the frames (1 warm-up, median of 5).

    Set up (inputs uploaded, handles created, every handle and worker thread warmed up) at bench start, like a
    long-lived service; run() is the timed stream.  Its HIP streams are the process's shared worker streams
    (streams.py): with streams created ad hoc per leg, whichever leg created its streams second could get two of
    them on one hardware queue (this leg 0.16 -> 0.20 ms/frame, the configs[3] leg 19 -> 24 ms)."""

    def __init__(self, args, L, synth, torch, frames):
        self.args, self.L, self.synth, self.torch, self.frames = args, L, synth, torch, frames
        depth, color, ext = frames
        intr_t = synth.REF_INTRINSICS_1280
        self.W, self.H = intr_t[0], intr_t[1]
        self.npx = self.W * self.H
        self.nf = depth.shape[0]
        self.d16 = torch.from_numpy(depth.view(np.int16)).cuda().view(torch.uint16).contiguous()
        self.col = torch.from_numpy(color).cuda().contiguous()
        self.exts = np.ascontiguousarray(ext, dtype=np.float64).reshape(self.nf, 16)
        intr = L.ot_intrinsics(self.W, self.H, *intr_t[2:])
        self.B, self.T = max(1, args.filter_batch), max(1, args.filter_streams)
        self.nb = (self.nf + self.B - 1) // self.B
        self.handles = []
        for _ in range(self.T):
            h = C.c_void_p()
            L.call("ot_rgbd_filter_create", C.byref(intr), self.B, 1000.0, 5.0, 0.005, 20, 2.0, C.byref(h))
            self.handles.append(h)
        self.streams = importlib.import_module(PKG + ".streams").worker_streams(self.T)
        from concurrent.futures import ThreadPoolExecutor

        self.pool = ThreadPoolExecutor(max_workers=self.T)
        # warm-up: every handle and every worker thread (thread-local scratch) on the batches with the most points
        for _ in range(2):
            for _ in self.pool.map(lambda t: self.worker(t, [t % self.nb]), range(self.T)):
                pass
        torch.cuda.synchronize()

    def worker(self, t, batches):
        L, B, nf, npx = self.L, self.B, self.nf, self.npx
        tot = [0, 0, 0]
        with self.torch.cuda.stream(self.streams[t]):
            s_ = C.c_void_p(self.streams[t].cuda_stream)
            for b in batches:
                f0 = b * B
                n = min(B, nf - f0)
                L.call("ot_rgbd_filter_run", self.handles[t], n, C.c_void_p(self.d16.data_ptr() + f0 * npx * 2),
                       C.c_void_p(self.col.data_ptr() + f0 * npx * 3),
                       self.exts[f0:f0 + n].ctypes.data_as(C.c_void_p), s_)
                P, K, KK = C.c_int64(0), C.c_int64(0), C.c_int64(0)
                L.call("ot_rgbd_filter_sizes", self.handles[t], C.byref(P), C.byref(K), C.byref(KK), None, None, None)
                tot = [tot[0] + P.value, tot[1] + K.value, tot[2] + KK.value]
            self.streams[t].synchronize()
        return tot

    def close(self):
        self.pool.shutdown()
        for h in self.handles:
            self.L.call("ot_rgbd_filter_destroy", h)
        self.handles = []
        del self.d16, self.col
        self.torch.cuda.empty_cache()

    def run(self):
        return filter_stream(self)


def filter_stream(fs):
    args, L, synth, torch = fs.args, fs.L, fs.synth, fs.torch
    depth, color, ext = fs.frames
    intr_t = synth.REF_INTRINSICS_1280
    W, H, nf, B, T, nb = fs.W, fs.H, fs.nf, fs.B, fs.T, fs.nb
    torch.cuda.synchronize()
    a0 = L.alloc_count()
    t0 = time.perf_counter()
    pts = vox = kept = 0
    for p_, v_, k_ in fs.pool.map(lambda t: fs.worker(t, list(range(t, nb, T))), range(T)):
        pts, vox, kept = pts + p_, vox + v_, kept + k_
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    allocs = L.alloc_count() - a0
    # CPU oracle: the same chain on frames 0 and nf // 2 (1 warm-up pass, median of 5 timed passes)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    sample = [0, nf // 2]

    def cpu_pass():
        n_pts = 0
        for f in sample:
            x, c = O.unproject(O.depth_to_float(depth[f], 1000.0, 5.0), color[f], intr_t, ext[f])
            v = O.voxel_down_sample(x, c, 0.005)[0]
            O.remove_statistical_outlier(v, 20, 2.0)
            n_pts += x.shape[0]
        return n_pts

    cpu_pass()
    times = []
    for _ in range(5):
        t1 = time.perf_counter()
        cpu_pts = cpu_pass()
        times.append(time.perf_counter() - t1)
    cdt = float(np.median(times))
    cores = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    bytes_frame = 5.0 * W * H + 15.0 * kept / nf
    return {"workload": f"configs[2]: {nf} distinct 1280x720 RGB-D frames, create_from_rgbd_image (depth_trunc 5 m) + "
                        f"voxel_down_sample(0.005) + remove_statistical_outlier(20, 2.0) + select_by_index per frame; "
                        f"batched device-resident chain, {B} frames per call, {T} calls in flight",
            "frames": nf, "distinct_frames": nf, "batch": B, "streams": T,
            "mpoints_per_s": round(pts / dt / 1e6, 2), "frames_per_s": round(nf / dt, 2),
            "ms_per_frame": round(dt * 1e3 / nf, 4), "points_per_frame": round(pts / nf),
            "voxels_per_frame": round(vox / nf), "kept_per_frame": round(kept / nf),
            "allocs_in_timed_region": allocs,
            # SURVEY 8(d) fused configs[2] pipeline bytes: 5*W*H (u16 depth + RGB8) + 15*K_kept per frame over the
            # wall time (intermediates not counted; the chain is sort / kNN bound)
            "roofline": {"bound": "hbm", "unit": "GB/s", "peak": HBM_PEAK_GBS,
                         "algorithmic_bytes_per_frame": round(bytes_frame),
                         "achieved": round(bytes_frame * nf / dt / 1e9, 2),
                         "frac": round(bytes_frame * nf / dt / 1e9 / HBM_PEAK_GBS, 5)},
            "kernel_roofline": _sor_roofline(args, fs.L),
            "cpu_baseline": {"mpoints_per_s": round(cpu_pts / cdt / 1e6, 3), "cores": cores, "kind": "port",
                             "sample": f"frames {sample} of the same stream, CPU oracle chain, 1 warm-up + median of 5"}}


def _sor_roofline(args, L):
    """The chain's dominant kernel, k_sor_knn (SOR stage 1), against the ceiling that binds it: vector-ALU issue
    (PMC SQ_ACTIVE_INST_VALU x 4 per SIMD-cycle of the dispatch, same build; tools/pmc.sh runs it on batches of
    --filter-batch frames of the same stream -- the entry's workload must say the batch this bench times).  Its HBM
    traffic per launch is reported beside it, with the algorithmic bytes (12 B per point read + 12 B per kept point,
    SURVEY 8(d)) when the entry records them."""
    ent, note = _pmc_entry(args, L, "k_sor_knn", {"batch": args.filter_batch})
    if not ent or ent.get("valu_busy_frac") is None:
        return {"kernel": "k_sor_knn", "bound": "valu", "frac": None, "source": note}
    cyc = ent.get("dispatch_cycles")
    out = {"kernel": "k_sor_knn", "bound": "valu", "frac": round(ent["valu_busy_frac"], 4),
           "valu_insts_per_launch": ent.get("valu_insts_per_launch"),
           "frames_per_launch": ent.get("config", {}).get("batch"),
           "dispatch_cycles": round(cyc) if cyc else None, "td_busy_frac": ent.get("td_busy_frac"),
           "hbm_bytes_per_launch": ent.get("bytes_per_launch"), "source": note}
    if ent.get("config", {}).get("algorithmic_bytes_per_launch"):
        alg = ent["config"]["algorithmic_bytes_per_launch"]
        out["algorithmic_bytes_per_launch"] = alg
        out["traffic_over_algorithmic"] = round(ent["bytes_per_launch"] / alg, 3)
    return out


def _pmc_entry(args, L, kernel, config):
    """The PMC summary of `kernel` from profiles/pmc_traffic.json -- only when the file was taken on this build
    (source hash) and the same workload; else (None, reason)."""
    try:
        with open(args.traffic) as f:
            tr = json.load(f)
    except Exception:
        return None, "no PMC file"
    ent = tr.get("kernels_traffic", {}).get(kernel)
    if not ent:
        return None, f"no PMC entry for {kernel}"
    if tr.get("source_hash") != L.source_hash():
        return None, f"stale PMC file (source hash {tr.get('source_hash')} != {L.source_hash()})"
    cfg = ent.get("config", tr.get("config", {}))
    if any(cfg.get(k) != v for k, v in config.items()):
        return None, f"PMC entry workload {cfg} != {config}"
    return ent, f"{os.path.relpath(args.traffic, ROOT)} (source hash {tr['source_hash']})"


def _traffic(args, L, kernel, config):
    """Measured HBM bytes per launch of `kernel` (same build and workload), else (None, reason)."""
    ent, note = _pmc_entry(args, L, kernel, config)
    return (ent["bytes_per_launch"] if ent else None), note


def cpu_baseline(depth, color, ext, intr_t, args):
    """CPU oracle (kind "port") on the --cpu-frames first frames of the same scan (default: all 256, the headline's
    whole step): 1 warm-up pass, then the median of 3 timed passes, each into a fresh volume; the per-pass spread is
    reported beside the median (host load moves it by +-20 % across boxes)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    O.lib()
    n = min(args.cpu_frames, depth.shape[0])
    dfs = [O.depth_to_float(depth[k], 1000.0, 3.0) for k in range(n)]

    def one_pass():
        vol = O.TSDF(args.voxel, args.sdf_trunc, 1, 4)
        t0 = time.perf_counter()
        for k in range(n):
            vol.integrate(dfs[k], color[k], intr_t, ext[k])
        return time.perf_counter() - t0

    one_pass()
    times = [one_pass() for _ in range(3)]
    dt = float(np.median(times))
    cores = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
    return {"value": round(n / dt, 3), "unit": "frames/s", "cores": cores, "kind": "port",
            "sample": f"{'all' if n == depth.shape[0] else 'first'} {n} of the {args.frames} frames, same synthetic "
                      f"scan, one fresh volume per pass (float64 colour state, as Open3D and the headline), 1 warm-up "
                      f"+ median of 3 passes, depth->float excluded (done before timing), OMP_NUM_THREADS={cores}",
            "pass_seconds": [round(t, 3) for t in times],
            "frames_per_s_min_max": [round(n / max(times), 3), round(n / min(times), 3)]}


if __name__ == "__main__":
    main()
