"""Where a chain walk's time goes (otx_chain_walk_trace): the sampling's area sum and CDF chains of a configs[3] object
mesh (object_scene(0), 64 frames, 5 mm), each walk event time-stamped with clock64 -- cycles spent per event kind
(run accepted / accepted after the 64-way search / serial chunk) and the walk's total.  Tool only."""
import ctypes as C
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
PKG = "object-triggered-3d-slam_amd"
KIND = {1: "run accepted", 2: "accepted after search", 3: "serial chunk"}


def main():
    synth = importlib.import_module(PKG + ".synth")
    depth, color, ext = synth.make_sequence(synth.object_scene(0), n_frames=64)
    import torch

    pkg = importlib.import_module(PKG)
    L = importlib.import_module(PKG + "._lib")
    integ = pkg.pipelines.integration
    intr = pkg.camera.PinholeCameraIntrinsic(*synth.REF_INTRINSICS_640)
    vol = integ.ScalableTSDFVolume(voxel_length=0.005, sdf_trunc=0.04, color_type=integ.TSDFVolumeColorType.RGB8)
    for k in range(64):
        vol.integrate(pkg.geometry.RGBDImage.create_from_color_and_depth(
            pkg.geometry.Image(color[k]), pkg.geometry.Image(depth[k]), convert_rgb_to_intensity=False), intr, ext[k])
    mesh = vol.extract_triangle_mesh()
    V, T = mesh._v.dev(), mesh._t.dev().long()
    p0, p1, p2 = V[T[:, 0]], V[T[:, 1]], V[T[:, 2]]
    x, y = p0 - p1, p0 - p2
    cr = torch.stack([x[:, 1] * y[:, 2] - x[:, 2] * y[:, 1], x[:, 2] * y[:, 0] - x[:, 0] * y[:, 2],
                      x[:, 0] * y[:, 1] - x[:, 1] * y[:, 0]], 1)
    areas = (0.5 * torch.sqrt((cr * cr).sum(1))).contiguous()
    s_ = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    cap = 1 << 14
    trace = torch.zeros(2 * cap, dtype=torch.int64, device="cuda")
    for name, d, cdf in (("sum", areas, 0), ("cdf", (areas / areas.sum()).contiguous(), 1)):
        out = torch.empty_like(d)
        for rep in range(3):  # the last repetition is reported (warm caches, tables uploaded)
            trace.zero_()
            L.call("otx_chain_walk_trace", C.c_void_p(d.data_ptr()), d.shape[0], cdf, C.c_void_p(out.data_ptr()),
                   C.c_void_p(trace.data_ptr()), cap, s_)
        t = trace.view(-1, 2).cpu().numpy().astype(np.uint64)
        t = t[t[:, 0] != 0]
        clk, kind = t[:, 0].astype(np.int64), (t[:, 1] & 0xFF).astype(np.int64)
        # each step: from its start event (kind 0) to the next start (or the end event)
        starts = np.nonzero(kind == 0)[0]
        per = {}
        pre = []
        for i, si in enumerate(starts):
            nxt = starts[i + 1] if i + 1 < len(starts) else len(kind) - 1
            ks = [int(x) for x in kind[si + 1:nxt + 1] if x in (1, 2, 3)]
            k = ks[0] if ks else 4
            per.setdefault(k, []).append(int(clk[nxt] - clk[si]))
            if k == 3:  # serial: step start -> first segment (metadata, the failed fast check, the values' wait)
                f5 = [j for j in range(si + 1, nxt) if kind[j] == 5]
                if f5:
                    pre.append(int(clk[f5[0]] - clk[si]))
        if pre:
            print(f"   serial steps: start -> first segment mean {np.mean(pre):.0f} cycles")
        # inside serial chunks: kind 5 = segment start, 6 = after the segment's scans (before its stores / float add)
        seg_a, seg_b = [], []
        for i in range(len(kind) - 1):
            if kind[i] == 5:
                seg_a.append(int(clk[i + 1] - clk[i]))  # start -> scans done
            if kind[i] == 6:
                seg_b.append(int(clk[i + 1] - clk[i]))  # scans done -> next event
        if seg_a:
            print(f"   segments {len(seg_a)}: start->scans mean {np.mean(seg_a):.0f} cycles, scans->next mean "
                  f"{np.mean(seg_b):.0f}")
        total = int(clk[-1] - clk[0])
        print(f"{name}: {len(starts)} steps, {total} cycles in the walk loop")
        for k, v in sorted(per.items()):
            print(f"   {KIND.get(k, k):24s} n={len(v):4d}  cycles total {sum(v):8d}  mean {np.mean(v):8.0f}  "
                  f"max {max(v):8d}")


if __name__ == "__main__":
    main()
