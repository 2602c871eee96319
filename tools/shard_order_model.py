"""Host models behind two round-6 sharding decisions (tool only):
  --order : list scheduling of a batch's integrate items (4 (unit, quarter) items per unit, cost 4 + frames seen,
            2,048 resident slots, dispatched in work-list order) for the configs[1] ring scan, per rank and 64-frame
            batch: arbitrary order vs heavy-first (two classes at >= 32 frames) vs longest-first (LPT);
  --interleave : sector ownership with K interleaved sub-sectors per rank (rank r owns sub-sectors r, r + N, ...):
            units per batch and staged-tile fraction per rank.
Uses tools/shard_sector_model.py's scan restatement (touch rule, footprints) and its cached scan."""
import argparse
import heapq
import importlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
PKG = "object-triggered-3d-slam_amd"


def makespan(costs, slots, order):
    h = [0.0] * slots
    heapq.heapify(h)
    for c in (costs[i] for i in order):
        t = heapq.heappop(h)
        heapq.heappush(h, t + c)
    return max(h)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--ranks", type=int, default=2)
    ap.add_argument("--interleave", default="1,2,4")
    ap.add_argument("--cache", default="/tmp/otslam_cfg1_scan.npz")
    a = ap.parse_args()
    M = importlib.import_module("shard_sector_model")
    synth = importlib.import_module(PKG + ".synth")
    intr = synth.REF_INTRINSICS_640
    if os.path.exists(a.cache):
        z = np.load(a.cache)
        depth, ext = z["depth"], z["ext"]
    else:
        depth, _, ext = synth.make_sequence_parallel(synth.Scene(seed=0), n_frames=256, intr=intr)
        np.savez(a.cache, depth=depth, ext=ext)
    L = 0.005 * 16
    W, H = intr[:2]
    tile = 16
    tx, ty = (W + tile - 1) // tile, (H + tile - 1) // tile
    per_frame = []
    for f in range(256):
        P = M.frame_samples(depth[f], ext[f], intr)
        per_frame.append(np.unique(M.touched(P, L, 0.04)[:, :3], axis=0))
    rng = np.random.default_rng(0)
    N = a.world
    print(f"list scheduling (2048 slots, item cost 4 + frames), {N} sector ranks and unsharded")
    for n, own in ((1, lambda k: np.zeros(len(k), int)), (N, lambda k: M.owner_sector(k, N, L, (0.0, 0.0)))):
        for r in range(min(n, a.ranks)):
            for b0 in range(0, 256, 64):
                cnt = {}
                for f in range(b0, b0 + 64):
                    k = per_frame[f]
                    for t in map(tuple, k[own(k) == r].tolist()):
                        cnt[t] = cnt.get(t, 0) + 1
                fr = np.array(list(cnt.values()) or [0], float)
                costs = np.repeat(4.0 + fr, 4)
                perm = rng.permutation(len(costs))
                heavy = [i for i in perm if costs[i] - 4.0 >= 32] + [i for i in perm if costs[i] - 4.0 < 32]
                print(f"  N {n} rank {r} batch {b0 // 64}: units {len(cnt):5d}  arbitrary {makespan(costs, 2048, perm):6.1f}"
                      f"  heavy-first {makespan(costs, 2048, heavy):6.1f}  LPT {makespan(costs, 2048, np.argsort(-costs, kind='stable')):6.1f}"
                      f"  bound {max(costs.sum() / 2048, costs.max()):6.1f}")
    print(f"interleaved sectors ({N} ranks x K sub-sectors each)")
    for K in [int(x) for x in a.interleave.split(",")]:
        own = lambda k, K=K: M.owner_sector(k, N * K, L, (0.0, 0.0)) % N
        for r in range(a.ranks):
            bu, bt = [], []
            for b0 in range(0, 256, 64):
                units, tiles = set(), 0
                for f in range(b0, b0 + 64):
                    k = per_frame[f]
                    mk = k[own(k) == r]
                    units.update(map(tuple, mk.tolist()))
                    rect = M.footprint_tiles(mk, ext[f], intr, 0.005, tile)
                    rect = rect[rect[:, 0] >= 0]
                    m = np.zeros((ty, tx), bool)
                    for x0, x1, y0, y1 in rect:
                        m[y0:y1 + 1, x0:x1 + 1] = True
                    tiles += int(m.sum())
                bu.append(len(units))
                bt.append(round(tiles / (64 * tx * ty), 3))
            print(f"  K {K} rank {r}: units per batch {bu}  staged tile fraction {bt}")


if __name__ == "__main__":
    main()
