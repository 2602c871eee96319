"""Deterministic synthetic RGB-D scenes and a writer for the reference dataset layout.

The reference ships no frames (its .gitignore:14-33 excludes every scan), so every benchmark and parity input
is generated here.  Scene: floor plane z = 0 plus axis-aligned boxes; cameras on a ring (radius 1.3 m,
height 0.9 m) looking at the object centre lifted 0.35 m; frame k of N at angle 2*pi*k/N.  Depth is the
optical-frame z of the first ray hit (float64 ray casting), plus Gaussian noise (sigma 1 mm), 0.5 % dropout
to 0, quantised to uint16 millimetres with round-half-even and zeroed above 5 m — the same conversion the
capture node applies (system_manager/src/scanner_node.cpp:277-281).  Colour is a procedural texture of the
hit point.  Noise comes from a counter-based hash, so any frame can be regenerated independently.

Pose files follow the ROS convention the reference caller expects: pose_ros = T_cam_optical @ inv(T_fix), so
that reconstruct_rgbd_filter.py:95 (`pose_optical = pose_ros @ T_fix`) recovers the optical camera pose.
"""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import numpy as np

# reconstruct_rgbd_filter.py:26-28 (Gazebo camera, hfov 1.02974 rad: model.sdf:377-437)
REF_INTRINSICS_640 = (640, 480, 565.6009, 565.6009, 320.5, 240.5)
# same hfov at 1280x720
REF_INTRINSICS_1280 = (1280, 720, 1131.2018, 1131.2018, 640.5, 360.5)

# reconstruct_rgbd_filter.py:32-37
T_FIX = np.array([[0, -1, 0, 0], [0, 0, -1, 0], [1, 0, 0, 0], [0, 0, 0, 1]], dtype=np.float64)
# reconstruct_rgbd_gt.py:52-57
T_FIX_GT = np.array([[0, 0, 1, 0], [-1, 0, 0, 0], [0, -1, 0, 0], [0, 0, 0, 1]], dtype=np.float64)

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _hash_u01(seed: int, ctr: np.ndarray) -> np.ndarray:
    """splitmix64(seed + (ctr+1)*golden) -> uniform [0,1) float64 (53 bits)."""
    with np.errstate(over="ignore"):
        z = np.uint64(seed & 0xFFFFFFFFFFFFFFFF) + (ctr.astype(np.uint64) + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


@dataclass
class Box:
    lo: tuple
    hi: tuple
    tint: tuple = (200, 60, 40)


@dataclass
class Scene:
    boxes: list = field(default_factory=lambda: [Box((-0.25, -0.25, 0.0), (0.25, 0.25, 0.7))])
    center: tuple = (0.0, 0.0)
    ring_radius: float = 1.3
    cam_height: float = 0.9
    look_height: float = 0.35
    noise_sigma: float = 0.001
    dropout: float = 0.005
    seed: int = 0


def object_scene(object_id: int) -> Scene:
    """Multi-object configs: object i on a 2 m grid, size varied by seed = object id."""
    rng = np.random.default_rng(object_id)
    cx, cy = 2.0 * (object_id % 4), 2.0 * (object_id // 4)
    hx, hy = rng.uniform(0.12, 0.3, size=2)
    hz = rng.uniform(0.3, 0.8)
    tint = tuple(int(v) for v in rng.integers(40, 220, size=3))
    return Scene(boxes=[Box((cx - hx, cy - hy, 0.0), (cx + hx, cy + hy, hz), tint)], center=(cx, cy),
                 seed=object_id)


def camera_pose(scene: Scene, k: int, n_frames: int) -> np.ndarray:
    """Optical camera-to-world pose (x right, y down, z forward) of ring frame k."""
    th = 2.0 * np.pi * k / n_frames
    cx, cy = scene.center
    pos = np.array([cx + scene.ring_radius * np.cos(th), cy + scene.ring_radius * np.sin(th), scene.cam_height])
    target = np.array([cx, cy, scene.look_height])
    f = target - pos
    f /= np.linalg.norm(f)
    r = np.cross(f, np.array([0.0, 0.0, 1.0]))
    r /= np.linalg.norm(r)
    d = np.cross(f, r)
    T = np.eye(4)
    T[:3, 0], T[:3, 1], T[:3, 2], T[:3, 3] = r, d, f, pos
    return T


def render(scene: Scene, T_cam: np.ndarray, intr=REF_INTRINSICS_640, frame_id: int = 0):
    """Ray-cast one frame.  Returns depth uint16 [h][w] (mm) and color uint8 [h][w][3] (RGB)."""
    w, h, fx, fy, cx, cy = intr
    jj, ii = np.meshgrid(np.arange(w, dtype=np.float64), np.arange(h, dtype=np.float64))
    dirs_c = np.stack([(jj - cx) / fx, (ii - cy) / fy, np.ones_like(jj)], axis=-1)
    R, o = T_cam[:3, :3], T_cam[:3, 3]
    d = dirs_c @ R.T
    t_best = np.full((h, w), np.inf)
    mat = np.zeros((h, w), np.int64)  # 0 none, 1 floor, 2+ box index
    with np.errstate(divide="ignore", invalid="ignore"):
        tf = np.where(d[..., 2] < 0, -o[2] / d[..., 2], np.inf)
        better = (tf > 0) & (tf < t_best)
        t_best = np.where(better, tf, t_best)
        mat = np.where(better, 1, mat)
        for bi, b in enumerate(scene.boxes):
            lo, hi = np.asarray(b.lo), np.asarray(b.hi)
            t1 = (lo - o) / d
            t2 = (hi - o) / d
            tmin = np.nanmax(np.minimum(t1, t2), axis=-1)
            tmax = np.nanmin(np.maximum(t1, t2), axis=-1)
            hit = (tmax >= np.maximum(tmin, 0.0)) & (tmin > 0)
            better = hit & (tmin < t_best)
            t_best = np.where(better, tmin, t_best)
            mat = np.where(better, 2 + bi, mat)
    valid = np.isfinite(t_best)
    t = np.where(valid, t_best, 0.0)
    p = o + d * t[..., None]
    # colour: 2 cm procedural texture + material tint
    cell = np.floor(p * 50.0).astype(np.int64)
    hsh = (cell[..., 0] * 73856093) ^ (cell[..., 1] * 19349663) ^ (cell[..., 2] * 83492791)
    tex = (hsh & 0x3F).astype(np.int64)
    col = np.zeros((h, w, 3), np.int64)
    col[mat == 1] = 110
    col += np.where(mat[..., None] == 1, tex[..., None], 0)
    for bi, b in enumerate(scene.boxes):
        m = mat == 2 + bi
        col[m] = np.asarray(b.tint, np.int64)[None, :] + tex[m][:, None] - 32
    col = np.clip(col, 0, 255).astype(np.uint8)
    # depth noise / dropout from a counter-based hash
    ctr = (np.int64(frame_id) * h + np.arange(h, dtype=np.int64)[:, None]) * w + np.arange(w, dtype=np.int64)[None, :]
    ctr = ctr.astype(np.uint64) * np.uint64(3)
    u1 = _hash_u01(scene.seed, ctr)
    u2 = _hash_u01(scene.seed, ctr + np.uint64(1))
    u3 = _hash_u01(scene.seed, ctr + np.uint64(2))
    gauss = np.sqrt(-2.0 * np.log(np.maximum(u1, 1e-300))) * np.cos(2.0 * np.pi * u2)
    depth_m = t + scene.noise_sigma * gauss
    depth_m = np.where(valid & (u3 >= scene.dropout), depth_m, 0.0)
    mm = np.rint(depth_m * 1000.0)
    mm = np.where((depth_m > 5.0) | (mm < 0), 0.0, mm)
    depth = np.clip(mm, 0, 65535).astype(np.uint16)
    return depth, col


def make_sequence(scene: Scene | None = None, n_frames: int = 16, intr=REF_INTRINSICS_640, frames=None):
    """Render frames of the ring sequence.  Returns depth [F][h][w] u16, color [F][h][w][3] u8, and the
    extrinsics [F][4][4] the reference caller would pass (inv(pose_ros @ T_fix))."""
    scene = scene or Scene()
    ks = range(n_frames) if frames is None else frames
    depths, colors, exts = [], [], []
    for k in ks:
        T = camera_pose(scene, k, n_frames)
        d, c = render(scene, T, intr, frame_id=k)
        depths.append(d)
        colors.append(c)
        pose_ros = T @ np.linalg.inv(T_FIX)
        exts.append(np.linalg.inv(pose_ros @ T_FIX))
    return np.stack(depths), np.stack(colors), np.stack(exts)


def render_frames(job):
    """Picklable worker for process pools: job = (scene, n_frames, intr, frame indices) -> make_sequence(...)."""
    scene, n_frames, intr, frames = job
    return make_sequence(scene, n_frames=n_frames, intr=intr, frames=frames)


def make_sequence_parallel(scene: Scene | None = None, n_frames: int = 16, intr=REF_INTRINSICS_640, frames=None,
                           workers: int = 16, chunk: int = 4):
    """make_sequence over a fork process pool (identical arrays; call before the process initialises the GPU)."""
    import multiprocessing as mp
    from concurrent.futures import ProcessPoolExecutor

    scene = scene or Scene()
    ks = list(range(n_frames) if frames is None else frames)
    jobs = [(scene, n_frames, intr, ks[i:i + chunk]) for i in range(0, len(ks), chunk)]
    if len(jobs) <= 1 or workers <= 1:
        return make_sequence(scene, n_frames=n_frames, intr=intr, frames=ks)
    with ProcessPoolExecutor(max_workers=min(workers, len(jobs)), mp_context=mp.get_context("fork")) as ex:
        parts = list(ex.map(render_frames, jobs))
    return tuple(np.concatenate([p[i] for p in parts]) for i in range(3))


def write_dataset(base_dir: str, label: str, depth, color, poses_ros, start_index: int = 1):
    """Write the reference dataset layout (scanner_node.cpp:260-302): color/<label>_<n>.jpg,
    depth/<label>_<n>.png (uint16 mm), poses/<label>_<n>.txt (4x4, %.6f).  Counter starts at 1."""
    from PIL import Image

    for sub in ("color", "depth", "poses"):
        os.makedirs(os.path.join(base_dir, sub), exist_ok=True)
    for k in range(depth.shape[0]):
        n = start_index + k
        Image.fromarray(np.ascontiguousarray(color[k]), mode="RGB").save(
            os.path.join(base_dir, "color", f"{label}_{n}.jpg"), quality=95)
        Image.fromarray(np.ascontiguousarray(depth[k]).astype(np.uint16)).save(
            os.path.join(base_dir, "depth", f"{label}_{n}.png"))
        np.savetxt(os.path.join(base_dir, "poses", f"{label}_{n}.txt"), poses_ros[k], fmt="%.6f")


def ros_poses(scene: Scene, n_frames: int) -> np.ndarray:
    return np.stack([camera_pose(scene, k, n_frames) @ np.linalg.inv(T_FIX) for k in range(n_frames)])


# ------------------------------------------------------------------------------------ 2-D laser scans (diff_node)
def _segments_of_boxes(boxes):
    segs = []
    for (x0, y0, x1, y1) in boxes:
        segs += [(x0, y0, x1, y0), (x1, y0, x1, y1), (x1, y1, x0, y1), (x0, y1, x0, y0)]
    return np.array(segs, np.float64).reshape(-1, 4)


def _raycast(px, py, angles, segs, range_max):
    """Nearest hit distance of rays from (px, py) at map angles against segments; inf when none <= range_max."""
    dx, dy = np.cos(angles)[:, None], np.sin(angles)[:, None]
    x0, y0, x1, y1 = (segs[:, k][None, :] for k in range(4))
    ex, ey = x1 - x0, y1 - y0
    den = dx * ey - dy * ex
    with np.errstate(divide="ignore", invalid="ignore"):
        t = ((x0 - px) * ey - (y0 - py) * ex) / den
        u = ((x0 - px) * dy - (y0 - py) * dx) / den
    ok = (np.abs(den) > 1e-12) & (t > 0) & (u >= 0) & (u <= 1)
    t = np.where(ok, t, np.inf).min(axis=1)
    return np.where(t <= range_max, t, np.inf)


def laser_scan_batch(n_scans=32, n_beams=720, seed=0, range_max=12.0):
    """Scan pairs for the change detector: the saved map (a 10 m x 8 m room with pillars) rendered as the virtual
    scan, and the current world (one pillar removed, two boxes added, 1 cm range noise, a few NaN returns) as the
    real scan, from a robot driving a loop.  Returns (real [B][N] f32, virtual [B][N] f32, poses [B][7] (tx ty tz
    qx qy qz qw), dts [B], angle_min, angle_increment, range_max)."""
    rng = np.random.default_rng(seed)
    room = [(-5.0, -4.0, 5.0, 4.0)]
    pillars = [(-2.2, -1.2, -1.8, -0.8), (1.8, 0.8, 2.2, 1.2), (-0.3, 2.0, 0.3, 2.6)]
    added = [(0.5, -2.5, 1.3, -1.9), (-3.5, 1.0, -2.9, 1.8)]
    saved = _segments_of_boxes(room + pillars)
    world = _segments_of_boxes(room + pillars[1:] + added)
    amin, ainc = -np.pi, 2 * np.pi / n_beams
    beam = (np.float32(amin) + np.arange(n_beams, dtype=np.float32) * np.float32(ainc)).astype(np.float64)
    real = np.empty((n_scans, n_beams), np.float32)
    virt = np.empty((n_scans, n_beams), np.float32)
    poses = np.zeros((n_scans, 7), np.float64)
    for b in range(n_scans):
        th = 2 * np.pi * b / n_scans
        px, py, yaw = 3.0 * np.cos(th), 2.2 * np.sin(th), th + np.pi / 2
        virt[b] = _raycast(px, py, beam + yaw, saved, range_max)
        r = _raycast(px, py, beam + yaw, world, range_max)
        r = r + np.where(np.isfinite(r), rng.normal(0, 0.01, n_beams), 0.0)
        r[rng.random(n_beams) < 0.003] = np.nan
        real[b] = r
        poses[b] = (px, py, 0.0, 0.0, 0.0, np.sin(yaw / 2), np.cos(yaw / 2))
    dts = np.full(n_scans, 0.1) + rng.uniform(0, 0.02, n_scans)
    return real, virt, poses, dts, float(np.float32(amin)), float(np.float32(ainc)), float(range_max)


def occupancy_pair(h=1024, w=1024, seed=0):
    """A saved occupancy grid (PGM convention: 0 occupied, 254 free, 205 unknown) and a newer grid of the same area
    with moved obstacles, newly explored free space and unknown cells — the two maps of 2d_selective_merge.py."""
    rng = np.random.default_rng(seed)
    old = np.full((h, w), 205, np.uint8)
    old[h // 8: 7 * h // 8, w // 8: 7 * w // 8] = 254
    for _ in range(40):
        r, c = rng.integers(h // 8, 7 * h // 8 - 20, 2)
        old[r:r + rng.integers(4, 20), c:c + rng.integers(4, 20)] = 0
    new = old.copy()
    new[: h // 4, :] = 205                                   # not re-observed
    new[7 * h // 8:, w // 4: 3 * w // 4] = 254               # newly explored
    for _ in range(25):
        r, c = rng.integers(h // 4, 7 * h // 8 - 20, 2)
        new[r:r + rng.integers(4, 20), c:c + rng.integers(4, 20)] = rng.choice([0, 254])
    noise = rng.random((h, w)) < 0.01
    new[noise] = rng.integers(195, 216, int(noise.sum()))   # values around the unknown band edges
    return old, new


def object_cloud(object_id: int, n_points: int = 100000, moved: bool = False):
    """A filtered object cloud as the reconstruction writes it (points on the visible box faces of
    object_scene(object_id), z >= 0.03), for the hybrid-map fusion configs.  `moved` = the object as the
    saved map last saw it for every third object (shifted 6 cm, 10 % fewer samples) — the change to detect."""
    sc = object_scene(object_id)
    b = sc.boxes[0]
    lo, hi = np.array(b.lo, np.float64), np.array(b.hi, np.float64)
    if moved and object_id % 3 == 0:
        lo, hi = lo + [0.06, 0.0, 0.0], hi + [0.06, 0.0, 0.0]
        n_points = int(n_points * 0.9)
    rng = np.random.default_rng(1000 + object_id + (7919 if moved else 0))
    u = rng.random((n_points, 3))
    face = rng.integers(0, 5, n_points)  # 4 sides + top
    p = lo + u * (hi - lo)
    ax = np.where(face < 2, 0, np.where(face < 4, 1, 2))
    side = np.where(face % 2 == 0, lo[ax], hi[ax])
    side = np.where(face == 4, hi[2], side)
    p[np.arange(n_points), ax] = side
    p += rng.normal(0, 0.002, p.shape)
    return p[p[:, 2] >= 0.03]


def room_occupancy(resolution=0.05, margin=1.0):
    """The saved map of laser_scan_batch's room as an OccupancyGrid (int8: 100 walls/pillars, 0 free, -1 outside),
    origin at (-5 - margin, -4 - margin).  Returns (grid [h][w] int8, resolution, (origin_x, origin_y))."""
    ox, oy = -5.0 - margin, -4.0 - margin
    w = int(round((10.0 + 2 * margin) / resolution))
    h = int(round((8.0 + 2 * margin) / resolution))
    xs = ox + (np.arange(w) + 0.5) * resolution
    ys = oy + (np.arange(h) + 0.5) * resolution
    X, Y = np.meshgrid(xs, ys)
    g = np.full((h, w), -1, np.int8)
    inside = (X > -5.0) & (X < 5.0) & (Y > -4.0) & (Y < 4.0)
    g[inside] = 0
    wall = inside & ((X < -5.0 + resolution) | (X > 5.0 - resolution) | (Y < -4.0 + resolution) | (Y > 4.0 - resolution))
    g[wall] = 100
    for (x0, y0, x1, y1) in [(-2.2, -1.2, -1.8, -0.8), (1.8, 0.8, 2.2, 1.2), (-0.3, 2.0, 0.3, 2.6)]:
        g[(X >= x0) & (X <= x1) & (Y >= y0) & (Y <= y1)] = 100
    return g, resolution, (ox, oy)
