"""Synthetic scan-match inputs shaped like the reference's.

* Grids hold what a reference ScanMatchMap holds: every cell starts at the
  unknown value 0.3f (kMapUnknownCellProb, slam/slam_processor.h:264); each wall
  cell is set to 1.0f and splatted with the Gaussian kernel times the blur
  offset (OccuGridMap::SetCellOccuBlur, map/occu_grid_map.h:531-576; kernel
  GaussianBlur::InitKernel :83-105; max-composition of SetGridProbability,
  map/grid_map_cell.h:361-365). Free cells are never decremented because the
  scan-match maps run with just_update_occu_ = true (slam_processor.cpp:495,510).
* Scans are ray-cast from a ground-truth pose like a Hokuyo in
  worlds/willow-pr2-5cm.world:7-13 (1081 beams, 270.25 deg, 0.1-10 m); beam
  angles accumulate from angle_min in double from float32 message fields, and
  only ranges in (range_min, range_threshold) are kept
  (SlamNode::BuildRangeDataContainer, roborts_slam_node.cpp:290-311).

All generation is numpy, seeded; nothing here runs in the timed path.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass

import numpy as np

UNKNOWN = np.float32(0.3)


def blur_kernel(resolution: float, sigma: float, offset: float) -> tuple[int, np.ndarray]:
    """GaussianBlur kernel (occu_grid_map.h:83-105) times the occupancy offset,
    rounded to float as SetGridProbability's float parameter does."""
    half = int((sigma / resolution) * math.sqrt(math.log(2)))
    k = np.empty((2 * half + 1, 2 * half + 1), dtype=np.float32)
    for j in range(-half, half + 1):
        for i in range(-half, half + 1):
            d = math.hypot(i * resolution, j * resolution)
            z = math.exp(-0.5 * (d / sigma) ** 2)
            k[j + half, i + half] = np.float32(z * offset)
    return half, k


def splat_walls(wall: np.ndarray, resolution: float, sigma: float = None, offset: float = 0.88,
                base: np.float32 = UNKNOWN) -> np.ndarray:
    """Grid of probabilities from a boolean wall mask (max-composed blur)."""
    if sigma is None:
        sigma = 3 * resolution
    grid = np.full(wall.shape, base, dtype=np.float32)
    half, k = blur_kernel(resolution, sigma, offset)
    ys, xs = np.nonzero(wall)
    H, W = wall.shape
    for dj in range(-half, half + 1):
        for di in range(-half, half + 1):
            v = k[dj + half, di + half]
            yy, xx = ys + dj, xs + di
            ok = (yy >= 0) & (yy < H) & (xx >= 0) & (xx < W)
            cur = grid[yy[ok], xx[ok]]
            grid[yy[ok], xx[ok]] = np.where(cur < v, v, cur)
    grid[wall] = np.float32(1.0)
    return grid


def _draw_segment(wall: np.ndarray, x0, y0, x1, y1):
    n = int(max(abs(x1 - x0), abs(y1 - y0))) * 2 + 2
    xs = np.rint(np.linspace(x0, x1, n)).astype(np.int64)
    ys = np.rint(np.linspace(y0, y1, n)).astype(np.int64)
    H, W = wall.shape
    ok = (xs >= 0) & (xs < W) & (ys >= 0) & (ys < H)
    wall[ys[ok], xs[ok]] = True


def make_walls(size_x: int, size_y: int, rng: np.random.Generator, n_rooms: int = None,
               n_segments: int = None, margin: int = 8) -> np.ndarray:
    """Random indoor-like wall layout: an outer boundary, axis-aligned rooms
    with door gaps, and free segments at random angles."""
    wall = np.zeros((size_y, size_x), dtype=bool)
    area = size_x * size_y
    if n_rooms is None:
        n_rooms = max(2, area // 20000)
    if n_segments is None:
        n_segments = max(2, area // 40000)
    m = margin
    for (a, b, c, d) in ((m, m, size_x - m, m), (size_x - m, m, size_x - m, size_y - m),
                         (size_x - m, size_y - m, m, size_y - m), (m, size_y - m, m, m)):
        _draw_segment(wall, a, b, c, d)
    for _ in range(n_rooms):
        w = rng.integers(20, max(21, size_x // 4))
        h = rng.integers(20, max(21, size_y // 4))
        x = rng.integers(m, max(m + 1, size_x - m - w))
        y = rng.integers(m, max(m + 1, size_y - m - h))
        corners = [(x, y), (x + w, y), (x + w, y + h), (x, y + h), (x, y)]
        for (p, q) in zip(corners[:-1], corners[1:]):
            _draw_segment(wall, p[0], p[1], q[0], q[1])
        # a door gap on one side
        side = rng.integers(0, 4)
        gx, gy = corners[side]
        hx, hy = corners[side + 1]
        t = rng.uniform(0.2, 0.7)
        cx, cy = gx + (hx - gx) * t, gy + (hy - gy) * t
        r = 6
        wall[int(max(cy - r, 0)):int(cy + r), int(max(cx - r, 0)):int(cx + r)] = False
    for _ in range(n_segments):
        x0, y0 = rng.uniform(m, size_x - m), rng.uniform(m, size_y - m)
        ang = rng.uniform(0, 2 * math.pi)
        ln = rng.uniform(10, max(11, min(size_x, size_y) / 6))
        _draw_segment(wall, x0, y0, x0 + ln * math.cos(ang), y0 + ln * math.sin(ang))
    return wall


@dataclass
class World:
    """A synthetic map in the reference's frame conventions."""

    grid: np.ndarray       # float32 [size_y, size_x]
    wall: np.ndarray       # bool
    resolution: float
    offset: tuple          # map_offset_ (m): world_to_map = (w + offset) / resolution

    @property
    def size_x(self):
        return self.grid.shape[1]

    @property
    def size_y(self):
        return self.grid.shape[0]

    def world_of_cell(self, cx, cy):
        return (np.asarray(cx) * self.resolution - self.offset[0],
                np.asarray(cy) * self.resolution - self.offset[1])


def make_world(size_x: int, size_y: int, resolution: float = 0.05, seed: int = 20261015,
               sigma: float = None, offset_blur: float = 0.88) -> World:
    rng = np.random.default_rng(seed)
    wall = make_walls(size_x, size_y, rng)
    grid = splat_walls(wall, resolution, sigma, offset_blur)
    off = (size_x * resolution / 2, size_y * resolution / 2)
    return World(grid, wall, resolution, off)


@dataclass
class LaserSpec:
    """Hokuyo of worlds/willow-pr2-5cm.world:7-13 (fov 270.25 deg, 1081 samples)."""

    n_beams: int = 1081
    fov_deg: float = 270.25
    range_min: float = 0.1
    range_max: float = 10.0
    range_threshold_scale: float = 0.95   # config/simulatin_param.yaml:36

    @property
    def angle_min(self) -> np.float32:
        return np.float32(-math.radians(self.fov_deg) / 2)

    @property
    def angle_increment(self) -> np.float32:
        return np.float32(math.radians(self.fov_deg) / (self.n_beams - 1))

    @property
    def range_threshold(self) -> float:  # sensor_data_manager.h:43-48
        return self.range_min + self.range_threshold_scale * (self.range_max - self.range_min)


def _edt(wall: np.ndarray) -> np.ndarray:
    from scipy.ndimage import distance_transform_edt
    return distance_transform_edt(~wall).astype(np.float32)


def raycast_ranges(world: World, poses_world: np.ndarray, laser: LaserSpec, rng=None,
                   noise_m: float = 0.0, edt: np.ndarray = None) -> np.ndarray:
    """Ranges (float32, metres) for poses [M,3] (world x, y, theta) by sphere
    tracing a distance transform of the wall cells. inf where nothing is hit."""
    if edt is None:
        edt = _edt(world.wall)
    res = world.resolution
    poses = np.atleast_2d(np.asarray(poses_world, dtype=np.float64))
    M = poses.shape[0]
    a0, inc = float(laser.angle_min), float(laser.angle_increment)
    rel = a0 + inc * np.arange(laser.n_beams)
    ang = poses[:, 2:3] + rel[None, :]
    ox = (poses[:, 0:1] + world.offset[0]) / res
    oy = (poses[:, 1:2] + world.offset[1]) / res
    dx, dy = np.cos(ang).ravel(), np.sin(ang).ravel()
    ox = np.broadcast_to(ox, ang.shape).ravel()
    oy = np.broadcast_to(oy, ang.shape).ravel()
    t = np.full(ang.size, laser.range_min / res)
    tmax = laser.range_max / res
    hit = np.zeros(ang.size, dtype=bool)
    H, W = edt.shape
    act = np.arange(ang.size)          # indices of rays still marching
    for _ in range(400):
        if act.size == 0:
            break
        ta = t[act]
        ix = np.rint(ox[act] + ta * dx[act]).astype(np.int64)
        iy = np.rint(oy[act] + ta * dy[act]).astype(np.int64)
        inside = (ix >= 0) & (ix < W) & (iy >= 0) & (iy < H)
        d = np.where(inside, edt[np.clip(iy, 0, H - 1), np.clip(ix, 0, W - 1)], 1e9)
        newly = inside & (d < 0.5)
        hit[act[newly]] = True
        tn = ta + np.maximum(d - 1.0, 0.35)
        go = inside & ~newly & (tn <= tmax)
        t[act[go]] = tn[go]
        t[act[~inside | (tn > tmax)]] = tmax + 1
        act = act[go]
    t = t.reshape(ang.shape)
    hit = hit.reshape(ang.shape)
    r = t * res
    if noise_m > 0 and rng is not None:
        r = r + rng.normal(0.0, noise_m, size=r.shape)
    r = np.where(hit, r, np.inf)
    return r.astype(np.float32)


_BEAM_ANGLES: dict = {}


def beam_angles(laser: LaserSpec) -> np.ndarray:
    """Beam angles accumulated in double from the float32 angle_min by the
    float32 increment, one addition per beam (roborts_slam_node.cpp:294,306)."""
    key = (laser.n_beams, float(laser.angle_min), float(laser.angle_increment))
    if key not in _BEAM_ANGLES:
        a = np.empty(laser.n_beams)
        cur, inc = float(laser.angle_min), float(laser.angle_increment)
        for i in range(laser.n_beams):
            a[i] = cur
            cur += inc
        _BEAM_ANGLES[key] = a
    return _BEAM_ANGLES[key]


def scan_points(ranges: np.ndarray, laser: LaserSpec) -> np.ndarray:
    """Sensor-frame endpoints (metres) of one scan as BuildRangeDataContainer
    builds them; keep range_min < r < range_threshold."""
    ranges = np.asarray(ranges, dtype=np.float32)
    a = beam_angles(laser)
    d = ranges.astype(np.float64)
    keep = (d > float(np.float32(laser.range_min))) & (d < laser.range_threshold)
    return np.stack([np.cos(a[keep]) * d[keep], np.sin(a[keep]) * d[keep]], axis=1)


def sample_free_poses(world: World, n: int, rng: np.random.Generator, clearance_m: float = 0.6,
                      border_m: float = 1.0, edt: np.ndarray = None) -> np.ndarray:
    """n world poses in free space at least clearance_m from any wall."""
    if edt is None:
        edt = _edt(world.wall)
    res = world.resolution
    H, W = edt.shape
    b = int(border_m / res)
    cand = np.argwhere(edt[b:H - b, b:W - b] > clearance_m / res) + b
    # keep poses inside the boundary walls: flood from the centre region is
    # overkill here; the outer wall is at the margin, so interior == inside it.
    sel = cand[rng.integers(0, cand.shape[0], size=n)]
    cy, cx = sel[:, 0].astype(np.float64), sel[:, 1].astype(np.float64)
    wx, wy = world.world_of_cell(cx + rng.uniform(-0.4, 0.4, n), cy + rng.uniform(-0.4, 0.4, n))
    th = rng.uniform(-math.pi, math.pi, n)
    return np.stack([wx, wy, th], axis=1)


@dataclass
class ScanBatch:
    points_cells: np.ndarray   # [sum N, 2] map cells, sensor frame
    offsets: np.ndarray        # [S+1] int64
    true_poses: np.ndarray     # [S,3] world
    init_poses: np.ndarray     # [S,3] world (what the matcher starts from)


def make_scan_batch(world: World, n_scans: int, seed: int = 20261015, laser: LaserSpec = None,
                    init_offset=(0.12, -0.07, math.radians(4.0)), min_points: int = 50,
                    noise_m: float = 0.0) -> ScanBatch:
    """n_scans ray-cast scans at distinct free poses; init pose = truth + init_offset."""
    laser = laser or LaserSpec()
    rng = np.random.default_rng(seed)
    edt = _edt(world.wall)
    pts_list, poses = [], []
    need = n_scans
    while need > 0:
        cand = sample_free_poses(world, max(need + need // 8, 8), rng, edt=edt)
        rngs = raycast_ranges(world, cand, laser, rng, noise_m, edt=edt)
        for k in range(cand.shape[0]):
            if need == 0:
                break
            p = scan_points(rngs[k], laser)
            if p.shape[0] < min_points:
                continue
            pts_list.append(p * (1 / world.resolution))  # CreateFrom(range, 1/res)
            poses.append(cand[k])
            need -= 1
    true_poses = np.array(poses)
    init = true_poses + np.asarray(init_offset)[None, :]
    offs = np.zeros(n_scans + 1, dtype=np.int64)
    offs[1:] = np.cumsum([p.shape[0] for p in pts_list])
    return ScanBatch(np.ascontiguousarray(np.concatenate(pts_list, axis=0)), offs, true_poses,
                     np.ascontiguousarray(init))


@dataclass
class ScanStream:
    """A robot run for the online front-end (BASELINE config 5): per scan the
    sensor-frame endpoints in metres (before CreateFrom), the true pose and the
    odometry pose read with it."""

    points_m: list
    true_poses: np.ndarray   # [S,3] world
    odom_poses: np.ndarray   # [S,3] odometry frame (drifting)


def make_scan_stream(world: World, n_scans: int, seed: int = 20261015, laser: LaserSpec = None,
                     step_m: float = 0.05, turn_rad: float = 0.02, clearance_m: float = 0.8,
                     odom_noise=(0.004, 0.002)) -> ScanStream:
    """A collision-free drive of n_scans steps (step_m per scan, 2 m/s at 40 Hz
    for 0.05) with a slowly wandering heading; the robot turns away when the
    distance transform says a wall is near. Odometry integrates the true
    increments with multiplicative noise (odom_noise = translation, rotation)."""
    laser = laser or LaserSpec()
    rng = np.random.default_rng(seed)
    edt = _edt(world.wall)
    res = world.resolution
    H, W = edt.shape

    def clear(p):
        cx = int(round((p[0] + world.offset[0]) / res))
        cy = int(round((p[1] + world.offset[1]) / res))
        return 0 <= cx < W and 0 <= cy < H and edt[cy, cx] * res > clearance_m

    pose = sample_free_poses(world, 1, rng, clearance_m=1.5, edt=edt)[0]
    poses = [pose.copy()]
    while len(poses) < n_scans:
        th = pose[2] + rng.normal(0.0, turn_rad)
        for k in range(64):
            cand = np.array([pose[0] + step_m * math.cos(th), pose[1] + step_m * math.sin(th), th])
            if clear(cand):
                break
            th = pose[2] + (0.15 * (k + 1) if k % 2 == 0 else -0.15 * (k + 1))
        else:
            cand = np.array([pose[0], pose[1], pose[2] + 0.3])
        pose = cand
        poses.append(pose.copy())
    true = np.array(poses)
    odom = np.zeros_like(true)
    for k in range(1, n_scans):
        d = true[k] - true[k - 1]
        c, s = math.cos(-true[k - 1, 2]), math.sin(-true[k - 1, 2])
        lx, ly = c * d[0] - s * d[1], s * d[0] + c * d[1]  # increment in the robot frame
        lx *= 1 + rng.normal(0, odom_noise[0] / max(step_m, 1e-9))
        dth = d[2] * (1 + rng.normal(0, odom_noise[1] * 10))
        oc, os_ = math.cos(odom[k - 1, 2]), math.sin(odom[k - 1, 2])
        odom[k] = odom[k - 1] + np.array([oc * lx - os_ * ly, os_ * lx + oc * ly, dth])
    rngs = raycast_ranges(world, true, laser, edt=edt)
    pts = [scan_points(rngs[k], laser) for k in range(n_scans)]
    return ScanStream(pts, true, odom)


def hostile_grid(size_x: int, size_y: int, seed: int = 7) -> np.ndarray:
    """fp32 values spread over many binades (not exactly summable in fp64):
    only a kernel that keeps the reference's beam order stays bit-exact."""
    rng = np.random.default_rng(seed)
    mant = rng.uniform(0.5, 1.0, size=(size_y, size_x))
    expo = rng.integers(-30, 1, size=(size_y, size_x))
    return (mant * np.exp2(expo)).astype(np.float32)


def read_pgm(path: str) -> np.ndarray:
    """Binary (P5) PGM reader."""
    with open(path, "rb") as f:
        data = f.read()
    tokens, pos = [], 0
    while len(tokens) < 4:
        while data[pos:pos + 1].isspace():
            pos += 1
        if data[pos:pos + 1] == b"#":
            while data[pos:pos + 1] not in (b"\n", b""):
                pos += 1
            continue
        start = pos
        while not data[pos:pos + 1].isspace():
            pos += 1
        tokens.append(data[start:pos])
    pos += 1
    assert tokens[0] == b"P5"
    w, h, maxv = int(tokens[1]), int(tokens[2]), int(tokens[3])
    assert maxv < 256
    return np.frombuffer(data, dtype=np.uint8, count=w * h, offset=pos).reshape(h, w)


WILLOW_FIXTURE = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..",
                                               "tests", "golden", "willow_walls.npz"))


def willow_world(pad: int = 200, path: str = WILLOW_FIXTURE) -> World:
    """Config 4: the reference's willow-full-0.05 map
    (tests/golden/make_willow.py) padded by `pad` cells of unknown (0.3) on
    every side, walls splatted like the synthetic worlds. World offset: the
    map_offset_ that puts the yaml origin at cell (pad, pad)
    (world_to_map = Scaling(1/res) * Translation(offset), grid_map_base.h:68-69)."""
    f = np.load(path)
    h, w = (int(v) for v in f["shape"])
    wall = np.unpackbits(f["wall_bits"])[: h * w].reshape(h, w).astype(bool)
    res = float(f["resolution"])
    wall = np.pad(wall, pad, constant_values=False)
    grid = splat_walls(wall, res)
    origin = f["origin"]
    off = (-float(origin[0]) + pad * res, -float(origin[1]) + pad * res)
    return World(grid, wall, res, off)
