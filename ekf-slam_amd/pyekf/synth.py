"""Synthetic EKF-SLAM inputs (the stand-in for nusim's simulator and fake sensor).

This is input generation, not filter math: it plays the role of ``nusim``
(nusim/src/nusim.cpp:211-289 wheel integration with slip, :310-349 fake landmark sensor) so the
same odometry + marker streams can be fed to the HIP path, the CPU oracle and the benchmark.

* Robot drives a circle (nuturtle_control/src/circle.cpp:85-86: v = ω·r) sampled at ``tick_hz``
  joint-state ticks; the sensor fires every ``ticks_per_msg`` ticks (5 Hz at 200 Hz ticks,
  nusim.cpp:72,89).
* True wheel angles carry multiplicative slip noise U(-slip, slip) (nusim.cpp:224-227); the encoders
  report the commanded angles, so odometry drifts from the truth and the EKF has work to do.
* Each message carries landmark positions in the true body frame plus N(0, σ²) noise on x and y
  (nusim.cpp:317-346). ``basic_world`` reports every landmark with DELETE beyond ``max_range``
  (nusim.cpp:332-336); the large synthetic maps report the ``m`` nearest landmarks.

Seeds are explicit; every array is deterministic for a given argument set.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

ADD, DELETE = 0, 2  # visualization_msgs Marker actions

# basic_world.yaml:5-10 and diff_params.yaml:3-4 of the reference
BASIC_WORLD_LANDMARKS = np.array([[-0.5, -0.7], [0.8, -0.8], [0.4, 0.8], [-0.6, 0.65]])
BASIC_WORLD_THETA0 = 1.28
WHEEL_RADIUS = 0.033
TRACK_WIDTH = 0.160


@dataclass
class Scenario:
    n_landmarks: int          # filter slots N (state dim 3 + 2N)
    landmarks: np.ndarray     # [L, 2] true landmark positions, L <= N
    wheel: np.ndarray         # [T, ticks, 2] encoder wheel angles (left, right), cumulative rad
    ids: np.ndarray           # [T, M] int32 landmark ids (-1 = padding)
    actions: np.ndarray       # [T, M] int32 ADD / DELETE
    rel: np.ndarray           # [T, M, 2] body-frame marker positions (noisy)
    count: np.ndarray         # [T] markers per message
    truth: np.ndarray         # [T, 3] true (θ, x, y) at each sensor message
    track: float = TRACK_WIDTH
    radius: float = WHEEL_RADIUS

    @property
    def n_messages(self) -> int:
        return int(self.ids.shape[0])

    def corrections(self, start: int = 0, stop: int | None = None) -> int:
        """Number of non-DELETE markers (= EKF correction steps) in messages [start, stop):
        slam.cpp:205 skips only DELETE; ADD, MODIFY and DELETEALL are corrected."""
        stop = self.n_messages if stop is None else stop
        c = 0
        for t in range(start, stop):
            k = int(self.count[t])
            c += int(np.count_nonzero(self.actions[t, :k] != DELETE))
        return c


def _se2_step(pose, omega, vx):
    """Exact arc integration of a body twist (same kinematics as turtlelib integrate_twist)."""
    th, x, y = pose
    if omega == 0.0:
        dx, dy = vx, 0.0
    else:
        dx = vx / omega * math.sin(omega)
        dy = vx / omega * (1.0 - math.cos(omega))
    c, s = math.cos(th), math.sin(th)
    return (th + omega, x + c * dx - s * dy, y + s * dx + c * dy)


def make_scenario(n_landmarks: int, landmarks: np.ndarray, n_messages: int, *,
                  max_markers: int = 16, nearest: bool = True, start_pose=(0.0, 0.0, -1.0),
                  circle_radius: float = 1.0, omega: float = 0.5, tick_hz: float = 200.0,
                  ticks_per_msg: int = 40, sensor_sigma: float = 1e-3, slip: float = 0.02,
                  max_range: float = 5.0, seed: int = 20240317, shuffle: bool = False,
                  n_delete: int = 0) -> Scenario:
    """Generate a drive + sensing sequence. ``start_pose`` is (θ, x, y)."""
    rng = np.random.default_rng(seed)
    L = landmarks.shape[0]
    assert L <= n_landmarks
    v = omega * circle_radius
    wr = (v + omega * TRACK_WIDTH / 2.0) / WHEEL_RADIUS
    wl = (v - omega * TRACK_WIDTH / 2.0) / WHEEL_RADIUS
    dt = 1.0 / tick_hz
    m = L if not nearest else min(max_markers, L)
    M = m + n_delete
    wheel = np.zeros((n_messages, ticks_per_msg, 2))
    ids = np.full((n_messages, M), -1, dtype=np.int32)
    actions = np.zeros((n_messages, M), dtype=np.int32)
    rel = np.zeros((n_messages, M, 2))
    count = np.zeros(n_messages, dtype=np.int32)
    truth = np.zeros((n_messages, 3))
    enc = np.zeros(2)
    true_w = np.zeros(2)
    pose = tuple(float(p) for p in start_pose)
    for t in range(n_messages):
        for k in range(ticks_per_msg):
            cmd = np.array([wl, wr]) * dt
            enc = enc + cmd
            slipped = cmd * (1.0 + rng.uniform(-slip, slip, size=2))
            true_w = true_w + slipped
            om = WHEEL_RADIUS / TRACK_WIDTH * (-slipped[0] + slipped[1])
            vx = WHEEL_RADIUS / 2.0 * (slipped[0] + slipped[1])
            pose = _se2_step(pose, om, vx)
            wheel[t, k] = enc
        truth[t] = pose
        th, x, y = pose
        c, s = math.cos(th), math.sin(th)
        d = landmarks - np.array([x, y])
        # body frame: R(θ)ᵀ (p − x)
        bx = c * d[:, 0] + s * d[:, 1]
        by = -s * d[:, 0] + c * d[:, 1]
        dist = np.hypot(bx, by)
        if nearest:
            sel = np.argsort(dist, kind="stable")[:m]
            sel = sel[dist[sel] <= max_range]
        else:
            sel = np.arange(L)
        if shuffle:
            sel = rng.permutation(sel)
        k = len(sel)
        noise = rng.normal(0.0, sensor_sigma, size=(k, 2))
        ids[t, :k] = sel
        rel[t, :k, 0] = bx[sel] + noise[:, 0]
        rel[t, :k, 1] = by[sel] + noise[:, 1]
        actions[t, :k] = np.where(dist[sel] <= max_range, ADD, DELETE)
        if n_delete:
            far = rng.integers(0, n_landmarks, size=n_delete)
            ids[t, k:k + n_delete] = far
            rel[t, k:k + n_delete] = 100.0
            actions[t, k:k + n_delete] = DELETE
            k += n_delete
        count[t] = k
    return Scenario(n_landmarks, landmarks, wheel, ids, actions, rel, count, truth)


def basic_world(n_messages: int = 100, seed: int = 20240317, **kw) -> Scenario:
    """nusim basic_world (4 landmarks, θ0 = 1.28) in a 50-slot filter (slam.cpp:665)."""
    kw.setdefault("circle_radius", 0.3)
    kw.setdefault("nearest", False)
    return make_scenario(50, BASIC_WORLD_LANDMARKS, n_messages, seed=seed,
                         start_pose=(BASIC_WORLD_THETA0, 0.0, 0.0), **kw)


def random_landmarks(n: int, seed: int = 20240317, circle_radius: float = 1.0,
                     clearance: float = 0.3) -> np.ndarray:
    """N landmarks uniform in [-L, L]², L = 0.5·sqrt(N), kept `clearance` m off the circle path."""
    rng = np.random.default_rng(seed + 7919)
    half = 0.5 * math.sqrt(n)
    half = max(half, circle_radius + 2 * clearance + 0.5)
    out = np.zeros((n, 2))
    k = 0
    while k < n:
        p = rng.uniform(-half, half, size=(2 * n, 2))
        r = np.hypot(p[:, 0], p[:, 1])
        p = p[np.abs(r - circle_radius) >= clearance]
        take = min(n - k, len(p))
        out[k:k + take] = p[:take]
        k += take
    return out


def synthetic(n_landmarks: int, n_messages: int, seed: int = 20240317, max_markers: int = 16,
              **kw) -> Scenario:
    """SURVEY.md §8d synthetic map: N landmarks, unit circle at ω = 0.5, m nearest markers."""
    lm = random_landmarks(n_landmarks, seed)
    return make_scenario(n_landmarks, lm, n_messages, seed=seed, max_markers=max_markers, **kw)


def lidar_scans(poses, circles, arena=(10.0, 5.0), n_beams=360, sigma=0.0, seed=20240317,
                range_min=0.11, range_max=10.0):
    """Synthetic LaserScan ranges (float32 [P, n_beams]) for body poses [P, 3] = (θ, x, y): a lidar
    mounted −0.032 m along the body x axis (nusim.cpp:577), beam i at θ + i·2π/n_beams, exact ray
    casting against cylinders ``circles`` [(x, y, r)] and the walls of an axis-aligned arena centred
    on the origin, clamped to [range_min, range_max], plus N(0, σ²) noise (nusim.cpp:700-707).
    Scan inputs for the landmark front-end (include/landmarks.h); angle_min = 0,
    angle_increment = float32(2π / n_beams)."""
    poses = np.atleast_2d(np.asarray(poses, dtype=np.float64))
    th = poses[:, 0:1] + np.arange(n_beams)[None, :] * (2.0 * math.pi / n_beams)
    lx = (poses[:, 1] - 0.032 * np.cos(poses[:, 0]))[:, None]
    ly = (poses[:, 2] - 0.032 * np.sin(poses[:, 0]))[:, None]
    dx, dy = np.cos(th), np.sin(th)
    best = np.full(th.shape, np.inf)
    for (cx, cy, r) in circles:
        fx, fy = lx - cx, ly - cy
        bq = fx * dx + fy * dy
        disc = bq * bq - (fx * fx + fy * fy - r * r)
        with np.errstate(invalid="ignore"):
            t = -bq - np.sqrt(disc)
        hit = (disc >= 0.0) & (t > 0.0)
        best = np.where(hit, np.minimum(best, t), best)
    hx, hy = arena[0] / 2.0, arena[1] / 2.0
    with np.errstate(divide="ignore", invalid="ignore"):
        for den, lim, org in ((dx, hx, lx), (-dx, hx, -lx), (dy, hy, ly), (-dy, hy, -ly)):
            best = np.where(den > 1e-12, np.minimum(best, (lim - org) / den), best)
    best = np.clip(best, range_min, range_max)
    if sigma > 0.0:
        best = best + np.random.default_rng(seed).normal(0.0, sigma, best.shape)
    return best.astype(np.float32)


def lidar_world(n_scans: int = 426, n_obstacles: int = 20, seed: int = 20240317,
                arena=(5.0, 4.0), obstacle_r: float = 0.038, sigma: float = 1e-3):
    """Surrogate of BASELINE configs[4] (the rosbag2_2024_03_17-18_35_57 replay, whose .mcap payload
    is missing from the reference snapshot): the bag's shape — 87 s, 426 lidar scans at ≈ 5 Hz,
    ≈ 20 odometry ticks per scan, ≈ 20 landmarks (metadata.yaml:11-174) — as a unit-circle drive
    at 0.2 rad/s through ``n_obstacles`` cylinders, 360-beam scans by ``lidar_scans``.
    Returns (scenario with wheel ticks and truth, obstacles [(x, y, r)], scans float32 [T, 360])."""
    rng = np.random.default_rng(seed + 104729)
    obs = []
    while len(obs) < n_obstacles:
        p = rng.uniform([-arena[0] / 2 + 0.5, -arena[1] / 2 + 0.5],
                        [arena[0] / 2 - 0.5, arena[1] / 2 - 0.5])
        if abs(math.hypot(p[0], p[1]) - 1.0) < 0.35:
            continue
        if all(math.hypot(p[0] - q[0], p[1] - q[1]) > 0.5 for q in obs):
            obs.append((float(p[0]), float(p[1]), obstacle_r))
    lm = np.array([(x, y) for x, y, _ in obs])
    sc = make_scenario(50, lm, n_scans, circle_radius=1.0, omega=0.2, tick_hz=100.0,
                       ticks_per_msg=20, nearest=False, start_pose=(0.0, 1.0, 0.0), seed=seed)
    scans = lidar_scans(sc.truth, obs, arena=arena, n_beams=360, sigma=sigma, seed=seed + 1)
    return sc, obs, scans


def with_markers(sc: Scenario, markers) -> Scenario:
    """The scenario's drive with unknown-association marker arrays ``markers`` (per message a list
    of body-frame (x, y)) in place of its fake-sensor ones (the `landmarks` node's output feeding
    sensor_cb)."""
    T = sc.n_messages
    M = max(1, max(len(m) for m in markers))
    rel = np.zeros((T, M, 2))
    count = np.zeros(T, dtype=np.int32)
    for t, m in enumerate(markers):
        count[t] = len(m)
        if len(m):
            rel[t, :len(m)] = np.asarray(m, dtype=np.float64).reshape(-1, 2)
    return Scenario(sc.n_landmarks, sc.landmarks, sc.wheel, np.full((T, M), -1, np.int32),
                    np.zeros((T, M), np.int32), rel, count, sc.truth, sc.track, sc.radius)
