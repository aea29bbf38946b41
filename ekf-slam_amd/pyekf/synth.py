"""Synthetic EKF-SLAM inputs (the stand-in for nusim's simulator and fake sensor).

This is input generation, not filter math: it plays the role of ``nusim``
(nusim/src/nusim.cpp:211-289 wheel integration with slip, :310-349 fake landmark sensor) so the
same odometry + marker streams can be fed to the HIP path, the CPU oracle and the benchmark.

* The robot follows a commanded (v, ω) schedule sampled at ``tick_hz`` joint-state ticks; the
  sensor fires every ``ticks_per_msg`` ticks (5 Hz at 200 Hz ticks, nusim.cpp:72,89). The basic
  drive is a circle (nuturtle_control/src/circle.cpp:85-86: v = ω·r).
* True wheel angles carry multiplicative slip noise U(-slip, slip) (nusim.cpp:224-227) and the true
  pose is DiffDrive::FKin of them (nusim.cpp:230); the encoders report the commanded angles, so
  odometry drifts from the truth and the EKF has work to do.
* Each message carries landmark positions in the true body frame plus N(0, σ²) noise on x and y
  (nusim.cpp:317-346). ``basic_world`` reports every landmark with DELETE beyond ``max_range``
  (nusim.cpp:332-336); the large synthetic maps report the ``m`` nearest landmarks.
* Populated maps ("one untimed warm-up pass that initializes every landmark"):
  ``populated`` / ``swarm`` prefix the circle with a survey drive — an inward spiral with rings
  ``ring`` m apart over the whole field, ending on the unit circle at the field's centre — whose
  messages carry, of the landmarks within
  twice ``max_range`` (slip drifts the true path off the commanded spiral), the not-yet-sighted
  ones first, then the nearest; never none (the nearest, if nothing is in range). Every landmark is sighted by the
  end of the survey (asserted). Landmarks are placed at least ``clearance`` m from the true path of
  the whole drive (range 0 is the reference's unguarded NaN, slam.cpp:241-249).

Randomness is counter-based (splitmix64 of (seed, stream, index)): every draw of filter f with seed
``base + f`` is a pure function of its indices, so a whole swarm is generated array-at-a-time and
any filter can be regenerated alone (``Swarm.scenario(f)`` equals ``populated(..., seed=base+f)``).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np

ADD, MODIFY, DELETE, DELETEALL = 0, 1, 2, 3  # visualization_msgs Marker actions

# basic_world.yaml:5-10 and diff_params.yaml:3-4 of the reference
BASIC_WORLD_LANDMARKS = np.array([[-0.5, -0.7], [0.8, -0.8], [0.4, 0.8], [-0.6, 0.65]])
BASIC_WORLD_THETA0 = 1.28
WHEEL_RADIUS = 0.033
TRACK_WIDTH = 0.160

# sensor modes per message
SENSE_NEAREST, SENSE_SURVEY, SENSE_ALL = 0, 1, 2
SURVEY_RANGE = 2.0  # survey messages sense out to this multiple of max_range
# RNG streams
_S_SLIP, _S_NOISE, _S_MAP, _S_SHUFFLE, _S_DELETE = 1, 2, 3, 4, 5


@dataclass
class Scenario:
    n_landmarks: int          # filter slots N (state dim 3 + 2N)
    landmarks: np.ndarray     # [L, 2] true landmark positions, L <= N
    wheel: np.ndarray         # [T, ticks, 2] encoder wheel angles (left, right), cumulative rad
    ids: np.ndarray           # [T, M] int32 landmark ids (-1 = padding)
    actions: np.ndarray       # [T, M] int32 ADD / DELETE (MODIFY / DELETEALL: corrected too)
    rel: np.ndarray           # [T, M, 2] body-frame marker positions (noisy)
    count: np.ndarray         # [T] markers per message
    truth: np.ndarray         # [T, 3] true (θ, x, y) at each sensor message
    track: float = TRACK_WIDTH
    radius: float = WHEEL_RADIUS
    n_warm: int = 0           # leading survey messages (every landmark sighted by their end)

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


# ---- counter-based RNG ---------------------------------------------------------------------------
_G = np.uint64(0x9E3779B97F4A7C15)


def _mix64(z):
    """splitmix64's output function (uint64 arrays, wrapping arithmetic)."""
    z = np.asarray(z, dtype=np.uint64)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def rng_u64(seed, stream: int, idx):
    """64 random bits for draw ``idx`` of ``stream`` under ``seed`` (broadcasting arrays)."""
    with np.errstate(over="ignore"):
        key = _mix64(np.asarray(seed, dtype=np.uint64) * _G + np.uint64(stream))
        return _mix64(key + (np.asarray(idx, dtype=np.uint64) + np.uint64(1)) * _G)


def rng_uniform(seed, stream: int, idx):
    """U[0, 1) with 53 random bits."""
    return (rng_u64(seed, stream, idx) >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)


def rng_normal(seed, stream: int, idx):
    """N(0, 1) by Box–Muller from draws 2·idx, 2·idx + 1 of the stream."""
    idx = np.asarray(idx, dtype=np.uint64)
    u1 = 1.0 - rng_uniform(seed, stream, idx * np.uint64(2))  # (0, 1]
    u2 = rng_uniform(seed, stream, idx * np.uint64(2) + np.uint64(1))
    return np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * math.pi * u2)


# ---- commanded drives ----------------------------------------------------------------------------
@dataclass
class Drive:
    """Per-tick commanded body twist and per-message sensor mode."""
    v: np.ndarray              # [ticks_total] forward speed, m/s
    w: np.ndarray              # [ticks_total] yaw rate, rad/s
    sense: np.ndarray          # [T] SENSE_* per message
    ticks_per_msg: int
    tick_hz: float
    n_warm: int = 0
    start_pose: tuple | None = None  # true (θ, x, y) at the first tick (None: the caller's)


def circle_drive(n_messages: int, circle_radius=1.0, omega=0.5, tick_hz=200.0, ticks_per_msg=40,
                 sense=SENSE_NEAREST) -> Drive:
    nt = n_messages * ticks_per_msg
    return Drive(np.full(nt, omega * circle_radius), np.full(nt, omega),
                 np.full(n_messages, sense, np.int32), ticks_per_msg, tick_hz)


def survey_drive(half: float, n_messages: int, ring=3.0, v_survey=4.0, circle_radius=1.0,
                 omega=0.5, tick_hz=200.0, ticks_per_msg=40, max_range=5.0) -> Drive:
    """Inward spiral over the [-half, half]² field (radius shrinking ``ring`` m per turn, curvature
    1/r, at ``v_survey`` m/s) from the outer ring down to the unit circle, then ``n_messages`` of the
    circle (radius ``circle_radius`` at ``omega``) around the field's centre. The robot starts on
    the outer ring towards a corner, heading counter-clockwise (``Drive.start_pose``); the ring
    passes each corner within ``max_range`` − 1 m while it shrinks over the first turn. The spiral's
    messages sense in survey mode."""
    dt = 1.0 / tick_hz
    r_max = max(half * math.sqrt(2.0) - 0.5, circle_radius + ring)
    phi0 = 0.25 * math.pi
    r, v, w = r_max, [], []
    while r > circle_radius:
        om = v_survey / r
        v.append(v_survey)
        w.append(om)
        r -= ring / (2.0 * math.pi) * om * dt
    nw = -(-len(v) // ticks_per_msg)  # whole messages: pad with the unit circle at survey speed
    pad = nw * ticks_per_msg - len(v)
    v += [v_survey] * pad
    w += [v_survey / circle_radius] * pad
    c = circle_drive(n_messages, circle_radius, omega, tick_hz, ticks_per_msg)
    sense = np.concatenate([np.full(nw, SENSE_SURVEY, np.int32), c.sense])
    return Drive(np.concatenate([np.array(v), c.v]), np.concatenate([np.array(w), c.w]), sense,
                 ticks_per_msg, tick_hz, nw,
                 start_pose=(phi0 + 0.5 * math.pi, r_max * math.cos(phi0), r_max * math.sin(phi0)))


# ---- simulation ----------------------------------------------------------------------------------
def _compose(a, b):
    """geom.hpp compose (turtlelib Transform2D ``*``, se2d.cpp:57-75), vectorised; a, b = (θ, x, y)."""
    c, s = np.cos(a[0]), np.sin(a[0])
    return a[0] + b[0], c * b[1] - s * b[2] + a[1], s * b[1] + c * b[2] + a[2]


def _inverse(t):
    c, s = np.cos(t[0]), np.sin(t[0])
    return -t[0], -t[1] * c - t[2] * s, -t[2] * c + t[1] * s


def _fkin_step(config, dl, dr, radius=WHEEL_RADIUS, track=TRACK_WIDTH):
    """One DiffDrive::FKin update (diff_drive.cpp:10-28, geom.hpp DiffDrive::fkin) for wheel-angle
    increments (dl, dr): body twist → integrate_twist (se2d.cpp:127-138) → config · Δ."""
    om = radius / track * (-dl + dr)
    vx = radius / 2.0 * (dl + dr)
    zero = om == 0.0
    w = np.where(zero, 1.0, om)
    tsb = (np.zeros_like(om), 0.0 / w, -vx / w)
    d = _compose(_compose(_inverse(tsb), (w, np.zeros_like(om), np.zeros_like(om))), tsb)
    d = (np.where(zero, 0.0, d[0]), np.where(zero, vx, d[1]), np.where(zero, 0.0, d[2]))
    return _compose(config, d)


def _simulate(drive: Drive, seeds: np.ndarray, start_pose, slip: float):
    """True poses of F filters → (wheel [T, ticks, 2] encoder angles shared by all filters,
    truth [F, T, 3] at the messages, path [F, ticks_total, 2] positions).

    nusim's timer (nusim.cpp:222-230): each tick a wheel turns by its commanded increment ×
    (1 + U(−slip, slip)), and the true pose is DiffDrive::FKin of the accumulated true wheel angles
    from the start pose. The encoders here report the commanded angles (nusim reports the slipped
    ones), so odometry drifts from the truth and the filter has work to do. The device simulator
    (ekf-slam_amd/csrc/sim_kernels.hip) runs the same arithmetic, draw for draw."""
    F = seeds.shape[0]
    nt = drive.v.shape[0]
    tpm = drive.ticks_per_msg
    T = nt // tpm
    dt = 1.0 / drive.tick_hz
    wr = (drive.v + drive.w * TRACK_WIDTH / 2.0) / WHEEL_RADIUS * dt
    wl = (drive.v - drive.w * TRACK_WIDTH / 2.0) / WHEEL_RADIUS * dt
    cmd = np.stack([wl, wr], 1)                                         # [nt, 2]
    wheel = np.cumsum(cmd, 0).reshape(T, tpm, 2)
    k = np.arange(nt, dtype=np.uint64)
    u = rng_uniform(seeds[:, None, None], _S_SLIP,
                    (k[None, :, None] * np.uint64(2) + np.arange(2, dtype=np.uint64)))
    slipped = cmd[None] * (1.0 + slip * (2.0 * u - 1.0))                # [F, nt, 2]
    config = (np.full(F, float(start_pose[0])), np.full(F, float(start_pose[1])),
              np.full(F, float(start_pose[2])))
    phi_l = np.zeros(F)
    phi_r = np.zeros(F)
    path = np.zeros((F, nt, 2))
    truth = np.zeros((F, T, 3))
    for i in range(nt):
        nl = phi_l + slipped[:, i, 0]
        nr = phi_r + slipped[:, i, 1]
        config = _fkin_step(config, nl - phi_l, nr - phi_r)
        phi_l, phi_r = nl, nr
        path[:, i, 0] = config[1]
        path[:, i, 1] = config[2]
        if (i + 1) % tpm == 0:
            t = (i + 1) // tpm - 1
            truth[:, t, 0], truth[:, t, 1], truth[:, t, 2] = config
    return wheel, truth, path


def _place_landmarks(n: int, half: float, seeds: np.ndarray, path: np.ndarray, clearance: float):
    """n landmarks per filter, uniform in [-half, half]², at least ``clearance`` m from that
    filter's true path (rejection by nearest-neighbour distance to the path's tick positions,
    ≤ 2 cm apart, with that spacing added to the clearance)."""
    from scipy.spatial import cKDTree
    F = seeds.shape[0]
    out = np.zeros((F, n, 2))
    for f in range(F):
        tree = cKDTree(path[f])
        k, draw = 0, 0
        while k < n:
            m = 2 * n
            idx = np.arange(draw, draw + m, dtype=np.uint64)
            p = (2.0 * rng_uniform(seeds[f], _S_MAP, idx[:, None] * np.uint64(2) +
                                   np.arange(2, dtype=np.uint64)) - 1.0) * half
            draw += m
            d, _ = tree.query(p, k=1, distance_upper_bound=clearance + 0.02)
            p = p[~np.isfinite(d)]
            take = min(n - k, len(p))
            out[f, k:k + take] = p[:take]
            k += take
    return out


def _sense(drive: Drive, seeds, landmarks, truth, max_markers, max_range, sensor_sigma, shuffle,
           n_delete, n_landmarks):
    """Fake-sensor marker arrays for F filters → ids/actions [T, F, M], rel [T, F, M, 2], count."""
    F, T = truth.shape[0], truth.shape[1]
    L = landmarks.shape[1]
    mall = int(np.any(drive.sense == SENSE_ALL))
    m = min(max_markers, L)
    M = (L if mall else m) + n_delete
    ids = np.full((T, F, M), -1, np.int32)
    act = np.zeros((T, F, M), np.int32)
    rel = np.zeros((T, F, M, 2))
    cnt = np.zeros((T, F), np.int32)
    sighted = np.zeros((F, L), bool)
    warm_sighted = sighted.copy()
    ar = np.arange(L)
    for t in range(T):
        if t == drive.n_warm:
            warm_sighted = sighted.copy()
        th, x, y = truth[:, t, 0:1], truth[:, t, 1:2], truth[:, t, 2:3]
        c, s = np.cos(th), np.sin(th)
        dxl = landmarks[..., 0] - x
        dyl = landmarks[..., 1] - y
        bx = c * dxl + s * dyl            # body frame: R(θ)ᵀ (p − x)
        by = -s * dxl + c * dyl
        dist = np.hypot(bx, by)           # [F, L]
        mode = drive.sense[t]
        if mode == SENSE_ALL:
            sel = np.broadcast_to(ar, (F, L))
            k = np.full(F, L)
            a = np.where(dist <= max_range, ADD, DELETE)
        else:
            # the survey senses out to twice the range: slip drifts the true path off the
            # commanded spiral by metres over a survey, and every landmark must still be sighted
            rng = SURVEY_RANGE * max_range if mode == SENSE_SURVEY else max_range
            key = np.where(dist <= rng, dist, np.inf)
            if mode == SENSE_SURVEY:
                key = np.where(sighted & np.isfinite(key), key + 1e6, key)
            if mode == SENSE_SURVEY:  # a survey message is never empty: the nearest, out of range
                key = np.where(np.isfinite(key).any(1, keepdims=True), key,
                               np.where(dist == dist.min(1, keepdims=True), dist, np.inf))
            sel = np.argsort(key, axis=1, kind="stable")[:, :m]
            k = np.count_nonzero(np.isfinite(np.take_along_axis(key, sel, 1)), axis=1)
            a = np.full((F, L), ADD)
        W = sel.shape[1]
        valid = np.arange(W)[None, :] < k[:, None]
        if shuffle:  # a random order of the valid markers (invalid ones stay behind them)
            keys = rng_u64(seeds[:, None], _S_SHUFFLE, np.uint64(t) * np.uint64(M) +
                           np.arange(W, dtype=np.uint64))
            keys = np.where(valid, keys >> np.uint64(1), np.uint64(2 ** 63) + np.arange(W, dtype=np.uint64))
            sel = np.take_along_axis(sel, np.argsort(keys, axis=1, kind="stable"), 1)
        rows = np.arange(F)[:, None]
        ids[t, :, :W] = np.where(valid, sel, -1)
        act[t, :, :W] = np.where(valid, a[rows, sel], 0)
        rel[t, :, :W, 0] = np.where(valid, bx[rows, sel], 0.0)
        rel[t, :, :W, 1] = np.where(valid, by[rows, sel], 0.0)
        cnt[t] = k
        sighted[np.broadcast_to(rows, sel.shape)[valid], sel[valid]] = True
        if n_delete:
            j = np.arange(n_delete, dtype=np.uint64)
            far = (rng_u64(seeds[:, None], _S_DELETE, np.uint64(t) * np.uint64(n_delete) + j)
                   % np.uint64(n_landmarks)).astype(np.int32)
            for f in range(F):
                kf = int(cnt[t, f])
                ids[t, f, kf:kf + n_delete] = far[f]
                rel[t, f, kf:kf + n_delete] = 100.0
                act[t, f, kf:kf + n_delete] = DELETE
                cnt[t, f] = kf + n_delete
    # N(0, σ²) on every reported x, y (nusim.cpp:339-340; DELETE padding markers stay at 100 m)
    idx = (np.arange(T, dtype=np.uint64)[:, None, None] * np.uint64(M) +
           np.arange(M, dtype=np.uint64)[None, None, :]) * np.uint64(2)
    noise = sensor_sigma * np.stack([
        rng_normal(seeds[None, :, None], _S_NOISE, idx),
        rng_normal(seeds[None, :, None], _S_NOISE, idx + np.uint64(1))], -1)
    live = (np.arange(M)[None, None, :] < cnt[..., None]) & (rel[..., 0] != 100.0)
    rel = np.where(live[..., None], rel + noise, rel)
    if T == drive.n_warm:
        warm_sighted = sighted.copy()
    return ids, act, rel, cnt, warm_sighted


@dataclass
class Swarm:
    """F independent seeded runs over one commanded drive, arrays indexed [T, F, ...] (the
    ekf_replay / ekf_batch_sensor layout)."""
    n_landmarks: int
    seeds: np.ndarray        # [F] uint64
    landmarks: np.ndarray    # [F, L, 2]
    wheel: np.ndarray        # [T, ticks, 2] encoder angles (the commanded drive: every filter's)
    ids: np.ndarray          # [T, F, M]
    actions: np.ndarray      # [T, F, M]
    rel: np.ndarray          # [T, F, M, 2]
    count: np.ndarray        # [T, F]
    truth: np.ndarray        # [T, F, 3]
    n_warm: int = 0
    sighted: np.ndarray = field(default=None, repr=False)  # [F, L] by the survey's end
    cmd: np.ndarray = field(default=None, repr=False)      # [T·ticks, 2] commanded wheel increments
    sense: np.ndarray = field(default=None, repr=False)    # [T] SENSE_* per message
    start_pose: tuple = (0.0, 0.0, -1.0)                   # true (θ, x, y) at the first tick

    @property
    def n_filters(self) -> int:
        return int(self.seeds.shape[0])

    def scenario(self, f: int) -> Scenario:
        return Scenario(self.n_landmarks, self.landmarks[f], self.wheel, self.ids[:, f],
                        self.actions[:, f], self.rel[:, f], self.count[:, f], self.truth[:, f],
                        n_warm=self.n_warm)

    def corrections(self, start: int = 0, stop: int | None = None) -> int:
        sl = slice(start, stop)
        live = np.arange(self.ids.shape[2])[None, None, :] < self.count[sl][..., None]
        return int(np.count_nonzero(live & (self.actions[sl] != DELETE)))


def _generate(n_landmarks, drive: Drive, seeds, landmarks=None, half=None, *, max_markers=16,
              start_pose=(0.0, 0.0, -1.0), sensor_sigma=1e-3, slip=0.02, max_range=5.0,
              shuffle=False, n_delete=0, clearance=0.3, n_map=None) -> Swarm:
    seeds = np.asarray(seeds, dtype=np.uint64).reshape(-1)
    F = seeds.shape[0]
    if drive.start_pose is not None:
        start_pose = drive.start_pose
    wheel, truth, path = _simulate(drive, seeds, start_pose, slip)
    tpm = drive.ticks_per_msg
    dt = 1.0 / drive.tick_hz
    cmd = np.stack([(drive.v - drive.w * TRACK_WIDTH / 2.0) / WHEEL_RADIUS * dt,
                    (drive.v + drive.w * TRACK_WIDTH / 2.0) / WHEEL_RADIUS * dt], 1)
    cmd = cmd[:(drive.v.shape[0] // tpm) * tpm]
    if landmarks is None:
        landmarks = _place_landmarks(n_landmarks if n_map is None else n_map, half, seeds, path,
                                     clearance)
    else:
        landmarks = np.broadcast_to(np.asarray(landmarks, np.float64),
                                    (F,) + np.shape(landmarks)[-2:]).copy()
    assert landmarks.shape[1] <= n_landmarks
    ids, act, rel, cnt, sighted = _sense(drive, seeds, landmarks, truth, max_markers, max_range,
                                         sensor_sigma, shuffle, n_delete, n_landmarks)
    return Swarm(n_landmarks, seeds, landmarks, wheel, ids, act, rel, cnt,
                 np.ascontiguousarray(truth.transpose(1, 0, 2)), drive.n_warm, sighted, cmd,
                 drive.sense.copy(), tuple(float(v) for v in start_pose))


def make_scenario(n_landmarks: int, landmarks: np.ndarray, n_messages: int, *,
                  max_markers: int = 16, nearest: bool = True, start_pose=(0.0, 0.0, -1.0),
                  circle_radius: float = 1.0, omega: float = 0.5, tick_hz: float = 200.0,
                  ticks_per_msg: int = 40, sensor_sigma: float = 1e-3, slip: float = 0.02,
                  max_range: float = 5.0, seed: int = 20240317, shuffle: bool = False,
                  n_delete: int = 0) -> Scenario:
    """A circle drive + sensing sequence over a given map. ``start_pose`` is (θ, x, y)."""
    drive = circle_drive(n_messages, circle_radius, omega, tick_hz, ticks_per_msg,
                         SENSE_NEAREST if nearest else SENSE_ALL)
    sw = _generate(n_landmarks, drive, [seed], landmarks, max_markers=max_markers,
                   start_pose=start_pose, sensor_sigma=sensor_sigma, slip=slip,
                   max_range=max_range, shuffle=shuffle, n_delete=n_delete)
    return sw.scenario(0)


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
    """SURVEY.md §8d synthetic map: N landmarks, unit circle at ω = 0.5, m nearest markers (only
    the landmarks near the circle are ever sighted: see ``populated`` for a full map)."""
    lm = random_landmarks(n_landmarks, seed)
    return make_scenario(n_landmarks, lm, n_messages, seed=seed, max_markers=max_markers, **kw)


def field_half(n_landmarks: int) -> float:
    """landmarks uniform in [-L, L]², L = 0.5·√N m."""
    return max(0.5 * math.sqrt(n_landmarks), 2.0)


def swarm(n_landmarks: int, n_filters: int, n_messages: int, seed: int = 20240317,
          max_markers: int = 16, survey: bool = True, **kw) -> Swarm:
    """SURVEY.md §8d synthetic workload for ``n_filters`` independent filters, filter f seeded
    ``seed + f`` (its own map, slip and sensor noise): ``n_messages`` of the unit circle at
    ω = 0.5 with the m nearest markers, prefixed (``survey``) by the spiral warm-up that sights
    every landmark (``Swarm.n_warm`` messages)."""
    n_map = kw.pop("n_map", n_landmarks)  # landmarks placed (≤ N slots; the rest stay free for
    half = field_half(n_map)               # the association path's new landmarks)
    ring = kw.pop("ring", 3.0)
    v_survey = kw.pop("v_survey", 4.0)
    drive = (survey_drive(half, n_messages, ring=ring, v_survey=v_survey,
                          max_range=kw.get("max_range", 5.0)) if survey else
             circle_drive(n_messages))
    seeds = np.uint64(seed) + np.arange(n_filters, dtype=np.uint64)
    sw = _generate(n_landmarks, drive, seeds, half=half, max_markers=max_markers, n_map=n_map,
                   **kw)
    if survey and not sw.sighted.all():
        raise RuntimeError(f"survey left {int((~sw.sighted).sum())} landmarks unsighted")
    return sw


def populated(n_landmarks: int, n_messages: int, seed: int = 20240317, max_markers: int = 16,
              **kw) -> Scenario:
    """One filter of ``swarm``: the survey (``n_warm`` messages, every landmark sighted), then
    ``n_messages`` of the circle."""
    return swarm(n_landmarks, 1, n_messages, seed=seed, max_markers=max_markers, **kw).scenario(0)


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
