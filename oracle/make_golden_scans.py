"""Generate tests/golden/scans.npz with the numpy front-end oracle (oracle/landmarks_numpy.py).

ORACLE — TEST INFRASTRUCTURE ONLY. Run in the build container:
    python oracle/make_golden_scans.py
Each scan is a synthetic LaserScan (landmarks_numpy.synthetic_scan: exact ray casting against
cylinders and the arena walls, N(0, σ²) range noise) plus the oracle's laserCallback output
(landmarks.cpp:109-156): marker count (−1 where the reference throws: a scan without a cluster
break) and, per marker, (id, c_x, c_y, R). Cases:
  basic_world  the nusim basic_world obstacles (basic_world.yaml:8-10) seen from 24 poses of a
               circle drive, 360 beams, σ = 0.001
  wrap         an obstacle straddling beam 0, so cluster 0 wraps round the scan (landmarks.cpp:96)
  empty        a 2 m × 2 m room, walls only, no break anywhere: the reference throws (LM_NO_BREAK)
  crowded      40 random obstacles, 1440 beams, σ = 0.002
  maxbeams     LM_MAX_BEAMS (2048) beams, 25 obstacles
"""
from __future__ import annotations

import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)

import landmarks_numpy as L  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")
BASIC = [(-0.5, -0.7, 0.038), (0.8, -0.8, 0.038), (0.4, 0.8, 0.038), (-0.6, 0.65, 0.038)]


def _f32(v):
    return float(np.float32(v))


def make_cases(seed=20240317):
    rng = np.random.default_rng(seed)
    cases = []  # (name, ranges float32, angle_min, angle_inc)
    inc360 = _f32(2.0 * math.pi / 360.0)  # LaserScan stores angle_increment as float32
    for k in range(24):
        th = 2.0 * math.pi * k / 24
        pose = (th + math.pi / 2, math.cos(th) - 0.0, math.sin(th))
        r = L.synthetic_scan(pose, BASIC, sigma=0.001, rng=rng)
        cases.append(("basic_world", r, 0.0, inc360))
    # an obstacle dead ahead of the lidar (beam 0 and the last beams hit it)
    r = L.synthetic_scan((0.0, 0.0, 0.0), [(0.6, 0.0, 0.05), (-0.3, 0.9, 0.05)], sigma=0.0005,
                         rng=rng)
    cases.append(("wrap", r, 0.0, inc360))
    r = L.synthetic_scan((0.3, 0.2, -0.1), [], arena=(2.0, 2.0), sigma=0.001, rng=rng)
    cases.append(("empty", r, 0.0, inc360))
    for n_beams, n_obs, name, sig in ((1440, 40, "crowded", 0.002), (2048, 25, "maxbeams", 0.001)):
        for _ in range(3):
            obs = [(rng.uniform(-4.5, 4.5), rng.uniform(-2.2, 2.2), rng.uniform(0.03, 0.12))
                   for _ in range(n_obs)]
            pose = (rng.uniform(-math.pi, math.pi), rng.uniform(-1.0, 1.0), rng.uniform(-0.5, 0.5))
            r = L.synthetic_scan(pose, obs, n_beams=n_beams, sigma=sig, rng=rng)
            cases.append((name, r, _f32(-0.01), _f32(2.0 * math.pi / n_beams)))
    return cases


def main():
    cases = make_cases()
    maxm = 32
    names, counts = [], []
    ranges = np.full((len(cases), 2048), np.nan, dtype=np.float32)
    nbeams = np.zeros(len(cases), dtype=np.int32)
    amin = np.zeros(len(cases))
    ainc = np.zeros(len(cases))
    mk = np.zeros((len(cases), maxm, 4))
    for s, (name, r, a0, inc) in enumerate(cases):
        out = L.laser_callback(r, a0, inc)
        names.append(name)
        ranges[s, :len(r)] = r
        nbeams[s] = len(r)
        amin[s], ainc[s] = a0, inc
        counts.append(-1 if out is None else len(out))
        for i, m in enumerate(out or []):
            mk[s, i] = m
    np.savez_compressed(os.path.join(GOLD, "scans.npz"), names=np.array(names), ranges=ranges,
                        n_beams=nbeams, angle_min=amin, angle_inc=ainc,
                        counts=np.array(counts, dtype=np.int32), markers=mk)
    print("scans:", len(cases), "counts:", counts)


if __name__ == "__main__":
    main()
