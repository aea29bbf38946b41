"""ORACLE — TEST INFRASTRUCTURE ONLY.

numpy restatement of maxipalay/ekf-slam's lidar landmark front-end, the producer of the
association path's input:

* ``get_clusters``   — ``Landmarks::getClusters``, nuslam/src/landmarks.cpp:58-106
* ``check_circle``   — ``turtlelib::checkCircle``, turtlelib/src/landmark_detection.cpp:5-48
* ``fit_circle``     — ``turtlelib::fitCircle`` (Hyper fit), landmark_detection.cpp:50-135
* ``laser_callback`` — ``Landmarks::laserCallback``, landmarks.cpp:109-156

The reference's linear algebra is Armadillo over LAPACK: ``arma::svd`` (gesdd), ``arma::eig_sym``
(syevd), ``arma::solve`` (gesv). numpy.linalg calls the same LAPACK drivers (its bundled OpenBLAS
build), so this restatement follows the reference's arithmetic call for call.

Parity status: ``fit_circle`` is PINNED by the reference's known-answer tests
(turtlelib/tests/circle_tests.cpp:8-34, tests/test_landmarks.py). ``get_clusters``,
``check_circle`` and ``laser_callback`` have no reference test: restated from the source text,
parity UNPINNED beyond that.

Only ``tests/`` (and ``oracle/make_golden.py``) import this module; the product never does.
"""
from __future__ import annotations

import math

import numpy as np

from ekf_numpy import normalize_angle

LIDAR_X_OFFSET = 0.032      # landmarks.cpp:69 (base_scan sits 32 mm behind the body origin)
CLUSTER_THRESHOLD = 0.2     # landmarks.cpp:195
MAX_RADIUS = 0.2            # landmarks.cpp:145
MAX_RANGE = 2.0             # landmarks.cpp:145


def _dist(p, q):
    """turtlelib::distance, geometry2d.cpp:134-136"""
    return math.sqrt((p[0] - q[0]) ** 2 + (p[1] - q[1]) ** 2)


def scan_points(ranges, angle_min, angle_increment):
    """The beam endpoints of landmarks.cpp:66-70: the ranges are float32 (sensor_msgs/LaserScan)
    widened to double; the angle is normalize_angle(i·inc) + angle_min."""
    pts = []
    for i, r in enumerate(np.asarray(ranges, dtype=np.float32)):
        a = normalize_angle(float(i) * angle_increment) + angle_min
        r = float(r)
        pts.append((r * math.cos(a) - LIDAR_X_OFFSET, r * math.sin(a)))
    return pts


def get_clusters(ranges, angle_min, angle_increment, threshold=CLUSTER_THRESHOLD):
    """landmarks.cpp:58-106. A point farther than ``threshold`` from its predecessor ends the
    current cluster and is itself DROPPED (:81-86: the new cluster starts empty), possibly leaving
    empty clusters in the list. The last cluster is appended to the first when the scan's last
    point lies within ``threshold`` of the first cluster's first point (:94-103). With no break in
    the whole scan the reference throws (``clusters.at(0)`` on an empty list, :94): ``None``."""
    pts = scan_points(ranges, angle_min, angle_increment)
    clusters, cur, prev = [], [], None
    for i, p in enumerate(pts):
        if i == 0:
            cur.append(p)
        elif _dist(p, prev) <= threshold:
            cur.append(p)
        else:
            clusters.append(cur)
            cur = []
        prev = p
    if not clusters:
        return None
    if _dist(clusters[0][0], prev) <= threshold:
        clusters[0].extend(cur)
    else:
        clusters.append(cur)
    return clusters


def check_circle(cluster):
    """landmark_detection.cpp:5-48: inscribed angles of the interior points over the chord from
    the first to the last point; a circle when their sample std (N−1, arma::stddev) < 0.2 and
    1.3 < mean < 2.6."""
    p0, p1 = cluster[0], cluster[-1]
    ang = []
    for j in range(1, len(cluster) - 1):
        q = cluster[j]
        a = math.sqrt((p0[0] - q[0]) ** 2 + (p0[1] - q[1]) ** 2)
        b = math.sqrt((p1[0] - q[0]) ** 2 + (p1[1] - q[1]) ** 2)
        c = math.sqrt((p0[0] - p1[0]) ** 2 + (p0[1] - p1[1]) ** 2)
        with np.errstate(all="ignore"):
            x = np.float64(c * c - a * a - b * b) / np.float64(-2.0 * a * b)
            ang.append(float(np.arccos(x)))
    ang = np.array(ang)
    with np.errstate(all="ignore"):
        sd = float(np.std(ang, ddof=1)) if len(ang) > 1 else 0.0
        mn = float(np.mean(ang))
    return bool(sd < 0.2 and 1.3 < mn < 2.6)


def fit_circle(cluster):
    """landmark_detection.cpp:50-135 (Hyper fit, Al-Sharadqah & Chernov): (c_x, c_y, R)."""
    P = np.array(cluster, dtype=np.float64).reshape(-1, 2)
    n = P.shape[0]
    means = P.mean(axis=0)
    x = P[:, 0] - means[0]
    y = P[:, 1] - means[1]
    z = x ** 2 + y ** 2
    z_mean = z.mean()
    Z = np.stack([z, x, y, np.ones(n)], axis=1)
    H_inv = np.eye(4)
    H_inv[0, 0] = 0.0
    H_inv[3, 0] = 0.5
    H_inv[0, 3] = 0.5
    H_inv[3, 3] = -2.0 * z_mean
    _, s, Vt = np.linalg.svd(Z, full_matrices=False)  # s descending, like arma::svd
    V = Vt.T
    if s.min() < 10.0e-12:
        A = V[:, 3]
    else:
        Y = V @ np.diag(s) @ V.T
        Q = Y @ H_inv @ Y
        w, E = np.linalg.eigh(Q)                          # ascending, like arma::eig_sym
        idx, min_val = 0, 10.0e6
        for i in range(4):
            if w[i] < min_val and w[i] > 0.0:
                min_val, idx = w[i], i
        A = np.linalg.solve(Y, E[:, idx])
    a = -A[1] / 2.0 / A[0]
    b = -A[2] / 2.0 / A[0]
    R2 = (A[1] * A[1] + A[2] * A[2] - 4.0 * A[0] * A[3]) / 4.0 / A[0] / A[0]
    with np.errstate(invalid="ignore"):
        R = float(np.sqrt(R2))
    return float(a + means[0]), float(b + means[1]), R


def laser_callback(ranges, angle_min, angle_increment, threshold=CLUSTER_THRESHOLD):
    """landmarks.cpp:109-156: clusters of 4..39 points that pass check_circle are numbered in
    order (the marker id, :147); a fitted circle becomes a marker when R < 0.2 and its centre is
    within 2 m (:145). Returns a list of (id, c_x, c_y, R), or None where the reference throws."""
    clusters = get_clusters(ranges, angle_min, angle_increment, threshold)
    if clusters is None:
        return None
    cands = [c for c in clusters if 3 < len(c) < 40 and check_circle(c)]
    out = []
    for i, c in enumerate(cands):
        cx, cy, r = fit_circle(c)
        if r < MAX_RADIUS and math.sqrt(cx ** 2 + cy ** 2) < MAX_RANGE:
            out.append((i, cx, cy, r))
    return out


def synthetic_scan(pose, circles, arena=(10.0, 5.0), n_beams=360, sigma=0.0, rng=None,
                   range_min=0.11, range_max=10.0):
    """Test-input generator (not a reference function): exact ray casting of a lidar at
    ``pose`` = (θ, x, y) of the body, mounted −0.032 m along the body x axis (nusim.cpp:577), beam
    i at angle i·2π/n, against cylinders ``circles`` = [(x, y, r)] and the walls of an axis-aligned
    arena centred on the origin; ranges clamped to [range_min, range_max] then N(0, σ²) noise added
    (nusim.cpp:700-707). Returns float32 ranges."""
    th, px, py = pose
    lx, ly = px - 0.032 * math.cos(th), py - 0.032 * math.sin(th)
    hx, hy = arena[0] / 2.0, arena[1] / 2.0
    out = np.empty(n_beams, dtype=np.float32)
    for i in range(n_beams):
        a = th + i * 2.0 * math.pi / n_beams
        dx, dy = math.cos(a), math.sin(a)
        best = math.inf
        for (cx, cy, r) in circles:
            fx, fy = lx - cx, ly - cy
            bq = fx * dx + fy * dy
            cq = fx * fx + fy * fy - r * r
            disc = bq * bq - cq
            if disc >= 0.0:
                t = -bq - math.sqrt(disc)
                if t > 0.0:
                    best = min(best, t)
        for (den, lim, org) in ((dx, hx, lx), (-dx, hx, -lx), (dy, hy, ly), (-dy, hy, -ly)):
            if den > 1e-12:
                best = min(best, (lim - org) / den)
        best = min(max(best, range_min), range_max)
        if sigma > 0.0:
            best += rng.normal(0.0, sigma)
        out[i] = best
    return out
