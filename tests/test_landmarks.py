"""Landmark front-end oracle (oracle/landmarks_numpy.py) against the reference's own known-answer
tests and the committed scan fixtures. CPU only."""
import math
import os

import numpy as np
import pytest

import landmarks_numpy as L

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "scans.npz")

# turtlelib/tests/circle_tests.cpp:8-34 (tolerance 1e-4 there)
FIT_KATS = [
    ([(1, 7), (2, 6), (5, 8), (7, 7), (9, 5), (3, 7)], (4.615482, 2.807354, 4.8275)),
    ([(-1, 0), (-0.3, -0.06), (0.3, 0.1), (1, 0)], (0.4908357, -22.15212, 22.17979)),
]


@pytest.mark.parametrize("pts,want", FIT_KATS)
def test_oracle_fit_circle_kats(pts, want):
    got = L.fit_circle(pts)
    assert np.allclose(got, want, atol=1e-4, rtol=0)


def test_oracle_check_circle_arc_and_line():
    arc = [(0.05 * math.cos(t), 0.05 * math.sin(t)) for t in np.linspace(-1.2, 1.2, 9)]
    line = [(0.1 * k, 0.0) for k in range(9)]
    assert L.check_circle(arc)        # inscribed angles constant (= π − 1.2 ≈ 1.94 rad)
    assert not L.check_circle(line)   # π on a straight wall: mean > 2.6


def test_oracle_clusters_drop_breaking_point():
    """landmarks.cpp:81-86: the point that breaks a cluster belongs to none."""
    r = np.full(12, 1.0, dtype=np.float32)
    r[5] = 3.0  # far from both neighbours: breaks before and after itself
    cl = L.get_clusters(r, 0.0, np.float32(0.05))
    sizes = [len(c) for c in cl]
    # [0..4], then point 5 dropped (break), point 6 also a break (3 m → 1 m) and dropped, [7..11]
    # merged into cluster 0 (the scan's last point is near the first)?  0.55 rad apart: no
    assert sizes == [5, 0, 5]


def test_oracle_no_break_is_reference_exception():
    r = np.full(360, 0.5, dtype=np.float32)  # a circular room: no break anywhere
    assert L.get_clusters(r, 0.0, np.float32(2 * math.pi / 360)) is None
    assert L.laser_callback(r, 0.0, np.float32(2 * math.pi / 360)) is None


def test_golden_scans_reproduce():
    g = np.load(GOLD)
    assert len(g["names"]) >= 30 and -1 in g["counts"] and g["counts"].max() >= 10
    for s in range(len(g["names"])):
        n = int(g["n_beams"][s])
        out = L.laser_callback(g["ranges"][s, :n], float(g["angle_min"][s]),
                               float(g["angle_inc"][s]))
        if out is None:
            assert g["counts"][s] == -1
            continue
        assert len(out) == g["counts"][s]
        for i, m in enumerate(out):
            assert np.array_equal(np.array(m), g["markers"][s, i])


def test_golden_markers_near_true_obstacles():
    """Sanity of the synthetic scans: basic_world detections land on an obstacle (laser frame →
    world through the generating pose is not stored, so check radius only)."""
    g = np.load(GOLD)
    for s in np.flatnonzero(g["names"] == "basic_world"):
        for i in range(g["counts"][s]):
            assert abs(g["markers"][s, i, 3] - 0.038) < 0.01
