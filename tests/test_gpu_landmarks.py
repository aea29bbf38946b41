"""GPU parity of the landmark front-end (include/landmarks.h) against the numpy oracle and the
reference's known-answer tests. Tolerances: the reference KATs' 1e-4 (circle_tests.cpp:8-34);
against the oracle (same algorithm, LAPACK arithmetic) 1e-9 m on centres and radii for clusters
of real scans; classification decisions and marker ids exactly."""
import math
import os

import numpy as np
import pytest

import landmarks_numpy as L

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "scans.npz")


@pytest.fixture(scope="module")
def det():
    from pyekf.landmarks import Detector
    d = Detector(max_scans=4096, max_beams=2048)
    yield d
    d.close()


def test_fit_circle_kats(det):
    from test_landmarks import FIT_KATS
    got = det.fit_circles([p for p, _ in FIT_KATS])
    for g, (_, want) in zip(got, FIT_KATS):
        assert np.allclose(g, want, atol=1e-4, rtol=0)
    for g, (p, _) in zip(got, FIT_KATS):
        assert np.allclose(g, L.fit_circle(p), rtol=1e-9, atol=1e-9)


def test_fit_and_check_random_arcs(det):
    rng = np.random.default_rng(7)
    clusters = []
    for _ in range(500):
        n = int(rng.integers(4, 40))
        c = rng.uniform(-2, 2, 2)
        r = rng.uniform(0.02, 0.3)
        t0 = rng.uniform(-math.pi, math.pi)
        t = t0 + np.sort(rng.uniform(0, rng.uniform(0.5, 3.0), n))
        pts = np.stack([c[0] + r * np.cos(t), c[1] + r * np.sin(t)], 1)
        pts += rng.normal(0, rng.choice([1e-4, 1e-3, 5e-3]), pts.shape)
        clusters.append(pts)
    fits = det.fit_circles(clusters)
    want = np.array([L.fit_circle(c) for c in clusters])
    scale = np.maximum(1.0, np.abs(want))
    assert np.all(np.abs(fits - want) / scale < 1e-8), np.max(np.abs(fits - want) / scale)
    chk = det.check_circles(clusters)
    ref = np.array([L.check_circle(c) for c in clusters])
    assert chk.sum() > 50 and (~chk).sum() > 50
    assert np.array_equal(chk, ref)


def test_exact_circle_takes_null_vector_branch(det):
    """Noise-free points: s.min() < 1e-12 → A = V.col(3) (landmark_detection.cpp:97-98)."""
    t = np.linspace(0.2, 2.0, 12)
    pts = np.stack([0.5 + 0.1 * np.cos(t), -0.3 + 0.1 * np.sin(t)], 1)
    got = det.fit_circles([pts])[0]
    assert np.allclose(got, (0.5, -0.3, 0.1), atol=1e-9)


def _detect_golden(det, idx):
    g = np.load(GOLD)
    B = int(g["n_beams"][idx[0]])
    assert all(int(g["n_beams"][s]) == B for s in idx)
    cnt, mk = det.detect(g["ranges"][idx, :B], g["angle_min"][idx], g["angle_inc"][idx])
    return g, cnt, mk


@pytest.mark.parametrize("name", ["basic_world", "wrap", "empty", "crowded", "maxbeams"])
def test_detect_matches_golden(det, name):
    g = np.load(GOLD)
    idx = np.flatnonzero(g["names"] == name)
    g, cnt, mk = _detect_golden(det, idx)
    for k, s in enumerate(idx):
        assert cnt[k] == g["counts"][s], (name, s)
        for i in range(max(cnt[k], 0)):
            want = g["markers"][s, i]
            assert mk[k, i]["id"] == int(want[0])
            got = np.array([mk[k, i]["x"], mk[k, i]["y"], mk[k, i]["r"]])
            assert np.allclose(got, want[1:], rtol=0, atol=1e-9), (name, s, i, got - want[1:])


def test_detect_batch_of_4096_scans(det):
    """A swarm-sized batch: every scan's result equals the same scan detected alone."""
    g = np.load(GOLD)
    idx = np.flatnonzero(g["names"] == "basic_world")
    rng = np.random.default_rng(3)
    pick = rng.choice(idx, 4096)
    cnt, mk = det.detect(g["ranges"][pick, :360], g["angle_min"][pick], g["angle_inc"][pick])
    for s in np.unique(pick):
        c1, m1 = det.detect(g["ranges"][s:s + 1, :360], g["angle_min"][s:s + 1],
                            g["angle_inc"][s:s + 1])
        rows = np.flatnonzero(pick == s)
        assert np.all(cnt[rows] == c1[0])
        k = max(int(c1[0]), 0)  # slots past the count are not written
        assert np.all(mk[rows, :k] == m1[0, :k])


def test_marker_capacity_overflow_counts_all(det):
    g = np.load(GOLD)
    s = int(np.argmax(g["counts"]))
    B = int(g["n_beams"][s])
    cnt, mk = det.detect(g["ranges"][s:s + 1, :B], g["angle_min"][s:s + 1],
                         g["angle_inc"][s:s + 1], max_markers=3)
    assert cnt[0] == g["counts"][s] > 3
    assert [int(m["id"]) for m in mk[0]] == [int(v) for v in g["markers"][s, :3, 0]]


def test_nonfinite_ranges_break_clusters(det):
    """inf / nan returns (real lidars) break clusters exactly as the reference's comparisons do."""
    g = np.load(GOLD)
    s = int(np.flatnonzero(g["names"] == "basic_world")[5])
    r = g["ranges"][s, :360].copy()
    r[::37] = np.inf
    r[10:14] = np.nan
    cnt, mk = det.detect(r[None], g["angle_min"][s:s + 1], g["angle_inc"][s:s + 1])
    want = L.laser_callback(r, float(g["angle_min"][s]), float(g["angle_inc"][s]))
    assert cnt[0] == (-1 if want is None else len(want))
    for i, w in enumerate(want or []):
        assert mk[0, i]["id"] == w[0]
        assert np.allclose([mk[0, i]["x"], mk[0, i]["y"], mk[0, i]["r"]], w[1:], atol=1e-9)


def test_argument_errors(det):
    from pyekf import EkfError
    with pytest.raises(EkfError):
        det.check_circles([np.zeros((2, 2))])  # the reference needs ≥ 3 points
    with pytest.raises(EkfError):
        det.detect(np.zeros((1, 4096), np.float32), 0.0, 0.01)  # > max_beams
