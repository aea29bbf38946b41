"""The C oracle (literal dense and structured) against the golden fixtures of the numpy oracle.

Both restate nuslam/src/slam.cpp independently (see oracle/ekf_oracle.h for the parity status:
EKF parity is unpinned by the reference's own tests; this is the cross-check between the two
restatements). Tolerances: fp64 with the reference's 1e7 prior variance — first sightings cancel
≈1e7 against ≈1e7, so ≈1e-16·1e7/1e-2 relative noise reaches the state at the 1e-10 level.
"""
import numpy as np
import pytest

import orc
from conftest import GOLDEN_CASES, load_golden

POSE_TOL = 1e-8
SIGMA_TOL = 1e-8  # absolute = 1e-15 × the 1e7 prior variance (slam.cpp:130)


@pytest.mark.parametrize("literal", [False, True], ids=["structured", "literal"])
@pytest.mark.parametrize("name", GOLDEN_CASES)
def test_oracle_matches_golden(name, literal):
    sc, g = load_golden(name)
    o = orc.run_scenario(sc, bool(g["assoc"]), literal=literal)
    assert np.all(o["rcs"] == 0)
    assert np.abs(o["poses"] - g["poses"]).max() < POSE_TOL
    assert np.abs(o["tmo"] - g["tmo"]).max() < POSE_TOL
    assert np.abs(o["state"] - g["state"]).max() < POSE_TOL
    assert np.abs(o["sigma"] - g["sigma"]).max() < SIGMA_TOL
    assert o["counter"] == int(g["counter"])
    if int(g["assoc"]):
        assert np.array_equal(o["assoc_j"], g["assoc_j"])
        assert np.array_equal(o["assoc_new"], g["assoc_new"])


def test_oracle_error_paths():
    f = orc.OracleEKF(n_landmarks=3)
    rel = np.array([[1.0, 0.5]])
    assert f.fake_sensor_cb(np.array([3]), np.array([0]), rel) == -2      # id ≥ N
    assert f.fake_sensor_cb(np.array([], np.int32), np.array([], np.int32), np.zeros((0, 2))) == -3
    # capacity: four distinct far-apart landmarks in a 3-slot filter
    pts = np.array([[1.0, 0.0], [0.0, 3.0], [-4.0, 0.0], [0.0, -5.0]])
    rc, j, nw = f.sensor_cb(pts)
    assert rc == -2 and list(nw[:3]) == [1, 1, 1]


def test_oracle_delete_only_message_is_predict_only():
    f = orc.OracleEKF(n_landmarks=4)
    f.set_odom((0.1, 0.2, 0.0))
    assert f.fake_sensor_cb(np.array([0, 1]), np.array([2, 2]), np.ones((2, 2))) == 0
    x, S, tmo, _ = f.get()
    assert np.allclose(x[:3], [0.1, 0.2, 0.0]) and np.all(x[3:] == 0)
    assert np.allclose(np.diag(S)[:3], 1e-2)


@pytest.mark.parametrize("assoc", [False, True], ids=["known", "assoc"])
def test_oracle_joseph_modes_agree(assoc):
    """The opt-in Joseph form in the C oracle: the literal dense (I−KH)Σ(I−KH)ᵀ + KRKᵀ and the
    structured expansion Σ − K·HΣ − ΣHᵀ·Kᵀ + K·S·Kᵀ agree, and both stay within rounding of the
    reference's simple form (slam.cpp:264-265; equal in exact arithmetic with the optimal gain)."""
    from pyekf import synth
    sc = synth.synthetic(20, 30, seed=7, max_markers=6, shuffle=assoc)
    js = orc.run_scenario(sc, assoc, joseph=True)
    jl = orc.run_scenario(sc, assoc, joseph=True, literal=True)
    simple = orc.run_scenario(sc, assoc)
    assert js["counter"] == jl["counter"] == simple["counter"]
    assert np.abs(js["sigma"] - jl["sigma"]).max() < 1e-8
    assert np.abs(js["poses"] - jl["poses"]).max() < 1e-9
    assert np.abs(js["sigma"] - simple["sigma"]).max() < 3e-8
    assert np.abs(js["poses"] - simple["poses"]).max() < 1e-9


def test_numpy_oracle_joseph_matches_c():
    """bench.py's CPU leg of the Joseph workload (n1024_fp32_joseph): oracle/ekf_numpy.py's dense
    (I−KH)Σ(I−KH)ᵀ + KRKᵀ equals the C oracle's Joseph mode message by message (fake_sensor_cb,
    slam.cpp:180-316, with the update of :264-265 in Joseph form)."""
    import ekf_numpy
    import pyekf
    from pyekf import synth
    sc = synth.synthetic(20, 14, seed=5, max_markers=6)
    odom = pyekf.odometry(sc)
    d = ekf_numpy.DenseEKF(n_landmarks=20, joseph=True)
    ref = orc.OracleEKF(n_landmarks=20, joseph=True)
    for t in range(sc.n_messages):
        c = int(sc.count[t])
        d.t_odom_robot = tuple(odom[t])
        d.fake_sensor_cb(sc.ids[t, :c], sc.actions[t, :c], sc.rel[t, :c])
        ref.set_odom(odom[t])
        ref.fake_sensor_cb(sc.ids[t, :c], sc.actions[t, :c], sc.rel[t, :c])
        x = ref.get(sigma=False)[0]
        assert np.abs(d.state - x).max() < 1e-8, t
    x, S, _, _ = ref.get()
    assert np.abs(d.sigma - S).max() < 1e-7
