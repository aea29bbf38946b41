"""End to end on the GPU, the reference's lidar pipeline: LaserScan → `landmarks` node
(lm_detect) → MarkerArray → `slam` node sensor_cb (ekf_sensor, unknown association), against the
same pipeline in the oracles (landmarks_numpy.laser_callback → OracleEKF.sensor_cb).

Tolerances: detected marker positions 1e-9 m (front-end parity), association decisions exactly,
posterior poses 1e-8 (EKF parity, tests/test_gpu_parity.py)."""
import math

import numpy as np
import pytest

import landmarks_numpy as L
import orc

pytestmark = pytest.mark.gpu

BASIC = [(-0.5, -0.7, 0.038), (0.8, -0.8, 0.038), (0.4, 0.8, 0.038), (-0.6, 0.65, 0.038)]


def _drive(T):
    """Circle of radius 0.5 m about (0.1, 0) at 0.1 rad per message, perfect odometry."""
    out = []
    for t in range(T):
        a = 0.1 * t
        out.append((a + math.pi / 2, 0.1 + 0.5 * math.cos(a), 0.5 * math.sin(a)))
    return np.array(out)


def test_scan_to_posterior_matches_oracles():
    import pyekf
    from pyekf import synth
    from pyekf.landmarks import Detector
    T = 40
    poses = _drive(T)
    scans = synth.lidar_scans(poses, BASIC, sigma=0.001, seed=11)
    inc = float(np.float32(2 * math.pi / 360))
    det = Detector(max_scans=T, max_beams=360)
    cnt, mk = det.detect(scans, np.zeros(T), np.full(T, inc))
    ekf = pyekf.EKF(n_landmarks=50)
    ref = orc.OracleEKF(n_landmarks=50)
    seen = 0
    for t in range(T):
        want = L.laser_callback(scans[t], 0.0, inc)
        assert cnt[t] == len(want)
        got = np.array([[m["x"], m["y"]] for m in mk[t, :cnt[t]]]).reshape(-1, 2)
        ref_xy = np.array([[w[1], w[2]] for w in want]).reshape(-1, 2)
        assert np.abs(got - ref_xy).max(initial=0.0) < 1e-9
        # the slam node: odometry, then the detected MarkerArray through sensor_cb
        ekf.set_odom(poses[t])
        ref.set_odom(poses[t])
        if cnt[t] == 0:
            continue  # landmarks.cpp:153 publishes nothing for an empty detection
        seen += int(cnt[t])
        rc, j, nw = ekf.sensor(got)
        rrc, rj, rnw = ref.sensor_cb(ref_xy)
        assert rc == rrc == 0
        np.testing.assert_array_equal(j, rj)
        np.testing.assert_array_equal(nw, rnw)
        x = ekf.pose()
        xr = ref.get(sigma=False)[0][:3]
        assert np.abs(x - xr).max() < 1e-8, (t, x - xr)
    assert seen >= 20
    x, S, c = ekf.state()
    xr, Sr, _, cr = ref.get()
    assert c == cr >= 3
    assert np.abs(S - Sr).max() < 1e-6 * max(1.0, np.abs(Sr).max() / 1e7)
    det.close()
    ekf.close()


def test_rosbag_surrogate_pose_trace_matches_cpu():
    """BASELINE configs[4] surrogate (the bag's .mcap payload is missing; synth.lidar_world has its
    shape: 426 scans at 5 Hz, 20 odometry ticks per scan, 20 obstacles): scans → lm_detect →
    slam node (joint states + unknown-association MarkerArrays, slam_replay) on the GPU, against
    laser_callback → the C oracle's node loop. Pose trace within 1e-8 of the CPU pipeline."""
    import pyekf
    from pyekf import synth
    from pyekf.landmarks import Detector
    sc, _, scans = synth.lidar_world()
    T = len(scans)
    inc = float(np.float32(2 * math.pi / 360))
    det = Detector(max_scans=T, max_beams=360)
    cnt, mk = det.detect(scans, np.zeros(T), np.full(T, inc))
    det.close()
    gpu_mk = [[(m["x"], m["y"]) for m in mk[t, :cnt[t]]] for t in range(T)]
    cpu_mk = [[(w[1], w[2]) for w in L.laser_callback(scans[t], 0.0, inc)] for t in range(T)]
    for g, c in zip(gpu_mk, cpu_mk):
        assert len(g) == len(c)
        assert np.abs(np.array(g) - np.array(c)).max(initial=0.0) < 1e-9
    s = pyekf.Slam(n_landmarks=50, source=pyekf.SOURCE_ASSOC)
    rc, poses, tmo = s.replay(synth.with_markers(sc, gpu_mk))
    _, _, counter = s.filter_state(sigma=False)
    s.close()
    o = orc.run_scenario(synth.with_markers(sc, cpu_mk), True)
    assert counter == o["counter"] >= 10
    assert np.abs(poses - o["poses"]).max() < 1e-8
    assert np.abs(tmo - o["tmo"]).max() < 1e-8
