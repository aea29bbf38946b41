"""On-device Monte-Carlo inputs (include/ekf_sim.h) against their host
restatement (pyekf.synth) and the filter they feed against the C oracle.

The device runs nusim's slipping wheels + DiffDrive::FKin truth (nusim.cpp:222-230,
diff_drive.cpp:10-28), the encoders' odometry (slam.cpp:599-634) and the fake sensor
(nusim.cpp:317-346) with synth's counter-based draws, so:
* marker ids, actions and counts equal synth's exactly;
* true poses, odometry and marker positions agree to 1e-9 (the only difference is libm's sin / cos /
  log / atan2 against the device's, ≤ 1 ulp per call, over ~10³ sequential ticks);
* the filters fed on the device equal the C oracle fed the device's own recorded markers and
  odometry: basic_world 1e-8; on the populated survey maps state 5e-8 and Σ 1e-7. A chunk's
  factored update carries the 1e7 prior of its first sightings into its later corrections'
  products (K_c = r₀·Z_c, x += r₀·Zx), each rounding at ~1e7·ε: measured 1.06e-8 on
  the N=128 survey swarm below, where the two CPU restatements (oracle literal vs structured)
  differ by 1.0e-9 in state and 2.1e-8 in Σ.
"""
import numpy as np
import pytest

import orc
import pyekf
from pyekf import synth

pytestmark = pytest.mark.gpu

POSE_TOL = 1e-8
STATE_TOL_POPULATED = 5e-8
SIGMA_TOL = 1e-7
SIM_TOL = 1e-9


def _sim_for(e, sw, record=True, **kw):
    M = sw.ids.shape[2]
    m = min(16, sw.landmarks.shape[1])
    return pyekf.Sim(e, sw.landmarks, seed=int(sw.seeds[0]), ticks_per_msg=sw.wheel.shape[1],
                     max_markers=m, marker_stride=M, start_theta=sw.start_pose[0],
                     start_x=sw.start_pose[1], start_y=sw.start_pose[2], record=int(record), **kw)


def _check_inputs(sim, sw, t0=0):
    cnt, ids, act, rel = sim.markers()
    odom, truth = sim.poses()
    T = cnt.shape[0]
    sl = slice(t0, t0 + T)
    assert np.abs(truth - sw.truth[sl]).max() < SIM_TOL
    assert np.abs(odom - pyekf.odometry(sw.scenario(0))[sl]).max() < SIM_TOL
    np.testing.assert_array_equal(cnt, sw.count[sl])
    np.testing.assert_array_equal(ids, sw.ids[sl])
    np.testing.assert_array_equal(act, sw.actions[sl])
    assert np.abs(rel - sw.rel[sl]).max() < SIM_TOL
    return cnt, ids, act, rel, odom


def _oracle(N, cnt, ids, act, rel, odom, f, joseph=False):
    ref = orc.OracleEKF(n_landmarks=N, joseph=joseph)
    for t in range(cnt.shape[0]):
        ref.set_odom(odom[t])
        c = int(cnt[t, f])
        ref.fake_sensor_cb(ids[t, f, :c], act[t, f, :c], rel[t, f, :c])
    return ref.get()


@pytest.mark.parametrize("dtype", [pyekf.EKF_F64], ids=["f64"])
def test_sim_populated_swarm(dtype):
    """N=128 slots, 8 filters seeded base + f: the survey spiral (SENSE_SURVEY, every landmark
    sighted) then the circle (SENSE_NEAREST, 16 markers), all on the device, pipeline path."""
    N, F = 128, 8
    sw = synth.swarm(N, F, 12)
    e = pyekf.EKF(n_landmarks=N, n_filters=F, dtype=dtype)
    assert e.path == pyekf.EKF_PATH_PIPELINE
    sim = _sim_for(e, sw)
    sim.run(sw.cmd, sw.sense)
    cnt, ids, act, rel, odom = _check_inputs(sim, sw)
    for f in range(F):
        assert e.status(f) == 0
        x, S, c = e.state(f)
        xr, Sr, _, cr = _oracle(N, cnt, ids, act, rel, odom, f)
        assert c == cr
        assert np.abs(x - xr).max() < STATE_TOL_POPULATED, f
        assert np.abs(S - Sr).max() < SIGMA_TOL, f
    sim.close()
    e.close()


def test_sim_basic_world_resident_and_runs_continue():
    """configs[0]'s world for 64 filters on the resident path: every landmark reported, DELETE
    beyond range (SENSE_ALL, nusim.cpp:332-336). Two runs continue where the first stopped (wheel,
    odometry and message counters), equal to one host-generated drive."""
    F, T1, T2 = 64, 30, 20
    drive = synth.circle_drive(T1 + T2, 0.3, sense=synth.SENSE_ALL)
    seeds = np.uint64(777) + np.arange(F, dtype=np.uint64)
    sw = synth._generate(50, drive, seeds, synth.BASIC_WORLD_LANDMARKS,
                         start_pose=(synth.BASIC_WORLD_THETA0, 0.0, 0.0), max_range=0.8)
    assert (sw.actions == synth.DELETE).any() and (sw.actions == synth.ADD).any()
    e = pyekf.EKF(n_landmarks=50, n_filters=F)
    assert e.path == pyekf.EKF_PATH_RESIDENT
    sim = _sim_for(e, sw, max_range=0.8)
    tpm = sw.wheel.shape[1]
    parts = []
    for a, b in ((0, T1), (T1, T1 + T2)):
        sim.run(sw.cmd[a * tpm:b * tpm], sw.sense[a:b])
        parts.append(_check_inputs(sim, sw, a))
    cnt, ids, act, rel, odom = (np.concatenate(p) for p in zip(*parts))
    for f in (0, 17, 63):
        assert e.status(f) == 0
        x, S, _ = e.state(f)
        xr, Sr, _, _ = _oracle(50, cnt, ids, act, rel, odom, f)
        assert np.abs(x - xr).max() < POSE_TOL, f
        assert np.abs(S - Sr).max() < POSE_TOL, f
    sim.close()
    e.close()


def test_sim_schedules_and_host_replay_agree(monkeypatch):
    """The device-fed filter in the device-epoch and the event schedule (bit-identical), and the
    same markers through ekf_replay planned on the host (the descriptors differ only in z from the
    device's atan2 against glibc's): within 1e-9."""
    N, F = 64, 4
    sw = synth.swarm(N, F, 10)
    out = []
    for env in ("1", "0"):
        monkeypatch.setenv("EKF_DEVSYNC", env)
        e = pyekf.EKF(n_landmarks=N, n_filters=F)
        sim = _sim_for(e, sw)
        sim.run(sw.cmd, sw.sense)
        out.append([e.state(f) for f in range(F)])
        markers = sim.markers()
        odom = sim.poses()[0]
        sim.close()
        e.close()
    for (xa, Sa, _), (xb, Sb, _) in zip(*out):
        np.testing.assert_array_equal(xa, xb)
        np.testing.assert_array_equal(Sa, Sb)
    cnt, ids, act, rel = markers
    e = pyekf.EKF(n_landmarks=N, n_filters=F)
    e.replay(cnt, rel, np.repeat(odom[:, None], F, 1), ids=ids, actions=act)
    for f in range(F):
        x, S, _ = e.state(f)
        assert np.abs(x - out[0][f][0]).max() < 1e-9
        assert np.abs(S - out[0][f][1]).max() < 1e-8
    e.close()


def test_sim_then_host_call_predicts_from_the_sims_odometry():
    """After ekf_sim_run the handle's t_odom_robot is the run's last odometry pose (the device
    integrated the encoders, slam.cpp:599-634): a host ekf_batch_sensor with odom = NULL then
    predicts from it, as the oracle fed the same odometry does (fp64 pipeline, N = 64)."""
    N, F, T = 64, 2, 10
    sw = synth.swarm(N, F, T + 1)
    Tw = sw.count.shape[0] - 1  # the sim runs all but the last message; the host sends that one
    e = pyekf.EKF(n_landmarks=N, n_filters=F)
    sim = _sim_for(e, sw)
    tpm = sw.wheel.shape[1]
    sim.run(sw.cmd[:Tw * tpm], sw.sense[:Tw])
    cnt, ids, act, rel = sim.markers()
    odom = sim.poses()[0]
    t = Tw
    assert e.batch_sensor(sw.count[t], sw.rel[t], None, ids=sw.ids[t], actions=sw.actions[t]) == 0
    for f in range(F):
        ref = orc.OracleEKF(n_landmarks=N)
        for k in range(Tw):
            ref.set_odom(odom[k])
            c = int(cnt[k, f])
            ref.fake_sensor_cb(ids[k, f, :c], act[k, f, :c], rel[k, f, :c])
        c = int(sw.count[t, f])  # odometry unchanged since the run: t_odom_robot = odom[Tw - 1]
        ref.fake_sensor_cb(sw.ids[t, f, :c], sw.actions[t, f, :c], sw.rel[t, f, :c])
        x, S, _ = e.state(f)
        xr, Sr, _, _ = ref.get()
        assert e.status(f) == 0
        assert np.abs(x - xr).max() < STATE_TOL_POPULATED, f
        assert np.abs(S - Sr).max() < SIGMA_TOL, f
    sim.close()
    e.close()


def _runs(sim, sw, bounds):
    tpm = sw.wheel.shape[1]
    parts = []
    for a, b in bounds:
        sim.run(sw.cmd[a * tpm:b * tpm], sw.sense[a:b])
        parts.append(_check_inputs(sim, sw, a))
    return [np.concatenate(p) for p in zip(*parts)]


def test_sim_parallel_form_equals_sequential(monkeypatch):
    """Runs without SURVEY messages take the parallel form on the pipeline (the wheels per filter,
    then every (message, filter) sensed at once, planned by ekf_replay_device's planner): markers
    and poses equal synth's as the sequential kernel's do, and the filter equals the sequential
    form's to rounding (EKF_SIM_PARALLEL=0 plans each run on the host mirror: its first chunk gathers
    Σ_in from HBM where the device planner's rebuilds it from the chunk before, kLook, and the
    rebuild's MFMA sums D − K'·M' in another order than the Σ pass: ≤ 1e-14 relative, measured
    7e-15 on the state) and the oracle fed the markers. N = 128, 8 filters: the survey in one run
    (sequential), the circle in two runs."""
    N, F = 128, 8
    sw = synth.swarm(N, F, 14)
    w = sw.n_warm
    assert (sw.sense[:w] == synth.SENSE_SURVEY).any() and not (sw.sense[w:] == synth.SENSE_SURVEY).any()
    bounds = ((0, w), (w, w + 6), (w + 6, w + 14))
    out = []
    for env in ("1", "0"):
        monkeypatch.setenv("EKF_SIM_PARALLEL", env)
        e = pyekf.EKF(n_landmarks=N, n_filters=F)
        sim = _sim_for(e, sw)
        inputs = _runs(sim, sw, bounds)
        out.append(([e.state(f) for f in range(F)], [e.status(f) for f in range(F)]))
        sim.close()
        e.close()
    cnt, ids, act, rel, odom = inputs
    for f in range(F):
        (xa, Sa, ca), (xb, Sb, cb) = out[0][0][f], out[1][0][f]
        assert out[0][1][f] == 0 and out[1][1][f] == 0
        assert np.all(np.abs(xa - xb) <= 1e-12 * np.maximum(1.0, np.abs(xb))), f
        assert np.all(np.abs(Sa - Sb) <= 1e-12 * np.maximum(1.0, np.abs(Sb))), f
        assert ca == cb
        if f in (0, 5):
            xr, Sr, _, cr = _oracle(N, cnt, ids, act, rel, odom, f)
            assert ca == cr
            assert np.abs(xa - xr).max() < STATE_TOL_POPULATED, f
            assert np.abs(Sa - Sr).max() < SIGMA_TOL, f


def test_sim_parallel_form_sense_all_on_the_pipeline(monkeypatch):
    """basic_world (every landmark reported, DELETE beyond range: SENSE_ALL) forced onto the HBM
    pipeline (EKF_RESIDENT=0), so the parallel form runs it: inputs equal synth's, the filter the
    oracle's (1e-8), across two runs that continue one another."""
    monkeypatch.setenv("EKF_RESIDENT", "0")
    F, T1, T2 = 16, 12, 10
    drive = synth.circle_drive(T1 + T2, 0.3, sense=synth.SENSE_ALL)
    seeds = np.uint64(4242) + np.arange(F, dtype=np.uint64)
    sw = synth._generate(50, drive, seeds, synth.BASIC_WORLD_LANDMARKS,
                         start_pose=(synth.BASIC_WORLD_THETA0, 0.0, 0.0), max_range=0.8)
    assert (sw.actions == synth.DELETE).any()
    e = pyekf.EKF(n_landmarks=50, n_filters=F)
    assert e.path == pyekf.EKF_PATH_PIPELINE
    sim = _sim_for(e, sw, max_range=0.8)
    cnt, ids, act, rel, odom = _runs(sim, sw, ((0, T1), (T1, T1 + T2)))
    for f in (0, 9, 15):
        assert e.status(f) == 0
        x, S, _ = e.state(f)
        xr, Sr, _, _ = _oracle(50, cnt, ids, act, rel, odom, f)
        assert np.abs(x - xr).max() < POSE_TOL, f
        assert np.abs(S - Sr).max() < POSE_TOL, f
    sim.close()
    e.close()


@pytest.mark.parametrize("parallel", ["1", "0"], ids=["parallel", "sequential"])
def test_sim_joseph_on_the_pipeline(monkeypatch, parallel):
    """ekf_set_joseph on an HBM-pipeline handle: both forms write kJoseph chunks, one per message
    (the parallel form through ekf_replay_device's planner, the sequential one from k_sim) —
    basic_world forced onto the pipeline over two runs, against the oracle's Joseph mode fed the
    device's markers (1e-8)."""
    monkeypatch.setenv("EKF_RESIDENT", "0")
    monkeypatch.setenv("EKF_SIM_PARALLEL", parallel)
    F, T1, T2 = 4, 12, 10
    drive = synth.circle_drive(T1 + T2 + 1, 0.3, sense=synth.SENSE_ALL)
    seeds = np.uint64(5151) + np.arange(F, dtype=np.uint64)
    sw = synth._generate(50, drive, seeds, synth.BASIC_WORLD_LANDMARKS,
                         start_pose=(synth.BASIC_WORLD_THETA0, 0.0, 0.0), max_range=0.8)
    e = pyekf.EKF(n_landmarks=50, n_filters=F)
    assert e.path == pyekf.EKF_PATH_PIPELINE
    assert e.set_joseph(True) == pyekf.EKF_OK
    sim = _sim_for(e, sw, max_range=0.8)
    cnt, ids, act, rel, odom = _runs(sim, sw, ((0, T1), (T1, T1 + T2)))
    for f in (0, 3):
        assert e.status(f) == 0
        x, S, _ = e.state(f)
        xr, Sr, _, _ = _oracle(50, cnt, ids, act, rel, odom, f, joseph=True)
        assert np.abs(x - xr).max() < POSE_TOL, f
        assert np.abs(S - Sr).max() < POSE_TOL, f
    sim.close()
    e.close()
