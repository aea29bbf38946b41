"""Generate tests/golden/*.npz with the dense numpy oracle (oracle/ekf_numpy.py).

ORACLE — TEST INFRASTRUCTURE ONLY. Run in the build container:
    python oracle/make_golden.py
Each fixture holds the scenario inputs (encoder wheel angles per joint-state tick, marker ids /
actions / body-frame positions) and the oracle outputs (posterior pose and t_map_odom after every
sensor message, association decisions, final state, Σ and counter_obstacles).

The driver loop mirrors the reference node: every joint-state tick runs DiffDrive::FKin into
t_odom_robot (slam.cpp:599-634); every sensor message runs fake_sensor_cb (slam.cpp:180-316) or
sensor_cb (slam.cpp:318-530).
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(ROOT, "ekf-slam_amd"))

from ekf_numpy import DenseEKF, DiffDrive  # noqa: E402
from pyekf import synth  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden")


def run(sc: synth.Scenario, assoc: bool, **ekf_kw):
    ekf = DenseEKF(n_landmarks=sc.n_landmarks, **ekf_kw)
    dd = DiffDrive(sc.track, sc.radius)
    T = sc.n_messages
    poses = np.zeros((T, 3))
    tmo = np.zeros((T, 3))
    M = sc.ids.shape[1]
    assoc_j = np.full((T, M), -1, dtype=np.int32)
    assoc_new = np.zeros((T, M), dtype=np.int32)
    counters = np.zeros(T, dtype=np.int32)
    for t in range(T):
        for k in range(sc.wheel.shape[1]):
            ekf.t_odom_robot = dd.fkin(float(sc.wheel[t, k, 0]), float(sc.wheel[t, k, 1]))
        cnt = int(sc.count[t])
        if assoc:
            res = ekf.sensor_cb(sc.rel[t, :cnt])
            for i, (j, nw) in enumerate(res):
                assoc_j[t, i] = j
                assoc_new[t, i] = int(nw)
        else:
            ekf.fake_sensor_cb(sc.ids[t, :cnt], sc.actions[t, :cnt], sc.rel[t, :cnt])
        poses[t] = ekf.state[:3]
        tmo[t] = ekf.t_map_odom
        counters[t] = ekf.counter
    return dict(poses=poses, tmo=tmo, assoc_j=assoc_j, assoc_new=assoc_new, counters=counters,
                state=ekf.state, sigma=ekf.sigma, counter=ekf.counter)


def save(name, sc, out, assoc, **meta):
    path = os.path.join(GOLD, name + ".npz")
    np.savez_compressed(
        path, n_landmarks=sc.n_landmarks, landmarks=sc.landmarks, wheel=sc.wheel, ids=sc.ids,
        actions=sc.actions, rel=sc.rel, count=sc.count, truth=sc.truth, track=sc.track,
        radius=sc.radius, assoc=int(assoc), **out, **meta)
    print(f"{path}: T={sc.n_messages} corrections={sc.corrections()} "
          f"final pose={out['poses'][-1]} counter={out['counter']}")


def mixed_actions():
    """(6) basic_world with the markers' action field varied: only DELETE (2) is skipped by the
    reference (slam.cpp:205: `marker.action != DELETE`); ADD (0), MODIFY (1) and DELETEALL (3)
    markers are corrections like any other."""
    sc = synth.basic_world(60, n_delete=1, seed=20240319)
    rng = np.random.default_rng(6)
    for t in range(sc.n_messages):
        k = int(sc.count[t])
        for i in range(k):
            if sc.actions[t, i] != synth.DELETE:
                sc.actions[t, i] = rng.choice([0, 1, 3])
    assert np.isin(sc.actions, [1]).any() and np.isin(sc.actions, [3]).any()
    return sc


def main():
    os.makedirs(GOLD, exist_ok=True)
    if sys.argv[1:] == ["mixed_actions"]:  # add only this fixture (the others stay as committed)
        sc = mixed_actions()
        save("mixed_actions_known", sc, run(sc, False), False)
        return
    # (1) basic_world, known association, with one far DELETE marker per message (slam.cpp:205)
    sc = synth.basic_world(100, n_delete=1)
    save("basic_world_known", sc, run(sc, False), False)
    # (2) basic_world, unknown association (markers shuffled, ids stripped)
    sc = synth.basic_world(100, shuffle=True, seed=20240318)
    save("basic_world_assoc", sc, run(sc, True), True)
    # (3) small synthetic map, known association, 16 landmarks in 20 slots, 8 nearest per message
    lm = synth.random_landmarks(16, seed=11)
    sc = synth.make_scenario(20, lm, 80, max_markers=8, seed=11)
    save("synth16_known", sc, run(sc, False), False)
    # (4) same map, unknown association (exercises new-landmark creation and re-association)
    sc = synth.make_scenario(20, lm, 80, max_markers=8, seed=12, shuffle=True)
    save("synth16_assoc", sc, run(sc, True), True)
    # (5) crowded map: landmark pairs 0.25 m apart so Mahalanobis distances fall near the gate
    rng = np.random.default_rng(5)
    base = synth.random_landmarks(6, seed=5)
    crowd = np.concatenate([base, base + rng.normal(0, 0.18, size=base.shape)])
    sc = synth.make_scenario(24, crowd, 60, max_markers=6, seed=13, shuffle=True)
    save("crowded_assoc", sc, run(sc, True), True)
    # (6) MODIFY / DELETEALL actions are corrected, only DELETE is skipped
    sc = mixed_actions()
    save("mixed_actions_known", sc, run(sc, False), False)


if __name__ == "__main__":
    main()
