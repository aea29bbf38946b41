"""The synthetic workload generator (pyekf.synth, the stand-in for nusim): SURVEY.md §8d's inputs.

CPU-only: these check the generator's own contract — counter-based seeding per filter, the survey
warm-up sighting every landmark, the path clearance, and the marker semantics the reference's
callbacks see (slam.cpp:205: only DELETE is skipped).
"""
import numpy as np

from pyekf import synth


def test_counter_rng_is_a_pure_function_of_its_indices():
    a = synth.rng_u64(7, 3, np.arange(10))
    b = synth.rng_u64(np.uint64(7), 3, np.arange(10, dtype=np.uint64))
    assert np.array_equal(a, b)
    assert len(set(a.tolist())) == 10
    assert not np.array_equal(a, synth.rng_u64(8, 3, np.arange(10)))   # seed
    assert not np.array_equal(a, synth.rng_u64(7, 4, np.arange(10)))   # stream
    u = synth.rng_uniform(1, 1, np.arange(200000))
    assert 0.0 <= u.min() and u.max() < 1.0 and abs(u.mean() - 0.5) < 0.005
    z = synth.rng_normal(1, 2, np.arange(200000))
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1.0) < 0.01


def test_swarm_filters_are_their_own_seeded_runs():
    """Filter f of a swarm seeded s is exactly the single run seeded s + f."""
    sw = synth.swarm(64, 5, 8, seed=1000)
    for f in (0, 3):
        one = synth.populated(64, 8, seed=1000 + f)
        s = sw.scenario(f)
        assert np.array_equal(s.ids, one.ids) and np.array_equal(s.rel, one.rel)
        assert np.array_equal(s.landmarks, one.landmarks) and np.array_equal(s.wheel, one.wheel)
    # distinct filters see distinct maps and noise
    assert not np.array_equal(sw.landmarks[0], sw.landmarks[1])
    assert not np.array_equal(sw.rel[:, 0], sw.rel[:, 1])


def test_survey_sights_every_landmark_before_the_timed_messages():
    for N in (64, 256, 1024):
        sc = synth.populated(N, 4)
        w = sc.n_warm
        seen = np.unique(sc.ids[:w][(sc.ids[:w] >= 0) & (sc.actions[:w] != synth.DELETE)])
        assert seen.size == N and w > 0
        assert sc.n_messages == w + 4
        assert np.all(sc.count <= 16)


def test_landmarks_keep_clear_of_the_true_path():
    sc = synth.populated(256, 30)
    r = np.hypot(sc.rel[..., 0], sc.rel[..., 1])[sc.ids >= 0]
    assert r.min() > 0.3 - 5e-3  # clearance 0.3 m (sensor noise σ = 1e-3)


def test_circle_drive_sees_only_the_landmarks_near_it():
    """The plain circle (synth.synthetic) is why the survey exists: at N=1024 it sights ~35 ids."""
    sc = synth.synthetic(1024, 100)
    assert np.unique(sc.ids[sc.ids >= 0]).size < 64


def test_basic_world_reports_every_landmark_with_delete_beyond_range():
    sc = synth.basic_world(30, n_delete=1)
    assert np.all(sc.count == 5)
    assert np.all(sc.actions[:, 4] == synth.DELETE)
    assert sc.corrections() == 4 * 30
    sc.actions[0, 0] = synth.DELETEALL
    sc.actions[0, 1] = synth.MODIFY
    assert sc.corrections() == 4 * 30  # only DELETE is skipped (slam.cpp:205)
