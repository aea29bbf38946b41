"""HIP path (through the C-ABI) against the golden fixtures and the C oracle.

Tolerances (fp64): posterior poses / state 1e-8, Σ 1e-8 absolute (1e-15 of the reference's 1e7
prior variance, slam.cpp:130), association decisions exact. The HIP path folds a message's
corrections into one rank-(2+2m) Σ pass, so its summation order differs from the reference's
sequential dense algebra; the results agree to rounding.
"""
import numpy as np
import pytest

import orc
import pyekf
from conftest import GOLDEN_CASES, load_golden
from pyekf import synth

pytestmark = pytest.mark.gpu

POSE_TOL = 1e-8
SIGMA_TOL = 1e-8


def _replay_node(sc, assoc, dtype=pyekf.EKF_F64):
    s = pyekf.Slam(n_landmarks=sc.n_landmarks,
                   source=pyekf.SOURCE_ASSOC if assoc else pyekf.SOURCE_SIM, dtype=dtype,
                   track=sc.track, radius=sc.radius)
    rc, poses, tmo = s.replay(sc)
    x, S, cnt = s.filter_state()
    return rc, poses, tmo, x, S, cnt, s


@pytest.mark.parametrize("name", GOLDEN_CASES)
def test_node_replay_matches_golden(name):
    sc, g = load_golden(name)
    rc, poses, tmo, x, S, cnt, _ = _replay_node(sc, bool(g["assoc"]))
    assert rc == pyekf.EKF_OK
    assert np.abs(poses - g["poses"]).max() < POSE_TOL
    assert np.abs(tmo - g["tmo"]).max() < POSE_TOL
    assert np.abs(x - g["state"]).max() < POSE_TOL
    assert np.abs(S - g["sigma"]).max() < SIGMA_TOL
    assert cnt == int(g["counter"])


@pytest.mark.parametrize("name", [c for c in GOLDEN_CASES if "assoc" in c])
def test_association_decisions_match_golden(name):
    sc, g = load_golden(name)
    ekf = pyekf.EKF(n_landmarks=sc.n_landmarks)
    odom = pyekf.odometry(sc)
    for t in range(sc.n_messages):
        ekf.set_odom(odom[t])
        c = int(sc.count[t])
        rc, j, nw = ekf.sensor(sc.rel[t, :c])
        assert rc == 0
        assert np.array_equal(j, g["assoc_j"][t, :c]), t
        assert np.array_equal(nw, g["assoc_new"][t, :c]), t
    assert np.abs(ekf.pose() - g["poses"][-1]).max() < POSE_TOL


def test_fine_grained_surface_equals_callback():
    """predict()/correct()/posterior() one marker at a time == fake_sensor_cb (slam.cpp:180-316)."""
    sc, g = load_golden("basic_world_known")
    ekf = pyekf.EKF(n_landmarks=sc.n_landmarks)
    odom = pyekf.odometry(sc)
    for t in range(sc.n_messages):
        ekf.set_odom(odom[t])
        assert ekf.predict() == 0
        for i in range(int(sc.count[t])):
            if sc.actions[t, i] == pyekf.DELETE:
                continue
            assert ekf.correct(sc.ids[t, i], *sc.rel[t, i]) == 0
        assert ekf.posterior() == 0
        assert np.abs(ekf.pose() - g["poses"][t]).max() < POSE_TOL
        assert np.abs(ekf.map_odom() - g["tmo"][t]).max() < POSE_TOL
    x, S, _ = ekf.state()
    assert np.abs(S - g["sigma"]).max() < SIGMA_TOL


def test_fine_grained_associate_equals_callback():
    sc, g = load_golden("synth16_assoc")
    ekf = pyekf.EKF(n_landmarks=sc.n_landmarks)
    odom = pyekf.odometry(sc)
    for t in range(sc.n_messages):
        ekf.set_odom(odom[t])
        ekf.predict()
        for i in range(int(sc.count[t])):
            rc, j, nw = ekf.associate_correct(*sc.rel[t, i])
            assert rc == 0 and j == g["assoc_j"][t, i] and nw == g["assoc_new"][t, i]
        ekf.posterior()
    assert np.abs(ekf.pose() - g["poses"][-1]).max() < POSE_TOL


@pytest.mark.parametrize("assoc", [False, True], ids=["known", "assoc"])
def test_batched_filters_match_oracle(assoc):
    """8 independent filters in one handle (the swarm layout), each vs its own oracle run."""
    F, T, N = 8, 30, 20
    scs = [synth.make_scenario(N, synth.random_landmarks(12, seed=100 + f), T, max_markers=6,
                               seed=200 + f, shuffle=assoc) for f in range(F)]
    M = max(s.ids.shape[1] for s in scs)
    counts = np.zeros((T, F), np.int32)
    ids = np.full((T, F, M), -1, np.int32)
    act = np.zeros((T, F, M), np.int32)
    rel = np.zeros((T, F, M, 2))
    odom = np.zeros((T, F, 3))
    for f, s in enumerate(scs):
        m = s.ids.shape[1]
        counts[:, f] = s.count
        ids[:, f, :m] = s.ids
        act[:, f, :m] = s.actions
        rel[:, f, :m] = s.rel
        odom[:, f] = pyekf.odometry(s)
    ekf = pyekf.EKF(n_landmarks=N, n_filters=F)
    poses = ekf.replay(counts, rel, odom, ids=None if assoc else ids, actions=act, assoc=assoc,
                       poses=True)
    for f, s in enumerate(scs):
        o = orc.run_scenario(s, assoc)
        assert np.abs(poses[:, f] - o["poses"]).max() < POSE_TOL, f
        x, S, cnt = ekf.state(f)
        assert np.abs(S - o["sigma"]).max() < SIGMA_TOL, f
        assert cnt == o["counter"]


def test_long_message_is_chunked():
    """40 markers in one message → three Σ passes (EKF_MAX_CHUNK = 16), same result."""
    lm = synth.random_landmarks(40, seed=3)
    sc = synth.make_scenario(50, lm, 12, max_markers=40, seed=4)
    assert sc.count.max() > 16
    rc, poses, tmo, x, S, cnt, _ = _replay_node(sc, False)
    o = orc.run_scenario(sc, False)
    assert rc == 0
    assert np.abs(poses - o["poses"]).max() < POSE_TOL
    assert np.abs(S - o["sigma"]).max() < SIGMA_TOL


def test_repeated_landmark_in_one_message():
    """The same id twice in one message (two copies of its rows in the touched-index set)."""
    ekf = pyekf.EKF(n_landmarks=6)
    ref = orc.OracleEKF(n_landmarks=6)
    rng = np.random.default_rng(0)
    for t in range(10):
        od = (0.05 * t, 0.1 * t, 0.02 * t)
        ekf.set_odom(od)
        ref.set_odom(od)
        ids = np.array([1, 3, 1, 1, 4], np.int32)
        rel = np.array([[1.0, 0.2], [0.5, -1.0], [1.0, 0.2], [1.0, 0.21], [-0.7, 0.4]])
        rel = rel + rng.normal(0, 1e-3, rel.shape)
        assert ekf.fake_sensor(ids, np.zeros(5, np.int32), rel) == 0
        assert ref.fake_sensor_cb(ids, np.zeros(5, np.int32), rel) == 0
    x, S, _ = ekf.state()
    xr, Sr, _, _ = ref.get()
    assert np.abs(x - xr).max() < POSE_TOL
    assert np.abs(S - Sr).max() < SIGMA_TOL


def test_error_paths():
    ekf = pyekf.EKF(n_landmarks=3)
    x0, S0, _ = ekf.state()
    assert ekf.fake_sensor(np.array([3]), np.array([0]), np.array([[1.0, 0.5]])) == \
        pyekf.EKF_E_RANGE
    assert ekf.fake_sensor(np.zeros(0), np.zeros(0), np.zeros((0, 2))) == pyekf.EKF_E_EMPTY
    x1, S1, _ = ekf.state()
    assert np.array_equal(x0, x1) and np.array_equal(S0, S1)  # rejected atomically
    # DELETE-only message: predict only
    ekf.set_odom((0.1, 0.2, 0.0))
    assert ekf.fake_sensor(np.array([0, 1]), np.array([2, 2]), np.ones((2, 2))) == 0
    x, S, _ = ekf.state()
    assert np.allclose(x[:3], [0.1, 0.2, 0.0]) and np.all(x[3:] == 0)
    # capacity overflow on the association path (the reference indexes past the state)
    pts = np.array([[1.0, 0.0], [0.0, 3.0], [-4.0, 0.0], [0.0, -5.0]])
    rc, j, nw = ekf.sensor(pts)
    assert rc == pyekf.EKF_E_RANGE and list(nw[:3]) == [1, 1, 1] and j[3] == -1
    assert ekf.status() & pyekf.EKF_FLAG_RANGE


def test_set_get_state_roundtrip():
    sc, g = load_golden("synth16_known")
    ekf = pyekf.EKF(n_landmarks=sc.n_landmarks)
    ekf.set_state(g["state"], g["sigma"], tmo=g["tmo"][-1], counter=7)
    x, S, cnt = ekf.state()
    assert np.array_equal(x, g["state"]) and np.array_equal(S, g["sigma"]) and cnt == 7
    assert np.array_equal(ekf.map_odom(), g["tmo"][-1])


def _pipelined_final(sc, monkeypatch, env, dtype=pyekf.EKF_F64, F=1):
    """Replay every message in one call (one upload, chunks pipelined across the two streams)."""
    for k in ("EKF_SERIAL", "EKF_CU_SPLIT", "EKF_DEVSYNC"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    odom = pyekf.odometry(sc)
    e = pyekf.EKF(n_landmarks=sc.n_landmarks, n_filters=F, dtype=dtype)
    rep = lambda a: np.repeat(a[:, None], F, 1)  # noqa: E731
    e.replay(rep(sc.count), rep(sc.rel), rep(odom), ids=rep(sc.ids), actions=rep(sc.actions))
    out = [e.state(f) for f in range(F)]
    # no numeric skip and no epoch-poll timeout (EKF_FLAG_TIMEOUT = 4) in any schedule
    assert [e.status(f) for f in range(F)] == [0] * F, env
    e.close()
    return out


@pytest.mark.parametrize("F", [1, 4], ids=["1filter", "4filters"])
def test_pipelined_replay_sync_modes(monkeypatch, F):
    """Three schedules of the same replay, run without per-message synchronisation so chunks
    really overlap: the default device-epoch pipeline (one persistent chain launch walking every
    chunk beside the bulk stream), the event-synchronised two streams (EKF_DEVSYNC=0) and the
    single-stream order launch the same per-chunk arithmetic on the same data: bit-identical, and
    against the oracle. LDS is poisoned with NaNs first, so a chain that reads LDS it never wrote
    fails here every time."""
    sc = synth.synthetic(256, 30)
    pyekf.poison_lds()
    dev = _pipelined_final(sc, monkeypatch, {"EKF_DEVSYNC": "1"}, F=F)
    evt = _pipelined_final(sc, monkeypatch, {"EKF_DEVSYNC": "0"}, F=F)
    ser = _pipelined_final(sc, monkeypatch, {"EKF_SERIAL": "1"}, F=F)
    for (xd, Sd, cd), (xe, Se, ce), (xs, Ss, cs) in zip(dev, evt, ser):
        assert cd == ce == cs
        np.testing.assert_array_equal(xd, xs)
        np.testing.assert_array_equal(Sd, Ss)
        np.testing.assert_array_equal(xe, xs)
        np.testing.assert_array_equal(Se, Ss)
    o = orc.run_scenario(sc, False)
    x, S, _ = dev[0]
    assert np.abs(x - o["state"]).max() < 1e-7
    assert np.abs(S - o["sigma"]).max() < 1e-7


@pytest.mark.parametrize("F", [1, 4], ids=["1filter", "4filters"])
def test_pipelined_replay_sync_modes_multichunk(monkeypatch, F):
    """Messages of up to 24 markers span two chunks (the second chunk of a message rebuilds from
    the first, kLook within the message): the three schedules bit-identical (LDS poisoned)."""
    sc = synth.synthetic(96, 14, max_markers=24)
    assert sc.count.max() > 16  # some messages span two chunks
    pyekf.poison_lds()
    dev = _pipelined_final(sc, monkeypatch, {"EKF_DEVSYNC": "1"}, F=F)
    evt = _pipelined_final(sc, monkeypatch, {"EKF_DEVSYNC": "0"}, F=F)
    ser = _pipelined_final(sc, monkeypatch, {"EKF_SERIAL": "1"}, F=F)
    for (xd, Sd, cd), (xe, Se, ce), (xs, Ss, cs) in zip(dev, evt, ser):
        assert cd == ce == cs
        np.testing.assert_array_equal(xd, xs)
        np.testing.assert_array_equal(Sd, Ss)
        np.testing.assert_array_equal(xe, xs)
        np.testing.assert_array_equal(Se, Ss)


def test_pipelined_replay_fp32_n1024_sync_modes(monkeypatch):
    """Config 3 size, fp32 Σ, 24 messages pipelined: the device-epoch schedule (EKF_DEVSYNC=1,
    LDS poisoned first) and the single stream: bit-identical."""
    N, warm, T = 1024, 40, 24
    sc = synth.synthetic(N, warm + T)
    odom = pyekf.odometry(sc)
    e64 = pyekf.EKF(n_landmarks=N)
    e64.replay(sc.count[:warm, None], sc.rel[:warm, None], odom[:warm, None],
               ids=sc.ids[:warm, None], actions=sc.actions[:warm, None])
    x0, S0, c0 = e64.state()
    tmo0 = e64.map_odom()
    e64.close()
    res = []
    for env in ({"EKF_DEVSYNC": "1"}, {"EKF_SERIAL": "1"}):
        for k in ("EKF_SERIAL", "EKF_CU_SPLIT", "EKF_DEVSYNC"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        pyekf.poison_lds()
        e = pyekf.EKF(n_landmarks=N, dtype=pyekf.EKF_F32)
        e.set_state(x0, S0, tmo=tmo0, counter=c0)
        sl = slice(warm, warm + T)
        e.replay(sc.count[sl, None], sc.rel[sl, None], odom[sl, None], ids=sc.ids[sl, None],
                 actions=sc.actions[sl, None])
        res.append(e.state())
        assert e.status() == 0, env
        e.close()
    np.testing.assert_array_equal(res[0][0], res[1][0])
    np.testing.assert_array_equal(res[0][1], res[1][1])
    assert np.all(np.isfinite(res[0][1]))


@pytest.mark.parametrize("F,devsync", [(24, "0"), (24, "1"), (40, "0")],
                         ids=["24filters_xcdgrid", "24filters_devsync", "40filters_nocusplit"])
def test_many_filters_match_small_batch(F, devsync, monkeypatch):
    """≥16 filters take the XCD-aware Σ-pass grid, > 32 filters streams without a CU split;
    filter f replays scenario f % 8, and must equal the same scenario in an 8-filter handle bit for
    bit (the arithmetic per filter does not depend on the batch). devsync: both handles run the
    device-epoch schedule (EKF_DEVSYNC=1, LDS poisoned first)."""
    for k in ("EKF_SERIAL", "EKF_CU_SPLIT", "EKF_DEVSYNC"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("EKF_DEVSYNC", devsync)
    if devsync == "1":
        pyekf.poison_lds()
    N, T = 64, 12
    scs = [synth.synthetic(N, T, seed=100 + k) for k in range(8)]
    odo = [pyekf.odometry(s) for s in scs]
    M = max(s.ids.shape[1] for s in scs)

    def run(nf):
        cnt = np.zeros((T, nf), np.int32)
        ids = np.full((T, nf, M), -1, np.int32)
        act = np.zeros((T, nf, M), np.int32)
        rel = np.zeros((T, nf, M, 2))
        od = np.zeros((T, nf, 3))
        for f in range(nf):
            s = scs[f % 8]
            k = s.ids.shape[1]
            cnt[:, f] = s.count
            ids[:, f, :k] = s.ids
            act[:, f, :k] = s.actions
            rel[:, f, :k] = s.rel
            od[:, f] = odo[f % 8]
        e = pyekf.EKF(n_landmarks=N, n_filters=nf)
        e.replay(cnt, rel, od, ids=ids, actions=act)
        out = [e.state(f) for f in range(nf)]
        assert [e.status(f) for f in range(nf)] == [0] * nf
        e.close()
        return out

    big = run(F)
    small = run(8)
    for f in range(F):
        xs, Ss, cs = small[f % 8]
        xb, Sb, cb = big[f]
        assert cs == cb
        np.testing.assert_array_equal(xs, xb)
        np.testing.assert_array_equal(Ss, Sb)
        # the symmetric fp64 Σ pass (wide tiles here, narrow in the 8-filter handle) leaves Σ
        # exactly symmetric
        np.testing.assert_array_equal(Sb, Sb.T)


@pytest.mark.parametrize("name,dtype,N", [("basic_world_known", pyekf.EKF_F64, 12000),
                                          ("basic_world_assoc", pyekf.EKF_F64, 12000)],
                         ids=["known_n12000_fp64", "assoc_n12000_fp64"])
def test_maximum_size_prefix_equals_golden(name, dtype, N):
    """Size-independent property at a size whose Σ (n = 24 003, 4.6 GB per copy) is beyond 32-bit
    byte offsets: unused landmark slots never touch the used part of the state (their cross
    covariances stay exactly 0), so the N=50 golden fixture is a prefix of the N=12000 run. Same
    tolerances as at N=50; the slots past the fixture's stay exactly 0."""
    import dataclasses
    sc, g = load_golden(name)
    s = pyekf.Slam(n_landmarks=N, source=pyekf.SOURCE_ASSOC if bool(g["assoc"]) else
                   pyekf.SOURCE_SIM, dtype=dtype, track=sc.track, radius=sc.radius)
    rc, poses, tmo = s.replay(dataclasses.replace(sc, n_landmarks=N))
    x, _, cnt = s.filter_state(sigma=False)
    s.close()
    assert rc == pyekf.EKF_OK
    assert np.abs(poses - g["poses"]).max() < POSE_TOL
    assert np.abs(tmo - g["tmo"]).max() < POSE_TOL
    n0 = g["state"].shape[0]
    assert np.abs(x[:n0] - g["state"]).max() < POSE_TOL
    assert not np.any(x[n0:])
    assert cnt == int(g["counter"])


@pytest.mark.parametrize("resident", ["1", "0"], ids=["resident", "pipeline"])
def test_empty_and_all_delete_messages(monkeypatch, resident):
    """ekf_replay with counts[t][f] == 0 (that filter gets no message: nothing changes, as the
    oracle's fake_sensor_cb rejects an empty array — the reference throws at markers.at(0),
    slam.cpp:281) and with messages whose markers are all DELETE (predict + posterior only,
    slam.cpp:205). Four filters replay the same drive with different holes; each equals the oracle
    fed the same messages."""
    monkeypatch.setenv("EKF_RESIDENT", resident)
    sc = synth.basic_world(24, n_delete=1)
    odom = pyekf.odometry(sc)
    T, M, F = sc.n_messages, sc.ids.shape[1], 4
    cnt = np.repeat(sc.count[:, None], F, 1).astype(np.int32)
    ids = np.repeat(sc.ids[:, None], F, 1)
    act = np.repeat(sc.actions[:, None], F, 1).copy()
    rel = np.repeat(sc.rel[:, None], F, 1)
    cnt[5::4, 1] = 0                 # filter 1: every 4th message missing
    cnt[3:6, 2] = 0                  # filter 2: a run of missing messages
    act[7::3, 3] = synth.DELETE      # filter 3: every 3rd message all DELETE
    e = pyekf.EKF(n_landmarks=sc.n_landmarks, n_filters=F)
    poses = e.replay(cnt, rel, np.repeat(odom[:, None], F, 1), ids=ids, actions=act, poses=True)
    for f in range(F):
        ref = orc.OracleEKF(n_landmarks=sc.n_landmarks)
        for t in range(T):
            ref.set_odom(odom[t])
            c = int(cnt[t, f])
            ref.fake_sensor_cb(ids[t, f, :c], act[t, f, :c], rel[t, f, :c])
            assert np.abs(poses[t, f] - ref.get(sigma=False)[0][:3]).max() < POSE_TOL, (f, t)
        x, S, _ = e.state(f)
        xr, Sr, _, _ = ref.get()
        assert e.status(f) == 0
        assert np.abs(x - xr).max() < POSE_TOL, f
        assert np.abs(S - Sr).max() < SIGMA_TOL, f
    e.close()


@pytest.mark.gpu
def test_serial_gather_matches_small_batch(monkeypatch):
    """EKF_SERIAL_GATHER=1 (opt-in): the chains of a stream-ordered handle (> 32
    filters: one stream) gather their complete Σ_in instead of rebuilding it from the chunk before
    (kLook). Filter f replays scenario f % 8 and equals the same scenario in an 8-filter handle
    (events, kLook) to rounding — the gather and the rebuild round differently — and Σ stays
    exactly symmetric."""
    for k in ("EKF_SERIAL", "EKF_CU_SPLIT", "EKF_DEVSYNC", "EKF_SERIAL_GATHER"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("EKF_DEVSYNC", "0")
    N, T = 64, 12
    scs = [synth.synthetic(N, T, seed=100 + k) for k in range(8)]
    odo = [pyekf.odometry(s) for s in scs]
    M = max(s.ids.shape[1] for s in scs)

    def run(nf):
        cnt = np.zeros((T, nf), np.int32)
        ids = np.full((T, nf, M), -1, np.int32)
        act = np.zeros((T, nf, M), np.int32)
        rel = np.zeros((T, nf, M, 2))
        od = np.zeros((T, nf, 3))
        for f in range(nf):
            s = scs[f % 8]
            k = s.ids.shape[1]
            cnt[:, f] = s.count
            ids[:, f, :k] = s.ids
            act[:, f, :k] = s.actions
            rel[:, f, :k] = s.rel
            od[:, f] = odo[f % 8]
        e = pyekf.EKF(n_landmarks=N, n_filters=nf)
        e.replay(cnt, rel, od, ids=ids, actions=act)
        out = [e.state(f) for f in range(nf)]
        assert [e.status(f) for f in range(nf)] == [0] * nf
        e.close()
        return out

    small = run(8)
    monkeypatch.setenv("EKF_SERIAL_GATHER", "1")
    big = run(40)
    for f in range(40):
        xs, Ss, cs = small[f % 8]
        xb, Sb, cb = big[f]
        assert cs == cb
        np.testing.assert_allclose(xb, xs, rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(Sb, Ss, rtol=1e-12, atol=1e-9)
        np.testing.assert_array_equal(Sb, Sb.T)
