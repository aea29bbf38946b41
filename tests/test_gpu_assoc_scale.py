"""Unknown association (Slam::sensor_cb, nuslam/src/slam.cpp:318-530) at the shape bench.py times:
N = 1024 slots, G = 16 workgroups of k_assoc_msg per filter, ≈ 970 mapped landmarks and unmapped
ones in view of the drive (new-landmark commits at counter ≥ 960), through the C-ABI, against the
C oracle. Both exchange transports (XCD-local, the default here, and agent-coherent, EKF_AM_XCD=0),
every decision equal to the oracle's, the state within the tolerances of tests/test_gpu_scale.py
(fp64: poses 1e-8, state 5e-8, Σ 1e-7; fp32 Σ: poses 1e-6, state 1e-5, Σ 5e-5).

Also: more filters than the GPU holds workgroups at once (64 filters × 16 = 1 024 workgroups:
a filter's workgroups spin on each other, so the host launches them in groups the CUs hold at
once, ekf_api.cpp assoc_msg_group), the one-marker-per-launch route when a filter's workgroups
cannot all be resident (EKF_CU_SPLIT leaves the bulk stream one CU per XCD), the single-stream
schedule (EKF_SERIAL=1: the association runs on the main stream's narrower CU mask), and a forced
exchange timeout, which must reach the caller as EKF_E_TIMEOUT / EKF_FLAG_TIMEOUT."""
import json
import os

import numpy as np
import pytest

import orc
import pyekf
from pyekf import synth

pytestmark = pytest.mark.gpu

POSE_TOL, STATE_TOL, SIGMA_TOL = 1e-8, 5e-8, 1e-7
F32_POSE_TOL, F32_STATE_TOL, F32_SIGMA_TOL = 1e-6, 1e-5, 5e-5
ENV = ("EKF_SERIAL", "EKF_CU_SPLIT", "EKF_DEVSYNC", "EKF_AM_XCD", "EKF_AM_DROP",
       "EKF_AM_SPIN_LOG2", "EKF_ASSOC_MSG")
ERRORS = {}


@pytest.fixture(scope="module", autouse=True)
def _record_errors():
    yield
    out = os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "gpurun_out")
    os.makedirs(out, exist_ok=True)
    with open(os.path.join(out, "assoc_scale_errors.json"), "w") as fh:
        json.dump(ERRORS, fh, indent=1)


def _env(monkeypatch, **kv):
    for k in ENV:
        monkeypatch.delenv(k, raising=False)
    for k, v in kv.items():
        monkeypatch.setenv(k, v)


def _open_map(N, n_map, T, seed=20240317):
    """n_map landmarks surveyed with known ids into N slots; half of the landmarks the T circle
    messages see are relabelled to the top of the map and forgotten (their slots back at the prior,
    slam.cpp:127-132), so the drive meets mapped and unmapped landmarks. counter = mapped count."""
    sc = synth.populated(N, T, seed=seed, n_map=n_map, shuffle=True)
    w = sc.n_warm
    live = np.arange(sc.ids.shape[1])[None, :] < sc.count[w:, None]
    seen = np.unique(sc.ids[w:][live])
    unmapped = seen[::2]
    mapped = np.setdiff1d(np.arange(n_map), unmapped)
    perm = np.arange(N, dtype=np.int32)
    perm[mapped] = np.arange(mapped.size)
    perm[unmapped] = mapped.size + np.arange(unmapped.size)
    ids = np.where(sc.ids >= 0, perm[np.maximum(sc.ids, 0)], -1).astype(np.int32)
    sc = synth.Scenario(sc.n_landmarks, sc.landmarks, sc.wheel, ids, sc.actions, sc.rel,
                        sc.count, sc.truth, sc.track, sc.radius, sc.n_warm)
    counter = int(mapped.size)
    odom = pyekf.odometry(sc)
    e = pyekf.EKF(n_landmarks=N)
    e.replay(sc.count[:w, None], sc.rel[:w, None], odom[:w, None], ids=sc.ids[:w, None],
             actions=sc.actions[:w, None])
    x, S, _ = e.state()
    tmo = e.map_odom()
    assert e.status() == 0
    e.close()
    k = 3 + 2 * counter
    x[k:] = 0.0
    S[k:, :] = 0.0
    S[:, k:] = 0.0
    S[np.arange(k, S.shape[0]), np.arange(k, S.shape[0])] = 10e6
    return sc, odom, (x, S, tmo, counter)


def _oracle_run(N, sc, odom, ws, gate=2.0, joseph=False):
    x, S, tmo, cnt = ws
    ref = orc.OracleEKF(n_landmarks=N, mah_gate=gate, joseph=joseph)
    ref.set(x, S, tmo, x[:3], cnt)
    out = []
    for t in range(sc.n_warm, sc.n_messages):
        ref.set_odom(odom[t])
        out.append(ref.sensor_cb_dmin(sc.rel[t, :int(sc.count[t])]) + (ref.get(sigma=False)[0][:3],))
    return ref, out


def _gpu_sensor(N, sc, odom, ws, ref_out, dtype=pyekf.EKF_F64, gate=2.0, route=None,
                joseph=False):
    """ekf_sensor message by message (decisions read back), every decision against the oracle's."""
    x, S, tmo, cnt = ws
    e = pyekf.EKF(n_landmarks=N, dtype=dtype, mah_gate=gate)
    if joseph:
        assert e.set_joseph(True) == pyekf.EKF_OK
    if route is not None:
        assert e.assoc_route == route
    e.set_state(x, S, tmo=tmo, counter=cnt)
    perr, n_new, n_old = 0.0, 0, 0
    for i, t in enumerate(range(sc.n_warm, sc.n_messages)):
        e.set_odom(odom[t])
        rc, j, nw = e.sensor(sc.rel[t, :int(sc.count[t])])
        rr, jr, nr, _, pr = ref_out[i]
        assert rc == rr == 0
        assert np.array_equal(j, jr) and np.array_equal(nw, nr), (t, j, jr, nw, nr)
        n_new += int(nr.sum())
        n_old += int(nr.size - nr.sum())
        perr = max(perr, float(np.abs(e.pose() - pr).max()))
    xg, Sg, cg = e.state()
    assert e.status() == 0
    e.close()
    return perr, xg, Sg, cg, n_new, n_old


@pytest.fixture(scope="module")
def map1024():
    """bench.py's n1024_*_assoc shape: 1 024 slots, 980 landmarks placed, ≈ 970 of them mapped."""
    sc, odom, ws = _open_map(1024, 980, 10)
    assert 960 <= ws[3] < 1024 - 8
    ref, out = _oracle_run(1024, sc, odom, ws)
    return sc, odom, ws, ref.get(), out


@pytest.mark.parametrize("xcd", ["1", "0"], ids=["xcd_local", "agent"])
@pytest.mark.parametrize("dtype", [pyekf.EKF_F64, pyekf.EKF_F32], ids=["f64", "f32"])
def test_assoc_n1024_decisions(map1024, xcd, dtype, monkeypatch):
    """Every decision of 10 messages × 16 markers at N = 1024 (G = 16) equal to the oracle's, both
    branches of slam.cpp:421-440 taken, in both exchange transports; poses, state and Σ within
    the fp64 / fp32 tolerances."""
    _env(monkeypatch, EKF_AM_XCD=xcd)
    sc, odom, ws, (xr, Sr, _, cr), out = map1024
    route = pyekf.EKF_ASSOC_CHUNK_XCD if xcd == "1" else pyekf.EKF_ASSOC_CHUNK
    perr, xg, Sg, cg, n_new, n_old = _gpu_sensor(1024, sc, odom, ws, out, dtype, route=route)
    key = f"n1024_{'f64' if dtype == pyekf.EKF_F64 else 'f32'}_{'xcd' if xcd == '1' else 'agent'}"
    ERRORS[key] = {"new": n_new, "associated": n_old, "counter": int(cg), "pose": perr,
                   "state": float(np.abs(xg - xr).max()), "sigma": float(np.abs(Sg - Sr).max())}
    assert n_new > 0 and n_old > 0
    assert cg == cr > ws[3] >= 960
    pt, st, sg = ((POSE_TOL, STATE_TOL, SIGMA_TOL) if dtype == pyekf.EKF_F64 else
                  (F32_POSE_TOL, F32_STATE_TOL, F32_SIGMA_TOL))
    assert perr < pt
    assert np.abs(xg - xr).max() < st
    assert np.abs(Sg - Sr).max() < sg


@pytest.fixture(scope="module")
def map1024_joseph(map1024):
    """The same drive through the oracle's Joseph form (ekf_oracle.c orc_ekf_set_joseph)."""
    sc, odom, ws, _, _ = map1024
    ref, out = _oracle_run(1024, sc, odom, ws, joseph=True)
    return sc, odom, ws, ref.get(), out


@pytest.mark.parametrize("route", ["xcd_local", "agent", "marker"])
@pytest.mark.parametrize("dtype", [pyekf.EKF_F64, pyekf.EKF_F32], ids=["f64", "f32"])
def test_assoc_n1024_joseph(map1024_joseph, route, dtype, monkeypatch):
    """Unknown association in the Joseph form (ekf_set_joseph; slam.cpp:485-486's update as
    (I − KH)Σ(I − KH)ᵀ + KRKᵀ): whole chunks through k_assoc_msg<T, true> — every step's V_c·K_cᵀ
    on the lanes' blocks, in the crosses' history sums and as the chunk's Kcat / Mcat rows 2 + 2m..
    (one rank-(2 + 4m) Σ pass per chunk) — in both exchange transports, and the one-marker route
    (EKF_ASSOC_MSG=0). Every decision equal to the oracle's Joseph sensor_cb, poses, state and Σ
    within the fp64 / fp32 tolerances above — the fp32 one-marker route within 5e-6 / 1e-4 / 5e-5:
    it rounds Σ to fp32 once per marker (160 Σ passes against the chunk route's 10; measured
    2.3e-6 / 3.5e-5 / 8.1e-6)."""
    env = {"xcd_local": {"EKF_AM_XCD": "1"}, "agent": {"EKF_AM_XCD": "0"},
           "marker": {"EKF_ASSOC_MSG": "0"}}[route]
    _env(monkeypatch, **env)
    sc, odom, ws, (xr, Sr, _, cr), out = map1024_joseph
    want = {"xcd_local": pyekf.EKF_ASSOC_CHUNK_XCD, "agent": pyekf.EKF_ASSOC_CHUNK,
            "marker": pyekf.EKF_ASSOC_MARKER}[route]
    perr, xg, Sg, cg, n_new, n_old = _gpu_sensor(1024, sc, odom, ws, out, dtype, joseph=True)
    key = f"n1024_joseph_{'f64' if dtype == pyekf.EKF_F64 else 'f32'}_{route}"
    ERRORS[key] = {"new": n_new, "associated": n_old, "counter": int(cg), "pose": perr,
                   "state": float(np.abs(xg - xr).max()), "sigma": float(np.abs(Sg - Sr).max())}
    e = pyekf.EKF(n_landmarks=1024, dtype=dtype)
    assert e.set_joseph(True) == pyekf.EKF_OK
    assert e.assoc_route == want
    e.close()
    assert n_new > 0 and n_old > 0
    assert cg == cr > ws[3] >= 960
    pt, st, sg = ((POSE_TOL, STATE_TOL, SIGMA_TOL) if dtype == pyekf.EKF_F64 else
                  (F32_POSE_TOL, F32_STATE_TOL, F32_SIGMA_TOL) if route != "marker" else
                  (5e-6, 1e-4, 5e-5))
    assert perr < pt
    assert np.abs(xg - xr).max() < st
    assert np.abs(Sg - Sr).max() < sg


@pytest.mark.parametrize("dtype", [pyekf.EKF_F64, pyekf.EKF_F32], ids=["f64", "f32"])
def test_assoc_n1024_replay_equals_sensor(map1024, dtype, monkeypatch):
    """The batched path bench.py times (ekf_replay with assoc = 1: every message planned ahead, one
    upload) against ekf_sensor message by message from the same state: bit-identical state, and
    both transports bit-identical to each other."""
    sc, odom, ws, _, _ = map1024
    w = sc.n_warm
    x, S, tmo, cnt = ws
    res = []
    for xcd in ("1", "0"):
        _env(monkeypatch, EKF_AM_XCD=xcd)
        e = pyekf.EKF(n_landmarks=1024, dtype=dtype)
        e.set_state(x, S, tmo=tmo, counter=cnt)
        sl = slice(w, sc.n_messages)
        e.replay(sc.count[sl, None], sc.rel[sl, None], odom[sl, None], ids=None,
                 actions=sc.actions[sl, None], assoc=True)
        res.append(e.state())
        assert e.status() == 0
        e.close()
        e = pyekf.EKF(n_landmarks=1024, dtype=dtype)
        e.set_state(x, S, tmo=tmo, counter=cnt)
        for t in range(w, sc.n_messages):
            e.set_odom(odom[t])
            assert e.sensor(sc.rel[t, :int(sc.count[t])], decisions=False)[0] == 0
        res.append(e.state())
        e.close()
    for xg, Sg, cg in res[1:]:
        assert cg == res[0][2]
        np.testing.assert_array_equal(xg, res[0][0])
        np.testing.assert_array_equal(Sg, res[0][1])


@pytest.mark.parametrize("xcd", ["1", "0"], ids=["xcd_local", "agent"])
def test_assoc_n1024_near_the_gate(map1024, xcd, monkeypatch):
    """A gate 3e-4 below one marker's smallest existing distance (slam.cpp:401-408: the new slot
    wins only over a strictly larger minimum), N = 1024, both transports: every decision, the
    near-gate one included, equal to the oracle's."""
    _env(monkeypatch, EKF_AM_XCD=xcd)
    sc, odom, ws, _, out = map1024
    d = np.concatenate([o[3] for o in out])
    i0 = int(np.argmax((d > 0.5) & (d < 2.0)))
    assert 0.5 < d[i0] < 2.0
    gate = float(d[i0]) - 3e-4
    ref, out2 = _oracle_run(1024, sc, odom, ws, gate)
    d2 = np.concatenate([o[3] for o in out2])
    assert i0 in np.flatnonzero(np.abs(d2 - gate) < 1e-3)
    perr, xg, Sg, cg, n_new, n_old = _gpu_sensor(1024, sc, odom, ws, out2, gate=gate)
    xr, Sr, _, cr = ref.get()
    ERRORS["n1024_near_gate_" + ("xcd" if xcd == "1" else "agent")] = {
        "gate": gate, "new": n_new, "associated": n_old, "pose": perr,
        "state": float(np.abs(xg - xr).max())}
    assert cg == cr
    assert perr < POSE_TOL
    assert np.abs(xg - xr).max() < STATE_TOL
    assert np.abs(Sg - Sr).max() < SIGMA_TOL


@pytest.mark.parametrize("joseph", [False, True], ids=["simple", "joseph"])
@pytest.mark.parametrize("xcd", ["1", "0"], ids=["xcd_local", "agent"])
def test_assoc_more_filters_than_resident_workgroups(map1024, xcd, joseph, monkeypatch):
    """64 filters at N = 1024 in one handle: 1 024 workgroups of k_assoc_msg per chunk, more than
    the bulk stream's CUs hold at once, so the host splits the chunk into launches of co-resident
    filters (a filter's workgroups spin on each other; the Joseph kernel's larger LDS makes its
    groups smaller, `am_group_j`). Every filter ends bit-identical to a one-filter handle, whose
    state equals the oracle's (fp32 Σ tolerances; the oracle's Joseph mode for the Joseph form)."""
    sc, odom, ws, (xr, Sr, _, cr), _ = map1024
    w, T, F = sc.n_warm, 4, 64
    x, S, tmo, cnt = ws
    sl = slice(w, w + T)
    rep = lambda a: np.repeat(a[sl, None], F, axis=1)  # noqa: E731
    _env(monkeypatch, EKF_AM_XCD=xcd)
    e = pyekf.EKF(n_landmarks=1024, n_filters=F, dtype=pyekf.EKF_F32)
    if joseph:
        assert e.set_joseph(True) == pyekf.EKF_OK
        assert e.assoc_route != pyekf.EKF_ASSOC_MARKER
    for f in range(F):
        e.set_state(x, S, tmo=tmo, counter=cnt, f=f)
    e.replay(rep(sc.count), rep(sc.rel), rep(odom), ids=None, actions=rep(sc.actions), assoc=True)
    e.sync()
    assert [e.status(f) for f in range(F)] == [0] * F
    got = [e.state(f) for f in range(0, F, 9)] + [e.state(F - 1)]
    e.close()
    one = pyekf.EKF(n_landmarks=1024, dtype=pyekf.EKF_F32)
    if joseph:
        assert one.set_joseph(True) == pyekf.EKF_OK
    one.set_state(x, S, tmo=tmo, counter=cnt)
    one.replay(sc.count[sl, None], sc.rel[sl, None], odom[sl, None], ids=None,
               actions=sc.actions[sl, None], assoc=True)
    x1, S1, c1 = one.state()
    one.close()
    for xg, Sg, cg in got:
        assert cg == c1
        np.testing.assert_array_equal(xg, x1)
        np.testing.assert_array_equal(Sg, S1)
    ref = orc.OracleEKF(n_landmarks=1024, joseph=joseph)
    ref.set(x, S, tmo, x[:3], cnt)
    for t in range(w, w + T):
        ref.set_odom(odom[t])
        ref.sensor_cb(sc.rel[t, :int(sc.count[t])])
    xo, So, _, co = ref.get()
    assert c1 == co
    assert np.abs(x1 - xo).max() < F32_STATE_TOL
    assert np.abs(S1 - So).max() < F32_SIGMA_TOL


def test_assoc_n1024_serial_schedule(map1024, monkeypatch):
    """EKF_SERIAL=1 on a one-filter handle: k_assoc_msg runs on the main stream, whose CU mask holds
    4 CUs per XCD (8 resident workgroups per XCD < G = 16), so the route comes from those CUs —
    the agent placement, G / 8 workgroups per XCD — not from the bulk stream's (which would pick
    the XCD-local exchange and spin into its timeout). Every decision equal to the oracle's, fp64
    tolerances, no timeout."""
    _env(monkeypatch, EKF_SERIAL="1")
    sc, odom, ws, (xr, Sr, _, cr), out = map1024
    perr, xg, Sg, cg, n_new, n_old = _gpu_sensor(1024, sc, odom, ws, out,
                                                 route=pyekf.EKF_ASSOC_CHUNK)
    ERRORS["n1024_serial"] = {"new": n_new, "associated": n_old, "pose": perr,
                              "state": float(np.abs(xg - xr).max())}
    assert n_new > 0 and n_old > 0 and cg == cr
    assert perr < POSE_TOL
    assert np.abs(xg - xr).max() < STATE_TOL
    assert np.abs(Sg - Sr).max() < SIGMA_TOL


@pytest.fixture(scope="module")
def map2048():
    """2 048 slots (G = 32 workgroups per filter), 300 landmarks placed."""
    sc, odom, ws = _open_map(2048, 300, 4)
    ref, out = _oracle_run(2048, sc, odom, ws)
    return sc, odom, ws, ref.get(), out


@pytest.mark.parametrize("split,route", [(None, pyekf.EKF_ASSOC_CHUNK_XCD),
                                         ("31", pyekf.EKF_ASSOC_MARKER)],
                         ids=["chunks", "one_cu_per_xcd_marker_route"])
def test_assoc_route_by_residency(map2048, split, route, monkeypatch):
    """N = 2048: by default a filter's 32 workgroups fit one XCD's bulk CUs (XCD-local chunks); with
    EKF_CU_SPLIT=31 the bulk stream has one CU per XCD (16 resident workgroups < 32), so the
    handle routes every marker through its own launch (EKF_ASSOC_MARKER) instead of spinning into
    the exchange timeout. Both routes: every decision equal to the oracle's, fp64 tolerances."""
    if split is None:
        _env(monkeypatch)
    else:
        _env(monkeypatch, EKF_CU_SPLIT=split)
    sc, odom, ws, (xr, Sr, _, cr), out = map2048
    perr, xg, Sg, cg, n_new, n_old = _gpu_sensor(2048, sc, odom, ws, out, route=route)
    ERRORS["n2048_route_" + str(route)] = {"new": n_new, "associated": n_old, "pose": perr,
                                           "state": float(np.abs(xg - xr).max())}
    assert n_new > 0 and n_old > 0 and cg == cr
    assert perr < POSE_TOL
    assert np.abs(xg - xr).max() < STATE_TOL
    assert np.abs(Sg - Sr).max() < SIGMA_TOL


def test_assoc_exchange_timeout_is_reported(map1024, monkeypatch):
    """Fault injection (EKF_AM_DROP=1: the last workgroup never publishes its first exchange; polls
    bounded at 2^10): every workgroup's poll times out. The caller sees EKF_E_TIMEOUT from
    ekf_sensor, the filter's status carries EKF_FLAG_TIMEOUT, the report is made once, and a fresh
    handle afterwards runs clean."""
    sc, odom, ws, _, _ = map1024
    w = sc.n_warm
    x, S, tmo, cnt = ws
    _env(monkeypatch, EKF_AM_DROP="1", EKF_AM_SPIN_LOG2="10")
    e = pyekf.EKF(n_landmarks=1024)
    e.set_state(x, S, tmo=tmo, counter=cnt)
    e.set_odom(odom[w])
    rc, _, _ = e.sensor(sc.rel[w, :int(sc.count[w])])
    assert rc == pyekf.EKF_E_TIMEOUT
    assert e.status() & pyekf.EKF_FLAG_TIMEOUT
    e.sync()  # reported once
    e.close()
    _env(monkeypatch)
    e = pyekf.EKF(n_landmarks=1024)
    e.set_state(x, S, tmo=tmo, counter=cnt)
    e.set_odom(odom[w])
    assert e.sensor(sc.rel[w, :int(sc.count[w])])[0] == 0
    e.sync()
    assert e.status() == 0
    e.close()
