"""ekf_replay_device (include/ekf.h): a known-id replay whose inputs already live on the GPU, its
descriptors planned by k_plan_replay (plan_kernels.hip). Parity: the same replay through the
host planner (ekf_replay, plan_known in ekf_api.cpp) — the reference's fake_sensor_cb
(nuslam/src/slam.cpp:180-316) message by message — and the CPU oracle."""
import numpy as np
import pytest

import pyekf
from pyekf import synth
import orc

pytestmark = pytest.mark.gpu

# fp64, against the host planner. The two differ only in the bearing's atan2 (ocml on the device,
# glibc on the host, ≤ 1 ulp apart); a first sighting's 1e7 − (1e7 − δ) (the reference's prior,
# slam.cpp:130) amplifies that to ≈ 1e-11 on the new landmark's Σ entries, ≈ 2e-9 at most seen.
STATE_TOL = 1e-9
SIGMA_TOL = 1e-8


def _inputs(scs, F, T0, T1, holes=False):
    """counts/ids/actions/rel/odom [T][F](...) for messages [T0, T1) of scenario f % len(scs)."""
    T = T1 - T0
    M = max(s.ids.shape[1] for s in scs)
    cnt = np.zeros((T, F), np.int32)
    ids = np.zeros((T, F, M), np.int32)
    act = np.zeros((T, F, M), np.int32)
    rel = np.zeros((T, F, M, 2))
    od = np.zeros((T, F, 3))
    for f in range(F):
        s = scs[f % len(scs)]
        k = s.ids.shape[1]
        cnt[:, f] = s.count[T0:T1]
        ids[:, f, :k] = s.ids[T0:T1]
        act[:, f, :k] = s.actions[T0:T1]
        rel[:, f, :k] = s.rel[T0:T1]
        od[:, f] = pyekf.odometry(s)[T0:T1]
    if holes and F > 1:
        cnt[1::3, 1] = 0                   # filter 1: every 3rd message missing
        act[2::4, F - 1] = synth.DELETE    # the last filter: every 4th message all DELETE
    return cnt, ids, act, rel, od


def _to_gpu(arrs):
    import torch
    cnt, ids, act, rel, od = arrs
    return (torch.from_numpy(cnt).cuda(), torch.from_numpy(ids).cuda(),
            torch.from_numpy(act).cuda(), torch.from_numpy(rel).cuda(), torch.from_numpy(od).cuda())


def _run(scs, N, F, spans, kinds, dtype=pyekf.EKF_F64, warm=None, holes=False, joseph=False):
    """Replay the spans [(T0, T1), ...] in order, span i through kinds[i] ('host' / 'device')."""
    e = pyekf.EKF(n_landmarks=N, n_filters=F, dtype=dtype)
    if joseph:
        assert e.set_joseph(True) == pyekf.EKF_OK
    if warm is not None:
        for f in range(F):
            x, S, tmo, c = warm
            e.set_state(x, S, tmo=tmo, counter=c, f=f)
    keep = []
    # the whole drive's inputs (holes at absolute message indices), cut into the spans
    full = _inputs(scs, F, spans[0][0], spans[-1][1], holes)
    for (t0, t1), kind in zip(spans, kinds):
        cnt, ids, act, rel, od = (np.ascontiguousarray(a[t0 - spans[0][0]:t1 - spans[0][0]])
                                  for a in full)
        if kind == "device":
            g = _to_gpu((cnt, ids, act, rel, od))
            keep.append(g)
            e.replay_device(g[0], g[3], g[4], g[1], g[2])
        else:
            e.replay(cnt, rel, od, ids=ids, actions=act)
    out = [e.state(f) for f in range(F)]
    st = [e.status(f) for f in range(F)]
    poses = np.stack([e.pose(f) for f in range(F)])
    e.close()
    return out, st, poses


def _close(a, b, tol, stol=SIGMA_TOL):
    for (xa, Sa, ca), (xb, Sb, cb) in zip(a, b):
        assert ca == cb
        assert np.abs(xa - xb).max() <= tol
        assert np.abs(Sa - Sb).max() <= stol


@pytest.mark.parametrize("F,env", [(1, {}), (4, {}), (1, {"EKF_DEVSYNC": "0"}),
                                   (4, {"EKF_SERIAL": "1"}), (3, {"EKF_STAGE": "0"})],
                         ids=["1filter", "4filters", "1filter_events", "4filters_serial",
                              "3filters_nostage"])
def test_device_replay_equals_host_replay(monkeypatch, F, env):
    """fp64 N = 96 (the HBM pipeline), 30 messages, every schedule: the device-planned replay ends
    where the host-planned one does, holes (empty and all-DELETE messages) included."""
    for k in ("EKF_SERIAL", "EKF_CU_SPLIT", "EKF_DEVSYNC", "EKF_STAGE"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    pyekf.poison_lds()
    scs = [synth.synthetic(96, 30, seed=7 + k) for k in range(3)]
    host, sh, ph = _run(scs, 96, F, [(0, 30)], ["host"], holes=True)
    dev, sd, pd = _run(scs, 96, F, [(0, 30)], ["device"], holes=True)
    assert sh == sd == [0] * F
    _close(host, dev, STATE_TOL)
    assert np.abs(ph - pd).max() <= STATE_TOL


def test_device_replay_chains_with_host_calls():
    """Host, device, device, host spans of one drive (the planning state goes down to the GPU,
    stays there between the two device calls, comes back for the host call) against the whole drive
    on the host, and filter 0 against the CPU oracle."""
    scs = [synth.synthetic(80, 40, seed=21 + k) for k in range(2)]
    spans = [(0, 8), (8, 20), (20, 31), (31, 40)]
    mixed, sm, _ = _run(scs, 80, 2, spans, ["host", "device", "device", "host"])
    host, sh, _ = _run(scs, 80, 2, [(0, 40)], ["host"])
    assert sm == sh == [0, 0]
    _close(host, mixed, STATE_TOL)
    o = orc.run_scenario(scs[0], False)
    assert np.abs(mixed[0][0] - o["state"]).max() < 1e-7
    assert np.abs(mixed[0][1] - o["sigma"]).max() < 1e-7


@pytest.mark.parametrize("env", [{}, {"EKF_SERIAL": "0"}, {"EKF_CU_SPLIT": "8"}],
                         ids=["36filters_serial", "36filters_events", "36filters_device_epochs"])
def test_device_device_host_handover_36_filters(monkeypatch, env):
    """36 filters (more than 32: one stream by default; EKF_SERIAL=0 keeps the chain and bulk
    streams with HIP events; a CU split of 8 per XCD holds all 36 chains, so device epochs), fp64
    N = 96 (the HBM pipeline), spans device → device → host of one drive with holes. The second device call's first chunks need the Σ passes two back, which belong to the
    first device call; the host call adopts the device's planning state. Round 4 saw exactly this
    hand-over off by 3.29 on the state under a since-removed schedule; the wait that fixed it
    (a device replay's chain waits for the pass two back) is what this test pins, against the whole
    drive planned on the host, without any pairing of filters.
    The events case failed intermittently until round 6 (2 of 5 runs, one filter's pose 6.1 rad
    off): the chain kernel's LDS zeroing raced with its own npose_ci initialisation when its waves
    ran at different paces on CUs shared with the bulk stream (k_chain); it gates."""
    for k in ("EKF_SERIAL", "EKF_CU_SPLIT", "EKF_DEVSYNC", "EKF_STAGE"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    pyekf.poison_lds()
    F = 36
    scs = [synth.synthetic(96, 30, seed=51 + k) for k in range(4)]
    spans = [(0, 11), (11, 20), (20, 30)]
    mixed, sm, pm = _run(scs, 96, F, spans, ["device", "device", "host"], holes=True)
    for k in ("EKF_SERIAL", "EKF_CU_SPLIT", "EKF_DEVSYNC", "EKF_STAGE"):
        monkeypatch.delenv(k, raising=False)
    host, sh, ph = _run(scs, 96, F, [(0, 30)], ["host"], holes=True)
    assert sm == sh == [0] * F
    _close(host, mixed, STATE_TOL)
    assert np.abs(ph - pm).max() <= STATE_TOL


@pytest.mark.parametrize("env", [{}, {"EKF_SERIAL": "0"}, {"EKF_CU_SPLIT": "8"}],
                         ids=["36filters_serial", "36filters_events", "36filters_device_epochs"])
def test_joseph_handover_36_filters(monkeypatch, env):
    """The hand-over above in the Joseph form (k_chain<T, true> in multi-filter launches, one
    kJoseph chunk per message planned on the host and on the device): device → device → host spans
    against the whole drive planned on the host, in each schedule; then a switch to the simple
    form for the last span (ekf_set_joseph drops every filter's rebuild: its next chunk gathers)
    against the same switch on the host."""
    for k in ("EKF_SERIAL", "EKF_CU_SPLIT", "EKF_DEVSYNC", "EKF_STAGE"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    pyekf.poison_lds()
    F = 36
    scs = [synth.synthetic(96, 30, seed=61 + k) for k in range(4)]
    spans = [(0, 11), (11, 20), (20, 30)]
    mixed, sm, pm = _run(scs, 96, F, spans, ["device", "device", "host"], holes=True, joseph=True)
    for k in ("EKF_SERIAL", "EKF_CU_SPLIT", "EKF_DEVSYNC", "EKF_STAGE"):
        monkeypatch.delenv(k, raising=False)
    host, sh, ph = _run(scs, 96, F, [(0, 30)], ["host"], holes=True, joseph=True)
    assert sm == sh == [0] * F
    _close(host, mixed, STATE_TOL)
    assert np.abs(ph - pm).max() <= STATE_TOL
    # the form switched between spans: Joseph device span, then the simple form on the device
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    full = _inputs(scs, F, 0, 30, True)
    res = []
    for kinds in (("device", "device"), ("host", "host")):
        e = pyekf.EKF(n_landmarks=96, n_filters=F)
        assert e.set_joseph(True) == pyekf.EKF_OK
        keep = []
        for (t0, t1), kind, jos in zip([(0, 15), (15, 30)], kinds, (True, False)):
            assert e.set_joseph(jos) == pyekf.EKF_OK
            cnt, ids, act, rel, od = (np.ascontiguousarray(a[t0:t1]) for a in full)
            if kind == "device":
                g = _to_gpu((cnt, ids, act, rel, od))
                keep.append(g)
                e.replay_device(g[0], g[3], g[4], g[1], g[2])
            else:
                e.replay(cnt, rel, od, ids=ids, actions=act)
        res.append(([e.state(f) for f in range(F)], [e.status(f) for f in range(F)]))
        e.close()
    assert res[0][1] == res[1][1] == [0] * F
    _close(res[1][0], res[0][0], STATE_TOL)


def test_posterior_then_device_replay(monkeypatch):
    """ekf_posterior enqueues k_posterior on the main stream, reading its descriptor in the upload
    buffer; with device epochs the next ekf_replay_device plans on the bulk stream and rewrites that
    buffer, so it must wait for the posterior first (ekf_api.cpp main_unordered). Four filters:
    host span, a posterior per filter, device span — against the single-stream schedule (planner
    and posterior in one stream order): bit-identical state and t_map_odom."""
    scs = [synth.synthetic(80, 24, seed=31 + k) for k in range(4)]
    F = 4
    full = _inputs(scs, F, 0, 24)
    res = []
    for env in ({"EKF_DEVSYNC": "1"}, {"EKF_SERIAL": "1"}):
        for k in ("EKF_SERIAL", "EKF_CU_SPLIT", "EKF_DEVSYNC", "EKF_STAGE"):
            monkeypatch.delenv(k, raising=False)
        for k, v in env.items():
            monkeypatch.setenv(k, v)
        e = pyekf.EKF(n_landmarks=80, n_filters=F)
        cnt, ids, act, rel, od = (np.ascontiguousarray(a[:8]) for a in full)
        e.replay(cnt, rel, od, ids=ids, actions=act)
        for f in range(F):
            e.posterior(f)
        g = _to_gpu(tuple(np.ascontiguousarray(a[8:]) for a in full))
        e.replay_device(g[0], g[3], g[4], g[1], g[2])
        res.append(([e.state(f) for f in range(F)], [e.map_odom(f) for f in range(F)],
                    [e.status(f) for f in range(F)]))
        e.close()
    (sa, ta, fa), (sb, tb, fb) = res
    assert fa == fb == [0] * F
    for (xa, Sa, ca), (xb, Sb, cb) in zip(sa, sb):
        assert ca == cb
        np.testing.assert_array_equal(xa, xb)
        np.testing.assert_array_equal(Sa, Sb)
    np.testing.assert_array_equal(np.stack(ta), np.stack(tb))


def test_device_replay_fp32_n1024():
    """The headline shape: fp32 N = 1024 from an fp64 survey, 24 messages of 16 markers through the
    device planner (bench.py's timed entry point) against the host planner (the staged rebuild
    operands and the fp32 patch are planned on the GPU too) and against the fp64 oracle."""
    N, warm, T = 1024, 40, 24
    sc = synth.synthetic(N, warm + T)
    assert sc.ids.shape[1] <= 16  # EKF_MAX_CHUNK: one chunk per message
    e64 = pyekf.EKF(n_landmarks=N)
    odom = pyekf.odometry(sc)
    e64.replay(sc.count[:warm, None], sc.rel[:warm, None], odom[:warm, None],
               ids=sc.ids[:warm, None], actions=sc.actions[:warm, None])
    x0, S0, c0 = e64.state()
    ws = (x0, S0, e64.map_odom(), c0)
    e64.close()
    host, sh, _ = _run([sc], N, 1, [(warm, warm + T)], ["host"], dtype=pyekf.EKF_F32, warm=ws)
    dev, sd, _ = _run([sc], N, 1, [(warm, warm + T)], ["device"], dtype=pyekf.EKF_F32, warm=ws)
    assert sh == sd == [0]
    (xh, Sh, ch), (xd, Sd, cd) = host[0], dev[0]
    assert ch == cd
    assert np.abs(xh - xd).max() < 1e-6
    assert np.abs(Sh - Sd).max() < 1e-6
    assert np.all(np.isfinite(Sd))
    # the timed entry point itself against the fp64 oracle (fake_sensor_cb, slam.cpp:180-316) from
    # the same warm state, at the fp32 tolerances of tests/test_gpu_scale.py: pose 1e-6, state
    # 1e-5, Σ 5e-5 absolute
    ref = orc.OracleEKF(n_landmarks=N)
    ref.set(x0, S0, ws[2], x0[:3], c0)
    for t in range(warm, warm + T):
        ref.set_odom(odom[t])
        c = int(sc.count[t])
        ref.fake_sensor_cb(sc.ids[t, :c], sc.actions[t, :c], sc.rel[t, :c])
    xr, Sr, _, cr = ref.get()
    assert cd == cr
    assert np.abs(xd[:3] - xr[:3]).max() < 1e-6
    assert np.abs(xd - xr).max() < 1e-5
    assert np.abs(Sd - Sr).max() < 5e-5


def test_device_replay_rejects():
    """No resident handles, at most EKF_MAX_CHUNK markers per message (one chunk)."""
    import torch
    sc = synth.synthetic(96, 4)
    g = _to_gpu(_inputs([sc], 1, 0, 4))
    e = pyekf.EKF(n_landmarks=20)  # fp64, n = 43: the resident path
    with pytest.raises(pyekf.EkfError):
        e.replay_device(g[0], g[3], g[4], g[1], g[2])
    e.close()
    e = pyekf.EKF(n_landmarks=96)
    wide = torch.zeros((4, 1, 17, 2), dtype=torch.float64, device="cuda")
    with pytest.raises(pyekf.EkfError):
        e.replay_device(g[0], wide, g[4], torch.zeros((4, 1, 17), dtype=torch.int32, device="cuda"))
    with pytest.raises(ValueError):  # host arrays are not device inputs
        e.replay_device(g[0].cpu(), g[3], g[4], g[1], g[2])
    e.replay_device(g[0], g[3], g[4], g[1], g[2])
    e.sync()
    assert e.status() == 0
    e.close()


@pytest.mark.parametrize("F,env", [(1, {}), (4, {}), (3, {"EKF_DEVSYNC": "0"}),
                                   (2, {"EKF_SERIAL": "1"})],
                         ids=["1filter", "4filters", "3filters_events", "2filters_serial"])
def test_device_replay_joseph_equals_host(monkeypatch, F, env):
    """Joseph form (ekf_set_joseph) through the device planner: one kJoseph chunk per message
    (plan_kernels.hip), as the host plans it (plan_known, kMaxJoseph = kMaxChunk). fp64 N = 96, up
    to 12 markers per message, holes (empty and all-DELETE messages): the two end alike, and filter
    0 equals the C oracle's Joseph mode."""
    for k in ("EKF_SERIAL", "EKF_CU_SPLIT", "EKF_DEVSYNC", "EKF_STAGE"):
        monkeypatch.delenv(k, raising=False)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    pyekf.poison_lds()
    scs = []
    for k in range(3):  # messages of 12, 5, 8, 9 and 1 markers
        s0 = synth.synthetic(96, 30, seed=7 + k, max_markers=12)
        cnt = np.minimum(s0.count, np.roll([12, 5, 8, 9, 1], k)[np.arange(30) % 5]).astype(s0.count.dtype)
        scs.append(synth.Scenario(s0.n_landmarks, s0.landmarks, s0.wheel, s0.ids, s0.actions,
                                  s0.rel, cnt, s0.truth, s0.track, s0.radius))
    assert scs[0].count.max() == 12 and scs[0].count.min() == 1
    host, sh, ph = _run(scs, 96, F, [(0, 30)], ["host"], holes=True, joseph=True)
    dev, sd, pd = _run(scs, 96, F, [(0, 30)], ["device"], holes=True, joseph=True)
    assert sh == sd == [0] * F
    _close(host, dev, STATE_TOL)
    assert np.abs(ph - pd).max() <= STATE_TOL
    o = orc.run_scenario(scs[0], False, joseph=True)
    assert np.abs(dev[0][0] - o["state"]).max() < 1e-7
    assert np.abs(dev[0][1] - o["sigma"]).max() < 1e-7


@pytest.mark.parametrize("dtype", [pyekf.EKF_F32, pyekf.EKF_F64], ids=["f32", "f64"])
def test_device_replay_joseph_n1024(dtype):
    """The Joseph form at the headline shape (bench.py --workload n1024_fp32_joseph): N = 1024 from
    an fp64 survey, 12 messages of 16 markers through the device planner — one chunk per message,
    its V_c·K_cᵀ terms folded into its one rank-66 Σ pass — against the fp64 oracle's
    Joseph mode from the same state, at the fp32 tolerances of tests/test_gpu_scale.py (pose 1e-6,
    state 1e-5, Σ 5e-5) or the fp64 populated-map ones (state 5e-8, Σ 1e-7)."""
    N, warm, T = 1024, 40, 12
    sc = synth.synthetic(N, warm + T)
    assert sc.count[warm:].max() == 16
    e64 = pyekf.EKF(n_landmarks=N)
    odom = pyekf.odometry(sc)
    e64.replay(sc.count[:warm, None], sc.rel[:warm, None], odom[:warm, None],
               ids=sc.ids[:warm, None], actions=sc.actions[:warm, None])
    x0, S0, c0 = e64.state()
    ws = (x0, S0, e64.map_odom(), c0)
    e64.close()
    dev, sd, _ = _run([sc], N, 1, [(warm, warm + T)], ["device"], dtype=dtype, warm=ws,
                      joseph=True)
    assert sd == [0]
    xd, Sd, cd = dev[0]
    assert np.all(np.isfinite(Sd))
    ref = orc.OracleEKF(n_landmarks=N, joseph=True)
    ref.set(x0, S0, ws[2], x0[:3], c0)
    for t in range(warm, warm + T):
        ref.set_odom(odom[t])
        c = int(sc.count[t])
        ref.fake_sensor_cb(sc.ids[t, :c], sc.actions[t, :c], sc.rel[t, :c])
    xr, Sr, _, cr = ref.get()
    assert cd == cr
    if dtype == pyekf.EKF_F32:
        assert np.abs(xd[:3] - xr[:3]).max() < 1e-6
        assert np.abs(xd - xr).max() < 1e-5
        assert np.abs(Sd - Sr).max() < 5e-5
    else:
        assert np.abs(xd - xr).max() < 5e-8
        assert np.abs(Sd - Sr).max() < 1e-7
