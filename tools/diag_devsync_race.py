"""Dev diagnostic: the opt-in device-epoch pipeline (EKF_DEVSYNC=1) against the single-stream order
(EKF_SERIAL=1) on the 4-filter N=256 replay of test_pipelined_replay_sync_modes and the 24-filter
N=64 replay of test_many_filters_match_small_batch, repeated in one process with a resident-path
handle and an fp32 N=1024 handle created and freed between repetitions (memory reuse, other
kernels in between); prints non-finite counts, max differences and status flags
(EKF_FLAG_NUMERIC = 2, EKF_FLAG_TIMEOUT = 4). Usage: diag_devsync_race.py [iterations]."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ekf-slam_amd"), os.path.join(ROOT, "oracle")]
import pyekf  # noqa: E402
from pyekf import synth  # noqa: E402

CASES = {"n256x4": (256, 4, synth.synthetic(256, 30)), "n64x24": (64, 24, synth.synthetic(64, 12))}


def run(case, env):
    N, F, sc = CASES[case]
    odom = pyekf.odometry(sc)
    rep = lambda a: np.repeat(a[:, None], F, 1)  # noqa: E731
    for k in ("EKF_SERIAL", "EKF_DEVSYNC", "EKF_RESIDENT"):
        os.environ.pop(k, None)
    os.environ.update(env)
    e = pyekf.EKF(n_landmarks=N, n_filters=F)
    e.replay(rep(sc.count), rep(sc.rel), rep(odom), ids=rep(sc.ids), actions=rep(sc.actions))
    out = [e.state(f) for f in range(F)]
    st = [e.status(f) for f in range(F)]
    e.close()
    return out, st


def other_work():
    r = pyekf.Slam(n_landmarks=50, source=pyekf.SOURCE_ASSOC)
    r.replay(synth.basic_world(20, shuffle=True), poses=False)
    r.filter_state()
    r.close()
    e = pyekf.EKF(n_landmarks=1024, dtype=pyekf.EKF_F32)
    e.close()


refs = {c: run(c, {"EKF_SERIAL": "1"})[0] for c in CASES}
for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 10):
    for c in CASES:
        other_work()
        out, st = run(c, {"EKF_DEVSYNC": "1"})
        bad = sum(int(np.count_nonzero(~np.isfinite(o[1]))) for o in out)
        dx = max(float(np.nanmax(np.abs(o[0] - r[0]))) for o, r in zip(out, refs[c]))
        flags = sorted(set(st))
        print(f"iter {it} {c}: nonfinite Σ entries {bad} max|dx| {dx:.2e} status {flags}",
              flush=True)
