"""Dev diagnostic: the device-epoch pipeline (EKF_DEVSYNC default) against the single-stream order
(EKF_SERIAL=1) on the 4-filter N=256 replay of test_pipelined_replay_sync_modes, repeated in one
process; prints non-finite counts, max differences and the status flags (EKF_FLAG_TIMEOUT = 4)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ekf-slam_amd"), os.path.join(ROOT, "oracle")]
import pyekf  # noqa: E402
from pyekf import synth  # noqa: E402

F = 4
sc = synth.synthetic(256, 30)
odom = pyekf.odometry(sc)
rep = lambda a: np.repeat(a[:, None], F, 1)  # noqa: E731


def run(env):
    for k in ("EKF_SERIAL", "EKF_DEVSYNC"):
        os.environ.pop(k, None)
    os.environ.update(env)
    e = pyekf.EKF(n_landmarks=256, n_filters=F)
    e.replay(rep(sc.count), rep(sc.rel), rep(odom), ids=rep(sc.ids), actions=rep(sc.actions))
    out = [e.state(f) for f in range(F)]
    st = [e.status(f) for f in range(F)]
    e.close()
    return out, st


ref, _ = run({"EKF_SERIAL": "1"})
for it in range(int(sys.argv[1]) if len(sys.argv) > 1 else 10):
    out, st = run({})
    bad = [int(np.count_nonzero(~np.isfinite(o[1]))) + int(np.count_nonzero(~np.isfinite(o[0])))
           for o in out]
    dx = max(float(np.nanmax(np.abs(o[0] - r[0]))) for o, r in zip(out, ref))
    print(f"iter {it}: nonfinite {bad} max|dx| {dx:.2e} status {st}", flush=True)
