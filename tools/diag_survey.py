"""Where does a populated-map survey replay on the GPU leave the C oracle? (diagnostic)

Replays synth.populated(N, T)'s messages through ekf_replay under several schedules and prints, per
variant, the first message whose posterior pose differs from the oracle's by more than 1e-8 and the
final state error. Usage: python tools/diag_survey.py N [T]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ekf-slam_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

import orc  # noqa: E402
import pyekf  # noqa: E402
from pyekf import synth  # noqa: E402

N = int(sys.argv[1])
T = int(sys.argv[2]) if len(sys.argv) > 2 else 10
sc = synth.populated(N, T)
odom = pyekf.odometry(sc)
W = sc.n_messages
ref = orc.OracleEKF(n_landmarks=N)
op = np.zeros((W, 3))
for t in range(W):
    ref.set_odom(odom[t])
    c = int(sc.count[t])
    ref.fake_sensor_cb(sc.ids[t, :c], sc.actions[t, :c], sc.rel[t, :c])
    op[t] = ref.get(sigma=False)[0][:3]
xr = ref.get(sigma=False)[0]
print(f"N={N} messages={W} (survey {sc.n_warm}) markers/msg {sc.count.mean():.2f} max {sc.count.max()}",
      flush=True)


def run(env, per_msg=False, dtype=pyekf.EKF_F64, upto=None):
    for k in ("EKF_SERIAL", "EKF_DEVSYNC", "EKF_CU_SPLIT", "EKF_RESIDENT"):
        os.environ.pop(k, None)
    os.environ.update(env)
    e = pyekf.EKF(n_landmarks=N, dtype=dtype)
    if per_msg:
        p = np.zeros((W, 1, 3))
        for t in range(W):
            sl = slice(t, t + 1)
            p[t] = e.replay(sc.count[sl, None], sc.rel[sl, None], odom[sl, None],
                            ids=sc.ids[sl, None], actions=sc.actions[sl, None], poses=True)[0]
    elif upto is not None:  # one persistent replay of the first `upto` messages, status only
        sl = slice(0, upto)
        e.replay(sc.count[sl, None], sc.rel[sl, None], odom[sl, None], ids=sc.ids[sl, None],
                 actions=sc.actions[sl, None])
        st = e.status()
        e.close()
        return st
    else:
        p = e.replay(sc.count[:, None], sc.rel[:, None], odom[:, None], ids=sc.ids[:, None],
                     actions=sc.actions[:, None], poses=True)
    x, _, _ = e.state(sigma=False)
    st = e.status()
    e.close()
    d = np.abs(p[:, 0] - op).max(1)
    bad = np.nonzero(d > 1e-8)[0]
    first = int(bad[0]) if len(bad) else -1
    info = ""
    if first >= 0:
        info = (f" count[first]={int(sc.count[first])} d[first]={d[first]:.3e} "
                f"d[first-1]={d[first - 1] if first else 0:.3e}")
    print(f"{str(env):40s} per_msg={per_msg} status={st} first_bad={first} "
          f"max_pose={d.max():.3e} final_state={np.abs(x - xr).max():.3e}{info}", flush=True)


for env, pm in (({}, False), ({"EKF_SERIAL": "1"}, False), ({"EKF_DEVSYNC": "1"}, False),
                ({}, True), ({"EKF_SERIAL": "1"}, True)):
    run(env, pm)

# the first prefix of one persistent (no per-message sync) replay whose status is non-zero
for env in ({}, {"EKF_DEVSYNC": "0"}):
    lo, hi = 0, W
    if run(env, upto=W) == 0:
        print(f"{env}: full persistent replay status 0", flush=True)
        continue
    while hi - lo > 1:
        mid = (lo + hi) // 2
        if run(env, upto=mid):
            hi = mid
        else:
            lo = mid
    print(f"{env}: status first non-zero after message {hi - 1} (count {int(sc.count[hi - 1])}, "
          f"previous {int(sc.count[hi - 2])})", flush=True)
