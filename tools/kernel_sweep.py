"""Dev tool: per-kernel device time (HIP events inside libekfslam) over N, m and dtype."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ekf-slam_amd"))
import pyekf  # noqa: E402
from pyekf import synth  # noqa: E402


def run(N, m, dtype, F=1, T=40):
    T = 2 * T
    sc = synth.synthetic(N, T, max_markers=m) if N > 50 else synth.basic_world(T)
    odom = pyekf.odometry(sc)
    e = pyekf.EKF(n_landmarks=N, n_filters=F, dtype=dtype)
    cnt = np.repeat(sc.count[:, None], F, 1)
    rel = np.repeat(sc.rel[:, None], F, 1)
    ids = np.repeat(sc.ids[:, None], F, 1)
    act = np.repeat(sc.actions[:, None], F, 1)
    od = np.repeat(odom[:, None], F, 1)
    h = T // 2
    e.replay(cnt[:5], rel[:5], od[:5], ids=ids[:5], actions=act[:5])
    e.sync()
    t0 = time.perf_counter()
    e.replay(cnt[5:h], rel[5:h], od[5:h], ids=ids[5:h], actions=act[5:h])
    e.sync()
    wall = (time.perf_counter() - t0) / (h - 5)
    e.profile(True)
    e.replay(cnt[h:], rel[h:], od[h:], ids=ids[h:], actions=act[h:])
    e.sync()
    ns, ms_s = e.profile_read(0)
    ng, ms_g = e.profile_read(1)
    nf, ms_f = e.profile_read(3)
    e.close()
    return wall * 1e6, ms_g / ng * 1e3, ms_s / ns * 1e3, ms_f / nf * 1e3


print(f"{'N':>5} {'m':>3} {'dt':>4} {'F':>4} | {'wall/msg us':>11} {'chain us':>9} {'factor us':>9} {'sigma us':>9}")
for N, m, dt, F in [(50, 4, 0, 1), (256, 1, 0, 1), (256, 4, 0, 1), (256, 16, 0, 1),
                    (1024, 1, 1, 1), (1024, 4, 1, 1), (1024, 16, 1, 1), (1024, 16, 0, 1),
                    (256, 16, 0, 64)]:
    w, g, s, fa = run(N, m, dt, F)
    print(f"{N:5d} {m:3d} {'f32' if dt else 'f64':>4} {F:4d} | {w:11.1f} {g:9.1f} {fa:9.1f} {s:9.1f}",
          flush=True)
