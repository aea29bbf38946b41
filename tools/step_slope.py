"""Dev tool: production wall time per message vs markers per message (pipelined replay, one
filter), to separate the per-correction cost from the per-message cost."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ekf-slam_amd"))
import pyekf  # noqa: E402
from pyekf import synth  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
dt = int(sys.argv[2]) if len(sys.argv) > 2 else 1
T = 200
for m in (1, 2, 4, 8, 12, 16):
    sc = synth.synthetic(N, T + 40, max_markers=m)
    odom = pyekf.odometry(sc)
    e = pyekf.EKF(n_landmarks=N, dtype=dt)
    if dt:  # fp32 starts warm (first sightings need fp64): seen landmarks only after a f64 lap
        pass
    a = dict(ids=sc.ids[:, None], actions=sc.actions[:, None])
    e.replay(sc.count[:40, None], sc.rel[:40, None], odom[:40, None], ids=sc.ids[:40, None],
             actions=sc.actions[:40, None])
    e.sync()
    best = 1e9
    for rep in range(3):
        t0 = time.perf_counter()
        e.replay(sc.count[40:, None], sc.rel[40:, None], odom[40:, None], ids=sc.ids[40:, None],
                 actions=sc.actions[40:, None])
        e.sync()
        best = min(best, (time.perf_counter() - t0) / T)
    mean_m = float(np.mean(sc.count[40:]))
    print(f"m={m:2d} (mean {mean_m:5.2f})  {best * 1e6:7.2f} us/message", flush=True)
    e.close()
