"""Dev diagnostic: the N=1024 fp32 warm-state replay of tests/test_gpu_parity.py, repeated in one
process; reports non-finite Σ entries (where) and the status flags after each run."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ekf-slam_amd"), os.path.join(ROOT, "oracle")]
import pyekf  # noqa: E402
from pyekf import synth  # noqa: E402

N, warm, T = 1024, 63, 40
sc = synth.synthetic(N, warm + T)
odom = pyekf.odometry(sc)
ekf64 = pyekf.EKF(n_landmarks=N)
ekf64.replay(sc.count[:warm, None], sc.rel[:warm, None], odom[:warm, None],
             ids=sc.ids[:warm, None], actions=sc.actions[:warm, None])
x, S, cnt = ekf64.state()
tmo = ekf64.map_odom()
ekf64.close()
for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 3):
    for poses_flag in (True, False):
        e = pyekf.EKF(n_landmarks=N, dtype=pyekf.EKF_F32)
        e.set_state(x, S, tmo=tmo, counter=cnt)
        e.replay(sc.count[warm:, None], sc.rel[warm:, None], odom[warm:, None],
                 ids=sc.ids[warm:, None], actions=sc.actions[warm:, None], poses=poses_flag)
        x32, S32, _ = e.state()
        bad = np.argwhere(~np.isfinite(S32))
        print(f"rep {rep} poses={poses_flag}: nonfinite {len(bad)} status {e.status()} "
              f"rows {sorted(set(bad[:, 0].tolist()))[:12]} cols {sorted(set(bad[:, 1].tolist()))[:12]}"
              f" x finite {np.all(np.isfinite(x32))}", flush=True)
        e.close()
