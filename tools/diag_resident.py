"""Dev diagnostic: per-filter max |Σ − oracle| and |x − oracle| for the resident path and the HBM
pipeline on the ragged swarm of tests/test_gpu_resident.py."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ekf-slam_amd"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "tests")]
import orc  # noqa: E402
import pyekf  # noqa: E402
from pyekf import synth  # noqa: E402
from test_gpu_resident import _stack  # noqa: E402

F, T, N = 48, 24, 40
assoc = len(sys.argv) > 1 and sys.argv[1] == "assoc"
scs = [synth.make_scenario(N, synth.random_landmarks(10 + f % 20, seed=300 + f), T,
                           max_markers=4 + f % 9, seed=400 + f, shuffle=assoc) for f in range(F)]
counts, ids, act, rel, odom = _stack(scs, T)
refs = [orc.run_scenario(s, assoc) for s in scs]
lit = []
res = {}
for resident in ("1", "0"):
    os.environ["EKF_RESIDENT"] = resident
    e = pyekf.EKF(n_landmarks=N, n_filters=F)
    e.replay(counts, rel, odom, ids=None if assoc else ids, actions=act, assoc=assoc)
    res[resident] = [e.state(f) for f in range(F)]
    e.close()
for f in range(F):
    o = refs[f]
    r = res["1"][f]
    p = res["0"][f]
    print(f, "res S %.2e x %.2e | pipe S %.2e x %.2e | res-pipe S %.2e" % (
        np.abs(r[1] - o["sigma"]).max(), np.abs(r[0] - o["state"]).max(),
        np.abs(p[1] - o["sigma"]).max(), np.abs(p[0] - o["state"]).max(),
        np.abs(r[1] - p[1]).max()))
for k, f in enumerate([]):
    print("literal vs structured oracle", f, "%.2e" % np.abs(lit[k]["sigma"] - refs[f]["sigma"]).max())
