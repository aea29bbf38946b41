import sys, os, numpy as np
sys.path.insert(0, "ekf-slam_amd")
import pyekf
from pyekf import synth
N, T = 64, 12
scs = [synth.synthetic(N, T, seed=100 + k) for k in range(8)]
odo = [pyekf.odometry(s) for s in scs]
M = max(s.ids.shape[1] for s in scs)
def run(nf):
    cnt = np.zeros((T, nf), np.int32); ids = np.full((T, nf, M), -1, np.int32)
    act = np.zeros((T, nf, M), np.int32); rel = np.zeros((T, nf, M, 2)); od = np.zeros((T, nf, 3))
    for f in range(nf):
        s = scs[f % 8]; k = s.ids.shape[1]
        cnt[:, f] = s.count; ids[:, f, :k] = s.ids; act[:, f, :k] = s.actions; rel[:, f, :k] = s.rel; od[:, f] = odo[f % 8]
    e = pyekf.EKF(n_landmarks=N, n_filters=nf)
    e.replay(cnt, rel, od, ids=ids, actions=act)
    out = [(e.state(f), e.status(f)) for f in range(nf)]
    e.close()
    return out
ref = run(8)
for nf in (8, 9, 15, 16, 17, 24):
    big = run(nf)
    bad = []
    for f in range(nf):
        (x, S, c), st = big[f]
        (xr, Sr, cr), _ = ref[f % 8]
        dx = np.abs(x - xr).max(); dS = np.abs(S - Sr).max()
        if dx > 0 or dS > 0 or st: bad.append((f, float(dx), float(dS), st))
    print(nf, "bad", bad[:8], len(bad))
