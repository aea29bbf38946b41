"""Dev tool: unknown association at scale (sensor_cb, slam.cpp:318-530) on the HBM pipeline.

A populated N-landmark map (the survey warm-up sights every landmark, counter = N), then T circle
messages with the ids stripped, replayed with on-device decisions (ekf_replay, assoc=1): each
marker is k_assoc over every known landmark, then a one-marker chunk (chain, factors, Σ pass).
Prints one JSON line: corrections/s end to end and the device time per kernel (HIP events).

  python tools/assoc_bench.py [N] [f32|f64] [T] [K]      (default 1024 f64 8, K = N − 64 known
  landmarks: room for the new ones a marker may start)
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ekf-slam_amd"))
import pyekf  # noqa: E402
from pyekf import synth  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
DT = sys.argv[2] if len(sys.argv) > 2 else "f64"
T = int(sys.argv[3]) if len(sys.argv) > 3 else 8
K = int(sys.argv[4]) if len(sys.argv) > 4 else N - 64
sc = synth.populated(N, 2 * T + 2, n_map=K)
odom = pyekf.odometry(sc)
w = sc.n_warm


def replay(e, sl, assoc):
    ids = None if assoc else sc.ids[sl, None]
    e.replay(sc.count[sl, None], sc.rel[sl, None], odom[sl, None], ids=ids,
             actions=sc.actions[sl, None], assoc=assoc)


e64 = pyekf.EKF(n_landmarks=N)
replay(e64, slice(0, w), False)
x, S, cnt = e64.state()
tmo = e64.map_odom()
e64.close()
e = pyekf.EKF(n_landmarks=N, dtype=pyekf.EKF_F32 if DT == "f32" else pyekf.EKF_F64)
e.set_state(x, S, tmo=tmo, counter=K)  # the survey sighted landmarks 0..K−1 (slam.cpp:351-356)
replay(e, slice(w, w + 2), True)  # warm-up (first launches, code objects)
e.sync()
t0 = time.perf_counter()
replay(e, slice(w + 2, w + 2 + T), True)
e.sync()
dt = time.perf_counter() - t0
e.profile(True)  # device time per kernel over the next T messages (HIP events per launch)
replay(e, slice(w + 2 + T, w + 2 + 2 * T), True)
e.sync()
names = {2: "k_assoc", 1: "k_chain", 3: "k_factors", 0: "k_sigma_pass"}
dev = {}
for k, nm in names.items():
    n, ms = e.profile_read(k)
    dev[nm] = {"launches": n, "avg_us": 1e3 * ms / max(n, 1)}
e.profile(False)
corr = int(sc.count[w + 2:w + 2 + T].sum())
st = e.status()
_, _, cnt2 = e.state()
e.close()
print(json.dumps({"workload": f"assoc_n{N}_{DT}", "n_landmarks": N, "counter_start": K,
                  "counter_end": int(cnt2), "messages": T, "corrections": corr,
                  "corrections_per_s": corr / dt, "us_per_correction": 1e6 * dt / corr,
                  "status": st, "device": dev}))
