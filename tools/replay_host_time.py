"""Host planning share of ekf_replay at one filter: the time ekf_replay takes to return (plan,
upload, enqueue — the GPU runs asynchronously) against the time to the GPU's completion.
Usage (repo root, GPU box): python tools/replay_host_time.py [--n 1024] [--msgs 200]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "ekf-slam_amd"))
import bench  # noqa: E402
import pyekf  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n", type=int, default=1024)
ap.add_argument("--msgs", type=int, default=200)
a = ap.parse_args()
sw, odom, _ = bench.build_inputs(a.n, 1, 3 * a.msgs, 20240317, 16, 0)
e = pyekf.EKF(n_landmarks=a.n, n_filters=1, dtype=pyekf.EKF_F64, device=0)
nw = sw.n_warm


def rp(lo, hi):
    s = slice(lo, hi)
    e.replay(sw.count[s], sw.rel[s], odom[s], ids=sw.ids[s], actions=sw.actions[s])


rp(0, nw + a.msgs)
e.sync()
for k in range(3):
    lo = nw + a.msgs * (1 + k % 2)
    t0 = time.perf_counter()
    rp(lo, lo + a.msgs)
    t1 = time.perf_counter()
    e.sync()
    t2 = time.perf_counter()
    print(f"run {k}: replay returns after {1e6 * (t1 - t0):.0f} us, GPU done after {1e6 * (t2 - t0):.0f} us "
          f"({1e6 * (t2 - t0) / a.msgs:.1f} us per message)", flush=True)
