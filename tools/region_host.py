"""Dev tool: host-side composition of the bench's timed region (N = 1024 fp32, device-planned
replay of K messages): enqueue (ekf_replay_device), the library's sync (ekf_sync), then
torch.cuda.synchronize — median over R regions in one process, for the bench's order of the two
syncs and the reverse order.  Usage: python tools/region_host.py [K] [R]"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ekf-slam_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402
import pyekf  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
R = int(sys.argv[2]) if len(sys.argv) > 2 else 30
N, W = 1024, 5
sw, odom, _ = bench.build_inputs(N, 1, W + R * K, 20240317, 16, 0)
torch.cuda.set_device(0)
e64 = pyekf.EKF(n_landmarks=N)
sl = slice(0, sw.n_warm)
e64.replay(sw.count[sl], sw.rel[sl], odom[sl], ids=sw.ids[sl], actions=sw.actions[sl])
x, S, cnt = e64.state(0)
tmo = e64.map_odom(0)
e64.close()
e = pyekf.EKF(n_landmarks=N, dtype=pyekf.EKF_F32)
e.set_state(x, S, tmo=tmo, counter=cnt)
dev = torch.device("cuda", 0)
g = [torch.from_numpy(np.ascontiguousarray(a, dtype=d)).to(dev) for a, d in
     ((sw.count, np.int32), (sw.ids, np.int32), (sw.actions, np.int32), (sw.rel, np.float64),
      (odom, np.float64))]
torch.cuda.synchronize()
rows = [(t.data_ptr(), t[0].numel() * t.element_size()) for t in g]


def msgs(a, b):
    pc, pi, pa, pr, po = (base + a * rb for base, rb in rows)
    e.replay_device_raw(b - a, sw.ids.shape[2], pc, pr, po, pi, pa)


t = sw.n_warm
msgs(t, t + W)
t += W
res = {"lib then torch": [], "torch then lib": [], "torch only (lib after the clock)": []}
for r in range(R):
    mode = list(res)[r % 3]
    e.sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    msgs(t, t + K)
    t1 = time.perf_counter()
    if mode == "lib then torch":
        e.sync()
        t2 = time.perf_counter()
        torch.cuda.synchronize()
    elif mode == "torch then lib":
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        e.sync()
    else:
        torch.cuda.synchronize()
        t2 = time.perf_counter()
    t3 = time.perf_counter()
    if mode.startswith("torch only"):
        e.sync()
    t += K
    res[mode].append(((t1 - t0) * 1e6, (t2 - t1) * 1e6, (t3 - t2) * 1e6, (t3 - t0) * 1e6))
print(f"N={N} fp32, {K} messages per region, {R} regions (medians, us): enqueue, first sync, "
      "second sync, region; status", e.status())
for k, v in res.items():
    a = np.median(np.array(v), axis=0)
    print(f"  {k:34s} enqueue {a[0]:7.1f}  sync1 {a[1]:7.1f}  sync2 {a[2]:6.1f}  region {a[3]:7.1f}"
          f"  -> {K * 16 / a[3] * 1e6:.4g} corrections/s")
