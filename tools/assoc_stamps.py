"""Dev tool: k_assoc_msg's per-step phase times (libekfslam_diag.so, s_memrealtime at 100 MHz) on
the n1024 association workload: workgroup 0 and the last workgroup, the last launch.
  EKF_LIB=libekfslam_diag.so python tools/assoc_stamps.py [f32|f64]"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ekf-slam_amd"))
import pyekf  # noqa: E402
from pyekf import synth  # noqa: E402

N = 1024
DT = sys.argv[1] if len(sys.argv) > 1 else "f32"
sc = synth.populated(N, 6, n_map=N - 64)
odom = pyekf.odometry(sc)
w = sc.n_warm
e64 = pyekf.EKF(n_landmarks=N)
e64.replay(sc.count[:w, None], sc.rel[:w, None], odom[:w, None], ids=sc.ids[:w, None],
           actions=sc.actions[:w, None])
x, S, _ = e64.state()
tmo = e64.map_odom()
e64.close()
e = pyekf.EKF(n_landmarks=N, dtype=pyekf.EKF_F32 if DT == "f32" else pyekf.EKF_F64)
e.set_state(x, S, tmo=tmo, counter=N - 64)
for t in range(w, w + 4):
    e.replay(sc.count[t:t + 1, None], sc.rel[t:t + 1, None], odom[t:t + 1, None], assoc=True)
    e.sync()
L = pyekf.lib()
L.ekf_diag_am_stamps.argtypes = [C.c_void_p]
st = np.zeros((2, 17, 8), dtype=np.uint64)
L.ekf_diag_am_stamps(st.ctypes.data)
for wg in range(2):
    t0 = int(st[wg, 16, 0])
    print(f"workgroup {'0' if wg == 0 else 'last'}: total {(int(st[wg, 16, 1]) - t0) / 100:.2f} us")
    for c in range(16):
        s0, s1, s2, s3, s4, s5 = (int(v) for v in st[wg, c, :6])
        if s0 == 0:
            continue
        hist = f" (history sums {(s5 - s3) / 100:5.2f})" if s5 else ""
        print(f"  step {c:2d} at {(s0 - t0) / 100:7.2f}: score+argmin {(s1 - s0) / 100:6.2f} "
              f"exchange {(s2 - s1) / 100:6.2f} loads {(s3 - s2) / 100:6.2f} "
              f"math {(s4 - s3) / 100:6.2f} us{hist}")
