"""Dev tool: phase stamps (s_memtime cycles) of the chain kernel's last chunk, filter 0, in the
pipelined replay (libekfslam_diag.so; build: make -C ekf-slam_amd diag)."""
import ctypes as C
import os
import sys

import numpy as np

os.environ["EKF_LIB"] = "libekfslam_diag.so"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ekf-slam_amd"))
import pyekf  # noqa: E402
from pyekf import synth  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
T = 40
sc = synth.synthetic(N, T) if os.environ.get("STAMPS_MAP") != "populated" else synth.populated(N, T)
odom = pyekf.odometry(sc)
e = pyekf.EKF(n_landmarks=N)
e.replay(sc.count[:, None], sc.rel[:, None], odom[:, None], ids=sc.ids[:, None],
         actions=sc.actions[:, None])
e.sync()
L = pyekf.lib()
st = (C.c_ulonglong * 256)()
L.ekf_diag_stamps.argtypes = [C.c_void_p, C.c_int]
assert L.ekf_diag_stamps(st, 256) == 0
s = np.array(st[:], dtype=np.int64)
t0 = s[0]
names = {1: "A0", 21: "kLook: gathers landed", 3: "kLook: R, C, D (prev predict)",
         7: "kLook: K', M' tiles", 5: "kLook: x[U]", 6: "A1 done (P tiles)",
         2: "predict (steps start)", 12: "steps+final pass", 16: "epi: rec stores issued",
         40: "chunk end"}
for k in (1, 21, 3, 7, 5, 6, 2, 12, 16, 40):
    print(f"{names[k]:24s} {s[k] - t0:8d}")
m = int(sc.count[-1])
steps = [s[64 + 8 * c] - t0 for c in range(m)]
print("step starts:", steps)
for c in (0, 1, m // 2, m - 2):
    b = 64 + 8 * c
    d = [s[b + k + 1] - s[b + k] for k in range(6)]
    print(f"step {c}: start {d[0]}  S,inv,nu {d[1]}  pdone wait+Bx reads {d[2]}  K,M,x,publish {d[3]}"
          f"  geometry(c+1)+cross update {s[b + 6] - s[b + 4]}  -> next {s[b + 8] - s[b + 6]}")
    print(f"   wave3: pub seen at {s[192 + 2 * c] - s[b]}, pdone at {s[193 + 2 * c] - s[b]} "
          f"(wave0 publish at {s[b + 4] - s[b]}, next-step pdone wait at {s[b + 8 + 2] - s[b]})")
e.close()
