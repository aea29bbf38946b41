"""Dev tool: phase stamps (s_memtime cycles) of the chain kernel's last chunk, filter 0, in the
pipelined replay (libekfslam_diag.so; build: make -C ekf-slam_amd diag).

  python tools/chain_stamps.py [N] [f32|f64]   (default 1024 f32: configs[2]'s headline shape —
  the fp64 survey lap, then fp32 circle messages from its state, as bench.py runs it)
  With the block builder (the default of a one-filter device-epoch handle) also its phases
  during the chunk before."""
import ctypes as C
import os
import sys

import numpy as np

os.environ.setdefault("EKF_LIB", "libekfslam_diag.so")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ekf-slam_amd"))
import pyekf  # noqa: E402
from pyekf import synth  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
DT = sys.argv[2] if len(sys.argv) > 2 else "f32"
T = 40
sw = synth.swarm(N, 1, T, seed=20240317, max_markers=16)
sc = sw.scenario(0)
odom = pyekf.odometry(sc)
w = sc.n_warm


# EKF_STAMP_F=<filters>: the same messages replayed by that many filters of one handle (the swarm's
# schedule: event hand-offs beyond 32 filters); the stamps are filter 0's
F = int(os.environ.get("EKF_STAMP_F", "1"))


def replay(e, sl):
    rep = lambda a: np.ascontiguousarray(np.repeat(a[sl, None], F, axis=1))  # noqa: E731
    e.replay(rep(sc.count), rep(sc.rel), rep(odom), ids=rep(sc.ids), actions=rep(sc.actions))


e64 = pyekf.EKF(n_landmarks=N, n_filters=F)
replay(e64, slice(0, w))
if DT == "f32":
    x, S, cnt = e64.state()
    tmo = e64.map_odom()
    e64.close()
    e = pyekf.EKF(n_landmarks=N, dtype=pyekf.EKF_F32)
    e.set_state(x, S, tmo=tmo, counter=cnt)
else:
    e = e64
if os.environ.get("EKF_STAMP_JOSEPH") == "1":  # the Joseph-form chain (ekf_set_joseph)
    assert e.set_joseph(True) == 0
replay(e, slice(w, w + T))
e.sync()
print("status", e.status())
L = pyekf.lib()
st = (C.c_ulonglong * 2048)()
L.ekf_diag_stamps.argtypes = [C.c_void_p, C.c_int]
assert L.ekf_diag_stamps(st, 2048) == 0
ring = np.array(st[:], dtype=np.int64).reshape(4, 512)
# the ring holds the last four chunks; WHICH=1 (default) the one before the last (it rebuilt the
# last chunk's block: the steady state), 0 the last
order = np.argsort(ring[:, 0])[::-1]
s = ring[order[int(os.environ.get("WHICH", "1"))]]
t0 = s[0]
names = {14: "A0: early loads issued", 1: "A0", 21: "kLook: loads landed", 3: "kLook: R, C, D (prev predict)",
         7: "kLook: K', M' tiles", 5: "kLook: x[U]", 6: "A1 done (P tiles)",
         2: "predict (steps start)", 12: "steps+final pass", 16: "epi: rec stores issued",
         40: "chunk end", 10: "  wave1 P tiles done", 11: "  wave2 P tiles done",
         13: "  wave3 P tiles done", 8: "  wave2 predicted pose", 9: "  wave3 x[U]",
         15: "  raw R, C, D stored", 17: "  (prev predict barrier)", 18: "  (diag block dump)",
         19: "  drain + barrier, wave 0 enters"}
print(f"N={N} {DT}, chunk {-1 - int(os.environ.get('WHICH', '1'))} of {T} messages (cycles from "
      f"the chunk's stamp 0); chunk starts of the ring, relative: {sorted(ring[:, 0] - ring[:, 0].min())}")
for k in (14, 1, 21, 15, 17, 3, 7, 5, 10, 11, 13, 8, 9, 6, 2, 18, 19, 12, 16, 40):
    print(f"{names[k]:24s} {s[k] - t0:8d}")
m = int(sc.count[w + T - 1 - int(os.environ.get("WHICH", "1"))])
steps = [int(s[64 + 8 * c] - t0) for c in range(m)]
print("step starts:", steps)
print("mean step:", (steps[-1] - steps[0]) / max(m - 1, 1))
for c in (0, 1, m // 2, m - 2):
    b = 64 + 8 * c
    d = [s[b + k + 1] - s[b + k] for k in range(6)]
    print(f"step {c}: start {d[0]}  S,inv,nu {d[1]}  pdone wait+Bx reads {d[2]}  K,M,x,publish {d[3]}"
          f"  geometry(c+1)+cross update {s[b + 6] - s[b + 4]}  -> next {s[b + 8] - s[b + 6]}")
    print(f"   wave3: pub seen at {s[192 + 2 * c] - s[b]}, pdone at {s[193 + 2 * c] - s[b]} "
          f"(wave0 publish at {s[b + 4] - s[b]}, next-step pdone wait at {s[b + 8 + 2] - s[b]})")
    print(f"   wave1 Z_c done at {s[320 + c] - s[b]}, wave2 Y_c done at {s[360 + c] - s[b]} (from wave 0's step start)")
    if os.environ.get("EKF_STAMP_JOSEPH") == "1":
        print(f"   wave1 pub seen {s[460 + c] - s[b]}, C done {s[480 + c] - s[b]}; wave2 pub seen "
              f"{s[400 + c] - s[b]}, zdone seen {s[420 + c] - s[b]}, D done {s[440 + c] - s[b]}")
