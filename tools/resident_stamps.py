"""Dev tool: s_memtime phase stamps of the resident kernel (thread 0, first workgroup) over the
first 64 known-association corrections of a basic_world-sized replay (libekfslam_diag.so;
build: make -C ekf-slam_amd diag). Per correction: 0 start, 5 gather issued, 1 after the barrier,
2 geometry (ẑ, H), 3 S, S⁻¹, ν, 4 update done."""
import ctypes as C
import os
import sys

import numpy as np

os.environ["EKF_LIB"] = "libekfslam_diag.so"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ekf-slam_amd"))
import pyekf  # noqa: E402
from pyekf import synth  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 50
assoc = len(sys.argv) > 2 and sys.argv[2] == "assoc"
sc = synth.make_scenario(N, synth.random_landmarks(20, seed=5), 30, max_markers=4, shuffle=assoc)
odom = pyekf.odometry(sc)
e = pyekf.EKF(n_landmarks=N)
print("path", e.path, "assoc" if assoc else "known")
e.replay(sc.count[:, None], sc.rel[:, None], odom[:, None], ids=None if assoc else sc.ids[:, None],
         actions=sc.actions[:, None], assoc=assoc)
e.sync()
L = pyekf.lib()
st = (C.c_ulonglong * 512)()
L.ekf_diag_res_stamps.argtypes = [C.c_void_p, C.c_int]
assert L.ekf_diag_res_stamps(st, 512) == 0
s = np.array(st[:], dtype=np.int64).reshape(64, 8)
for k in range(0, 24):
    r = s[k]
    nxt = s[k + 1][0] - r[0]
    pre = (f"gatherA+barrier {r[6]-r[0]:5d} wave0 assoc+barrier {r[7]-r[6]:5d} gatherB {r[5]-r[7]:5d}"
           if assoc else f"gather {r[5]-r[0]:5d}")
    print(f"corr {k:2d}: {pre} barrier {r[1]-r[5]:5d} geom {r[2]-r[1]:5d} "
          f"S {r[3]-r[2]:5d} update {r[4]-r[3]:5d} -> next start {nxt:6d}")
