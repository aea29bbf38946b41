"""Round-2 diagnostic: the chain's initial block Σ[U, U] (predict folded in) at the first chunk
of a replay prefix in the device-epoch and the event-synchronised schedule, from the diag
library's dump (EKF_LIB=libekfslam_diag.so, `make -C ekf-slam_amd diag`). Prints which block
entries differ, classified by whether their row / column index is new to the chunk."""
import os
import sys

os.environ["EKF_LIB"] = "libekfslam_diag.so"
sys.argv = [sys.argv[0]]
HERE = os.path.dirname(os.path.abspath(__file__))
exec(open(os.path.join(HERE, "diag_numeric.py")).read().split("for env in ({},)")[0])
import ctypes as C  # noqa: E402

lib = pyekf.lib()
P = int(os.environ.get("DIAG_PREFIX", "33"))
t = P - 1


def blocks(env):
    state_after(P, env)
    b = np.zeros((64, 35, 36))
    x = np.zeros((64, 35))
    assert lib.ekfslam_diag_read_blocks(b.ctypes.data_as(C.c_void_p), x.ctypes.data_as(C.c_void_p)) == 0
    return b[t & 63, :, :35], x[t & 63]


bc, xc = blocks({})
bn, xn = blocks({"EKF_DEVSYNC": "0"})
U, Up = ucols(t), ucols(t - 1)
nu = len(U)
new = [u not in Up for u in U]
print(f"chunk {t}: |U| {nu}, new positions {[a for a in range(nu) if new[a]]}", flush=True)
D = np.abs(bc[:nu, :nu] - bn[:nu, :nu])
print(f"x[U] max dev {np.abs(xc[:nu] - xn[:nu]).max():.3e} at {np.argmax(np.abs(xc[:nu] - xn[:nu]))}")
for kind, sel in (("old-old", lambda a, b: not new[a] and not new[b]),
                  ("old-new", lambda a, b: not new[a] and new[b]),
                  ("new-old", lambda a, b: new[a] and not new[b]),
                  ("new-new", lambda a, b: new[a] and new[b])):
    ents = [(a, b) for a in range(nu) for b in range(nu) if sel(a, b)]
    dv = [D[a, b] for a, b in ents]
    worst = sorted(zip(dv, ents), reverse=True)[:5]
    print(f"{kind}: {len(ents)} entries, max dev {max(dv) if dv else 0:.3e}; worst "
          f"{[(e, f'{d:.2e}', f'{bc[e]:.6e}', f'{bn[e]:.6e}') for d, e in worst]}", flush=True)
