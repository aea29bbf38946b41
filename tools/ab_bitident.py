"""Dev tool: is a rebuilt library bit-identical to a reference build on the GPU?

  python tools/ab_bitident.py <libA.so> <libB.so>   (names inside ekf-slam_amd/, EKF_LIB)

Each library runs the same replays in its own child process (the headline fp32 N = 1024 device
replay from an fp64 survey, fp64 N = 1024, messages of two chunks, the Joseph form, four filters
with event hand-offs, unknown association); the final states are compared bit for bit. A pure
performance change of the kernels (same formulas, same summation order) must print "identical"."""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, "gpurun_out")


def child(tag):
    sys.path.insert(0, os.path.join(ROOT, "ekf-slam_amd"))
    import pyekf
    from pyekf import synth
    res = {}

    def env(**kv):
        for k in ("EKF_SERIAL", "EKF_DEVSYNC", "EKF_STAGE", "EKF_CU_SPLIT"):
            os.environ.pop(k, None)
        os.environ.update(kv)

    def keep(name, e, F=1):
        for f in range(F):
            x, S, c = e.state(f)
            res[f"{name}_x{f}"], res[f"{name}_S{f}"] = x, S
            res[f"{name}_st{f}"] = np.array([e.status(f), c])

    # headline: fp64 survey, then fp32 N = 1024 through the device planner, and fp64 host-planned
    env()
    N, warm, T = 1024, 40, 24
    sc = synth.synthetic(N, warm + T)
    odom = pyekf.odometry(sc)
    e64 = pyekf.EKF(n_landmarks=N)
    e64.replay(sc.count[:warm, None], sc.rel[:warm, None], odom[:warm, None],
               ids=sc.ids[:warm, None], actions=sc.actions[:warm, None])
    x0, S0, c0 = e64.state()
    tmo = e64.map_odom()
    keep("survey64", e64)
    sl = slice(warm, warm + T)
    e64.replay(sc.count[sl, None], sc.rel[sl, None], odom[sl, None], ids=sc.ids[sl, None],
               actions=sc.actions[sl, None])
    keep("n1024_f64", e64)
    e64.close()
    import torch
    g = [torch.from_numpy(np.ascontiguousarray(a[sl, None])).cuda() for a in
         (sc.count, sc.ids, sc.actions, sc.rel, odom)]
    e = pyekf.EKF(n_landmarks=N, dtype=pyekf.EKF_F32)
    e.set_state(x0, S0, tmo=tmo, counter=c0)
    e.replay_device(g[0], g[3], g[4], g[1], g[2])
    keep("n1024_f32_dev", e)
    e.close()
    # messages of two chunks, fp64, device epochs and events
    sc = synth.synthetic(96, 14, max_markers=24)
    odom = pyekf.odometry(sc)
    for name, kv in (("multi_dev", {}), ("multi_evt", {"EKF_DEVSYNC": "0"})):
        env(**kv)
        e = pyekf.EKF(n_landmarks=96)
        e.replay(sc.count[:, None], sc.rel[:, None], odom[:, None], ids=sc.ids[:, None],
                 actions=sc.actions[:, None])
        keep(name, e)
        e.close()
    # Joseph
    env()
    e = pyekf.EKF(n_landmarks=96)
    e.set_joseph(True)
    e.replay(sc.count[:, None], sc.rel[:, None], odom[:, None], ids=sc.ids[:, None],
             actions=sc.actions[:, None])
    keep("joseph", e)
    e.close()
    # four filters, N = 256, events; and one stream
    sc = synth.synthetic(256, 20)
    odom = pyekf.odometry(sc)
    rep = lambda a: np.ascontiguousarray(np.repeat(a[:, None], 4, 1))  # noqa: E731
    for name, kv in (("f4_evt", {"EKF_DEVSYNC": "0"}), ("f4_ser", {"EKF_SERIAL": "1"})):
        env(**kv)
        e = pyekf.EKF(n_landmarks=256, n_filters=4)
        e.replay(rep(sc.count), rep(sc.rel), rep(odom), ids=rep(sc.ids), actions=rep(sc.actions))
        keep(name, e, 4)
        e.close()
    # unknown association (sensor_cb), fp64 and fp32
    env()
    sc = synth.synthetic(96, 20, shuffle=True)
    odom = pyekf.odometry(sc)
    for name, dt in (("assoc64", pyekf.EKF_F64), ("assoc32", pyekf.EKF_F32)):
        e = pyekf.EKF(n_landmarks=96, dtype=dt)
        e.replay(sc.count[:, None], sc.rel[:, None], odom[:, None], ids=None,
                 actions=sc.actions[:, None], assoc=True)
        keep(name, e)
        e.close()
    # digests only (a whole fp64 Σ at N = 1024 is 34 MB): bit-identical ⇔ equal digests
    import hashlib
    import json
    dig = {k: [hashlib.sha256(np.ascontiguousarray(v).tobytes()).hexdigest(),
               float(np.nansum(np.abs(v.astype(float))))] for k, v in res.items()}
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, f"ab_{tag}.json"), "w") as fh:
        json.dump(dig, fh)


def main():
    if len(sys.argv) == 3 and sys.argv[1] == "--child":
        return child(sys.argv[2])
    a, b = sys.argv[1], sys.argv[2]
    for lib in (a, b):
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", lib],
                           env=dict(os.environ, EKF_LIB=lib), timeout=600)
        if r.returncode:
            print(f"child {lib} failed: rc {r.returncode}")
            return r.returncode
    import json
    A = json.load(open(os.path.join(OUT, f"ab_{a}.json")))
    B = json.load(open(os.path.join(OUT, f"ab_{b}.json")))
    bad = [f"{k}: sum|v| {A[k][1]:.17g} vs {B[k][1]:.17g}" for k in A if A[k][0] != B.get(k, [""])[0]]
    print("identical" if not bad else "DIFFER:\n  " + "\n  ".join(bad))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
