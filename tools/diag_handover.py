"""Dev diagnostic: the 36-filter device → device → host hand-over of
tests/test_gpu_replay_device.py::test_device_device_host_handover_36_filters under the two-stream
event schedule (EKF_SERIAL=0), repeated in one process per hand-off variant (EKF_DBG_ORDER bit mask,
ekf_api.cpp) and per span layout, each run against the whole drive planned on the host (one
stream). Prints per (variant, layout) the failing runs and, for each, the failing filters and their
largest state difference. Usage: diag_handover.py [repetitions]."""
import os
import sys
import time

import ctypes as C

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the EKF_DBG_ORDER instrumentation is compiled into the diagnostic library only
os.environ.setdefault("EKF_LIB", "libekfslam_diag.so")  # (make -C ekf-slam_amd diag)
sys.path[:0] = [os.path.join(ROOT, "ekf-slam_amd"), os.path.join(ROOT, "oracle")]
import pyekf  # noqa: E402
from pyekf import synth  # noqa: E402

F, N, T = 36, 96, 30
SCS = [synth.synthetic(N, T, seed=51 + k) for k in range(4)]


def inputs():
    M = max(s.ids.shape[1] for s in SCS)
    cnt = np.zeros((T, F), np.int32)
    ids = np.zeros((T, F, M), np.int32)
    act = np.zeros((T, F, M), np.int32)
    rel = np.zeros((T, F, M, 2))
    od = np.zeros((T, F, 3))
    for f in range(F):
        s = SCS[f % len(SCS)]
        k = s.ids.shape[1]
        cnt[:, f] = s.count[:T]
        ids[:, f, :k] = s.ids[:T]
        act[:, f, :k] = s.actions[:T]
        rel[:, f, :k] = s.rel[:T]
        od[:, f] = pyekf.odometry(s)[:T]
    cnt[1::3, 1] = 0
    act[2::4, F - 1] = synth.DELETE
    return cnt, ids, act, rel, od


FULL = inputs()


def run(spans, kinds, env):
    import torch
    for k in ("EKF_SERIAL", "EKF_CU_SPLIT", "EKF_DEVSYNC", "EKF_STAGE", "EKF_DBG_ORDER"):
        os.environ.pop(k, None)
    os.environ.update(env)
    e = pyekf.EKF(n_landmarks=N, n_filters=F)
    keep = []
    for (t0, t1), kind in zip(spans, kinds):
        cnt, ids, act, rel, od = (np.ascontiguousarray(a[t0:t1]) for a in FULL)
        if kind == "device":
            g = tuple(torch.from_numpy(a).cuda() for a in (cnt, ids, act, rel, od))
            keep.append(g)
            e.replay_device(g[0], g[3], g[4], g[1], g[2])
        else:
            e.replay(cnt, rel, od, ids=ids, actions=act)
    xs = np.stack([e.state(f, sigma=False)[0] for f in range(F)])
    st = [e.status(f) for f in range(F)]
    cnt = (C.c_uint * 6)()
    if int(env.get("EKF_DBG_ORDER", "0")) & (1024 | 2048):
        pyekf._check(pyekf.lib().ekf_debug_counters(e.h, cnt, 6), "ekf_debug_counters")
    e.close()
    return xs, st, list(cnt)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    pyekf.poison_lds()
    layouts = {
        "d,d,h": ([(0, 11), (11, 20), (20, 30)], ["device", "device", "host"]),
        "d,d": ([(0, 11), (11, 20)], ["device", "device"]),
        "d": ([(0, 30)], ["device"]),
        "h,h,h": ([(0, 11), (11, 20), (20, 30)], ["host", "host", "host"]),
    }
    refs = {}
    for name, (spans, _) in layouts.items():
        end = spans[-1][1]
        refs[name] = run([(0, end)], ["host"], {})[0]
    variants = [0, 2048, 3072, 768 + 2048, 1 + 2048]
    if len(sys.argv) > 2:
        variants = [int(v) for v in sys.argv[2].split(",")]
    t0 = time.time()
    for name, (spans, kinds) in layouts.items():
        for v in variants:
            fails, cnts = [], [0] * 6
            for r in range(reps):
                xs, st, cn = run(spans, kinds, {"EKF_SERIAL": "0", "EKF_DBG_ORDER": str(v)})
                cnts = [a + b for a, b in zip(cnts, cn)]
                d = np.abs(xs - refs[name]).max(axis=1)
                bad = np.nonzero(d > 1e-9)[0]
                if len(bad) or any(st):
                    fails.append((r, [(int(f), float(d[f])) for f in bad[:6]], len(bad),
                                  [s for s in st if s]))
            print(f"[{time.time() - t0:6.1f}s] layout {name:6s} dbg {v:3d}: {len(fails)}/{reps} "
                  f"failed; unseen producer epochs: chains {cnts[0]}, factors {cnts[1]} "
                  f"(of {cnts[2]} chain checks); stale launch epochs: chain {cnts[3]}, factors {cnts[4]}, "
                  f"pass {cnts[5]}", flush=True)
            for fl in fails:
                print(f"    run {fl[0]}: {fl[2]} filters off, first {fl[1]}, status {fl[3]}",
                      flush=True)


if __name__ == "__main__":
    main()
