"""Dev diagnostic for the event-schedule hand-over (tools/diag_handover.py): the same 36-filter device
replay with EKF_DBG_ORDER=4096 (+ extra bits), which makes every chain log checksums of what it read
and wrote and runs a checksum kernel before each chain (Σ_in', x_in', record', t_map_odom as left in
memory), after each factor kernel (x_out, Kcat, Mcat) and after each Σ pass (Σ_out). The serial
schedule's log is the reference; for every events run whose final state differs, the first
(launch, kind, filter, slot) whose checksum differs is printed. Usage: diag_dlog.py [runs] [extra EKF_DBG_ORDER bits, e.g. 8192 for
the checksum kernels]."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the EKF_DBG_ORDER instrumentation is compiled into the diagnostic library only
os.environ.setdefault("EKF_LIB", "libekfslam_diag.so")  # (make -C ekf-slam_amd diag)
sys.path[:0] = [os.path.join(ROOT, "ekf-slam_amd"), os.path.join(ROOT, "oracle"),
                os.path.join(ROOT, "tools")]
import pyekf  # noqa: E402
import diag_handover as dh  # noqa: E402

KINDS = 21
STEP0 = 5  # kChainLogKind: chain step c logs as kind 5 + c (wave 0)
KNAME = {3: "pre-chain memory", 0: "chain reads/writes", 4: "factor reads/writes",
         1: "after factors", 2: "after pass"}
SLOTS = {3: ["Σ_in'", "x_in'", "rec'", "tmo", "Σ_in", "x_in"],
         0: ["desc", "tmo", "Σ' gathered", "x'", "rec' loaded", "rec out", "tmo out", "-"],
         1: ["x_out", "Kcat", "Mcat"], 2: ["Σ_out"],
         4: ["desc", "record read", "Σ_in rows read", "x_in read", "x_out written"]}
for _c in range(16):
    KNAME[STEP0 + _c] = f"chain step {_c}"
    SLOTS[STEP0 + _c] = ["S, S^-1 (lane 0)", "nu, zhat, H (lane 0)", "ka kb mm (rows)",
                         "xr xq cross operands", "K (rows)", "x after step", "pk pm after cross",
                         "rn qn read ahead"]


def run(env, spans=((0, 30),), kinds=("device",)):
    import torch
    for k in ("EKF_SERIAL", "EKF_CU_SPLIT", "EKF_DEVSYNC", "EKF_STAGE", "EKF_DBG_ORDER"):
        os.environ.pop(k, None)
    os.environ.update(env)
    e = pyekf.EKF(n_landmarks=dh.N, n_filters=dh.F)
    keep = []
    for (t0, t1), kind in zip(spans, kinds):
        a = tuple(np.ascontiguousarray(v[t0:t1]) for v in dh.FULL)
        if kind == "device":
            g = tuple(torch.from_numpy(v).cuda() for v in a)
            keep.append(g)
            e.replay_device(g[0], g[3], g[4], g[1], g[2])
        else:
            e.replay(a[0], a[3], a[4], ids=a[1], actions=a[2])
    xs = np.stack([e.state(f, sigma=False)[0] for f in range(dh.F)])
    log = np.zeros(KINDS * 64 * 64 * 8, np.uint64)
    pyekf._check(pyekf.lib().ekf_debug_log(e.h, log.ctypes.data_as(C.POINTER(C.c_ulonglong))),
                 "ekf_debug_log")
    e.close()
    return xs, log.reshape(KINDS, 64, 64, 8)


def first_diffs(log, ref, limit=12):
    out = []
    for seq in range(64):
        for kind in (3, 0, *range(STEP0, STEP0 + 16), 4, 1, 2):
            ne = log[kind, seq] != ref[kind, seq]
            if kind == 3:  # Σ_in / x_in before a kLook chain: the pass before may still run (events)
                ne[:, 4:] = False
            d = np.nonzero(ne)
            for f, slot in zip(*d):
                out.append((seq, KNAME[kind], int(f), SLOTS[kind][slot] if slot < len(SLOTS[kind])
                            else slot))
            if len(out) >= limit:
                return out
    return out


def main():
    runs = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    bits = 4096 + (int(sys.argv[2]) if len(sys.argv) > 2 else 0)
    pyekf.poison_lds()
    ref_x, ref = run({"EKF_SERIAL": "1", "EKF_DBG_ORDER": str(bits)})
    x2, ref2 = run({"EKF_SERIAL": "1", "EKF_DBG_ORDER": str(bits)})
    print(f"serial twice: state equal {np.array_equal(ref_x, x2)}, log equal "
          f"{np.array_equal(ref, ref2)}", flush=True)
    for r in range(runs):
        xs, log = run({"EKF_SERIAL": "0", "EKF_DBG_ORDER": str(bits)})
        d = np.abs(xs - ref_x).max(axis=1)
        bad = np.nonzero(d > 1e-9)[0]
        lg, rf = log.copy(), ref.copy()
        lg[3, :, :, 4:] = rf[3, :, :, 4:] = 0
        same_log = np.array_equal(lg, rf)
        print(f"run {r}: {len(bad)} filters off {[(int(f), round(float(d[f]), 4)) for f in bad[:4]]}, "
              f"log equal {same_log}", flush=True)
        if not same_log:
            for t in first_diffs(log, ref):
                print("    first diff: launch %d, %s, filter %d, %s" % t, flush=True)


if __name__ == "__main__":
    main()
