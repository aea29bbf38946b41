"""Round-2 diagnostic: a populated N=1024 fp64 survey variant (inward spiral from
half·√2 − 1 + ring·0.75 with 4 m rings, survey range = max_range) on which the GPU set
EKF_FLAG_NUMERIC while the C oracle reported no skip. Bisects the persistent replay to the first
flagged message, then replays up to it message by message (synchronised) and prints the oracle's
innovation covariance S for each marker of that message."""
import math
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "ekf-slam_amd"), os.path.join(ROOT, "oracle")]
import numpy as np  # noqa: E402

import orc  # noqa: E402
import pyekf  # noqa: E402
from pyekf import synth  # noqa: E402


def survey_r2b(half, n_messages, ring=4.0, v_survey=4.0, circle_radius=1.0, omega=0.5,
               tick_hz=200.0, ticks_per_msg=40, max_range=5.0):
    dt = 1.0 / tick_hz
    r_max = max(half * math.sqrt(2.0) - (max_range - 1.0) + 0.75 * ring, circle_radius + ring)
    phi0 = 0.25 * math.pi
    r, v, w = r_max, [], []
    while r > circle_radius:
        om = v_survey / r
        v.append(v_survey)
        w.append(om)
        r -= ring / (2.0 * math.pi) * om * dt
    nw = -(-len(v) // ticks_per_msg)
    pad = nw * ticks_per_msg - len(v)
    v += [v_survey] * pad
    w += [v_survey / circle_radius] * pad
    c = synth.circle_drive(n_messages, circle_radius, omega, tick_hz, ticks_per_msg)
    sense = np.concatenate([np.full(nw, synth.SENSE_SURVEY, np.int32), c.sense])
    return synth.Drive(np.concatenate([np.array(v), c.v]), np.concatenate([np.array(w), c.w]),
                       sense, ticks_per_msg, tick_hz, nw,
                       start_pose=(phi0 + 0.5 * math.pi, r_max * math.cos(phi0),
                                   r_max * math.sin(phi0)))


synth.SURVEY_RANGE = 1.0
N = 1024
half = synth.field_half(N)
sw = synth._generate(N, survey_r2b(half, 10), [20240317], half=half)
sc = sw.scenario(0)
odom = pyekf.odometry(sc)
W = sc.n_messages
print(f"messages {W}, survey {sc.n_warm}, unsighted {int((~sw.sighted).sum())}", flush=True)


def status_after(upto, env=None):
    for k in ("EKF_SERIAL", "EKF_DEVSYNC"):
        os.environ.pop(k, None)
    os.environ.update(env or {})
    e = pyekf.EKF(n_landmarks=N)
    sl = slice(0, upto)
    e.replay(sc.count[sl, None], sc.rel[sl, None], odom[sl, None], ids=sc.ids[sl, None],
             actions=sc.actions[sl, None])
    st = e.status()
    x, S, _ = e.state()
    e.close()
    return st, x, S


def state_after(upto, env):
    for k in ("EKF_SERIAL", "EKF_DEVSYNC"):
        os.environ.pop(k, None)
    os.environ.update(env)
    e = pyekf.EKF(n_landmarks=N)
    sl = slice(0, upto)
    e.replay(sc.count[sl, None], sc.rel[sl, None], odom[sl, None], ids=sc.ids[sl, None],
             actions=sc.actions[sl, None])
    x, S, _ = e.state()
    e.close()
    return x, S


def ucols(t):
    c = int(sc.count[t])
    return [0, 1, 2] + [v for j in sc.ids[t, :c] for v in (3 + 2 * int(j), 4 + 2 * int(j))]


for env in ({},):  # (the device-epoch default)
    lo, hi = 0, W
    def bad(k):
        xd, Sd = state_after(k, env)
        xe, Se = state_after(k, {"EKF_DEVSYNC": "0"})
        return np.abs(xd - xe).max() > 1e-6 or not np.isfinite(Sd).all() or \
            np.abs(Sd - Se).max() > 1e-6
    if not bad(W):
        print(f"{env}: devsync equals events over the whole replay", flush=True)
        continue
    while hi - lo > 1:
        mid = (lo + hi) // 2
        if bad(mid):
            hi = mid
        else:
            lo = mid
    t = hi - 1
    xd, Sd = state_after(hi, env)
    xe, Se = state_after(hi, {"EKF_DEVSYNC": "0"})
    D = np.abs(Sd - Se)
    D[~np.isfinite(D)] = 1e300
    r, c = np.nonzero(D > 1e-6)
    print(f"{env}: first deviating message {t} (count {int(sc.count[t])}); x dev "
          f"{np.abs(xd - xe).max():.3e}; Σ bad entries {len(r)}", flush=True)
    U, Up, Upp = ucols(t), ucols(t - 1), ucols(t - 2)
    print("  U   ", U, flush=True)
    print("  U'  ", Up, flush=True)
    print("  U'' ", Upp, flush=True)
    print("  new in U vs U':", [u for u in U if u not in Up], flush=True)
    rows = sorted(set(r.tolist()))
    cols = sorted(set(c.tolist()))
    print(f"  bad rows ({len(rows)}): {rows[:40]}", flush=True)
    print(f"  bad cols ({len(cols)}): {cols[:40]}", flush=True)
    print(f"  bad x: {np.nonzero(np.abs(xd - xe) > 1e-6)[0][:40].tolist()}", flush=True)

for env in ({}, {"EKF_DEVSYNC": "0"}, {"EKF_SERIAL": "1"}):
    st, _, _ = status_after(W, env)
    print(f"{env}: full replay status {st}", flush=True)
st, _, _ = status_after(W)
if st:
    lo, hi = 0, W
    while hi - lo > 1:
        mid = (lo + hi) // 2
        if status_after(mid)[0]:
            hi = mid
        else:
            lo = mid
    t = hi - 1
    c = int(sc.count[t])
    print(f"first flagged message {t}: count {c} ids {sc.ids[t, :c].tolist()}", flush=True)
    print(f"previous ids {sc.ids[t - 1, :int(sc.count[t - 1])].tolist()}", flush=True)
    _, xg, Sg = status_after(t)
    ref = orc.OracleEKF(n_landmarks=N)
    for k in range(t):
        ref.set_odom(odom[k])
        ck = int(sc.count[k])
        ref.fake_sensor_cb(sc.ids[k, :ck], sc.actions[k, :ck], sc.rel[k, :ck])
    xr, Sr, _, _ = ref.get()
    print(f"state before it: |dx| {np.abs(xg - xr).max():.3e} |dS| {np.abs(Sg - Sr).max():.3e} "
          f"finite {np.isfinite(Sg).all()}", flush=True)
    for j in sc.ids[t, :c]:
        a = 3 + 2 * int(j)
        print(f"  id {int(j)}: x {xr[a]:.4f} {xr[a + 1]:.4f} var {Sr[a, a]:.4e} "
              f"gpu var {Sg[a, a]:.4e}", flush=True)
    ref.set_odom(odom[t])
    print("oracle rc", ref.fake_sensor_cb(sc.ids[t, :c], sc.actions[t, :c], sc.rel[t, :c]))
