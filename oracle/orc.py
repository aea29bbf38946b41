"""ctypes binding of the C oracle (oracle/ekf_oracle.c).

ORACLE — TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the product package.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "libekf_oracle.so")
_lib = None

_dp = np.ctypeslib.ndpointer(dtype=np.float64, flags="C_CONTIGUOUS")
_ip = np.ctypeslib.ndpointer(dtype=np.int32, flags="C_CONTIGUOUS")


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        L.orc_normalize_angle.restype = C.c_double
        L.orc_normalize_angle.argtypes = [C.c_double]
        for fn in ("orc_tf_compose",):
            getattr(L, fn).argtypes = [_dp, _dp, _dp]
        L.orc_tf_inv.argtypes = [_dp, _dp]
        L.orc_integrate_twist.argtypes = [C.c_double, C.c_double, C.c_double, _dp]
        L.orc_fkin.argtypes = [_dp, C.c_double, C.c_double, _dp]
        L.orc_ekf_create.restype = C.c_void_p
        L.orc_ekf_create.argtypes = [C.c_int, C.c_double, C.c_double, C.c_double, C.c_double,
                                     C.c_int]
        L.orc_ekf_destroy.argtypes = [C.c_void_p]
        L.orc_ekf_dim.argtypes = [C.c_void_p]
        L.orc_ekf_set_odom.argtypes = [C.c_void_p, C.c_double, C.c_double, C.c_double]
        L.orc_ekf_predict.argtypes = [C.c_void_p]
        L.orc_ekf_correct.argtypes = [C.c_void_p, C.c_int, C.c_double, C.c_double]
        L.orc_ekf_associate_correct.argtypes = [C.c_void_p, C.c_double, C.c_double,
                                                C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.orc_ekf_posterior.argtypes = [C.c_void_p]
        L.orc_ekf_fake_sensor_cb.argtypes = [C.c_void_p, C.c_int, _ip, _ip, _dp]
        L.orc_ekf_sensor_cb.argtypes = [C.c_void_p, C.c_int, _dp, _ip, _ip]
        L.orc_ekf_get.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        L.orc_ekf_set.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                  C.c_uint]
        L.orc_ekf_get_prev.argtypes = [C.c_void_p, _dp]
        L.orc_ekf_set_joseph.argtypes = [C.c_void_p, C.c_int]
        L.orc_ekf_last_dmin.restype = C.c_double
        L.orc_ekf_last_dmin.argtypes = [C.c_void_p]
        _lib = L
    return _lib


def normalize_angle(a: float) -> float:
    return lib().orc_normalize_angle(a)


def tf_compose(a, b):
    out = np.zeros(3)
    lib().orc_tf_compose(np.asarray(a, float), np.asarray(b, float), out)
    return out


def tf_inv(a):
    out = np.zeros(3)
    lib().orc_tf_inv(np.asarray(a, float), out)
    return out


def integrate_twist(w, vx, vy):
    out = np.zeros(3)
    lib().orc_integrate_twist(w, vx, vy, out)
    return out


class DiffDrive:
    def __init__(self, track, radius):
        self.dd = np.array([track, radius, 0, 0, 0, 0, 0], dtype=np.float64)

    def fkin(self, left, right):
        out = np.zeros(3)
        lib().orc_fkin(self.dd, float(left), float(right), out)
        return out


class OracleEKF:
    """One filter of the C oracle. literal=True is the reference's dense O(n³) arithmetic."""

    def __init__(self, n_landmarks=50, q_noise=1e-2, r_noise=1e-2, init_var=10e6,
                 mah_gate=2.0, literal=False, joseph=False):
        self.N = n_landmarks
        self.n = 3 + 2 * n_landmarks
        self.h = lib().orc_ekf_create(n_landmarks, q_noise, r_noise, init_var, mah_gate,
                                      int(literal))
        if joseph:
            lib().orc_ekf_set_joseph(self.h, 1)

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_ekf_destroy(self.h)
            self.h = None

    def set_odom(self, pose):
        lib().orc_ekf_set_odom(self.h, float(pose[0]), float(pose[1]), float(pose[2]))

    def predict(self):
        lib().orc_ekf_predict(self.h)

    def correct(self, mid, rx, ry) -> int:
        return lib().orc_ekf_correct(self.h, int(mid), float(rx), float(ry))

    def posterior(self):
        lib().orc_ekf_posterior(self.h)

    def fake_sensor_cb(self, ids, actions, rel_xy) -> int:
        ids = np.ascontiguousarray(ids, dtype=np.int32)
        act = np.ascontiguousarray(actions, dtype=np.int32)
        rel = np.ascontiguousarray(rel_xy, dtype=np.float64).reshape(-1)
        return lib().orc_ekf_fake_sensor_cb(self.h, len(ids), ids, act, rel)

    def sensor_cb(self, rel_xy):
        rel = np.ascontiguousarray(rel_xy, dtype=np.float64).reshape(-1)
        m = rel.size // 2
        j = np.zeros(max(m, 1), dtype=np.int32)
        nw = np.zeros(max(m, 1), dtype=np.int32)
        rc = lib().orc_ekf_sensor_cb(self.h, m, rel, j, nw)
        return rc, j[:m], nw[:m]

    def sensor_cb_dmin(self, rel_xy):
        """sensor_cb (slam.cpp:318-530) marker by marker, as orc_ekf_sensor_cb runs it, also
        returning each marker's smallest existing Mahalanobis distance (tests near the gate)."""
        rel = np.ascontiguousarray(rel_xy, dtype=np.float64).reshape(-1, 2)
        m = rel.shape[0]
        j = np.zeros(m, dtype=np.int32)
        nw = np.zeros(m, dtype=np.int32)
        dmin = np.zeros(m)
        rc = -3 if m == 0 else 0
        if m:
            lib().orc_ekf_predict(self.h)
            for i in range(m):
                jj, nn = C.c_int(-1), C.c_int(0)
                e = lib().orc_ekf_associate_correct(self.h, float(rel[i, 0]), float(rel[i, 1]),
                                                    C.byref(jj), C.byref(nn))
                j[i], nw[i] = jj.value, nn.value
                dmin[i] = lib().orc_ekf_last_dmin(self.h)
                if e and not rc:
                    rc = e
            lib().orc_ekf_posterior(self.h)
        return rc, j, nw, dmin

    def get(self, sigma=True):
        x = np.zeros(self.n)
        S = np.zeros((self.n, self.n)) if sigma else None
        tmo = np.zeros(3)
        cnt = C.c_uint(0)
        lib().orc_ekf_get(self.h, x.ctypes.data, S.ctypes.data if sigma else None,
                          tmo.ctypes.data, C.addressof(cnt))
        return x, S, tmo, cnt.value

    def prev(self):
        p = np.zeros(3)
        lib().orc_ekf_get_prev(self.h, p)
        return p

    def set(self, state=None, sigma=None, tmo=None, prev=None, counter=0):
        keep = [None if a is None else np.ascontiguousarray(a, dtype=np.float64)
                for a in (state, sigma, tmo, prev)]
        lib().orc_ekf_set(self.h, *(None if a is None else a.ctypes.data for a in keep),
                          int(counter))


def run_scenario(sc, assoc: bool, literal=False, **kw):
    """Drive the oracle through a synth.Scenario the way the reference node would."""
    ekf = OracleEKF(n_landmarks=sc.n_landmarks, literal=literal, **kw)
    dd = DiffDrive(sc.track, sc.radius)
    T = sc.n_messages
    M = sc.ids.shape[1]
    poses = np.zeros((T, 3))
    tmo = np.zeros((T, 3))
    aj = np.full((T, M), -1, dtype=np.int32)
    an = np.zeros((T, M), dtype=np.int32)
    rcs = np.zeros(T, dtype=np.int32)
    for t in range(T):
        for k in range(sc.wheel.shape[1]):
            ekf.set_odom(dd.fkin(sc.wheel[t, k, 0], sc.wheel[t, k, 1]))
        c = int(sc.count[t])
        if assoc:
            rc, j, nw = ekf.sensor_cb(sc.rel[t, :c])
            aj[t, :c] = j
            an[t, :c] = nw
        else:
            rc = ekf.fake_sensor_cb(sc.ids[t, :c], sc.actions[t, :c], sc.rel[t, :c])
        rcs[t] = rc
        x, _, tm, _ = ekf.get(sigma=False)
        poses[t] = x[:3]
        tmo[t] = tm
    x, S, tm, cnt = ekf.get()
    return dict(poses=poses, tmo=tmo, assoc_j=aj, assoc_new=an, state=x, sigma=S, counter=cnt,
                rcs=rcs)
