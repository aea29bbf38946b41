"""ctypes binding of libekfslam.so (include/ekf.h, include/slam_core.h, include/landmarks.h,
include/ekf_sim.h).

The binding is plumbing for tests and bench.py; the product is the C-ABI library. Loading fails
loudly when the HIP library has not been built — there is no CPU fallback anywhere in this package.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(PKG_DIR, os.environ.get("EKF_LIB", "libekfslam.so"))

EKF_OK, EKF_E_ARG, EKF_E_RANGE, EKF_E_EMPTY, EKF_E_NUMERIC, EKF_E_HIP, EKF_E_NOMEM = \
    0, -1, -2, -3, -4, -5, -6
EKF_E_TIMEOUT = -7
EKF_FLAG_RANGE, EKF_FLAG_NUMERIC, EKF_FLAG_TIMEOUT = 1, 2, 4
EKF_ASSOC_MARKER, EKF_ASSOC_CHUNK, EKF_ASSOC_CHUNK_XCD = 0, 1, 2
EKF_SCHED_DEVSYNC, EKF_SCHED_SERIAL = 1, 4
EKF_SCHED_BUILDER = 2  # deprecated, never set (include/ekf.h)
EKF_F64, EKF_F32 = 0, 1
EKF_PATH_PIPELINE, EKF_PATH_RESIDENT = 0, 1
ADD, DELETE = 0, 2
SOURCE_SIM, SOURCE_ASSOC = 0, 1

# every symbol include/ekf.h and include/slam_core.h declare
EXPORTS = [
    "ekf_config_default", "ekf_strerror", "ekf_create", "ekf_destroy", "ekf_dims", "ekf_get_path",
    "ekf_get_assoc_route", "ekf_get_schedule",
    "ekf_set_odom",
    "ekf_fake_sensor", "ekf_sensor", "ekf_batch_sensor", "ekf_replay", "ekf_replay_device",
    "ekf_predict",
    "ekf_correct", "ekf_associate_correct", "ekf_posterior", "ekf_sync", "ekf_flush", "ekf_get_pose",
    "ekf_get_map_odom", "ekf_get_state", "ekf_set_state", "ekf_get_status", "ekf_defer",
    "ekf_set_joseph",
    "ekf_reset", "slam_reset",
    "ekf_profile_enable", "ekf_profile_read", "ekf_sigma_pass_bytes", "ekf_normalize_angle",
    "ekf_debug_poison_lds",
    "slam_create", "slam_destroy", "slam_joint_states", "slam_markers", "slam_initial_pose",
    "slam_odom", "slam_map_odom", "slam_filter", "slam_replay", "slam_integrate_odometry",
    "lm_create", "lm_destroy", "lm_detect", "lm_fit_circles", "lm_check_circles",
    "lm_last_kernel_us",
    "ekf_sim_config_default", "ekf_sim_create", "ekf_sim_destroy", "ekf_sim_run",
    "ekf_sim_markers", "ekf_sim_poses",
]
SENSE_NEAREST, SENSE_SURVEY, SENSE_ALL = 0, 1, 2


class EkfError(RuntimeError):
    def __init__(self, rc: int, what: str = ""):
        self.rc = rc
        super().__init__(f"{what}: {lib().ekf_strerror(rc).decode()} ({rc})")


class SimConfig(C.Structure):
    _fields_ = [("seed", C.c_ulonglong), ("f0", C.c_int), ("ticks_per_msg", C.c_int),
                ("slip", C.c_double), ("sensor_sigma", C.c_double), ("max_range", C.c_double),
                ("max_markers", C.c_int), ("marker_stride", C.c_int),
                ("wheel_radius", C.c_double), ("track_width", C.c_double),
                ("start_theta", C.c_double), ("start_x", C.c_double), ("start_y", C.c_double),
                ("record", C.c_int)]


class Config(C.Structure):
    _fields_ = [("n_landmarks", C.c_int), ("n_filters", C.c_int), ("dtype", C.c_int),
                ("q_noise", C.c_double), ("r_noise", C.c_double), ("init_var", C.c_double),
                ("mah_gate", C.c_double), ("device", C.c_int)]


_lib = None
_vp, _ip, _dp, _i, _d = C.c_void_p, C.POINTER(C.c_int), C.POINTER(C.c_double), C.c_int, C.c_double


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: build it with `make -C {PKG_DIR}` "
                               "(or __graft_entry__.build()); there is no CPU fallback")
        L = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        sig = {
            "ekf_config_default": (None, [C.POINTER(Config)]),
            "ekf_strerror": (C.c_char_p, [_i]),
            "ekf_create": (_i, [C.POINTER(_vp), C.POINTER(Config)]),
            "ekf_destroy": (_i, [_vp]),
            "ekf_dims": (_i, [_vp, _ip, _ip, _ip]),
            "ekf_get_path": (_i, [_vp, _ip]),
            "ekf_get_assoc_route": (_i, [_vp, _ip]),
            "ekf_get_schedule": (_i, [_vp, _ip]),
            "ekf_set_odom": (_i, [_vp, _i, _d, _d, _d]),
            "ekf_fake_sensor": (_i, [_vp, _i, _i, _vp, _vp, _vp]),
            "ekf_sensor": (_i, [_vp, _i, _i, _vp, _vp, _vp]),
            "ekf_batch_sensor": (_i, [_vp, _i, _i, _vp, _vp, _vp, _vp, _vp]),
            "ekf_replay": (_i, [_vp, _i, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp]),
            "ekf_replay_device": (_i, [_vp, _i, _i, _vp, _vp, _vp, _vp, _vp]),
            "ekf_predict": (_i, [_vp, _i]),
            "ekf_correct": (_i, [_vp, _i, _i, _d, _d]),
            "ekf_associate_correct": (_i, [_vp, _i, _d, _d, _ip, _ip]),
            "ekf_posterior": (_i, [_vp, _i]),
            "ekf_sync": (_i, [_vp]),
            "ekf_flush": (_i, [_vp]),
            "ekf_get_pose": (_i, [_vp, _i, _vp]),
            "ekf_get_map_odom": (_i, [_vp, _i, _vp]),
            "ekf_get_state": (_i, [_vp, _i, _vp, _vp, _vp]),
            "ekf_set_state": (_i, [_vp, _i, _vp, _vp, _vp, C.c_uint]),
            "ekf_get_status": (_i, [_vp, _i, C.POINTER(C.c_uint)]),
            "ekf_defer": (_i, [_vp, _i]),
            "ekf_set_joseph": (_i, [_vp, _i]),
            "ekf_reset": (_i, [_vp, _i]),
            "slam_reset": (_i, [_vp]),
            "ekf_profile_enable": (_i, [_vp, _i]),
            "ekf_profile_read": (_i, [_vp, _i, C.POINTER(C.c_longlong), _dp]),
            "ekf_sigma_pass_bytes": (C.c_double, [_vp, _i]),
            "ekf_normalize_angle": (C.c_double, [_d]),
            "ekf_debug_poison_lds": (_i, [_i]),
            "slam_create": (_i, [C.POINTER(_vp), C.POINTER(Config), _d, _d, _i]),
            "slam_destroy": (_i, [_vp]),
            "slam_joint_states": (_i, [_vp, _d, _d]),
            "slam_markers": (_i, [_vp, _i, _vp, _vp, _vp]),
            "slam_initial_pose": (_i, [_vp, _d, _d, _d]),
            "slam_odom": (_i, [_vp, _vp]),
            "slam_map_odom": (_i, [_vp, _vp]),
            "slam_filter": (_vp, [_vp]),
            "slam_replay": (_i, [_vp, _i, _i, _vp, _i, _vp, _vp, _vp, _vp, _vp, _vp]),
            "slam_integrate_odometry": (_i, [_d, _d, _i, _i, _vp, _vp]),
            "lm_create": (_i, [C.POINTER(_vp), _i, _i, _i]),
            "lm_destroy": (_i, [_vp]),
            "lm_detect": (_i, [_vp, _i, _i, _vp, _vp, _vp, _d, _vp, _i, _vp]),
            "lm_fit_circles": (_i, [_vp, _i, _vp, _vp, _vp]),
            "lm_check_circles": (_i, [_vp, _i, _vp, _vp, _vp]),
            "lm_last_kernel_us": (_i, [_vp, _dp]),
            "ekf_sim_config_default": (None, [C.POINTER(SimConfig)]),
            "ekf_sim_create": (_i, [C.POINTER(_vp), _vp, C.POINTER(SimConfig), _i, _vp]),
            "ekf_sim_destroy": (_i, [_vp]),
            "ekf_sim_run": (_i, [_vp, _i, _vp, _vp]),
            "ekf_sim_markers": (_i, [_vp, _vp, _vp, _vp, _vp]),
            "ekf_sim_poses": (_i, [_vp, _vp, _vp]),
        }
        for name, (res, argt) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = argt
        _lib = L
    return _lib


def _ptr(a):
    return None if a is None else a.ctypes.data


def _dptr(x, dtype):
    """A device buffer for ekf_replay_device: None, an int address, or a contiguous torch tensor
    of the given dtype on the GPU."""
    if x is None or isinstance(x, int):
        return x
    if not (x.is_cuda and x.is_contiguous() and x.dtype == dtype):
        raise ValueError(f"device input must be a contiguous {dtype} GPU tensor")
    return x.data_ptr()


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def _i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


def make_config(n_landmarks=50, n_filters=1, dtype=EKF_F64, q_noise=1e-2, r_noise=1e-2,
                init_var=10e6, mah_gate=2.0, device=0) -> Config:
    c = Config()
    lib().ekf_config_default(C.byref(c))
    c.n_landmarks, c.n_filters, c.dtype = n_landmarks, n_filters, dtype
    c.q_noise, c.r_noise, c.init_var, c.mah_gate, c.device = (q_noise, r_noise, init_var,
                                                             mah_gate, device)
    return c


def _check(rc, what):
    if rc != EKF_OK:
        raise EkfError(rc, what)
    return rc


class EKF:
    """A handle of F independent filters (F = 1: one slam node's filter)."""

    def __init__(self, n_landmarks=50, n_filters=1, dtype=EKF_F64, **kw):
        self.cfg = make_config(n_landmarks, n_filters, dtype, **kw)
        h = C.c_void_p()
        _check(lib().ekf_create(C.byref(h), C.byref(self.cfg)), "ekf_create")
        self.h = h
        n, ld, nf = C.c_int(), C.c_int(), C.c_int()
        lib().ekf_dims(self.h, C.byref(n), C.byref(ld), C.byref(nf))
        self.n, self.ld, self.F = n.value, ld.value, nf.value
        self.N = n_landmarks
        p = C.c_int()
        _check(lib().ekf_get_path(self.h, C.byref(p)), "ekf_get_path")
        self.path = p.value  # EKF_PATH_PIPELINE | EKF_PATH_RESIDENT
        _check(lib().ekf_get_assoc_route(self.h, C.byref(p)), "ekf_get_assoc_route")
        self.assoc_route = p.value  # EKF_ASSOC_*
        _check(lib().ekf_get_schedule(self.h, C.byref(p)), "ekf_get_schedule")
        self.schedule = p.value  # EKF_SCHED_* bits

    def close(self):
        if getattr(self, "h", None):
            lib().ekf_destroy(self.h)
            self.h = None

    __del__ = close

    # callbacks
    def set_odom(self, pose, f=0):
        return lib().ekf_set_odom(self.h, f, float(pose[0]), float(pose[1]), float(pose[2]))

    def fake_sensor(self, ids, actions, rel_xy, f=0) -> int:
        ids, act, rel = _i32(ids), _i32(actions), _f64(rel_xy)
        return lib().ekf_fake_sensor(self.h, f, len(ids), _ptr(ids), _ptr(act), _ptr(rel))

    def sensor(self, rel_xy, f=0, decisions=True):
        rel = _f64(rel_xy)
        m = rel.size // 2
        j = np.zeros(max(m, 1), np.int32)
        nw = np.zeros(max(m, 1), np.int32)
        rc = lib().ekf_sensor(self.h, f, m, _ptr(rel), _ptr(j) if decisions else None,
                              _ptr(nw) if decisions else None)
        return rc, j[:m], nw[:m]

    def batch_sensor(self, counts, rel_xy, odom=None, ids=None, actions=None, assoc=False):
        counts, rel = _i32(counts), _f64(rel_xy)
        m_max = rel.shape[1]
        ids = None if ids is None else _i32(ids)
        actions = None if actions is None else _i32(actions)
        odom = None if odom is None else _f64(odom)
        return lib().ekf_batch_sensor(self.h, int(assoc), m_max, _ptr(counts), _ptr(ids),
                                      _ptr(actions), _ptr(rel), _ptr(odom))

    def replay(self, counts, rel_xy, odom, ids=None, actions=None, assoc=False, poses=False):
        """counts[T][F], rel_xy[T][F][M][2], odom[T][F][3]."""
        counts, rel, odom = _i32(counts), _f64(rel_xy), _f64(odom)
        T, M = rel.shape[0], rel.shape[2]
        ids = None if ids is None else _i32(ids)
        actions = None if actions is None else _i32(actions)
        out = np.zeros((T, self.F, 3)) if poses else None
        rc = lib().ekf_replay(self.h, int(assoc), T, M, _ptr(counts), _ptr(ids), _ptr(actions),
                              _ptr(rel), _ptr(odom), _ptr(out))
        _check(rc, "ekf_replay")
        return out

    def replay_device(self, counts, rel_xy, odom, ids, actions=None):
        """ekf_replay_device: known-id replay whose inputs are GPU tensors already on this handle's
        device — counts [T,F] int32, rel_xy [T,F,M,2] float64, odom [T,F,3] float64, ids / actions
        [T,F,M] int32 (M <= EKF_MAX_CHUNK). Asynchronous; keep the tensors alive until a sync."""
        import torch
        T, M = int(rel_xy.shape[0]), int(rel_xy.shape[2])
        rc = lib().ekf_replay_device(self.h, T, M, _dptr(counts, torch.int32),
                                     _dptr(ids, torch.int32), _dptr(actions, torch.int32),
                                     _dptr(rel_xy, torch.float64), _dptr(odom, torch.float64))
        _check(rc, "ekf_replay_device")

    def replay_device_raw(self, T, M, counts, rel_xy, odom, ids, actions=0):
        """ekf_replay_device on raw device addresses (ints: the same layouts as replay_device):
        no tensor work on the caller's path (bench.py's timed region)."""
        _check(lib().ekf_replay_device(self.h, T, M, counts, ids, actions or None, rel_xy, odom),
               "ekf_replay_device")

    # fine-grained
    def predict(self, f=0):
        return lib().ekf_predict(self.h, f)

    def correct(self, mid, rx, ry, f=0):
        return lib().ekf_correct(self.h, f, int(mid), float(rx), float(ry))

    def associate_correct(self, rx, ry, f=0):
        j, nw = C.c_int(-1), C.c_int(0)
        rc = lib().ekf_associate_correct(self.h, f, float(rx), float(ry), C.byref(j), C.byref(nw))
        return rc, j.value, nw.value

    def posterior(self, f=0):
        return lib().ekf_posterior(self.h, f)

    # state
    def sync(self):
        _check(lib().ekf_sync(self.h), "ekf_sync")

    def flush(self):
        """Submit what is planned, without waiting (ekf_flush)."""
        _check(lib().ekf_flush(self.h), "ekf_flush")

    def pose(self, f=0):
        p = np.zeros(3)
        _check(lib().ekf_get_pose(self.h, f, _ptr(p)), "ekf_get_pose")
        return p

    def map_odom(self, f=0):
        p = np.zeros(3)
        _check(lib().ekf_get_map_odom(self.h, f, _ptr(p)), "ekf_get_map_odom")
        return p

    def state(self, f=0, sigma=True):
        x = np.zeros(self.n)
        S = np.zeros((self.n, self.n)) if sigma else None
        cnt = C.c_uint(0)
        _check(lib().ekf_get_state(self.h, f, _ptr(x), _ptr(S), C.byref(cnt)), "ekf_get_state")
        return x, S, cnt.value

    def set_state(self, state, sigma=None, tmo=None, counter=0, f=0):
        state = _f64(state)
        sigma = None if sigma is None else _f64(sigma)
        tmo = None if tmo is None else _f64(tmo)
        _check(lib().ekf_set_state(self.h, f, _ptr(state), _ptr(sigma), _ptr(tmo), counter),
               "ekf_set_state")

    def defer(self, on=True):
        _check(lib().ekf_defer(self.h, int(on)), "ekf_defer")

    def reset(self, f=-1):
        _check(lib().ekf_reset(self.h, f), "ekf_reset")

    def set_joseph(self, on=True) -> int:
        return lib().ekf_set_joseph(self.h, int(on))

    def status(self, f=0) -> int:
        fl = C.c_uint(0)
        _check(lib().ekf_get_status(self.h, f, C.byref(fl)), "ekf_get_status")
        return fl.value

    def profile(self, enable=True):
        lib().ekf_profile_enable(self.h, int(enable))

    def profile_read(self, kernel):
        n, ms = C.c_longlong(0), C.c_double(0)
        _check(lib().ekf_profile_read(self.h, kernel, C.byref(n), C.byref(ms)), "profile_read")
        return n.value, ms.value

    def sigma_pass_bytes(self, filters=None):
        return lib().ekf_sigma_pass_bytes(self.h, self.F if filters is None else filters)


class Slam:
    """slam_core: the reference node's callbacks (include/slam_core.h)."""

    def __init__(self, n_landmarks=50, source=SOURCE_SIM, dtype=EKF_F64, track=0.160,
                 radius=0.033, **kw):
        self.cfg = make_config(n_landmarks, 1, dtype, **kw)
        h = C.c_void_p()
        _check(lib().slam_create(C.byref(h), C.byref(self.cfg), track, radius, source),
               "slam_create")
        self.h = h
        self.n = 3 + 2 * n_landmarks
        p = C.c_int()
        _check(lib().ekf_get_path(lib().slam_filter(self.h), C.byref(p)), "ekf_get_path")
        self.path = p.value

    def close(self):
        if getattr(self, "h", None):
            lib().slam_destroy(self.h)
            self.h = None

    __del__ = close

    def reset(self):
        """A fresh node on the same handle (slam_reset)."""
        _check(lib().slam_reset(self.h), "slam_reset")

    def set_joseph(self, on=True) -> int:
        return lib().ekf_set_joseph(lib().slam_filter(self.h), int(on))

    def profile(self, enable=True):
        lib().ekf_profile_enable(lib().slam_filter(self.h), int(enable))

    def profile_read(self, kernel):
        n, ms = C.c_longlong(0), C.c_double(0)
        _check(lib().ekf_profile_read(lib().slam_filter(self.h), kernel, C.byref(n), C.byref(ms)),
               "profile_read")
        return n.value, ms.value

    def joint_states(self, left, right):
        return lib().slam_joint_states(self.h, float(left), float(right))

    def markers(self, ids, actions, rel_xy):
        rel = _f64(rel_xy)
        ids = None if ids is None else _i32(ids)
        actions = None if actions is None else _i32(actions)
        return lib().slam_markers(self.h, rel.size // 2, _ptr(ids), _ptr(actions), _ptr(rel))

    def initial_pose(self, x, y, theta):
        return lib().slam_initial_pose(self.h, x, y, theta)

    def odom(self):
        p = np.zeros(3)
        lib().slam_odom(self.h, _ptr(p))
        return p

    def map_odom(self):
        p = np.zeros(3)
        _check(lib().slam_map_odom(self.h, _ptr(p)), "slam_map_odom")
        return p

    def filter_state(self, sigma=True):
        ekf = lib().slam_filter(self.h)
        n = self.n
        x = np.zeros(n)
        S = np.zeros((n, n)) if sigma else None
        cnt = C.c_uint(0)
        _check(lib().ekf_get_state(ekf, 0, _ptr(x), _ptr(S), C.byref(cnt)), "ekf_get_state")
        return x, S, cnt.value

    def replay(self, sc, poses=True):
        """Drive a synth.Scenario (wheel ticks + marker arrays) natively through the node mirror."""
        T, ticks = sc.wheel.shape[0], sc.wheel.shape[1]
        M = sc.ids.shape[1]
        wheel, counts = _f64(sc.wheel), _i32(sc.count)
        ids, act, rel = _i32(sc.ids), _i32(sc.actions), _f64(sc.rel)
        out_p = np.zeros((T, 3)) if poses else None
        out_t = np.zeros((T, 3)) if poses else None
        rc = lib().slam_replay(self.h, T, ticks, _ptr(wheel), M, _ptr(counts), _ptr(ids),
                               _ptr(act), _ptr(rel), _ptr(out_p), _ptr(out_t))
        return rc, out_p, out_t


class Sim:
    """ekf_sim_t: on-device Monte-Carlo inputs for an EKF handle (include/ekf_sim.h)."""

    def __init__(self, ekf, landmarks, **cfg):
        c = SimConfig()
        lib().ekf_sim_config_default(C.byref(c))
        for k, v in cfg.items():
            setattr(c, k, v)
        self.cfg = c
        self.F = ekf.F
        lm = _f64(np.broadcast_to(np.asarray(landmarks, np.float64),
                                  (ekf.F,) + np.shape(landmarks)[-2:]))
        self.L = lm.shape[1]
        self.h = C.c_void_p()
        _check(lib().ekf_sim_create(C.byref(self.h), ekf.h, C.byref(c), self.L, _ptr(lm)),
               "ekf_sim_create")
        self.T = 0

    def run(self, wheel_cmd, sense=None):
        """wheel_cmd[T·ticks][2] commanded wheel increments per tick; sense[T] or None."""
        cmd = _f64(wheel_cmd).reshape(-1, 2)
        T = cmd.shape[0] // self.cfg.ticks_per_msg
        sn = None if sense is None else _i32(sense)
        _check(lib().ekf_sim_run(self.h, T, _ptr(cmd), _ptr(sn)), "ekf_sim_run")
        self.T = T

    def markers(self):
        """The last run's inputs as ekf_replay takes them: counts [T,F], ids/actions [T,F,M],
        rel [T,F,M,2]."""
        T, F, M = self.T, self.F, self.cfg.marker_stride
        cnt = np.zeros((T, F), np.int32)
        ids = np.zeros((T, F, M), np.int32)
        act = np.zeros((T, F, M), np.int32)
        rel = np.zeros((T, F, M, 2))
        _check(lib().ekf_sim_markers(self.h, _ptr(cnt), _ptr(ids), _ptr(act), _ptr(rel)),
               "ekf_sim_markers")
        return cnt, ids, act, rel

    def poses(self):
        """(odom [T, 3], truth [T, F, 3]) of the last run."""
        odom = np.zeros((self.T, 3))
        truth = np.zeros((self.T, self.F, 3))
        _check(lib().ekf_sim_poses(self.h, _ptr(odom), _ptr(truth)), "ekf_sim_poses")
        return odom, truth

    def close(self):
        if getattr(self, "h", None) and self.h.value:
            lib().ekf_sim_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def poison_lds(device=0):
    """ekf_debug_poison_lds: every CU's LDS filled with a NaN pattern (tests: unwritten LDS reads
    then fail deterministically)."""
    _check(lib().ekf_debug_poison_lds(device), "ekf_debug_poison_lds")


def odometry(sc, track=None, radius=None):
    """t_odom_robot at each sensor message of a scenario, integrated natively by the product's
    DiffDrive::fkin (slam_integrate_odometry) — input preparation for ekf_replay."""
    track = sc.track if track is None else track
    radius = sc.radius if radius is None else radius
    wheel = _f64(sc.wheel)
    T, ticks = wheel.shape[0], wheel.shape[1]
    out = np.zeros((T, 3))
    _check(lib().slam_integrate_odometry(track, radius, T, ticks, _ptr(wheel), _ptr(out)),
           "slam_integrate_odometry")
    return out
