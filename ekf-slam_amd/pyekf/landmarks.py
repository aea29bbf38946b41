"""ctypes wrapper of include/landmarks.h — the lidar landmark front-end (nuslam/src/landmarks.cpp,
turtlelib/src/landmark_detection.cpp) on the GPU. Plumbing for tests and bench.py."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import EKF_OK, EkfError, lib

LM_MAX_BEAMS, LM_MAX_CLUSTER, LM_NO_BREAK = 2048, 39, -1
MARKER_DTYPE = np.dtype([("x", "<f8"), ("y", "<f8"), ("r", "<f8"), ("id", "<i4"), ("pad", "<i4")])


def _check(rc, what):
    if rc != EKF_OK:
        raise EkfError(rc, what)


def _clusters(clusters):
    offs = np.zeros(len(clusters) + 1, dtype=np.int32)
    offs[1:] = np.cumsum([len(c) for c in clusters])
    xy = np.ascontiguousarray(np.concatenate([np.asarray(c, dtype=np.float64).reshape(-1, 2)
                                              for c in clusters]), dtype=np.float64)
    return offs, xy


class Detector:
    """Batched Landmarks::laserCallback (landmarks.cpp:109-156): S scans per call."""

    def __init__(self, max_scans=1, max_beams=360, device=0):
        self.h = C.c_void_p()
        _check(lib().lm_create(C.byref(self.h), max_scans, max_beams, device), "lm_create")

    def close(self):
        if self.h:
            lib().lm_destroy(self.h)
            self.h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def detect(self, ranges, angle_min, angle_inc, threshold=0.2, max_markers=32):
        """ranges [S, B] float32 → (counts [S], markers [S, max_markers] structured array)."""
        r = np.ascontiguousarray(ranges, dtype=np.float32)
        if r.ndim == 1:
            r = r[None]
        S, B = r.shape
        am = np.ascontiguousarray(np.broadcast_to(np.asarray(angle_min, np.float64), (S,)))
        ai = np.ascontiguousarray(np.broadcast_to(np.asarray(angle_inc, np.float64), (S,)))
        out = np.zeros((S, max_markers), dtype=MARKER_DTYPE)
        cnt = np.zeros(S, dtype=np.int32)
        _check(lib().lm_detect(self.h, S, B, r.ctypes.data, am.ctypes.data, ai.ctypes.data,
                               threshold, out.ctypes.data, max_markers, cnt.ctypes.data),
               "lm_detect")
        return cnt, out

    def markers(self, ranges, angle_min, angle_inc, threshold=0.2, max_markers=32):
        """One scan → list of (id, x, y, r) like the oracle's laser_callback (None: no break)."""
        cnt, out = self.detect(ranges, angle_min, angle_inc, threshold, max_markers)
        if cnt[0] == LM_NO_BREAK:
            return None
        return [(int(m["id"]), float(m["x"]), float(m["y"]), float(m["r"]))
                for m in out[0][:min(int(cnt[0]), max_markers)]]

    def fit_circles(self, clusters):
        offs, xy = _clusters(clusters)
        out = np.zeros((len(clusters), 3))
        _check(lib().lm_fit_circles(self.h, len(clusters), offs.ctypes.data, xy.ctypes.data,
                                    out.ctypes.data), "lm_fit_circles")
        return out

    def check_circles(self, clusters):
        offs, xy = _clusters(clusters)
        out = np.zeros(len(clusters), dtype=np.int32)
        _check(lib().lm_check_circles(self.h, len(clusters), offs.ctypes.data, xy.ctypes.data,
                                      out.ctypes.data), "lm_check_circles")
        return out.astype(bool)

    def last_kernel_us(self):
        us = C.c_double()
        _check(lib().lm_last_kernel_us(self.h, C.byref(us)), "lm_last_kernel_us")
        return us.value
