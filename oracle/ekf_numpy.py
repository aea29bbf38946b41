"""ORACLE — TEST INFRASTRUCTURE ONLY.

Dense numpy (fp64, BLAS dgemm) restatement of the EKF in maxipalay/ekf-slam
``nuslam/src/slam.cpp``, written the way the reference writes it: a dense At for the predict
(slam.cpp:194-198), a dense 2×n H (slam.cpp:240-249), ``K = Σ Hᵀ inv(HΣHᵀ+R)`` (slam.cpp:252) and the
dense ``Σ ← (I − KH) Σ`` (slam.cpp:264-265). numpy's matmul goes to the bundled OpenBLAS dgemm, the
closest available stand-in for the Armadillo+BLAS arithmetic of the reference build.

Only ``oracle/make_golden.py`` (fixture generation, in the build container) and ``tests/`` use it.
It is never shipped to or imported by the product path.

Parity status: EKF parity UNPINNED — no reference test covers slam.cpp and the reference cannot be
built or run here. turtlelib helpers are pinned by the reference's KATs
(tests/test_oracle_kat.py).
"""
from __future__ import annotations

import math

import numpy as np

PI = 3.14159265358979323846
MARKER_DELETE = 2  # visualization_msgs::msg::Marker::DELETE


def normalize_angle(rad: float) -> float:
    """turtlelib/src/geometry2d.cpp:5-14"""
    diff = math.fmod(rad + PI, 2.0 * PI)
    if diff <= 0.0:
        return diff + PI
    return diff - PI


def tf_compose(lhs, rhs):
    """turtlelib/src/se2d.cpp:66-75 — transforms are (θ, x, y)."""
    c, s = math.cos(lhs[0]), math.sin(lhs[0])
    return (lhs[0] + rhs[0], c * rhs[1] - s * rhs[2] + lhs[1], s * rhs[1] + c * rhs[2] + lhs[2])


def tf_inv(t):
    """turtlelib/src/se2d.cpp:57-63"""
    c, s = math.cos(t[0]), math.sin(t[0])
    return (-t[0], -t[1] * c - t[2] * s, -t[2] * c + t[1] * s)


def integrate_twist(omega, vx, vy):
    """turtlelib/src/se2d.cpp:127-138"""
    if omega == 0.0:
        return (0.0, vx, vy)
    tsb = (0.0, vy / omega, -vx / omega)
    tbs = tf_inv(tsb)
    return tf_compose(tf_compose(tbs, (omega, 0.0, 0.0)), tsb)


class DiffDrive:
    """turtlelib/src/diff_drive.cpp:5-28 (FKin only)."""

    def __init__(self, track: float, radius: float):
        self.track, self.radius = track, radius
        self.phi_l = self.phi_r = 0.0
        self.config = (0.0, 0.0, 0.0)

    def fkin(self, rad_left: float, rad_right: float):
        dl, dr = rad_left - self.phi_l, rad_right - self.phi_r
        omega = self.radius / self.track * (-dl + dr)
        vx = self.radius / 2.0 * (dl + dr)
        self.config = tf_compose(self.config, integrate_twist(omega, vx, 0.0))
        self.phi_l, self.phi_r = rad_left, rad_right
        return self.config


def inv2(a: np.ndarray) -> np.ndarray:
    """Armadillo's closed-form tiny 2×2 inverse used by arma::inv (slam.cpp:252, :401, :476)."""
    det = a[0, 0] * a[1, 1] - a[0, 1] * a[1, 0]
    return np.array([[a[1, 1] / det, -a[0, 1] / det], [-a[1, 0] / det, a[0, 0] / det]])


class DenseEKF:
    """Filter members of slam.cpp:657-676; constructor init slam.cpp:127-139."""

    def __init__(self, n_landmarks=50, q_noise=1.0e-2, r_noise=1.0e-2, init_var=10e6,
                 mah_threshold=2.0, joseph=False):
        self.N = n_landmarks
        # opt-in Joseph form (BASELINE.json north_star; the reference uses (I − KH)Σ):
        # Σ ← (I − KH)Σ(I − KH)ᵀ + K·R·Kᵀ, dense, as the C oracle's literal Joseph mode
        self.joseph = joseph
        self.n = n = 2 * n_landmarks + 3
        self.sigma = np.zeros((n, n))
        self.sigma[3:, 3:] = np.eye(n - 3) * init_var
        self.q_bar = np.zeros((n, n))
        self.q_bar[:3, :3] = np.eye(3) * q_noise
        self.R = np.eye(2) * r_noise
        self.state = np.zeros(n)
        self.mah_threshold = mah_threshold
        self.counter = 0
        self.t_map_odom = (0.0, 0.0, 0.0)
        self.prev = (0.0, 0.0, 0.0)
        self.t_odom_robot = (0.0, 0.0, 0.0)

    # slam.cpp:184-198
    def predict(self):
        cur = tf_compose(self.t_map_odom, self.t_odom_robot)
        self.state[0] = normalize_angle(cur[0])
        self.state[1] = cur[1]
        self.state[2] = cur[2]
        dx = cur[1] - self.prev[1]
        dy = cur[2] - self.prev[2]
        At = np.eye(self.n)
        At[1, 0] = -dy
        At[2, 0] = dx
        self.sigma = At @ self.sigma @ At.T + self.q_bar

    def _h(self, k):
        """ẑ and dense H for landmark slot k (slam.cpp:219-249)."""
        s = self.state
        j = 3 + 2 * k
        est_range = math.sqrt((s[j] - s[1]) ** 2 + (s[j + 1] - s[2]) ** 2)
        est_bearing = normalize_angle(math.atan2(s[j + 1] - s[2], s[j] - s[1]) - s[0])
        dx, dy = s[j] - s[1], s[j + 1] - s[2]
        d = dx * dx + dy * dy
        H = np.zeros((2, self.n))
        H[0, 1] = -dx / math.sqrt(d)
        H[0, 2] = -dy / math.sqrt(d)
        H[1, 0] = -1.0
        H[1, 1] = dy / d
        H[1, 2] = -dx / d
        H[0, j] = dx / math.sqrt(d)
        H[0, j + 1] = dy / math.sqrt(d)
        H[1, j] = -dy / d
        H[1, j + 1] = dx / d
        return np.array([est_range, est_bearing]), H

    def _correct(self, k, z):
        """slam.cpp:251-267"""
        z_hat, H = self._h(k)
        K = (self.sigma @ H.T) @ inv2((H @ self.sigma) @ H.T + self.R)
        z_diff = z - z_hat
        z_diff[1] = normalize_angle(z_diff[1])
        self.state = self.state + K @ z_diff
        if self.joseph:
            ikh = np.eye(self.n) - K @ H
            self.sigma = (ikh @ self.sigma) @ ikh.T + (K @ self.R) @ K.T
        else:
            self.sigma = (np.eye(self.n) - K @ H) @ self.sigma
        self.state[0] = normalize_angle(self.state[0])

    @staticmethod
    def _meas(rx, ry):
        return np.array([math.sqrt(rx ** 2 + ry ** 2), math.atan2(ry, rx)])

    def correct_known(self, mid, rx, ry):
        """slam.cpp:207-268"""
        z = self._meas(rx, ry)
        j = 3 + 2 * mid
        if self.state[j] == 0.0 and self.state[j + 1] == 0.0:
            self.state[j] = self.state[1] + z[0] * math.cos(z[1] + self.state[0])
            self.state[j + 1] = self.state[2] + z[0] * math.sin(z[1] + self.state[0])
        self._correct(mid, z)

    def associate_correct(self, rx, ry):
        """slam.cpp:345-488. Returns (landmark index, is_new)."""
        if self.counter >= self.N:
            raise IndexError("counter_obstacles overflow (reference throws on state() bounds)")
        z = self._meas(rx, ry)
        s = self.counter
        self.state[3 + 2 * s] = self.state[1] + z[0] * math.cos(z[1] + self.state[0])
        self.state[4 + 2 * s] = self.state[2] + z[0] * math.sin(z[1] + self.state[0])
        self.counter += 1
        dists = np.empty(self.counter)
        for k in range(self.counter):
            if k == self.counter - 1:
                dists[k] = self.mah_threshold
                continue
            z_hat, H = self._h(k)
            psi = (H @ self.sigma) @ H.T + self.R
            z_diff = z - z_hat
            z_diff[1] = normalize_angle(z_diff[1])
            dists[k] = (z_diff @ inv2(psi)) @ z_diff
        # arma::index_min: first minimum; NaN never selected
        best, bestd = -1, math.inf
        for k in range(self.counter):
            if dists[k] < bestd:
                best, bestd = k, dists[k]
        is_new = best == self.counter - 1 and bestd >= self.mah_threshold
        if not is_new:
            self.counter -= 1
            self.state[3 + 2 * self.counter] = 0.0
            self.state[4 + 2 * self.counter] = 0.0
        self._correct(best, z)
        return best, is_new

    def posterior(self):
        """slam.cpp:273-277, :291"""
        filt = (self.state[0], self.state[1], self.state[2])
        self.t_map_odom = tf_compose(filt, tf_inv(self.t_odom_robot))
        self.prev = filt

    def fake_sensor_cb(self, ids, actions, rel_xy):
        """slam.cpp:180-316 (publishing omitted)."""
        self.predict()
        for i in range(len(ids)):
            if actions[i] == MARKER_DELETE:  # slam.cpp:205: only DELETE (2) is skipped
                continue
            self.correct_known(int(ids[i]), float(rel_xy[i, 0]), float(rel_xy[i, 1]))
        self.posterior()

    def sensor_cb(self, rel_xy):
        """slam.cpp:318-530 (publishing omitted)."""
        self.predict()
        out = []
        for i in range(len(rel_xy)):
            out.append(self.associate_correct(float(rel_xy[i, 0]), float(rel_xy[i, 1])))
        self.posterior()
        return out
