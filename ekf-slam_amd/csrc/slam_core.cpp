// ROS-free mirror of the reference `slam` node's callbacks over the EKF C-ABI (include/slam_core.h).
#include "slam_core.h"

#include <new>

#include "geom.hpp"

using ekfslam::DiffDrive;
using ekfslam::Pose2;

struct slam_core {
  ekf_t ekf = nullptr;
  DiffDrive ddrive;              // slam.cpp:86, :642
  Pose2 t_odom_robot{};          // slam.cpp:650
  double track = 0.160, radius = 0.033;
  int source = SLAM_SOURCE_SIM;
};

extern "C" {

int slam_create(slam_t* out, const ekf_config* cfg, double track, double radius, int source) {
  if (!out || track <= 0.0 || radius <= 0.0) return EKF_E_ARG;
  slam_core* s = new (std::nothrow) slam_core;
  if (!s) return EKF_E_NOMEM;
  s->track = track;
  s->radius = radius;
  s->ddrive = DiffDrive(track, radius);
  s->source = source;
  const int rc = ekf_create(&s->ekf, cfg);
  if (rc) {
    delete s;
    return rc;
  }
  *out = s;
  return EKF_OK;
}

int slam_destroy(slam_t s) {
  if (!s) return EKF_E_ARG;
  if (s->ekf) ekf_destroy(s->ekf);
  delete s;
  return EKF_OK;
}

// slam.cpp:599-634: t_odom_robot = ddrive.FKin(position[0], position[1])
int slam_joint_states(slam_t s, double left, double right) {
  if (!s) return EKF_E_ARG;
  s->t_odom_robot = s->ddrive.fkin(left, right);
  return ekf_set_odom(s->ekf, 0, s->t_odom_robot.theta, s->t_odom_robot.x, s->t_odom_robot.y);
}

int slam_markers(slam_t s, int m, const int* ids, const int* actions, const double* rel_xy) {
  if (!s) return EKF_E_ARG;
  if (s->source == SLAM_SOURCE_SIM) return ekf_fake_sensor(s->ekf, 0, m, ids, actions, rel_xy);
  return ekf_sensor(s->ekf, 0, m, rel_xy, nullptr, nullptr);
}

// slam.cpp:575-597: restart the DiffDrive and set t_odom_robot (Σ and the state are untouched)
int slam_initial_pose(slam_t s, double x, double y, double theta) {
  if (!s) return EKF_E_ARG;
  s->ddrive = DiffDrive(s->track, s->radius);
  s->t_odom_robot = Pose2{theta, x, y};
  return ekf_set_odom(s->ekf, 0, theta, x, y);
}

int slam_odom(slam_t s, double* p) {
  if (!s || !p) return EKF_E_ARG;
  p[0] = s->t_odom_robot.theta;
  p[1] = s->t_odom_robot.x;
  p[2] = s->t_odom_robot.y;
  return EKF_OK;
}

int slam_map_odom(slam_t s, double* p) {
  if (!s) return EKF_E_ARG;
  return ekf_get_map_odom(s->ekf, 0, p);
}

ekf_t slam_filter(slam_t s) { return s ? s->ekf : nullptr; }

int slam_reset(slam_t s) {
  if (!s) return EKF_E_ARG;
  s->ddrive = DiffDrive(s->track, s->radius);
  s->t_odom_robot = Pose2{};
  const int rc = ekf_reset(s->ekf, 0);
  if (rc) return rc;
  return ekf_set_odom(s->ekf, 0, 0.0, 0.0, 0.0);
}

int slam_replay(slam_t s, int T, int ticks, const double* wheel, int m_max, const int* counts,
                const int* ids, const int* actions, const double* rel_xy, double* out_pose,
                double* out_tmo) {
  if (!s || T < 0 || ticks < 0 || !wheel || !counts || (m_max > 0 && !rel_xy)) return EKF_E_ARG;
  int first_rc = EKF_OK;
  const bool defer = !out_pose && !out_tmo;
  if (defer) ekf_defer(s->ekf, 1);
  for (int t = 0; t < T; ++t) {
    for (int k = 0; k < ticks; ++k) {
      const double* w = wheel + (static_cast<size_t>(t) * ticks + k) * 2;
      slam_joint_states(s, w[0], w[1]);
    }
    const size_t o = static_cast<size_t>(t) * m_max;
    const int rc = slam_markers(s, counts[t], ids ? ids + o : nullptr,
                                actions ? actions + o : nullptr, rel_xy + 2 * o);
    if (rc && !first_rc) first_rc = rc;
    if (out_pose) ekf_get_pose(s->ekf, 0, out_pose + 3 * static_cast<size_t>(t));
    if (out_tmo) ekf_get_map_odom(s->ekf, 0, out_tmo + 3 * static_cast<size_t>(t));
  }
  if (defer) {
    const int rc = ekf_defer(s->ekf, 0);
    if (rc && !first_rc) first_rc = rc;
  }
  return first_rc;
}

int slam_integrate_odometry(double track, double radius, int T, int ticks, const double* wheel,
                            double* out) {
  if (track <= 0.0 || radius <= 0.0 || T < 0 || ticks < 0 || !wheel || !out) return EKF_E_ARG;
  DiffDrive dd(track, radius);
  Pose2 p{};
  for (int t = 0; t < T; ++t) {
    for (int k = 0; k < ticks; ++k) {
      const double* w = wheel + (static_cast<size_t>(t) * ticks + k) * 2;
      p = dd.fkin(w[0], w[1]);
    }
    out[3 * static_cast<size_t>(t)] = p.theta;
    out[3 * static_cast<size_t>(t) + 1] = p.x;
    out[3 * static_cast<size_t>(t) + 2] = p.y;
  }
  return EKF_OK;
}

}  // extern "C"
