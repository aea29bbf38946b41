/*
 * slam_core.h — ROS-free mirror of maxipalay/ekf-slam's `slam` node (nuslam/src/slam.cpp) over ekf.h.
 *
 * Keeps the node's host-side state exactly where the reference keeps it — the DiffDrive odometry
 * (turtlelib diff_drive) and t_odom_robot — and forwards each subscription callback to the EKF
 * C-ABI. An rclcpp node (or the replay drivers in tests/ and bench.py) calls:
 *   slam_joint_states   ← Slam::jointStateCallback   (slam.cpp:599-634)
 *   slam_markers        ← Slam::fake_sensor_cb / Slam::sensor_cb (slam.cpp:180-316 / :318-530),
 *                         chosen by sensor_source "sim" / "assoc" (slam.cpp:115-125)
 *   slam_initial_pose   ← Slam::poseCallback         (slam.cpp:575-597)
 *   slam_map_odom       → the map→odom TF the node broadcasts (slam.cpp:281-289)
 */
#ifndef EKFSLAM_SLAM_CORE_H
#define EKFSLAM_SLAM_CORE_H
#include "ekf.h"
#ifdef __cplusplus
extern "C" {
#endif

typedef struct slam_core* slam_t;

#define SLAM_SOURCE_SIM 0   /* known ids: nusim/fake_sensor → fake_sensor_cb */
#define SLAM_SOURCE_ASSOC 1 /* unknown ids: green/detected_obstacles → sensor_cb */

int slam_create(slam_t* out, const ekf_config* cfg, double track_width, double wheel_radius,
                int sensor_source);
int slam_destroy(slam_t s);
/* joint_states: left/right wheel angles (rad) */
int slam_joint_states(slam_t s, double left, double right);
/* one MarkerArray; ids/actions ignored for SLAM_SOURCE_ASSOC (may be NULL) */
int slam_markers(slam_t s, int m, const int* ids, const int* actions, const double* rel_xy);
int slam_initial_pose(slam_t s, double x, double y, double theta);
/* A fresh node on the same handle: the filter back to its constructor state (ekf_reset), the
 * DiffDrive and t_odom_robot back to the origin (slam.cpp:86, :650). */
int slam_reset(slam_t s);
int slam_odom(slam_t s, double* theta_x_y);    /* t_odom_robot */
int slam_map_odom(slam_t s, double* theta_x_y); /* t_map_odom (synchronises) */
ekf_t slam_filter(slam_t s);
/* Replay a recorded run natively: per message, `ticks` joint_states (wheel[T][ticks][2]) then one
 * MarkerArray (counts[T], ids/actions[T][m_max], rel_xy[T][m_max][2]). out_pose / out_tmo
 * [T][3] (nullable) receive the posterior pose and t_map_odom after each message. Returns the
 * first non-OK status (processing continues, like a node that logs and carries on). With no
 * per-message output the messages are planned on the host and submitted together (ekf_defer):
 * asynchronous on return, like ekf_replay. */
int slam_replay(slam_t s, int T, int ticks, const double* wheel, int m_max, const int* counts,
                const int* ids, const int* actions, const double* rel_xy, double* out_pose,
                double* out_tmo);
/* t_odom_robot after each message's `ticks` joint_states, from a fresh DiffDrive (replay input
 * preparation): wheel[T][ticks][2] → out_odom[T][3]. */
int slam_integrate_odometry(double track_width, double wheel_radius, int T, int ticks,
                            const double* wheel, double* out_odom);

#ifdef __cplusplus
}
#endif
#endif
