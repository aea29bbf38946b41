/* On-device Monte-Carlo inputs for a filter handle: nusim's wheel
 * integration with slip and its fake landmark sensor, for every filter of an ekf_t, feeding the
 * filter with no host round trip.
 *
 * Replaces, per filter f (seeded seed + f0 + f, counter-based splitmix64 draws):
 *   nusim timer_callback   nusim/src/nusim.cpp:222-230  wheel angle += commanded increment ×
 *                                                      (1 + U(−slip, slip)); true pose =
 *                                                      DiffDrive::FKin(true wheel angles)
 *                                                      (turtlelib/src/diff_drive.cpp:10-28)
 *   slam jointStateCallback nuslam/src/slam.cpp:599-634 t_odom_robot = FKin(encoder angles): the
 *                                                      encoders report the COMMANDED angles — a
 *                                                      deliberate change from nusim, whose encoders
 *                                                      publish the slipped wheel_pos_l/r
 *                                                      (nusim.cpp:272-273), so its odometry follows
 *                                                      the truth; here odometry drifts from the
 *                                                      truth and the filter has work to do
 *   nusim sensor_timer_callback nusim.cpp:317-346      marker = landmark in the true body frame
 *                                                      + N(0, σ²) on x and y; ADD within range,
 *                                                      DELETE beyond (mode ALL) or the m nearest
 *                                                      in range (NEAREST)
 * and the host's per-message planning of ekf_replay (known association): the device writes each
 * message's descriptor itself, so a swarm replay is a few launches per upload window.
 * The same arithmetic, draw for draw, is restated on the host by pyekf.synth (the test oracle of
 * this path); the filter then equals oracle/ runs fed the device's own markers.
 *
 * Collisions with obstacles (nusim.cpp:232-254) are not modelled: landmarks are placed clear of
 * the path. Unknown association (ids stripped) is not supported here (ekf_replay is). */
#ifndef EKF_SIM_H
#define EKF_SIM_H

#include "ekf.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ekf_sim* ekf_sim_t;

#define EKF_SENSE_NEAREST 0 /* the m nearest landmarks within max_range, nearest first */
#define EKF_SENSE_SURVEY 1  /* within 2·max_range, not-yet-sighted first, never empty */
#define EKF_SENSE_ALL 2     /* every landmark in id order, DELETE beyond max_range */

typedef struct {
  unsigned long long seed; /* filter f of the handle draws from seed + f0 + f */
  int f0;                  /* global index of the handle's filter 0 (one handle per rank) */
  int ticks_per_msg;       /* joint-state ticks per sensor message (nusim: 200 Hz / 5 Hz = 40) */
  double slip;             /* slip_fraction (nusim.cpp:224-227) */
  double sensor_sigma;     /* σ of the marker x, y noise (nusim.cpp:339-340) */
  double max_range;        /* sensor range, m */
  int max_markers;         /* m ≤ 16 for NEAREST / SURVEY messages */
  int marker_stride;       /* M: noise draws of message t, marker i use index t·M + i (≥ m; ≥ L
                            * when any message senses ALL) */
  double wheel_radius, track_width;               /* diff_params.yaml: 0.033, 0.160 */
  double start_theta, start_x, start_y;           /* true start pose (odometry starts at 0) */
  int record;              /* keep markers and poses for ekf_sim_markers / ekf_sim_poses */
} ekf_sim_config;

void ekf_sim_config_default(ekf_sim_config* c);

/* landmarks[F][L][2]: filter f's map (true positions); L ≤ 1024, ≤ the handle's n_landmarks.
 * ticks_per_msg ≤ 64 (one lane per tick). The simulator keeps its own true and odometry
 * poses and message counter across runs. */
int ekf_sim_create(ekf_sim_t* out, ekf_t filter, const ekf_sim_config* cfg, int n_map,
                   const double* landmarks);
int ekf_sim_destroy(ekf_sim_t s);

/* T messages: wheel_cmd[T·ticks_per_msg][2] commanded wheel-angle increments per tick (rad, left,
 * right; every filter's), sense[T] EKF_SENSE_* per message (NULL: NEAREST). Simulates, senses and
 * plans on the device, then runs the filter over the T messages (asynchronous like ekf_replay; the
 * call waits only for the device planning). A filter with no marker in a message gets no message
 * (as ekf_replay with counts 0). Afterwards the handle's t_odom_robot is the run's last odometry
 * pose, as if ekf_set_odom had been called with it (the next host-planned call predicts from it).
 * With ekf_set_joseph on, the chunks are Joseph-form ones. */
int ekf_sim_run(ekf_sim_t s, int T, const double* wheel_cmd, const int* sense);

/* With cfg.record: the last run's inputs as ekf_replay would take them — counts[T][F],
 * ids/actions[T][F][M], rel_xy[T][F][M][2] (M = marker_stride) — and odom[T][3] (t_odom_robot) and
 * truth[T][F][3] (θ, x, y). Synchronises. */
int ekf_sim_markers(ekf_sim_t s, int* counts, int* ids, int* actions, double* rel_xy);
int ekf_sim_poses(ekf_sim_t s, double* odom, double* truth);

#ifdef __cplusplus
}
#endif
#endif
