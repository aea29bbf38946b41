/*
 * ORACLE — TEST INFRASTRUCTURE ONLY. Never linked into, loaded by, or called from the product
 * library (ekf-slam_amd/). Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load it, and only as the checker / the timed CPU baseline.
 *
 * Plain-C restatement of the EKF-SLAM path of maxipalay/ekf-slam (snapshot 2025-02-26):
 *   nuslam/src/slam.cpp            predict / known-association correction / Mahalanobis association
 *   turtlelib/src/geometry2d.cpp   normalize_angle
 *   turtlelib/src/se2d.cpp         Transform2D compose / inv, integrate_twist
 *   turtlelib/src/diff_drive.cpp   DiffDrive::FKin
 *
 * Parity status:
 *   - turtlelib helpers: PINNED by the reference's own known-answer tests
 *     (turtlelib/tests/test_geometry2d.cpp:8-17, test_se2d.cpp:152-251, test_diff_drive.cpp:7-99),
 *     transcribed in tests/test_oracle_kat.py.
 *   - EKF (slam.cpp): PARITY UNPINNED. No reference test covers slam.cpp and the reference cannot be
 *     built or executed in this environment (no Armadillo / ROS 2; executing reference sources was
 *     refused). The restatement is cross-checked between two independent forms:
 *     this C file (literal dense O(n^3) and structured O(n^2) modes) and oracle/ekf_numpy.py
 *     (dense numpy/BLAS), which generated tests/golden/.
 */
#ifndef EKF_ORACLE_H
#define EKF_ORACLE_H
#ifdef __cplusplus
extern "C" {
#endif

/* ---- turtlelib restatement ---- */
double orc_normalize_angle(double rad);
/* transforms are {theta, x, y} */
void orc_tf_compose(const double* lhs, const double* rhs, double* out);
void orc_tf_inv(const double* t, double* out);
void orc_integrate_twist(double omega, double vx, double vy, double* out);
/* dd = {track, radius, phi_left, phi_right, cfg_theta, cfg_x, cfg_y} (7 doubles, updated in place) */
void orc_fkin(double* dd, double rad_left, double rad_right, double* out);

/* ---- EKF restatement ---- */
typedef struct orc_ekf orc_ekf;
orc_ekf* orc_ekf_create(int n_landmarks, double q_noise, double r_noise, double init_var,
                        double mah_gate, int literal);
void orc_ekf_destroy(orc_ekf* f);
int  orc_ekf_dim(const orc_ekf* f);
/* opt-in Joseph-form update (I−KH)Σ(I−KH)ᵀ + KRKᵀ in place of slam.cpp:264-265's (I−KH)Σ */
void orc_ekf_set_joseph(orc_ekf* f, int on);
void orc_ekf_set_odom(orc_ekf* f, double theta, double x, double y);   /* t_odom_robot */
void orc_ekf_predict(orc_ekf* f);                                        /* slam.cpp:184-198 */
int  orc_ekf_correct(orc_ekf* f, int id, double rel_x, double rel_y);    /* slam.cpp:207-268 */
int  orc_ekf_associate_correct(orc_ekf* f, double rel_x, double rel_y, int* j, int* is_new);
void orc_ekf_posterior(orc_ekf* f);                                      /* slam.cpp:273-291 */
/* whole callbacks: actions[i] != 0 means DELETE (skipped on the fake path, slam.cpp:205) */
int  orc_ekf_fake_sensor_cb(orc_ekf* f, int m, const int* ids, const int* actions,
                            const double* rel_xy);
int  orc_ekf_sensor_cb(orc_ekf* f, int m, const double* rel_xy, int* assoc_out, int* new_out);
void orc_ekf_get(const orc_ekf* f, double* state, double* sigma, double* tmo, unsigned* counter);
void orc_ekf_set(orc_ekf* f, const double* state, const double* sigma, const double* tmo,
                 const double* prev, unsigned counter);
void orc_ekf_get_prev(const orc_ekf* f, double* prev);
/* test diagnostics: the smallest existing Mahalanobis distance of the last association (INFINITY
 * when there was no existing landmark), to build decisions near the gate */
double orc_ekf_last_dmin(const orc_ekf* f);

#ifdef __cplusplus
}
#endif
#endif
