/*
 * ekf.h — C-ABI of the MI355X-native EKF-SLAM update path (libekfslam.so).
 *
 * Drop-in boundary for the EKF inside maxipalay/ekf-slam's `slam` node (nuslam/src/slam.cpp).
 * The reference has no predict()/update()/associate() functions: the filter is inline code inside
 * two ROS 2 subscription callbacks. Each entry point below names the reference lines it replaces.
 * Plain C types only (no HIP / torch types); every call returns a status code and never throws.
 *
 * Threading: one handle is not thread-safe (the reference runs every callback on one executor
 * thread, slam.cpp:683); distinct handles are independent. The handle owns its device memory and a
 * private HIP stream; host arrays are caller-owned and copied in. Calls are asynchronous on the
 * handle's stream unless stated otherwise; ekf_get_* and ekf_sync synchronise.
 */
#ifndef EKFSLAM_EKF_H
#define EKFSLAM_EKF_H
#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ---- */
#define EKF_OK 0
#define EKF_E_ARG (-1)     /* bad argument / handle */
#define EKF_E_RANGE (-2)   /* landmark id >= N, or counter_obstacles overflow: the reference's
                              Armadillo bounds check throws (slam.cpp:213, :351) */
#define EKF_E_EMPTY (-3)   /* empty MarkerArray: the reference throws at msg.markers.at(0)
                              (slam.cpp:281, :498) */
#define EKF_E_NUMERIC (-4) /* singular or non-finite innovation covariance S (slam.cpp:252) */
#define EKF_E_HIP (-5)     /* HIP runtime error */
#define EKF_E_NOMEM (-6)
#define EKF_E_TIMEOUT (-7) /* a device hand-off (cross-stream epoch or k_assoc_msg's exchange
                              between a filter's workgroups) was not seen within its bounded poll:
                              the flagged filters' state after that message is undefined. Reported
                              once by the next ekf_sync / ekf_sensor / ekf_associate_correct;
                              ekf_get_status names the filters (EKF_FLAG_TIMEOUT). No reference
                              counterpart (the reference has no device). */

/* status flag bits (ekf_get_status), accumulated on the device */
#define EKF_FLAG_RANGE 1u   /* a marker was skipped: id >= N / map full (slam.cpp:213, :351) */
#define EKF_FLAG_NUMERIC 2u /* a marker was skipped: S singular or non-finite (slam.cpp:252) */
#define EKF_FLAG_TIMEOUT 4u /* a device poll timed out: this filter's state is undefined
                               (EKF_E_TIMEOUT) */

#define EKF_F64 0
#define EKF_F32 1 /* Σ stored and contracted in fp32; state and all O(n) math stay fp64 */

#define EKF_MARKER_ADD 0
#define EKF_MARKER_DELETE 2 /* visualization_msgs::msg::Marker::DELETE (skipped, slam.cpp:205) */

#define EKF_MAX_CHUNK 16 /* markers folded into one Σ pass; longer messages are split */

typedef struct ekf_ctx* ekf_t;

/* Filter parameters. Defaults = the reference's hard-coded members (slam.cpp:665-671, :130). */
typedef struct {
  int n_landmarks; /* N, state dim n = 3 + 2N (slam.cpp:665: 50)                 */
  int n_filters;   /* independent filters in one handle (Monte-Carlo swarm); 1 = one slam node */
  int dtype;       /* EKF_F64 | EKF_F32                                              */
  double q_noise;  /* Q̄ = q·I₃ on the pose block (slam.cpp:135-136, :666: 1e-2)     */
  double r_noise;  /* R = r·I₂ (slam.cpp:139, :667: 1e-2)                          */
  double init_var; /* landmark prior variance (slam.cpp:130: 10e6 = 1e7)           */
  double mah_gate; /* Mahalanobis gate on the squared distance (slam.cpp:671: 2.0)  */
  int device;      /* HIP device ordinal                                            */
} ekf_config;

void ekf_config_default(ekf_config* cfg);
const char* ekf_strerror(int status);

/* Filter construction: Σ₀ = diag(0,0,0, init_var·I_2N), state = 0, Q̄, R (slam.cpp:127-139, :674). */
int ekf_create(ekf_t* out, const ekf_config* cfg);
int ekf_destroy(ekf_t h);
/* n = 3+2N, ld = Σ row stride in elements, n_filters */
int ekf_dims(ekf_t h, int* n, int* ld, int* n_filters);

/* Which device path the handle runs (fixed at ekf_create):
 *   EKF_PATH_PIPELINE  Σ in HBM; per chunk of ≤ EKF_MAX_CHUNK markers a chain, a factor kernel and
 *                      one low-rank Σ pass (any n, fp64 or fp32);
 *   EKF_PATH_RESIDENT  fp64 with n ≤ EKF_RESIDENT_MAX_N (the reference's N = 50 map): one launch
 *                      per upload, Σ held in a workgroup's registers across all its messages.
 * The environment variable EKF_RESIDENT=0 forces the pipeline (both give the same results up to
 * summation order). */
#define EKF_PATH_PIPELINE 0
#define EKF_PATH_RESIDENT 1
#define EKF_RESIDENT_MAX_N 128
int ekf_get_path(ekf_t h, int* path);

/* How unknown association (ekf_sensor, ekf_associate_correct, assoc replays) runs on the pipeline
 * (fixed at ekf_create; same decisions either way, slam.cpp:344-440):
 *   EKF_ASSOC_CHUNK_XCD  a chunk of <= EKF_MAX_CHUNK markers per launch, one workgroup per 64
 *                        landmark slots, a filter's workgroups on one XCD exchanging through its L2;
 *   EKF_ASSOC_CHUNK      the same kernel with the workgroups anywhere (agent-coherent exchange;
 *                        EKF_AM_XCD=0 forces it);
 *   EKF_ASSOC_MARKER     one marker per launch (resident path, EKF_ASSOC_MSG=0, or a map whose
 *                        ceil(N/64) workgroups the CUs cannot hold at once).
 * The Joseph form (ekf_set_joseph) takes the chunk routes too, with its own kernel instantiation;
 * the route reported is the one in effect for the current form. */
#define EKF_ASSOC_MARKER 0
#define EKF_ASSOC_CHUNK 1
#define EKF_ASSOC_CHUNK_XCD 2
int ekf_get_assoc_route(ekf_t h, int* route);

/* The handle's schedule (fixed at ekf_create), bit flags:
 *   EKF_SCHED_DEVSYNC  <= 32 filters: the chain and bulk streams get disjoint CU masks and hand off
 *                      through device epochs (EKF_DEVSYNC=0: HIP events between the two streams);
 *   EKF_SCHED_SERIAL   every kernel on one stream. The default for > 32 filters (their Σ passes
 *                      fill every CU, so two streams overlap nothing; the staged rebuild operands
 *                      are off there too, EKF_STAGE=1 restores them); EKF_SERIAL=1 forces it for
 *                      any handle, EKF_SERIAL=0 keeps two streams (HIP events) for > 32 filters.
 * Every schedule gives bit-identical results.
 *   EKF_SCHED_BUILDER  deprecated: a block-builder schedule of earlier releases, retired; the bit is
 *                      never set (the name stays so that code written against it still compiles). */
#define EKF_SCHED_DEVSYNC 1
#define EKF_SCHED_BUILDER 2
#define EKF_SCHED_SERIAL 4
int ekf_get_schedule(ekf_t h, int* flags);

/* ---- the callbacks (fast path) ---- */

/* t_odom_robot ← DiffDrive::FKin output (slam.cpp:633, jointStateCallback :599-634). */
int ekf_set_odom(ekf_t h, int filter, double theta, double x, double y);

/* Slam::fake_sensor_cb (slam.cpp:180-316) minus ROS publishing: predict with the current
 * t_odom_robot, one correction per non-DELETE marker (ids known), posterior t_map_odom.
 * ids are validated before anything changes (EKF_E_RANGE). rel_xy = body-frame (x, y) pairs. */
int ekf_fake_sensor(ekf_t h, int filter, int m, const int* ids, const int* actions,
                    const double* rel_xy);

/* Slam::sensor_cb (slam.cpp:318-530) minus ROS publishing: predict, then per marker the
 * Mahalanobis nearest-neighbour association (:344-440) and the correction (:443-488).
 * If assoc_out/is_new_out are non-NULL the call synchronises and returns the decisions. */
int ekf_sensor(ekf_t h, int filter, int m, const double* rel_xy, int* assoc_out,
               int* is_new_out);

/* All filters of the handle at once, one message per filter (the swarm / replay path).
 * counts[F], ids/actions[F][m_max], rel_xy[F][m_max][2], odom[F][3] (t_odom_robot per filter,
 * NULL = keep). ids may be NULL with assoc=1 (unknown association). Asynchronous.
 * counts[f] == 0: filter f gets no message this step and nothing of it changes (as ekf_fake_sensor
 * rejects an empty array, EKF_E_EMPTY: the reference throws at msg.markers.at(0), slam.cpp:281);
 * a message whose markers are all DELETE is a predict + posterior (slam.cpp:205). */
int ekf_batch_sensor(ekf_t h, int assoc, int m_max, const int* counts, const int* ids,
                     const int* actions, const double* rel_xy, const double* odom);

/* Replay T messages through ekf_batch_sensor (arrays as there, with a leading [T] axis):
 * counts[T][F], ids/actions[T][F][m_max], rel_xy[T][F][m_max][2], odom[T][F][3].
 * out_pose[T][F][3] (nullable) receives each posterior pose and makes every message synchronous. */
int ekf_replay(ekf_t h, int assoc, int T, int m_max, const int* counts, const int* ids,
               const int* actions, const double* rel_xy, const double* odom, double* out_pose);

/* ekf_replay with known ids (assoc = 0) whose inputs already live in device memory of the
 * handle's GPU (same layouts; d_actions nullable): the descriptors are planned on the GPU (one
 * chunk per message, so m_max <= EKF_MAX_CHUNK, in either form; no resident handle: EKF_E_ARG)
 * and no input crosses PCIe. The measurement (range, bearing) of slam.cpp:208-210 is computed on
 * the GPU (correctly rounded sqrt; the bearing's atan2 may differ from glibc's in the last bit).
 * Inputs are not validated on the host: an id outside [0, N) is skipped by the correction and
 * sets EKF_FLAG_RANGE in the filter's status. Asynchronous; the inputs must stay valid until the
 * next synchronising call (ekf_sync, a state read). The handle's planning state comes back to the
 * host at the next host-planned call or state access. */
int ekf_replay_device(ekf_t h, int T, int m_max, const int* d_counts, const int* d_ids,
                      const int* d_actions, const double* d_rel_xy, const double* d_odom);

/* ---- the finer-grained surface (north_star: predict()/update()/associate()) ---- */

/* Predict (slam.cpp:184-198): deferred and folded into the next Σ pass. */
int ekf_predict(ekf_t h, int filter);
/* One known-association correction (slam.cpp:207-268), predict folded in if pending. */
int ekf_correct(ekf_t h, int filter, int landmark_id, double rel_x, double rel_y);
/* One association + correction (slam.cpp:345-488). Synchronous when j/is_new non-NULL. */
int ekf_associate_correct(ekf_t h, int filter, double rel_x, double rel_y, int* j, int* is_new);
/* Posterior (slam.cpp:273-291): t_map_odom = T(x, y, θ)·t_odom_robot⁻¹. */
int ekf_posterior(ekf_t h, int filter);

/* Joseph-form covariance update, opt-in (off by default, like the reference, which applies
 * Σ ← (I − KH)Σ at slam.cpp:264-265): Σ ← (I − KH)Σ(I − KH)ᵀ + KRKᵀ for every later correction.
 * Equal in exact arithmetic with the optimal gain; it differs only in rounding. Resident path: its
 * own kernel instantiation. HBM pipeline (fp32 and fp64): the same chunks of <= 16 markers, each
 * folded into one Σ pass of rank 2 + 4m (K_c·M_c and (Σ_cHᵀ − K_c·S_c)·K_cᵀ per correction), so one
 * Σ pass per message as in the simple form. A switch makes each filter's next chunk gather its rows
 * from Σ (the chunk before cannot be rebuilt across forms). */
int ekf_set_joseph(ekf_t h, int on);

/* Deferred submission. While on, the callbacks above only plan their work on the host; the plan
 * goes to the device in one upload (and, on the resident path, one kernel launch) when it reaches
 * 8192 descriptors, when a synchronising call below needs the state, or when deferral is turned
 * off (which submits what is planned). Off by default: each callback is submitted as it is made.
 * A replay driver with no per-message outputs (slam_replay) turns it on. */
int ekf_defer(ekf_t h, int on);

/* Back to the constructor's state (slam.cpp:127-139) on the device for filter `filter`, or every
 * filter when filter < 0: Σ₀, state 0, t_map_odom identity, counter 0, status clear. Host-side
 * odometry set by ekf_set_odom is kept. Synchronises. */
int ekf_reset(ekf_t h, int filter);

/* Submits what the host has planned (deferred callbacks included) without waiting for it: after
 * it, a device-wide synchronisation (hipDeviceSynchronize) covers all of the handle's work. */
int ekf_flush(ekf_t h);

/* ---- state access (synchronising) ---- */
/* Waits for everything submitted; EKF_E_TIMEOUT if a device hand-off timed out since the last
 * report (see EKF_E_TIMEOUT). */
int ekf_sync(ekf_t h);
int ekf_get_pose(ekf_t h, int filter, double* theta_x_y);
int ekf_get_map_odom(ekf_t h, int filter, double* theta_x_y); /* t_map_odom */
/* state[n] (fp64), sigma[n*n] row-major fp64 (nullable), counter (nullable) */
int ekf_get_state(ekf_t h, int filter, double* state, double* sigma, unsigned* counter);
/* overwrite a filter (fixtures / resync after an association flip); t_map_odom nullable.
 * fp64 pipeline handles keep Σ exactly symmetric (the Σ pass computes the upper triangle and
 * mirrors it), so sigma's upper triangle is taken and mirrored below the diagonal; the reference's
 * own (I − KH)Σ (slam.cpp:264-265) is symmetric up to rounding. fp32 and resident handles store
 * sigma as given. */
int ekf_set_state(ekf_t h, int filter, const double* state, const double* sigma,
                  const double* t_map_odom, unsigned counter);
int ekf_get_status(ekf_t h, int filter, unsigned* flags); /* and clears them */

/* ---- helpers ---- */
/* turtlelib::normalize_angle (geometry2d.cpp:5-14): maps into (-π, π], -π → π. */
double ekf_normalize_angle(double rad);

/* ---- measurement ---- */
/* Per-kernel device time (0 = Σ pass, 1 = chain, 2 = association, 3 = factors, 4 = resident filter
 * kernel) from HIP events
 * carried by each timed dispatch (hipExtLaunchKernelGGL start/stop events: the kernel's own
 * execution, on the stream it runs on). Off by default. */
int ekf_profile_enable(ekf_t h, int enable);
int ekf_profile_read(ekf_t h, int kernel, long long* launches, double* total_ms);
/* Bytes the Σ pass must move per launch for the current handle: fp32 2·n²·w·F (Σ_in read, Σ_out
 * written); fp64 (n(n+1)/2 + n²)·w·F (the symmetric pass reads Σ_in's upper triangle). */
double ekf_sigma_pass_bytes(ekf_t h, int filters_in_launch);

/* ---- diagnostics ---- */
/* Fill every CU's LDS on `device` with a NaN bit pattern (default stream, synchronising): LDS then
 * holds what an arbitrary earlier kernel could have left, so a kernel that reads LDS it never
 * wrote produces a non-finite result deterministically instead of rarely (used by tests/). */
int ekf_debug_poison_lds(int device);

#ifdef __cplusplus
}
#endif
#endif
