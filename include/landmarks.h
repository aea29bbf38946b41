/*
 * landmarks.h — C-ABI of the MI355X-native lidar landmark front-end (libekfslam.so).
 *
 * Drop-in for the producer of the association path's input in maxipalay/ekf-slam: the
 * `landmarks` node (nuslam/src/landmarks.cpp) and turtlelib's circle classification / fitting
 * (turtlelib/src/landmark_detection.cpp). Its MarkerArray output is what `slam`'s sensor_cb
 * consumes (ekf_sensor / slam_markers with SOURCE_ASSOC). SURVEY.md §8f row 1.
 *
 * Batched: one call takes S scans (independent robots / filters of a Monte-Carlo swarm, or
 * consecutive scans of one robot), one wavefront per scan on the GPU. Plain C types only; every
 * call returns an EKF_* status code (ekf.h) and never throws. One handle is not thread-safe;
 * calls synchronise the handle's stream before returning host results.
 */
#ifndef EKFSLAM_LANDMARKS_H
#define EKFSLAM_LANDMARKS_H
#ifdef __cplusplus
extern "C" {
#endif

#define LM_MAX_BEAMS 2048       /* beams per scan (LDS-resident)                           */
#define LM_MAX_CLUSTER 39       /* clusters of 4..39 points are fitted (landmarks.cpp:122)  */
#define LM_NO_BREAK (-1)        /* per-scan count: the scan has no cluster break; the
                                   reference throws at clusters.at(0) (landmarks.cpp:94)    */

typedef struct lm_ctx* lm_t;

/* One detected obstacle: visualization_msgs::Marker fields the slam node reads
 * (landmarks.cpp:146-148): id = index among circle-classified clusters, (x, y) = circle centre
 * in the laser frame, r = fitted radius (the marker's scale is 2r). */
typedef struct {
  double x, y, r;
  int id;
  int pad;
} lm_marker;

/* Handle with device buffers for up to max_scans scans of max_beams beams (≤ LM_MAX_BEAMS). */
int lm_create(lm_t* out, int max_scans, int max_beams, int device);
int lm_destroy(lm_t h);

/* Landmarks::laserCallback (landmarks.cpp:109-156) for S scans of B beams each.
 *   ranges       [S][B] float (sensor_msgs/LaserScan::ranges)
 *   angle_min    [S], angle_inc [S]: the messages' angle_min / angle_increment
 *   threshold    cluster break distance (landmarks.cpp:195: 0.2)
 *   markers      [S][max_markers] out; counts [S] out: published markers of each scan (those
 *                beyond max_markers are counted, not written), or LM_NO_BREAK.
 * Beam i's point is r_i·(cos, sin)(normalize_angle(i·inc) + angle_min) − (0.032, 0)
 * (landmarks.cpp:66-70). Returns EKF_OK even when some scans report LM_NO_BREAK. */
int lm_detect(lm_t h, int n_scans, int n_beams, const float* ranges, const double* angle_min,
              const double* angle_inc, double threshold, lm_marker* markers, int max_markers,
              int* counts);

/* turtlelib::fitCircle (landmark_detection.cpp:50-135) on n_clusters point sets: cluster c is
 * xy[2·offsets[c] .. 2·offsets[c+1]) as (x, y) pairs; out[3c..3c+2] = (c_x, c_y, R).
 * Any cluster size ≥ 1 (the node only fits 4..39 points). */
int lm_fit_circles(lm_t h, int n_clusters, const int* offsets, const double* xy, double* out);

/* turtlelib::checkCircle (landmark_detection.cpp:5-48) on the same layout; out[c] = 0 / 1.
 * Clusters need ≥ 3 points (the reference's angle vector has size − 2 entries). */
int lm_check_circles(lm_t h, int n_clusters, const int* offsets, const double* xy, int* out);

/* Per-kernel device time of the last lm_detect (HIP events around the dispatch), microseconds. */
int lm_last_kernel_us(lm_t h, double* us);

#ifdef __cplusplus
}
#endif
#endif
