// Landmark front-end launchers (defined in lm_kernels.hip, called by lm_api.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include "landmarks.h"

namespace lmk {

// One circle candidate (a cluster of 4..39 points) of the batch-wide list.
struct Cand {
  int scan, s0, n0, s1, n, pass;
  double cx, cy, r;
};

// Clusters with ≥ 4 points in a scan of B beams: each needs 4 points and a dropped break point.
inline int max_candidates(int B) { return B / 5 + 2; }
// The candidate list is split into regions (scan s → region s mod kRegions), one counter each.
constexpr int kRegions = 64;
inline size_t candidate_capacity(int S, int B) {
  return static_cast<size_t>(kRegions) * ((S + kRegions - 1) / kRegions) * max_candidates(B);
}

// Device workspace of lm_detect for up to S scans of B beams.
struct DetectWork {
  double* px;    // [S][B] beam points
  double* py;
  Cand* cand;    // [candidate_capacity(S, B)]: kRegions dense lists
  int* gcount;   // [kRegions] candidates in each region's list
  int* sbase;    // [S] first candidate of each scan
  int* sncand;   // [S] candidates of each scan (LM_NO_BREAK: no cluster break)
};

// Clusters, circle test, Hyper fit, marker compaction (k_clusters → k_candidates → k_markers).
hipError_t launch_detect(const float* ranges, int n_scans, int n_beams, const double* angle_min,
                         const double* angle_inc, double threshold, lm_marker* out,
                         int max_markers, int* counts, const DetectWork& w, hipStream_t st);
// One lane per point set: fitCircle / checkCircle on clusters given by offsets.
hipError_t launch_fit(int n_clusters, const int* offsets, const double* xy, double* out,
                      hipStream_t st);
hipError_t launch_check(int n_clusters, const int* offsets, const double* xy, int* out,
                        hipStream_t st);

}  // namespace lmk
