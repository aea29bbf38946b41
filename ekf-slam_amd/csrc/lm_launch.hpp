// Landmark front-end launchers (defined in lm_kernels.hip, called by lm_api.cpp).
#pragma once
#include <hip/hip_runtime.h>

#include "landmarks.h"

namespace lmk {

// One wavefront per scan: clusters, circle test, Hyper fit, marker compaction (k_detect).
hipError_t launch_detect(const float* ranges, int n_scans, int n_beams, const double* angle_min,
                         const double* angle_inc, double threshold, lm_marker* out,
                         int max_markers, int* counts, hipStream_t st);
// One lane per point set: fitCircle / checkCircle on clusters given by offsets.
hipError_t launch_fit(int n_clusters, const int* offsets, const double* xy, double* out,
                      hipStream_t st);
hipError_t launch_check(int n_clusters, const int* offsets, const double* xy, int* out,
                        hipStream_t st);

}  // namespace lmk
