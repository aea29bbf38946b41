// Host runtime behind include/landmarks.h: device buffers, the handle's stream and the batched
// laserCallback (nuslam/src/landmarks.cpp:109-156) over lm_kernels.hip.
#include <hip/hip_runtime.h>

#include <new>

#include "ekf.h"
#include "landmarks.h"
#include "lm_launch.hpp"

struct lm_ctx {
  int max_scans = 0, max_beams = 0, device = 0;
  hipStream_t stream = nullptr;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  float* d_ranges = nullptr;
  double* d_amin = nullptr;
  double* d_ainc = nullptr;
  int* d_counts = nullptr;
  lm_marker* d_markers = nullptr;
  int marker_cap = 0;  // markers per scan the device buffer holds
  lmk::DetectWork work{};
  // lm_fit_circles / lm_check_circles staging (grown on demand)
  int* d_offs = nullptr;
  double* d_xy = nullptr;
  double* d_out = nullptr;
  size_t cap_c = 0, cap_p = 0;
  bool timed = false;
};

namespace {

int grow(void** p, size_t bytes) {
  if (*p) hipFree(*p);
  *p = nullptr;
  return hipMalloc(p, bytes) == hipSuccess ? EKF_OK : EKF_E_NOMEM;
}

// fitCircle / checkCircle inputs → device (offsets validated on the host)
int stage_clusters(lm_t h, int nc, const int* offs, const double* xy) {
  if (!h || nc <= 0 || !offs || !xy || offs[0] != 0) return EKF_E_ARG;
  for (int c = 0; c < nc; ++c)
    if (offs[c + 1] <= offs[c]) return EKF_E_ARG;
  const size_t np = static_cast<size_t>(offs[nc]);
  if (static_cast<size_t>(nc) > h->cap_c) {
    if (grow(reinterpret_cast<void**>(&h->d_offs), sizeof(int) * (nc + 1)) ||
        grow(reinterpret_cast<void**>(&h->d_out), sizeof(double) * 3 * nc))
      return EKF_E_NOMEM;
    h->cap_c = nc;
  }
  if (np > h->cap_p) {
    if (grow(reinterpret_cast<void**>(&h->d_xy), sizeof(double) * 2 * np)) return EKF_E_NOMEM;
    h->cap_p = np;
  }
  if (hipSetDevice(h->device) != hipSuccess ||
      hipMemcpyAsync(h->d_offs, offs, sizeof(int) * (nc + 1), hipMemcpyHostToDevice, h->stream) !=
          hipSuccess ||
      hipMemcpyAsync(h->d_xy, xy, sizeof(double) * 2 * np, hipMemcpyHostToDevice, h->stream) !=
          hipSuccess)
    return EKF_E_HIP;
  return EKF_OK;
}

}  // namespace

extern "C" {

int lm_create(lm_t* out, int max_scans, int max_beams, int device) {
  if (!out || max_scans <= 0 || max_beams < 2 || max_beams > LM_MAX_BEAMS) return EKF_E_ARG;
  *out = nullptr;
  lm_ctx* h = new (std::nothrow) lm_ctx;
  if (!h) return EKF_E_NOMEM;
  h->max_scans = max_scans;
  h->max_beams = max_beams;
  h->device = device;
  const size_t S = max_scans;
  if (hipSetDevice(device) != hipSuccess || hipStreamCreate(&h->stream) != hipSuccess ||
      hipEventCreate(&h->e0) != hipSuccess || hipEventCreate(&h->e1) != hipSuccess) {
    lm_destroy(h);
    return EKF_E_HIP;
  }
  if (hipMalloc(&h->d_ranges, sizeof(float) * S * max_beams) != hipSuccess ||
      hipMalloc(&h->d_amin, sizeof(double) * S) != hipSuccess ||
      hipMalloc(&h->d_ainc, sizeof(double) * S) != hipSuccess ||
      hipMalloc(&h->d_counts, sizeof(int) * S) != hipSuccess ||
      hipMalloc(&h->work.px, sizeof(double) * S * max_beams) != hipSuccess ||
      hipMalloc(&h->work.py, sizeof(double) * S * max_beams) != hipSuccess ||
      hipMalloc(&h->work.cand, sizeof(lmk::Cand) * lmk::candidate_capacity(max_scans, max_beams)) !=
          hipSuccess ||
      hipMalloc(&h->work.gcount, sizeof(int) * lmk::kRegions) != hipSuccess ||
      hipMalloc(&h->work.sbase, sizeof(int) * S) != hipSuccess ||
      hipMalloc(&h->work.sncand, sizeof(int) * S) != hipSuccess) {
    lm_destroy(h);
    return EKF_E_NOMEM;
  }
  *out = h;
  return EKF_OK;
}

int lm_destroy(lm_t h) {
  if (!h) return EKF_E_ARG;
  hipSetDevice(h->device);
  if (h->stream) hipStreamSynchronize(h->stream);
  for (void* p : {static_cast<void*>(h->d_ranges), static_cast<void*>(h->d_amin),
                  static_cast<void*>(h->d_ainc), static_cast<void*>(h->d_counts),
                  static_cast<void*>(h->d_markers), static_cast<void*>(h->d_offs),
                  static_cast<void*>(h->d_xy), static_cast<void*>(h->d_out),
                  static_cast<void*>(h->work.px), static_cast<void*>(h->work.py),
                  static_cast<void*>(h->work.cand), static_cast<void*>(h->work.gcount),
                  static_cast<void*>(h->work.sbase), static_cast<void*>(h->work.sncand)})
    if (p) hipFree(p);
  if (h->e0) hipEventDestroy(h->e0);
  if (h->e1) hipEventDestroy(h->e1);
  if (h->stream) hipStreamDestroy(h->stream);
  delete h;
  return EKF_OK;
}

int lm_detect(lm_t h, int S, int B, const float* ranges, const double* amin, const double* ainc,
              double thr, lm_marker* markers, int max_markers, int* counts) {
  if (!h || S <= 0 || S > h->max_scans || B < 2 || B > h->max_beams || !ranges || !amin ||
      !ainc || !counts || max_markers < 0 || (max_markers > 0 && !markers))
    return EKF_E_ARG;
  if (hipSetDevice(h->device) != hipSuccess) return EKF_E_HIP;
  const int cap = max_markers > 0 ? max_markers : 1;
  if (cap > h->marker_cap) {
    if (grow(reinterpret_cast<void**>(&h->d_markers),
             sizeof(lm_marker) * static_cast<size_t>(h->max_scans) * cap))
      return EKF_E_NOMEM;
    h->marker_cap = cap;
  }
  const size_t nr = static_cast<size_t>(S) * B;
  if (hipMemcpyAsync(h->d_ranges, ranges, sizeof(float) * nr, hipMemcpyHostToDevice, h->stream) !=
          hipSuccess ||
      hipMemcpyAsync(h->d_amin, amin, sizeof(double) * S, hipMemcpyHostToDevice, h->stream) !=
          hipSuccess ||
      hipMemcpyAsync(h->d_ainc, ainc, sizeof(double) * S, hipMemcpyHostToDevice, h->stream) !=
          hipSuccess)
    return EKF_E_HIP;
  if (hipEventRecord(h->e0, h->stream) != hipSuccess) return EKF_E_HIP;
  if (lmk::launch_detect(h->d_ranges, S, B, h->d_amin, h->d_ainc, thr, h->d_markers, cap,
                         h->d_counts, h->work, h->stream) != hipSuccess)
    return EKF_E_HIP;
  if (hipEventRecord(h->e1, h->stream) != hipSuccess) return EKF_E_HIP;
  h->timed = true;
  if (hipMemcpyAsync(counts, h->d_counts, sizeof(int) * S, hipMemcpyDeviceToHost, h->stream) !=
      hipSuccess)
    return EKF_E_HIP;
  if (max_markers > 0 &&
      hipMemcpyAsync(markers, h->d_markers, sizeof(lm_marker) * static_cast<size_t>(S) * cap,
                     hipMemcpyDeviceToHost, h->stream) != hipSuccess)
    return EKF_E_HIP;
  return hipStreamSynchronize(h->stream) == hipSuccess ? EKF_OK : EKF_E_HIP;
}

int lm_fit_circles(lm_t h, int nc, const int* offs, const double* xy, double* out) {
  if (!out) return EKF_E_ARG;
  if (int rc = stage_clusters(h, nc, offs, xy)) return rc;
  if (lmk::launch_fit(nc, h->d_offs, h->d_xy, h->d_out, h->stream) != hipSuccess ||
      hipMemcpyAsync(out, h->d_out, sizeof(double) * 3 * nc, hipMemcpyDeviceToHost, h->stream) !=
          hipSuccess)
    return EKF_E_HIP;
  return hipStreamSynchronize(h->stream) == hipSuccess ? EKF_OK : EKF_E_HIP;
}

int lm_check_circles(lm_t h, int nc, const int* offs, const double* xy, int* out) {
  if (!out) return EKF_E_ARG;
  for (int c = 0; offs && c < nc; ++c)
    if (offs[c + 1] - offs[c] < 3) return EKF_E_ARG;  // the reference's angle vector needs n − 2 ≥ 1
  if (int rc = stage_clusters(h, nc, offs, xy)) return rc;
  int* dout = reinterpret_cast<int*>(h->d_out);  // 3·nc doubles ≥ nc ints
  if (lmk::launch_check(nc, h->d_offs, h->d_xy, dout, h->stream) != hipSuccess ||
      hipMemcpyAsync(out, dout, sizeof(int) * nc, hipMemcpyDeviceToHost, h->stream) != hipSuccess)
    return EKF_E_HIP;
  return hipStreamSynchronize(h->stream) == hipSuccess ? EKF_OK : EKF_E_HIP;
}

int lm_last_kernel_us(lm_t h, double* us) {
  if (!h || !us || !h->timed) return EKF_E_ARG;
  float ms = 0.0f;
  if (hipEventElapsedTime(&ms, h->e0, h->e1) != hipSuccess) return EKF_E_HIP;
  *us = 1e3 * ms;
  return EKF_OK;
}

}  // extern "C"
