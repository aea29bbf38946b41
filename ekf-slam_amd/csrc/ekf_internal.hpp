// Runtime internals shared by the filter runtime (ekf_api.cpp) and the on-device simulator
// (sim_api.cpp): how a device-written plan of known-association messages runs on a handle.
#pragma once
#include <hip/hip_runtime.h>

#include "ekf.h"
#include "ekf_device.hpp"
#include "ekf_launch.hpp"

namespace ekfslam {

struct HandleInfo {
  int F, N, n, dtype, device;
  bool resident;  // n ≤ kResidentMaxN fp64: one resident launch per plan
  bool joseph;    // ekf_set_joseph is on (the HBM pipeline then needs one marker per chunk)
  hipStream_t stream;
  hipStream_t bulk;  // the factors / Σ-pass stream (the main stream when serial)
};

// Runs everything the host has planned so far (flush) and describes the handle.
int handle_info(ekf_t h, HandleInfo* out);
// The parity each filter's next chunk reads (host mirror).
int handle_parity(ekf_t h, int* parity);
// T messages whose descriptors the device wrote into dd[t·F + f] on the handle's main stream (one
// known-association chunk per message, the first of each filter non-pipelined), and for the
// resident path the plan entries dplan[T]. Enqueues the filter kernels behind them; then the host
// mirror takes parity_after[F], odom_after[F][3] (t_odom_robot after the plan's last message, the
// predict input of the next host-planned call), no pending predict, and a non-pipelined next chunk.
int run_device_plan(ekf_t h, const MsgDesc* dd, const PlanEntry* dplan, int T,
                    const int* parity_after, const double* odom_after);

}  // namespace ekfslam
