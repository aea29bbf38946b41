// On-device simulator launcher (sim_kernels.hip), called by sim_api.cpp.
#pragma once
#include <hip/hip_runtime.h>

#include "ekf_device.hpp"

namespace ekfslam {

constexpr int kSimMaxMap = 1024;  // landmarks per filter map (16 per lane of the sensing wave)

// Per-filter simulator state kept on the device across runs: the true pose and the odometry pose
// (θ, x, y) after the last simulated tick.
struct alignas(16) SimState {
  double truth[3], odom[3];
};

struct SimArgs {
  const double* cmd;       // [T·tpm][2] commanded wheel increments of this run
  const int* sense;        // [T] EKF_SENSE_*, nullptr: NEAREST
  const double* lm;        // [F][L][2]
  unsigned* sighted;       // [F][(L + 31) / 32] survey bitsets
  SimState* st;            // [F]
  int* par;                // [F] parity the filter's next chunk reads (in / out)
  MsgDesc* desc;           // [T][F]
  int* out_ids;            // record: [T][F][M] (nullptr: not recorded)
  int* out_act;
  double* out_rel;         // [T][F][M][2]
  int* out_cnt;            // [T][F]
  double* out_truth;       // [T][F][3]
  double* out_odom;        // [T][3] (filter 0's wave)
  unsigned long long seed;
  long long tick0, msg0;   // global tick / message index of this run's first
  int f0, F, L, T, tpm, m, M, N;
  int joseph;              // the descriptors carry kJoseph (ekf_set_joseph on the HBM pipeline)
  double slip, sigma, range, radius, track;
  double start[3];
};

hipError_t launch_sim(const SimArgs& a, hipStream_t s);
// A run without SURVEY messages (no sighted set carried between messages): k_sim_pose walks the
// wheels per filter into truth_all / odom_all [T][F][3], then k_sim_sense senses every (t, f) in
// parallel into the record arrays (out_ids / out_act / out_rel / out_cnt, required); no descriptors.
hipError_t launch_sim_parallel(const SimArgs& a, double* truth_all, double* odom_all, hipStream_t s);

}  // namespace ekfslam
