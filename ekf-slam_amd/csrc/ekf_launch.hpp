// Kernel launchers (defined in ekf_kernels.hip, called by the host runtime in ekf_api.cpp).
// Optional e0/e1: timing events carried by the dispatch itself (kernel execution time).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>

#include "ekf_device.hpp"

namespace ekfslam {

// Everything a launch needs to find filter f's buffers. Filters [f0, f0 + grid.y) take part;
// desc[k] describes filter f0 + k.
template <typename T>
struct PassArgs {
  T* sig[2];            // Σ ping-pong copies, filter 0
  size_t sig_stride;    // elements between filters
  double* x[2];         // state ping-pong copies, filter 0
  size_t x_stride;
  T* kcat;              // [KW][ldk] per filter (row k = one rank-1 factor over rows i)
  T* mcat;              // [KW][ldk] per filter (row k = one rank-1 factor over cols c)
  size_t km_stride;
  int ldk;
  FilterCtl* ctl;
  ChunkRec* rec;        // [2][rec_stride]: chunk records by Σ parity (chain → factors, next chain)
  size_t rec_stride;
  StageRec<T>* stage;   // [2][rec_stride]: rebuild operands staged for a kLook chain (kStageIn)
  unsigned* sync;       // device epochs (ekf_device.hpp kSync*)
  unsigned* fatal;      // host-mapped word: set when any poll of the handle timed out (flag_timeout)
  unsigned seq;         // this launch pair's sequence number; its epochs are seq + 1
  unsigned need_sigma;  // chain: wait until the Σ-pass epoch reaches this (0 = no wait)
  unsigned need_plan;   // chain: the launch's descriptors are planned once the kSyncPlan count
                        // reaches this (ekf_replay_device's planner on the bulk stream; 0 = no wait)
  unsigned pub_sigma;   // factors: publish this Σ-pass epoch first (the previous chunk's pass, 0 = none)
  int first_ready;      // chain: the launch's first chunk skips its Σ-epoch poll (the host joined
                        // the bulk stream before it, and the last pass published no epoch)
  int polls;            // 1: the streams hand off through device epochs (kernels poll them);
                        // 0: stream order / events order everything, no poll and no epoch kernel
  int gather;           // chain (dev A/B, EKF_SERIAL_GATHER=1): in stream order every chunk
                        // gathers its complete Σ_in instead of a kLook rebuild
  const MsgDesc* desc;
  int desc_stride;      // descriptors between consecutive chunks of a chain launch
  int n, ld, N, f0;
  double q, r, gate;
  int joseph;           // resident path: Joseph-form Σ update (ekf_set_joseph)
  int dbg;              // dev only (EKF_DBG_ORDER >> 8, tools/diag_handover.py): 1 agent acquire at
                        // the start of chain / factors / Σ pass, 2 agent release at their end,
                        // 4 count hand-offs whose producer epoch is not yet visible (sync[48..]),
                        // 8 check launch epochs, 16 chain / factor kernels log checksums (dlog), 32 k_dbg_sum
                        // kernels around them (EKF_DBG_ORDER 8192)
  unsigned long long* dlog;  // dev only: [kDlogKinds][64 seq][64 filters][8 slots] wrapping sums
};
constexpr int kDlogKinds = 21;  // 0 chain, 1-3 k_dbg_sum, 4 factor kernel, 5 + c chain step c
// dev only: checksums of what a kernel pair left in memory (kind 1: after the factor kernel, x_out
// Kcat Mcat; 2: after the Σ pass, Σ_out; 3: before the chain, Σ_in' x_in' record' tmo Σ_in x_in)
template <typename T>
hipError_t launch_dbg_sum(const PassArgs<T>& a, int n_filters, int kind, hipStream_t s);

// Chain kernel: the chunk's sequential corrections on the |U|×|U| block (predict folded in),
// one workgroup per filter → ChunkRec.
// nchunks consecutive chunks in one launch (descriptors a.desc[i·a.desc_stride + filter]).
template <typename T>
hipError_t launch_chain(const PassArgs<T>& a, int n_filters, int nchunks, hipStream_t s,
                        hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr);

// Factor kernel: Kcat = R·Z, Mcat = Y·C on f64 MFMA and the new state. 16 rows / columns per wave.
template <typename T>
hipError_t launch_factors(const PassArgs<T>& a, int n_filters, hipStream_t s,
                      hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr);

// Σ pass: Σ_out = Σ_in + Q − Kcatᵀ·Mcat on MFMA, one tile per wave, then k_patch_stage (fp32: the
// chain's fp64 Σ[U,U] over its block; stage: some filter's descriptor has kStageOut, fp32 checks
// on the device). publish: launch the Σ-pass epoch kernel behind it; otherwise the next chunk's
// factor kernel publishes it (PassArgs::pub_sigma).
template <typename T>
hipError_t launch_sigma_pass(const PassArgs<T>& a, int n_filters, bool publish, bool stage, hipStream_t s,
                      hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr);

// Mahalanobis nearest-neighbour association for one marker per filter (one workgroup each).
template <typename T>
hipError_t launch_assoc(const PassArgs<T>& a, int n_filters, hipStream_t s,
                      hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr);

// Unknown association, a whole chunk of ≤ kMaxChunk markers in one launch (ekf_assoc.hip): the
// scratch of the handle's k_assoc_msg (per filter: hist [kMaxChunk][Np], cur [kMaxChunk + 1][Np],
// granules [kMaxChunk + 1][G][4], Np = G·kAmSlots ≥ N).
struct AmArgs {
  AmHist* hist;
  AmCur* cur;
  unsigned long long* gran;
  size_t hist_stride, cur_stride, gran_stride;  // elements between filters
  int G;                                        // workgroups per filter
  int xcd;  // XCD-local placement: 8 blocks per workgroup, a filter's G on one XCD (k_assoc_msg)
  unsigned spin;  // bounded polls per exchange (EKF_FLAG_TIMEOUT beyond; EKF_AM_SPIN_LOG2)
  int drop;       // fault injection (EKF_AM_DROP=1, tests only): the last workgroup never
                  // publishes its first exchange, so every workgroup's poll times out
};
// Workgroups of k_assoc_msg one CU holds at once (its LDS bounds it), for the co-residency check:
// a filter's G workgroups spin on each other, so all of them must fit the bulk stream's CUs
// (per XCD in the XCD-local placement) at once, or the host routes the markers through the
// one-marker-per-launch path instead (ekf_api.cpp am_route). joseph: the Joseph-form kernel (its
// history rows are 96 bytes, so its LDS is larger).
int assoc_msg_blocks_per_cu(bool f32, bool joseph);
// Scores, decides and corrects every marker of the chunk (slam.cpp:338-488) and writes the chunk's
// Kcat / Mcat, the new state, t_map_odom and the decisions; the Σ pass then runs as for a known-id
// chunk. One grid (G, n_filters) of 64-lane workgroups; a filter's G workgroups exchange each
// step's argmin through granules.
template <typename T>
hipError_t launch_assoc_msg(const PassArgs<T>& a, const AmArgs& b, int n_filters, hipStream_t s,
                            hipEvent_t e0 = nullptr, hipEvent_t e1 = nullptr);

// Posterior t_map_odom for filters with no pending Σ pass.
template <typename T>
hipError_t launch_posterior(const PassArgs<T>& a, int n_filters, hipStream_t s);

// Resident path (ekf_resident.hip): n ≤ kResidentMaxN, fp64. One plan entry = the descriptors
// desc[off + f − f0] of filters [f0, f0 + nf) (kind as ekf_api.cpp's Launch: 0 known chunk,
// 1 association + correction, 2 posterior only). One 1024-thread workgroup per filter
// [flo, flo + nfil) keeps Σ and x in registers across every entry of the plan.
constexpr int kResidentMaxN = 128;
struct alignas(16) PlanEntry {
  int off, f0, nf, kind;
};
hipError_t launch_resident(const PassArgs<double>& a, const PlanEntry* plan, int nplan, int flo,
                           int nfil, hipStream_t s, hipEvent_t e0 = nullptr,
                           hipEvent_t e1 = nullptr);

// Known-association replay planned on the GPU (plan_kernels.hip, ekf_replay_device): a filter's
// planning state between messages — ekf_api.cpp's host mirror of it — before and after a replay.
struct alignas(16) PlanState {
  int parity;    // Σ / x copy that is "in"
  int prev_m;    // markers of the filter's last pipelined chunk (−1: none, the next one gathers)
  int pending;   // a predict is pending (folded into the next chunk)
  int pad;
  int prev_ids[kMaxChunk];
  double odom[3];  // t_odom_robot of the last message
  double pad2;
};
struct ReplayArgs {
  const int* counts;      // [T][F]
  const int* ids;         // [T][F][M]
  const int* actions;     // [T][F][M] or null
  const double* rel;      // [T][F][M][2]
  const double* odom;     // [T][F][3]
  const PlanState* st_in; // [F]
  PlanState* st_out;      // [F]
  MsgDesc* desc;          // [T][F]
  int T, F, M, N;
  int joseph;             // 1: Joseph form (every chunk flagged kJoseph)
  int stage;              // staged rebuild operands (kStageOut / kStageIn)
  unsigned* plan_count;   // non-null: every wave adds 1 here once its descriptor is stored (the
                          // chain polls it instead of waiting for the planner's kernel boundary)
};
hipError_t launch_plan_replay(const ReplayArgs& a, hipStream_t s);

// Σ₀ diagonal: Σ[i][i] = v for i ≥ 3 (the rest is zero-filled by the caller).
template <typename T>
hipError_t launch_init_diag(T* sig, size_t stride, int n, int ld, double v, int nf, hipStream_t s);

// Diagnostics: n_blocks workgroups each fill kPoisonLdsBytes of LDS with `pattern` (three fit a
// CU's 160 KiB, so a grid of ≥ 3·256 blocks covers every CU's LDS).
constexpr int kPoisonLdsBytes = 53 * 1024;
hipError_t launch_poison_lds(unsigned long long pattern, int n_blocks, hipStream_t s);

}  // namespace ekfslam
