// Known-association replay planned on the GPU (ekf_replay_device, include/ekf.h): for every
// message t and filter f the MsgDesc that ekf_api.cpp's plan_known writes on the host for the
// same inputs (one chunk per message, m ≤ kMaxChunk), built from inputs already in HBM.
//
// One wave per (t, f), all in parallel. What a host plan carries from chunk to chunk is found by
// scanning the counts instead: the filter's previous active message (its markers are this
// chunk's U' for the kLook rebuild), the one after next (the kStageOut operands of the chunk
// after next), and the active messages before t (the parity).
// A message with count 0 is no message (ekf_batch_sensor: the filter sits the step out); one
// whose markers are all DELETE is a predict + posterior (slam.cpp:205), as on the host.
// Joseph form (A.joseph = 1): the same chunks, flagged kJoseph (kMaxJoseph = kMaxChunk markers).
#include <hip/hip_runtime.h>

#include "ekf.h"
#include "ekf_device.hpp"
#include "ekf_launch.hpp"

namespace ekfslam {
namespace {

struct PlanShared {
  MsgDesc d;
  int ids[4][kMaxChunk];  // compacted (non-DELETE) ids of t, prev, next, next2
  int m[4];
};

}  // namespace

// highest / lowest set bit of a 64-bit mask (−1: none)
__device__ __forceinline__ int hi_bit(unsigned long long b) { return b ? 63 - __clzll(b) : -1; }
__device__ __forceinline__ int lo_bit(unsigned long long b) { return b ? __ffsll(static_cast<long long>(b)) - 1 : -1; }

__global__ __launch_bounds__(64) void k_plan_replay(ReplayArgs A) {
  __shared__ PlanShared sh;
  const int t = blockIdx.x, f = blockIdx.y, lane = threadIdx.x;
  const int F = A.F, M = A.M, T = A.T;
  const size_t tf = static_cast<size_t>(t) * F + f;
  auto cnt = [&](int tt) { return A.counts[static_cast<size_t>(tt) * F + f]; };
  const PlanState& s0 = A.st_in[f];
  // ---- round trip 1: the counts of messages t − 64 .. t + 63 (bit l of lo ↔ t − 64 + l, of hi ↔
  // t + l); the neighbours almost always lie in this window, the loops below are the fallback ----
  const int tlo = t - 64 + lane, thi = t + lane;
  const unsigned long long blo = __ballot(tlo >= 0 && cnt(tlo) > 0);
  const unsigned long long bhi = __ballot(thi < T && cnt(thi) > 0);
  int before = __popcll(blo);  // active messages before t: the parity flips once per chunk
  for (int base = 0; base < t - 64; base += 64)
    before += __popcll(__ballot(base + lane < t - 64 && cnt(base + lane) > 0));
  auto scan_back = [&](int from) {  // largest tt ≤ from with a message, −1: none
    for (int base = from; base >= 0; base -= 64) {
      const int tt = base - lane;
      const unsigned long long b = __ballot(tt >= 0 && cnt(tt) > 0);
      if (b) return base - lo_bit(b);
    }
    return -1;
  };
  auto scan_fwd = [&](int from) {  // smallest tt ≥ from with a message, −1: none
    for (int base = from; base < T; base += 64) {
      const int tt = base + lane;
      const unsigned long long b = __ballot(tt < T && cnt(tt) > 0);
      if (b) return base + lo_bit(b);
    }
    return -1;
  };
  const bool active = bhi & 1ull;
  int prev = hi_bit(blo), prev2 = hi_bit(prev >= 0 ? blo & ~(1ull << prev) : 0ull);
  prev = prev >= 0 ? t - 64 + prev : scan_back(t - 65);
  prev2 = prev2 >= 0 ? t - 64 + prev2 : (prev > 0 ? scan_back(min(prev - 1, t - 65)) : -1);
  const unsigned long long bn = bhi & ~1ull;
  int next = lo_bit(bn), next2 = lo_bit(next >= 0 ? bn & ~(1ull << next) : 0ull);
  next = next >= 0 ? t + next : scan_fwd(t + 64);
  next2 = next2 >= 0 ? t + next2 : (next >= 0 ? scan_fwd(max(next + 1, t + 64)) : -1);
  const bool last_wave = t == T - 1;  // also writes the filter's state after the replay
  const int last = active ? t : prev;
  // ---- round trip 2: the markers of t, prev, next, next2 (slots 0..3), t's bearings and odom ----
  const int mi[4] = {active ? t : -1, active || last_wave ? prev : -1, active ? next : -1,
                     active ? next2 : -1};
  int id4[4], c4[4];
  bool del4[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    c4[k] = mi[k] >= 0 ? min(cnt(mi[k]), M) : 0;
    const size_t o = (static_cast<size_t>(mi[k] >= 0 ? mi[k] : 0) * F + f) * M + min(lane, M - 1);
    id4[k] = M > 0 ? A.ids[o] : 0;
    del4[k] = A.actions && M > 0 && A.actions[o] == EKF_MARKER_DELETE;
  }
  const size_t o0 = tf * M + min(lane, M - 1);
  const double rx = M > 0 ? A.rel[2 * o0] : 0.0, ry = M > 0 ? A.rel[2 * o0 + 1] : 0.0;
  const double od = lane < 3 ? A.odom[tf * 3 + lane] : 0.0;
  // the non-DELETE markers of each slot, compacted (slam.cpp:205's skip)
  int pos0 = 0;
  bool add0 = false;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const bool add = lane < c4[k] && !del4[k];
    const unsigned long long bal = __ballot(add);
    const int pos = static_cast<int>(__popcll(bal & ((1ull << lane) - 1ull)));
    if (lane < kMaxChunk) sh.ids[k][lane] = 0;
    if (lane == 0) sh.m[k] = min(static_cast<int>(__popcll(bal)), kMaxChunk);
    if (k == 0) {
      pos0 = pos;
      add0 = add;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    if (add && pos < kMaxChunk) sh.ids[k][pos] = id4[k];
  }
  uint4* dz = reinterpret_cast<uint4*>(&sh.d);
  for (int e = lane; e < static_cast<int>(sizeof(MsgDesc) / 16); e += 64) dz[e] = uint4{0, 0, 0, 0};
  __syncthreads();
  // ---- the filter's state after the replay (the host adopts it lazily) ----
  if (last_wave) {
    PlanState& so = A.st_out[f];
    const int ms = active ? sh.m[0] : sh.m[1];
    const int* li = active ? sh.ids[0] : sh.ids[1];
    if (lane == 0) {
      so.parity = s0.parity ^ ((before + (active ? 1 : 0)) & 1);
      so.prev_m = last >= 0 ? ms : s0.prev_m;
      so.pending = last >= 0 ? 0 : s0.pending;
      so.pad = 0;
    }
    if (lane < kMaxChunk) so.prev_ids[lane] = last >= 0 ? li[lane] : s0.prev_ids[lane];
    if (lane < 3) so.odom[lane] = od;
  }
  // ---- the descriptor of (t, f) ----
  if (active) {
    const int m = sh.m[0];
    const int prev_m = prev >= 0 ? sh.m[1] : s0.prev_m;
    MsgDesc& d = sh.d;
    if (add0 && pos0 < kMaxChunk) {  // z: slam.cpp:208-210 (std::pow(x, 2) is x·x; sqrt rounds alike)
      d.z[pos0][0] = sqrt(rx * rx + ry * ry);
      d.z[pos0][1] = atan2(ry, rx);
    }
    if (lane < kMaxChunk) {
      d.ids[lane] = sh.ids[0][lane];
      d.prev_ids[lane] = prev >= 0 ? sh.ids[1][lane] : (s0.prev_m >= 0 ? s0.prev_ids[lane] : 0);
    }
    if (lane < 3) d.odom[lane] = od;
    if (lane == 0) {
      int flags = kActive | kFirst | kLast | (A.joseph ? kJoseph : 0) | (prev_m >= 0 ? kLook : 0);
      // the chain two chunks on rebuilds from operands this chunk's Σ pass stages (plan_known:
      // both chunks in this plan); this chunk reads the ones staged two chunks back
      if (A.stage && prev_m >= 0 && prev2 >= 0) flags |= kStageIn;
      if (A.stage && next2 >= 0) {
        flags |= kStageOut;
        d.stg_m = sh.m[3];
        d.stg_pm = sh.m[2];
      }
      d.m = m;
      d.flags = flags;
      d.parity = s0.parity ^ (before & 1);
      d.prev_m = prev_m;
    }
    if (A.stage && next2 >= 0 && lane < kMaxChunk) {
      d.stg_ids[lane] = sh.ids[3][lane];
      d.stg_pids[lane] = sh.ids[2][lane];
    }
  }
  __syncthreads();
  uint4* gd = reinterpret_cast<uint4*>(A.desc + tf);
  for (int e = lane; e < static_cast<int>(sizeof(MsgDesc) / 16); e += 64) gd[e] = dz[e];
  if (A.plan_count) {  // the wave's stores (every lane's) complete, released, then counted; the
                       // explicit waits around the fence: the compiler may drop the fence's own
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_fetch_add(A.plan_count, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

hipError_t launch_plan_replay(const ReplayArgs& a, hipStream_t s) {
  if (a.T <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_plan_replay, dim3(a.T, a.F), dim3(64), 0, s, a);
  return hipGetLastError();
}

}  // namespace ekfslam
