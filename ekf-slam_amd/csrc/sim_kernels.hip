// On-device Monte-Carlo inputs (include/ekf_sim.h): one wavefront per filter walks a run's T
// messages in order — nusim's slipping wheels and DiffDrive::FKin truth (nusim/src/nusim.cpp:222-230,
// turtlelib/src/diff_drive.cpp:10-28) and the encoders' odometry (slam.cpp:599-634), the fake
// sensor (nusim.cpp:317-346) over the map on all 64 lanes, then the message's descriptor for the
// filter kernels (what ekf_api.cpp's plan_known writes on the host).
//
// FKin composes one arc per tick: config ← config · Δ_k. The ticks of a message are independent
// until that product, so lane j integrates tick j's arc and the wave composes the arcs with an
// inclusive scan (SE(2) composition is associative): log2(ticks) dependent compositions per
// message instead of one per tick. The host restatement (synth._simulate) composes tick by tick,
// so the two agree to rounding (≈1e-14 m per message), not bit for bit.
//
// Randomness is pyekf.synth's counter-based splitmix64, draw for draw: slip of wheel w at global
// tick k is uniform draw 2k + w of stream 1 under seed + f0 + f; the noise of marker i of message
// t is normal draw 2(t·M + i) (+1 for y) of stream 2. Compiled with -ffp-contract=off, so every
// product and sum rounds as numpy's does (synth.py is the host restatement this is tested against).
#include <hip/hip_runtime.h>

#include <climits>
#include <cmath>

#include "ekf_device.hpp"
#include "ekf_math.hpp"
#include "geom.hpp"
#include "sim_launch.hpp"

namespace ekfslam {
namespace {

constexpr unsigned long long kGolden = 0x9E3779B97F4A7C15ull;
constexpr unsigned long long kSlipStream = 1, kNoiseStream = 2;  // synth._S_SLIP, _S_NOISE
constexpr int kSenseNearest = 0, kSenseSurvey = 1, kSenseAll = 2;
constexpr double kSurveyRange = 2.0;  // synth.SURVEY_RANGE
constexpr int kPerLane = kSimMaxMap / 64;

__device__ __forceinline__ unsigned long long mix64(unsigned long long z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
__device__ __forceinline__ double uniform(unsigned long long seed, unsigned long long stream,
                                          unsigned long long idx) {
  const unsigned long long key = mix64(seed * kGolden + stream);
  return static_cast<double>(mix64(key + (idx + 1) * kGolden) >> 11) * 0x1p-53;
}
// N(0, 1) by Box–Muller from draws 2·idx, 2·idx + 1 (synth.rng_normal)
__device__ __forceinline__ double normal(unsigned long long seed, unsigned long long stream,
                                         unsigned long long idx) {
  const double u1 = 1.0 - uniform(seed, stream, 2 * idx);
  const double u2 = uniform(seed, stream, 2 * idx + 1);
  return sqrt(-2.0 * log(u1)) * cos(2.0 * M_PI * u2);
}

__device__ __forceinline__ double bcast(double v, int l) { return __shfl(v, l, 64); }

// the arc of one tick with wheel-angle increments (dl, dr) (DiffDrive::fkin's Δ)
__device__ __forceinline__ Pose2 arc(double dl, double dr, double radius, double track) {
  const Twist2 tw{radius / track * (-dl + dr), radius / 2.0 * (dl + dr), 0.0};
  return integrate_twist(tw);
}

// inclusive scan of compose over lanes 0..n−1 (lane j ends with Δ_0 · … · Δ_j)
__device__ __forceinline__ Pose2 scan_compose(Pose2 d, int lane) {
  for (int o = 1; o < 64; o <<= 1) {
    const Pose2 e{__shfl_up(d.theta, o, 64), __shfl_up(d.x, o, 64), __shfl_up(d.y, o, 64)};
    if (lane >= o) d = compose(e, d);
  }
  return d;
}

struct SimShared {
  double bx[kSimMaxMap], by[kSimMaxMap];
  unsigned sighted[kSimMaxMap / 32];
  int sel[kMaxChunk];
  int ids[kMaxChunk], prev_ids[kMaxChunk];
};

// One message's wheels (nusim.cpp:222-230, slam.cpp:599-634): lane j < tpm is tick j, the wave
// composes the ticks' arcs by a scan into the message's products (true, odometry; wave-uniform),
// which the true pose and the odometry then advance by.
__device__ __forceinline__ void arc_products(const SimArgs& A, unsigned long long seed, int t,
                                             int lane, Pose2& pt, Pose2& po) {
  Pose2 dt{0.0, 0.0, 0.0}, dot{0.0, 0.0, 0.0};  // identity past the message's ticks
  if (lane < A.tpm) {
    const size_t k = static_cast<size_t>(t) * A.tpm + lane;
    const double cl = A.cmd[2 * k], cr = A.cmd[2 * k + 1];
    const unsigned long long g = static_cast<unsigned long long>(A.tick0) + k;
    const double sl = cl * (1.0 + A.slip * (2.0 * uniform(seed, kSlipStream, 2 * g) - 1.0));
    const double sr = cr * (1.0 + A.slip * (2.0 * uniform(seed, kSlipStream, 2 * g + 1) - 1.0));
    dt = arc(sl, sr, A.radius, A.track);
    dot = arc(cl, cr, A.radius, A.track);
  }
  dt = scan_compose(dt, lane);
  dot = scan_compose(dot, lane);
  const int last = A.tpm - 1;
  pt = Pose2{bcast(dt.theta, last), bcast(dt.x, last), bcast(dt.y, last)};
  po = Pose2{bcast(dot.theta, last), bcast(dot.x, last), bcast(dot.y, last)};
}
__device__ __forceinline__ void wheels(const SimArgs& A, unsigned long long seed, int t, int lane,
                                       Pose2& truth, Pose2& odo) {
  Pose2 pt, po;
  arc_products(A, seed, t, lane, pt, po);
  truth = compose(truth, pt);
  odo = compose(odo, po);
}

// The fake sensor of one message at the true pose (th, px, py) (nusim.cpp:317-346): every
// landmark of the map `lm` in the true body frame R(θ)ᵀ(p − x) into sh.bx / sh.by (kMap), the
// selected landmarks into sh.sel (nearest first, or id order for ALL). Returns their count k.
// Without the map (k_sim_sense: no SURVEY message) `marker` recomputes a selected landmark's body
// frame position by the same expressions (the same bits), and the wave needs 64 B of LDS, not 16 KB.
template <bool kMap = true, typename Sh>
__device__ __forceinline__ int sense(const SimArgs& A, const double* lm, int mode, double th,
                                     double px, double py, Sh& sh, int lane) {
  const int L = A.L;
  const double c = cos(th), s = sin(th);
  const double rng = mode == kSenseSurvey ? kSurveyRange * A.range : A.range;
  double key[kPerLane];
  double dmin = INFINITY;
  bool any = false;
#pragma unroll
  for (int j = 0; j < kPerLane; ++j) {
    const int l = lane + 64 * j;
    key[j] = INFINITY;
    if (l < L) {
      const double dx = lm[2 * l] - px, dy = lm[2 * l + 1] - py;
      const double bx = c * dx + s * dy, by = -s * dx + c * dy;
      const double d = hypot(bx, by);
      if constexpr (kMap) {
        sh.bx[l] = bx;
        sh.by[l] = by;
      }
      dmin = fmin(dmin, d);
      double kk = d <= rng ? d : INFINITY;
      any = any || kk != INFINITY;
      if constexpr (kMap) {  // (SURVEY: a run with the map)
        if (mode == kSenseSurvey && kk != INFINITY && ((sh.sighted[l >> 5] >> (l & 31)) & 1u))
          kk = kk + 1e6;
      }
      key[j] = kk;
      if (mode == kSenseAll) key[j] = d;  // (the ADD / DELETE test below)
    }
  }
  if constexpr (kMap) __syncthreads();  // every lane's sh.bx / sh.by before the survey fallback
  int k = 0;
  if (mode == kSenseAll) {
    k = L;  // every landmark, in id order (L ≤ kMaxChunk, checked on the host)
    if (lane < L) sh.sel[lane] = lane;
  } else {
    if (kMap && mode == kSenseSurvey && !__any(any)) {  // never empty: the nearest, out of range
      for (int o = 32; o > 0; o >>= 1) dmin = fmin(dmin, __shfl_xor(dmin, o, 64));
      if constexpr (kMap) {
#pragma unroll
        for (int j = 0; j < kPerLane; ++j) {
          const int l = lane + 64 * j;
          if (l < L) key[j] = hypot(sh.bx[l], sh.by[l]) == dmin ? dmin : INFINITY;
        }
      }
    }
    // the m smallest keys, ties to the lower index (synth: a stable argsort)
    unsigned taken = 0;
    for (; k < A.m; ++k) {
      double best = INFINITY;
      int bi = INT_MAX;
#pragma unroll
      for (int j = 0; j < kPerLane; ++j) {
        const int l = lane + 64 * j;
        if (!((taken >> j) & 1u) && (key[j] < best || (key[j] == best && l < bi)) && l < L) {
          best = key[j];
          bi = l;
        }
      }
      // (smaller key, ties to the lower index: a strict total order, so the DPP tree of
      // ekf_math.hpp gives the pair the shuffle butterfly gave)
      wave_argmin(best, bi);
      if (best == INFINITY) break;  // wave-uniform
      if ((bi & 63) == lane) taken |= 1u << (bi >> 6);
      if (lane == 0) sh.sel[k] = bi;
    }
  }
  __syncthreads();
  return k;
}

// Marker `lane` < k of message `msg`: its landmark, the noisy body-frame position (draws
// 2·(msg·M + lane) and + 1 of stream 2) and ADD / DELETE (beyond range, mode ALL).
// (kMap false: the body frame position from the map `lm` at the true pose (th, px, py), as sense)
template <bool kMap = true, typename Sh>
__device__ __forceinline__ void marker(const SimArgs& A, unsigned long long seed, long long msg,
                                       int mode, int k, const Sh& sh, int lane, int* id,
                                       int* act, double* rx, double* ry, const double* lm = nullptr,
                                       double th = 0.0, double px = 0.0, double py = 0.0) {
  *id = -1;
  *act = 0;
  *rx = *ry = 0.0;
  if (lane < k) {
    *id = sh.sel[lane];
    double bx, by;
    if constexpr (kMap) {
      bx = sh.bx[*id];
      by = sh.by[*id];
    } else {
      const double c = cos(th), s = sin(th);
      const double dx = lm[2 * *id] - px, dy = lm[2 * *id + 1] - py;
      bx = c * dx + s * dy;
      by = -s * dx + c * dy;
    }
    const unsigned long long idx = (static_cast<unsigned long long>(msg) * A.M + lane) * 2;
    *rx = bx + A.sigma * normal(seed, kNoiseStream, idx);
    *ry = by + A.sigma * normal(seed, kNoiseStream, idx + 1);
    *act = mode == kSenseAll && !(hypot(bx, by) <= A.range) ? 2 : 0;  // DELETE
  }
}

// the message's markers as ekf_replay takes them (row `rowo` = t·F + f of the record arrays)
__device__ __forceinline__ void record_markers(const SimArgs& A, size_t rowo, int k, int id,
                                               int act, double rx, double ry, int lane) {
  const int M = A.M;
  for (int i = lane; i < M; i += 64) {
    const size_t o = rowo * M + i;
    A.out_ids[o] = i < k ? __shfl(id, i, 64) : -1;
    A.out_act[o] = i < k ? __shfl(act, i, 64) : 0;
    A.out_rel[2 * o] = i < k ? __shfl(rx, i, 64) : 0.0;
    A.out_rel[2 * o + 1] = i < k ? __shfl(ry, i, 64) : 0.0;
  }
  if (lane == 0) A.out_cnt[rowo] = k;
}

}  // namespace

__global__ __launch_bounds__(64) void k_sim(SimArgs A) {
  __shared__ SimShared sh;
  const int f = blockIdx.x, lane = threadIdx.x;
  const int L = A.L;
  const unsigned long long seed = A.seed + static_cast<unsigned long long>(A.f0 + f);
  SimState& S = A.st[f];
  const double* lm = A.lm + static_cast<size_t>(f) * L * 2;
  const int words = (L + 31) / 32;
  for (int w = lane; w < words; w += 64) sh.sighted[w] = A.sighted[static_cast<size_t>(f) * words + w];
  __syncthreads();  // (one wave: order the lanes' LDS writes before any lane reads another's word)
  // the true pose (slipping wheels) and the odometry (commanded encoder angles), wave-uniform
  Pose2 truth{S.truth[0], S.truth[1], S.truth[2]};
  Pose2 odo{S.odom[0], S.odom[1], S.odom[2]};
  int par = A.par[f];
  int prev_m = -1;       // the previous active chunk of this run (−1: the run's first gathers Σ_in)
  for (int t = 0; t < A.T; ++t) {
    const long long msg = A.msg0 + t;
    wheels(A, seed, t, lane, truth, odo);
    const double th = truth.theta, px = truth.x, py = truth.y;
    const double oth = odo.theta, ox = odo.x, oy = odo.y;
    if (A.out_truth && lane < 3)
      A.out_truth[(static_cast<size_t>(t) * A.F + f) * 3 + lane] = lane == 0 ? th : (lane == 1 ? px : py);
    if (A.out_odom && f == 0 && lane < 3)
      A.out_odom[static_cast<size_t>(t) * 3 + lane] = lane == 0 ? oth : (lane == 1 ? ox : oy);
    const int mode = A.sense ? A.sense[t] : kSenseNearest;
    const int k = sense(A, lm, mode, th, px, py, sh, lane);
    // ---- markers: noise, record, descriptor ----
    const size_t rowo = static_cast<size_t>(t) * A.F + f;
    int id, act;
    double rx, ry;
    marker(A, seed, msg, mode, k, sh, lane, &id, &act, &rx, &ry);
    if (lane < k && mode == kSenseSurvey) atomicOr(&sh.sighted[id >> 5], 1u << (id & 31));
    if (A.out_ids) record_markers(A, rowo, k, id, act, rx, ry, lane);
    // the filter's chunk: the non-DELETE markers in order (slam.cpp:205), z as slam.cpp:208-210
    const bool add = lane < k && act != 2;
    const unsigned long long bal = __ballot(add);
    const int m = __popcll(bal);
    const int pos = __popcll(bal & ((1ull << lane) - 1ull));
    MsgDesc* d = A.desc + rowo;
    double* dz = reinterpret_cast<double*>(d);
    for (int e = lane; e < static_cast<int>(sizeof(MsgDesc) / 8); e += 64) dz[e] = 0.0;
    __syncthreads();
    if (k == 0) continue;  // no marker: the filter gets no message (ekf_replay's counts 0)
    if (add) {
      d->ids[pos] = id;
      sh.ids[pos] = id;
      d->z[pos][0] = sqrt(rx * rx + ry * ry);  // std::pow(x, 2) is x·x rounded
      d->z[pos][1] = atan2(ry, rx);
    }
    if (lane == 0) {
      d->m = m;
      d->flags = kActive | kFirst | kLast | (prev_m >= 0 ? kLook : 0) | (A.joseph ? kJoseph : 0);
      d->parity = par;
      d->odom[0] = oth;
      d->odom[1] = ox;
      d->odom[2] = oy;
      d->prev_m = prev_m;
    }
    if (lane < kMaxChunk) d->prev_ids[lane] = prev_m >= 0 ? sh.prev_ids[lane] : 0;
    __syncthreads();
    if (lane < kMaxChunk) sh.prev_ids[lane] = lane < m ? sh.ids[lane] : 0;
    __syncthreads();
    prev_m = m;
    par ^= 1;
  }
  // state for the next run
  if (lane == 0) {
    S.truth[0] = truth.theta;
    S.truth[1] = truth.x;
    S.truth[2] = truth.y;
    S.odom[0] = odo.theta;
    S.odom[1] = odo.x;
    S.odom[2] = odo.y;
    A.par[f] = par;
  }
  for (int w = lane; w < words; w += 64) A.sighted[static_cast<size_t>(f) * words + w] = sh.sighted[w];
}

// ---- runs without SURVEY messages: every message sensed in parallel ----------------------------
// Only the survey's sighted set carries sensing state from one message to the next; without it a
// message's markers depend on its true pose alone. Pass 1 (k_sim_arcs, one wave per message and
// filter: each message's tick scan; then k_sim_pose, one wave per filter: the products composed in
// message order — the only sequential part) writes every message's true pose and odometry; pass 2 (k_sim_sense, one wave per message and filter, T·F in
// flight instead of F) senses and records the markers as ekf_replay takes them, and the device
// planner of ekf_replay_device (plan_kernels.hip) writes the descriptors from those. Same
// functions, draws and order as k_sim, so the same bits.
// Pass 1a: each message's tick products (one wave per (message, filter), in parallel) into
// truth_all / odom_all; pass 1b (k_sim_pose) composes them in message order over them.
__global__ __launch_bounds__(64) void k_sim_arcs(SimArgs A, double* truth_all, double* odom_all) {
  const int t = blockIdx.x, f = blockIdx.y, lane = threadIdx.x;
  const unsigned long long seed = A.seed + static_cast<unsigned long long>(A.f0 + f);
  Pose2 pt, po;
  arc_products(A, seed, t, lane, pt, po);
  const size_t o = (static_cast<size_t>(t) * A.F + f) * 3;
  if (lane < 3) {
    truth_all[o + lane] = lane == 0 ? pt.theta : (lane == 1 ? pt.x : pt.y);
    odom_all[o + lane] = lane == 0 ? po.theta : (lane == 1 ? po.x : po.y);
  }
}

__global__ __launch_bounds__(64) void k_sim_pose(SimArgs A, double* truth_all, double* odom_all) {
  const int f = blockIdx.x, lane = threadIdx.x;
  SimState& S = A.st[f];
  Pose2 truth{S.truth[0], S.truth[1], S.truth[2]};
  Pose2 odo{S.odom[0], S.odom[1], S.odom[2]};
  for (int t = 0; t < A.T; ++t) {
    const size_t o = (static_cast<size_t>(t) * A.F + f) * 3;
    // the message's products (k_sim_arcs), then the poses after it over them (same slot, same wave)
    truth = compose(truth, Pose2{truth_all[o], truth_all[o + 1], truth_all[o + 2]});
    odo = compose(odo, Pose2{odom_all[o], odom_all[o + 1], odom_all[o + 2]});
    if (lane < 3) {
      const double tv = lane == 0 ? truth.theta : (lane == 1 ? truth.x : truth.y);
      const double ov = lane == 0 ? odo.theta : (lane == 1 ? odo.x : odo.y);
      truth_all[o + lane] = tv;
      odom_all[o + lane] = ov;
      if (A.out_truth) A.out_truth[o + lane] = tv;
      if (A.out_odom && f == 0) A.out_odom[static_cast<size_t>(t) * 3 + lane] = ov;
    }
  }
  if (lane == 0) {
    S.truth[0] = truth.theta;
    S.truth[1] = truth.x;
    S.truth[2] = truth.y;
    S.odom[0] = odo.theta;
    S.odom[1] = odo.x;
    S.odom[2] = odo.y;
  }
}

struct SenseShared {
  int sel[kMaxChunk];
};
__global__ __launch_bounds__(64) void k_sim_sense(SimArgs A, const double* truth_all) {
  __shared__ SenseShared sh;
  const int t = blockIdx.x, f = blockIdx.y, lane = threadIdx.x;
  const unsigned long long seed = A.seed + static_cast<unsigned long long>(A.f0 + f);
  const size_t rowo = static_cast<size_t>(t) * A.F + f;
  const double th = truth_all[rowo * 3], px = truth_all[rowo * 3 + 1], py = truth_all[rowo * 3 + 2];
  const int mode = A.sense ? A.sense[t] : kSenseNearest;  // (never SURVEY here)
  const double* lm = A.lm + static_cast<size_t>(f) * A.L * 2;
  const int k = sense<false>(A, lm, mode, th, px, py, sh, lane);
  int id, act;
  double rx, ry;
  marker<false>(A, seed, A.msg0 + t, mode, k, sh, lane, &id, &act, &rx, &ry, lm, th, px, py);
  record_markers(A, rowo, k, id, act, rx, ry, lane);
}

hipError_t launch_sim(const SimArgs& a, hipStream_t s) {
  hipLaunchKernelGGL(k_sim, dim3(a.F), dim3(64), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_sim_parallel(const SimArgs& a, double* truth_all, double* odom_all, hipStream_t s) {
  hipLaunchKernelGGL(k_sim_arcs, dim3(a.T, a.F), dim3(64), 0, s, a, truth_all, odom_all);
  hipLaunchKernelGGL(k_sim_pose, dim3(a.F), dim3(64), 0, s, a, truth_all, odom_all);
  hipLaunchKernelGGL(k_sim_sense, dim3(a.T, a.F), dim3(64), 0, s, a,
                     static_cast<const double*>(truth_all));
  return hipGetLastError();
}

}  // namespace ekfslam
