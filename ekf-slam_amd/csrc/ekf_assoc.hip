// Unknown association (Slam::sensor_cb, nuslam/src/slam.cpp:318-530) for a whole chunk of markers
// in ONE launch, followed by a single Σ pass — instead of an association kernel, a chain, a factor
// kernel and a Σ pass per marker.
//
// Why it works. A chunk's corrections are Σ_{c+1} = Σ_c − K_c·M_c (slam.cpp:264-265, rank 2 each)
// on the predicted Σ_p (slam.cpp:321-335). Marker c's association (slam.cpp:358-440) reads, for every
// known landmark k, only the 5 × 5 block of Σ_c over {θ, x, y, kx, ky} and x_c at those indices. Those
// 16 entries per landmark evolve by the same rank-2 terms, so each landmark can carry its own block:
//   Σ_{c+1}[k, k] = Σ_c[k, k] − K_c[k]·M_c[:, k],  Σ_{c+1}[k, p] = Σ_c[k, p] − K_c[k]·M_c[:, p], …
// with K_c[k] = Σ_c[k, pA]·Hᵀ·S⁻¹ and M_c[:, k] = H·Σ_c[pA, k] over pA = {θ, x, y, jx, jy}. The only
// entries of Σ_c outside the blocks that a step needs are the crosses with its landmark j:
//   Σ_c[k, j] = Σ_p[k, j] − Σ_{c'<c} K_{c'}[k]·M_{c'}[:, j],   Σ_c[j, k] likewise,
// i.e. Σ_in (no predict term between landmarks) and the factor histories of k and of j. So:
//   * one lane per landmark slot, 64 slots per workgroup (wave 0; waves 1-2 only sum the history
//     terms, history_helper), G = ⌈N / 64⌉ workgroups per
//     filter; a lane keeps its slot's block and state in registers and its K / M history in LDS;
//   * per marker: every lane scores its landmark (k_assoc's expression, ekf_math.hpp assoc_dist),
//     a wave argmin (first index on ties, arma::index_min), then the G workgroups exchange their
//     (d, k) as tagged 8-byte granules (cdna_hip_programming.md Guideline 16, R2) and every one
//     takes the same decision: commit a new landmark (slam.cpp:421-422) or the argmin;
//   * the chosen landmark's block, state and history are read from write-through tables (every
//     lane publishes its slot's K, M and next block each step, drained before the granule), its
//     crosses with each lane's landmark are gathered from Σ_in; every workgroup then forms the same
//     S, S⁻¹, ν, K[pose], M[pose] and each lane its own K[k], M[k] — the chunk's Kcat / Mcat rows
//     for the Σ pass — and applies the step to its block and state.
// The Σ pass (k_sigma_pass, ekf_kernels.hip) then applies Σ_out = Σ_in + Q̄ − Kcatᵀ·Mcat once.
// fp32 Σ: a chunk that commits a new landmark also writes the final Σ[U, U] in fp64 (ChunkRec::Pend,
// the first sighting's 1e7 − (1e7 − δ), slam.cpp:130) for k_patch_stage, after a last exchange.
//
// In exact arithmetic this equals the reference's sequential dense algebra; the decisions are the
// reference's (tests/test_gpu_scale.py: every decision equal to the oracle's, new and known
// landmarks, a marker 3e-4 from the gate).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <climits>
#include <cstdint>

#include "ekf_device.hpp"
#include "ekf_launch.hpp"
#include "ekf_math.hpp"
#include "geom.hpp"

namespace ekfslam {

#include "ekf_sync.hpp"

// Diagnostic build only (tools/assoc_stamps.py): s_memrealtime (100 MHz) of workgroup 0 / the last
// workgroup, lane 0, per step and phase, of the last launch.
#ifdef EKF_DIAG_STAMPS
__device__ unsigned long long g_am_stamps[2][kMaxChunk + 1][8];
#define AM_STAMP(c, i)                                                                    \
  do {                                                                                    \
    if (blockIdx.y == 0 && threadIdx.x == 0 && (g == 0 || g == G - 1))                    \
      g_am_stamps[g == 0 ? 0 : 1][c][i] = __builtin_amdgcn_s_memrealtime();               \
  } while (0)
#else
#define AM_STAMP(c, i) \
  do {                 \
  } while (0)
#endif

namespace {


// Three waves per workgroup: wave 0 does everything below; waves 1 and 2 (history_helper) only sum
// each step's history terms of the lanes' crosses with the step's landmark (Σ_c[k, j], Σ_c[j, k]),
// the even steps' on wave 1 and the odd steps' on wave 2 — the two fma chains wave 0 interleaved
// alone before, so the same bits — while wave 0 forms the step's pose-level quantities, which do
// not need them.
constexpr int kAmThreads = 3 * kAmSlots;

// J: the Joseph form (ekf_set_joseph; every descriptor kJoseph). Each step then also subtracts
// V_c·K_cᵀ, V_c = Σ_c·Hᵀ − K_c·S_c (slam.cpp:264-265's update as (I − KH)Σ(I − KH)ᵀ + K·R·Kᵀ
// expanded, as k_chain's Joseph form), after the K_c·M_c term: the history carries V too.
template <bool J>
struct AmSharedT {
  static constexpr int HW = J ? 12 : 8;  // history doubles per (step, slot): K, M (, V)
  alignas(16) double hkm[kMaxChunk][kAmSlots][HW];  // wave 0's K_c[k] (0..3), M_c[:, k] (4..7)
                                       // (and V_c[k], 8..11), by lane: a lane's step in 64 (96)
                                       // contiguous bytes (ds_read_b128 × 4 (6))
  double es[2][8][kAmSlots];          // waves 1 / 2: the even / odd steps' history sums, by lane
  double jh[kMaxChunk][HW];           // the step's landmark: K (0..3), M (4..7) (, V) of every step
  double jc[18];                      // its block and state (AmCur, x included)
  double pb[kMaxChunk][18];           // fp32 patch: every marker's landmark's final block
  double pp[9];                       // fp32 patch: the final pose block
  int jl[kMaxChunk];                  // the chunk's landmark per marker (−1: skipped)
};

// The lane's predicted block of slot entries: Σ_p[k][b] = Σ[k][b] + Σ[k][0]·α_b,
// Σ_p[a][k] = Σ[a][k] + α_a·Σ[0][k] (k_assoc's expressions; At has α only in rows 1, 2).
template <typename T>
__device__ __forceinline__ void slot_block(const T* S, int ld, int ix, double a1, double a2,
                                           double (&kk)[4], double (&kp)[6], double (&pk)[6]) {
  const T* q0 = S + static_cast<size_t>(ix) * ld;
  const T* q1 = q0 + ld;
  double rk[2][3], rp[3][2];
#pragma unroll
  for (int b = 0; b < 3; ++b) {
    rk[0][b] = static_cast<double>(q0[b]);
    rk[1][b] = static_cast<double>(q1[b]);
  }
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    rp[a][0] = static_cast<double>(S[a * ld + ix]);
    rp[a][1] = static_cast<double>(S[a * ld + ix + 1]);
  }
  kk[0] = static_cast<double>(q0[ix]);
  kk[1] = static_cast<double>(q0[ix + 1]);
  kk[2] = static_cast<double>(q1[ix]);
  kk[3] = static_cast<double>(q1[ix + 1]);
#pragma unroll
  for (int e = 0; e < 2; ++e)
#pragma unroll
    for (int b = 0; b < 3; ++b) kp[3 * e + b] = rk[e][b] + rk[e][0] * alpha_of(b, a1, a2);
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int e = 0; e < 2; ++e) pk[2 * a + e] = rp[a][e] + alpha_of(a, a1, a2) * rp[0][e];
}

__device__ __forceinline__ unsigned long long ld_sc1_u64(const unsigned long long* p) {
  return __hip_atomic_load((const gu64*)(p), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
}

// Coherence of what a filter's G workgroups exchange within a launch (granules, tables). Loads are
// sc1 in both modes: they miss the CU's L1 and read the XCD's L2 coherently. Stores:
//  - agent mode (any placement): sc1, written through past the XCD's L2 to memory, where a reader
//    on another XCD finds them;
//  - XCD-local mode (all G workgroups on one XCD, established by `same_xcd` at the launch's start):
//    plain, so they stop in the L2 the workgroups share (the CU's L1 is write-through).
// Measured (tools/xcd_probe.hip, one-way hand-off between two CUs): same XCD, plain store + sc1
// load 224 ns, sc1 store + sc1 load 414 ns; across XCDs sc1 + sc1 564 ns (plain stores are never
// seen there); sc0 loads hit a stale L1 line forever. Every value a local-mode launch reads was
// written in that launch by a CU of the same XCD, so a stale L2 line from an earlier launch is
// never read (the granules carry the launch's tag).
// Loads go through a buffer descriptor of the filter's table (wave-uniform) with the entry's byte
// offset per lane.
constexpr int kAuxSc1 = 16;
__device__ __forceinline__ unsigned long long ld_x64(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __builtin_bit_cast(unsigned long long,
                            __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, kAuxSc1));
}
__device__ __forceinline__ double ld_xf64(__amdgpu_buffer_rsrc_t r, unsigned off) {
  return __longlong_as_double(static_cast<long long>(ld_x64(r, off)));
}
__device__ __forceinline__ void st_x64(unsigned long long* p, unsigned long long v, bool loc) {
  typedef unsigned u2 __attribute__((ext_vector_type(2)));
  if (loc)  // a plain store (no cache-policy bits), as the probe's
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, v), buf_rsrc(p, 8), 0, 0, 0);
  else
    __hip_atomic_store((gu64*)(p), v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// 16-byte table store: write-through past L2 (agent mode) or into the shared L2 (XCD-local)
template <bool LOC>
__device__ __forceinline__ void st_x2(__amdgpu_buffer_rsrc_t r, int off, double a, double b) {
  if (LOC) {
    typedef int i4 __attribute__((ext_vector_type(4)));
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i4, make_double2(a, b)), r, off, 0, 0);
  } else {
    st_wt2(r, off, a, b);
  }
}

// This lane's rows of the write-through tables. The buffer descriptor is built from the
// workgroup's block of 64 rows (wave-uniform, so it stays in SGPRs); the lane's row is the voffset.
// (A per-lane descriptor made hipcc wrap every store in a 64-iteration waterfall loop: ≈ 30 µs per
// step.)
template <bool LOC>
__device__ __forceinline__ void put_cur_m(AmCur* blk, int lane, const double (&kk)[4],
                                          const double (&kp)[6], const double (&pk)[6],
                                          const double (&xk)[2]) {
  const auto r = buf_rsrc(blk, kAmSlots * sizeof(AmCur));
  const int o = lane * static_cast<int>(sizeof(AmCur));
  st_x2<LOC>(r, o + 0, kk[0], kk[1]);
  st_x2<LOC>(r, o + 16, kk[2], kk[3]);
  st_x2<LOC>(r, o + 32, kp[0], kp[1]);
  st_x2<LOC>(r, o + 48, kp[2], kp[3]);
  st_x2<LOC>(r, o + 64, kp[4], kp[5]);
  st_x2<LOC>(r, o + 80, pk[0], pk[1]);
  st_x2<LOC>(r, o + 96, pk[2], pk[3]);
  st_x2<LOC>(r, o + 112, pk[4], pk[5]);
  st_x2<LOC>(r, o + 128, xk[0], xk[1]);
}
template <bool LOC>
__device__ __forceinline__ void put_hist_m(AmHist* blk, int lane, const double* h, int hw) {
  const auto r = buf_rsrc(blk, kAmSlots * sizeof(AmHist));
  const int o = lane * static_cast<int>(sizeof(AmHist));
  for (int t = 0; t < hw; t += 2) st_x2<LOC>(r, o + 8 * t, h[t], h[t + 1]);  // (hw: 8 or 12)
}

__device__ __forceinline__ void put_cur(AmCur* blk, int lane, const double (&kk)[4],
                                        const double (&kp)[6], const double (&pk)[6],
                                        const double (&xk)[2], bool loc) {
  if (loc) put_cur_m<true>(blk, lane, kk, kp, pk, xk);
  else put_cur_m<false>(blk, lane, kk, kp, pk, xk);
}
// h: K (4), M (4) and, hw = 12, V (4) — the lane's LDS history row layout
__device__ __forceinline__ void put_hist(AmHist* blk, int lane, const double* h, int hw, bool loc) {
  if (loc) put_hist_m<true>(blk, lane, h, hw);
  else put_hist_m<false>(blk, lane, h, hw);
}

// The G workgroups of a filter publish their (d, k) for exchange `c` and wait for everyone's:
// three 8-byte {tag, value} granules per workgroup (d's two halves, k), stored by lane 0 after the
// wave's write-through table stores have drained; lanes < G poll one workgroup's each. Returns the
// filter-wide argmin (the same in every workgroup), or a partial argmin and *timeout after `spin`
// polls — the filter's state is then undefined (EKF_FLAG_TIMEOUT, reported by the host as
// EKF_E_TIMEOUT). `drop`: fault injection, this workgroup does not publish (tests only).
__device__ __forceinline__ void exchange(unsigned long long* gran, int G, int g, int c,
                                         unsigned tag, double& d, int& k, bool* timeout, bool loc,
                                         unsigned spin, bool drop = false) {
  drain_stores();  // R1: this wave's table stores of the step are complete before its granule
  const int lane = threadIdx.x;
  unsigned long long* mine = gran + (static_cast<size_t>(c) * G + g) * 4;
  const unsigned long long hi = static_cast<unsigned long long>(tag) << 32;
  const unsigned long long bits = static_cast<unsigned long long>(__double_as_longlong(d));
  if (lane == 0 && !drop) {
    st_x64(mine + 0, hi | (bits & 0xffffffffull), loc);
    st_x64(mine + 1, hi | (bits >> 32), loc);
    st_x64(mine + 2, hi | static_cast<unsigned>(k), loc);
  }
  const auto gr = buf_rsrc(gran, static_cast<unsigned>((kMaxChunk + 1) * G * 4 * 8));
  double od = INFINITY;
  int ok = INT_MAX;
  for (int base = 0; base < G; base += 64) {
    const int w = base + lane;
    const unsigned src = static_cast<unsigned>(((c * G + (w < G ? w : 0)) * 4) * 8);
    for (unsigned spins = 0;; ++spins) {
      bool got = true;
      unsigned long long v0 = 0, v1 = 0, v2 = 0;
      if (w < G) {
        v0 = ld_x64(gr, src + 0);
        v1 = ld_x64(gr, src + 8);
        v2 = ld_x64(gr, src + 16);
        got = (v0 >> 32) == tag && (v1 >> 32) == tag && (v2 >> 32) == tag;
      }
      if (__all(got)) {
        if (w < G) {
          const double dv = __longlong_as_double(
              static_cast<long long>(((v1 & 0xffffffffull) << 32) | (v0 & 0xffffffffull)));
          const int kv = static_cast<int>(static_cast<unsigned>(v2));
          if (dv < od || (dv == od && kv < ok)) {
            od = dv;
            ok = kv;
          }
        }
        break;
      }
      if (spins >= spin) {
        *timeout = true;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  // loads of the published tables come after the poll (sc1: they bypass this CU's L1)
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  wave_argmin(od, ok);
  d = od;
  k = ok;
}

// Roll call of a launch in XCD-local placement: every workgroup of the filter publishes its XCD
// (HW_REG_XCC_ID) in word 3 of its step-0 granule, agent-coherent; workgroup 0 reads all G and
// publishes the launch's transport in word 3 of its step-1 granule (unused by the exchanges), and
// every other workgroup takes that one decision. XCD-local only if all G sit on one XCD; so every
// workgroup runs the same transport, also when a poll times out (workgroup 0 then publishes the
// agent transport; a workgroup that never sees the decision takes it too, and the timeout is
// flagged: EKF_FLAG_TIMEOUT, the filter's state is undefined).
__device__ bool same_xcd(unsigned long long* gran, int G, int g, unsigned tag, bool* timeout,
                         unsigned spin) {
  const unsigned xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11)) & 0xffffu;
  const int lane = threadIdx.x;
  const unsigned long long hi = static_cast<unsigned long long>(tag) << 32;
  unsigned long long* decision = gran + static_cast<size_t>(G) * 4 + 3;  // (c = 1, g = 0) word 3
  if (lane == 0) st_x64(gran + static_cast<size_t>(g) * 4 + 3, hi | xcc, false);
  if (g != 0) {
    for (unsigned spins = 0;; ++spins) {
      const unsigned long long v = ld_sc1_u64(decision);
      if ((v >> 32) == tag) return (v & 1ull) != 0;  // (the same address in every lane: uniform)
      if (spins >= spin) {
        *timeout = true;
        return false;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  bool same = true;
  for (int base = 0; base < G; base += 64) {
    const int w = base + lane;
    const unsigned long long* src = gran + static_cast<size_t>(w < G ? w : 0) * 4 + 3;
    for (unsigned spins = 0;; ++spins) {
      bool got = true;
      unsigned long long v = 0;
      if (w < G) {
        v = ld_sc1_u64(src);
        got = (v >> 32) == tag;
      }
      if (__all(got)) {
        if (w < G) same = same && static_cast<unsigned>(v & 0xffffu) == xcc;
        break;
      }
      if (spins >= spin) {
        *timeout = true;
        same = false;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  const bool all = __all(same) != 0;
  if (lane == 0) st_x64(decision, hi | (all ? 1ull : 0ull), false);
  return all;
}

// One history term of a lane's crosses with the step's landmark j: acc[0..3] += K_cc[k]·M_cc[:, j],
// acc[4..7] += K_cc[j]·M_cc[:, k] (slam.cpp:264-265's rank-2 terms at (k, j) and (j, k)). The
// operands (this lane's history, 4 × ds_read_b128, and j's, broadcast) are loaded apart from the
// fmas so that several terms' reads can be in flight together.
template <bool J>
struct HistOps {
  static constexpr int kV = AmSharedT<J>::HW / 2;
  double2 o[kV], jv[kV];
};
template <bool J>
__device__ __forceinline__ void hist_load(const AmSharedT<J>& sh, int cc, int lane, HistOps<J>& p) {
  const double2* hl = reinterpret_cast<const double2*>(sh.hkm[cc][lane]);
  const double2* jl = reinterpret_cast<const double2*>(sh.jh[cc]);
#pragma unroll
  for (int i = 0; i < HistOps<J>::kV; ++i) {
    p.o[i] = hl[i];
    p.jv[i] = jl[i];
  }
}
template <bool J>
__device__ __forceinline__ void hist_fma(const HistOps<J>& p, double (&acc)[8]) {
  const double ok0 = p.o[0].x, ok1 = p.o[0].y, ok2 = p.o[1].x, ok3 = p.o[1].y;
  const double om0 = p.o[2].x, om1 = p.o[2].y, om2 = p.o[3].x, om3 = p.o[3].y;
  const double jk[4] = {p.jv[0].x, p.jv[0].y, p.jv[1].x, p.jv[1].y};
  const double jm[4] = {p.jv[2].x, p.jv[2].y, p.jv[3].x, p.jv[3].y};
  acc[0] = fma(ok1, jm[2], fma(ok0, jm[0], acc[0]));
  acc[1] = fma(ok1, jm[3], fma(ok0, jm[1], acc[1]));
  acc[2] = fma(ok3, jm[2], fma(ok2, jm[0], acc[2]));
  acc[3] = fma(ok3, jm[3], fma(ok2, jm[1], acc[3]));
  acc[4] = fma(jk[1], om2, fma(jk[0], om0, acc[4]));
  acc[5] = fma(jk[1], om3, fma(jk[0], om1, acc[5]));
  acc[6] = fma(jk[3], om2, fma(jk[2], om0, acc[6]));
  acc[7] = fma(jk[3], om3, fma(jk[2], om1, acc[7]));
  if constexpr (J) {  // + V_cc[k]·K_cc[j]ᵀ at (k, j) and V_cc[j]·K_cc[k]ᵀ at (j, k)
    const double ov0 = p.o[4].x, ov1 = p.o[4].y, ov2 = p.o[5].x, ov3 = p.o[5].y;
    const double jv0 = p.jv[4].x, jv1 = p.jv[4].y, jv2 = p.jv[5].x, jv3 = p.jv[5].y;
    acc[0] = fma(ov1, jk[1], fma(ov0, jk[0], acc[0]));
    acc[1] = fma(ov1, jk[3], fma(ov0, jk[2], acc[1]));
    acc[2] = fma(ov3, jk[1], fma(ov2, jk[0], acc[2]));
    acc[3] = fma(ov3, jk[3], fma(ov2, jk[2], acc[3]));
    acc[4] = fma(jv1, ok1, fma(jv0, ok0, acc[4]));
    acc[5] = fma(jv1, ok3, fma(jv0, ok2, acc[5]));
    acc[6] = fma(jv3, ok1, fma(jv2, ok0, acc[6]));
    acc[7] = fma(jv3, ok3, fma(jv2, ok2, acc[7]));
  }
}

// Workgroup barrier ordering LDS only: the waves' global stores (tables, Kcat / Mcat rows) are not
// waited for here (__syncthreads' workgroup fence would drain them at every step).
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Waves 1 (par 0) and 2 (par 1): per step, after wave 0 has published j (sh.jl) and j's history
// (sh.jh) — barrier A — this lane's sums over the steps cc < c with cc ≡ par (mod 2) of
// K_cc[k]·M_cc[:, j] and K_cc[j]·M_cc[:, k] into sh.es[par], read by wave 0 after barrier B. Every
// wave passes both barriers at every step, whatever the step decides.
template <bool J>
__device__ __forceinline__ void history_helper(AmSharedT<J>& sh, int m, int k, int lane, int par) {
  for (int c = 0; c < m; ++c) {
    lds_barrier();  // A
    const int j = sh.jl[c];
    double e[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (j >= 0) {  // (uniform; the lane k = j ignores its sums)
      int cc = par;
      for (; cc + 6 < c; cc += 8) {  // four terms' reads in flight, then their fmas in order
        HistOps<J> p0, p1, p2, p3;
        hist_load(sh, cc, lane, p0);
        hist_load(sh, cc + 2, lane, p1);
        hist_load(sh, cc + 4, lane, p2);
        hist_load(sh, cc + 6, lane, p3);
        hist_fma(p0, e);
        hist_fma(p1, e);
        hist_fma(p2, e);
        hist_fma(p3, e);
      }
      for (; cc < c; cc += 2) {
        HistOps<J> p0;
        hist_load(sh, cc, lane, p0);
        hist_fma(p0, e);
      }
    }
#pragma unroll
    for (int t = 0; t < 8; ++t) sh.es[par][t][lane] = e[t];
    lds_barrier();  // B
  }
}

}  // namespace

template <typename T, bool J>
__global__ __launch_bounds__(kAmThreads) void k_assoc_msg(PassArgs<T> A, AmArgs B) {
  __shared__ AmSharedT<J> sh;
  constexpr int HW = AmSharedT<J>::HW;
  const int G = B.G, fy = blockIdx.y;
  // XCD-local placement (B.xcd): the grid has 8 blocks per workgroup; filter fy's workgroups are
  // the blocks x ≡ fy (mod 8), which round-robin dispatch puts on one XCD (checked: same_xcd)
  int g = blockIdx.x;
  if (B.xcd) {
    if ((g & 7) != (fy & 7)) return;
    g >>= 3;
  }
  const MsgDesc& d = A.desc[fy];
  const int flags = d.flags;
  if (!(flags & kActive)) return;  // (every workgroup of the filter)
  const int f = A.f0 + fy;
  const int lane = threadIdx.x & (kAmSlots - 1);
  const int N = A.N, ld = A.ld, ldk = A.ldk;
  const int Np = G * kAmSlots;
  const int k = g * kAmSlots + lane;  // this lane's landmark slot
  if (threadIdx.x >= kAmSlots) {  // waves 1, 2: the history sums only (uniform per wave)
    history_helper(sh, d.m, k, lane, (threadIdx.x >> 6) - 1);
    return;
  }
  const bool valid = k < N;
  const int ix = 3 + 2 * (valid ? k : N - 1);  // its state index (clamped for the loads)
  const T* S = A.sig[d.parity] + f * A.sig_stride;
  const double* xin = A.x[d.parity] + f * A.x_stride;
  double* xout = A.x[d.parity ^ 1] + f * A.x_stride;
  T* kc = A.kcat + f * A.km_stride;
  T* mc = A.mcat + f * A.km_stride;
  FilterCtl* ctl = A.ctl + f;
  AmHist* hist = B.hist + f * B.hist_stride;
  AmCur* cur = B.cur + f * B.cur_stride;
  unsigned long long* gran = B.gran + f * B.gran_stride;
  const int m = d.m;
  const double r_noise = A.r, gate = A.gate;
  const unsigned tagbase = (A.seq & 0x07ffffffu) << 5;
  bool timeout = false;
  unsigned status = 0;
  const bool loc = B.xcd && G > 1 && same_xcd(gran, G, g, tagbase | 31u, &timeout, B.spin);
  const auto cur_r = buf_rsrc(cur, static_cast<unsigned>(B.cur_stride * sizeof(AmCur)));
  const auto hist_r = buf_rsrc(hist, static_cast<unsigned>(B.hist_stride * sizeof(AmHist)));

  // ---- predict (slam.cpp:321-335): the pose, At's two entries, the pose block (every lane) ----
  double pose[3], a1, a2;
  predicted_pose(ctl->tmo, d, xin, pose, &a1, &a2);
  const bool first = (flags & kFirst) != 0;
  double Pp[3][3];
  {
  double raw[3][3];
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int b = 0; b < 3; ++b) raw[a][b] = static_cast<double>(S[a * ld + b]);
#pragma unroll
  for (int a = 0; a < 3; ++a)
#pragma unroll
    for (int b = 0; b < 3; ++b) {
      const double aa = alpha_of(a, a1, a2), ab = alpha_of(b, a1, a2);
      double v = raw[a][b] + aa * raw[0][b];
      v = v + (raw[a][0] + aa * raw[0][0]) * ab;
      if (first && a == b) v += A.q;
      Pp[a][b] = v;
    }
  }  // (raw: re-read for the factor rows at the end, not kept live through the steps)
  // the lane's slot: its predicted block and state
  double kk[4], kp[6], pk[6];
  slot_block(S, ld, ix, a1, a2, kk, kp, pk);
  double xk[2] = {xin[ix], xin[ix + 1]};
  unsigned s = ctl->counter;

  // the state at the chunk's start, for the first step's exchange
  if (valid && G > 1) put_cur(cur + g * kAmSlots, lane, kk, kp, pk, xk, loc);
  bool any_new = false;

  AM_STAMP(kMaxChunk, 0);
  for (int c = 0; c < m; ++c) {
    AM_STAMP(c, 0);
    const double z0 = d.z[c][0], z1 = d.z[c][1];
    // a full map: the reference's temporary landmark (slam.cpp:351-356) indexes the state out of
    // range and throws before any association; the marker is skipped (uniform: no exchange)
    const bool full = s >= static_cast<unsigned>(N);
    // ---- marker c's distance to this lane's landmark (slam.cpp:361-416) ----
    double key = INFINITY;
    if (!full && valid && k < static_cast<int>(s)) {
      double P[5][5];
#pragma unroll
      for (int a = 0; a < 3; ++a) {
#pragma unroll
        for (int b = 0; b < 3; ++b) P[a][b] = Pp[a][b];
        P[a][3] = pk[2 * a];
        P[a][4] = pk[2 * a + 1];
        P[3][a] = kp[a];
        P[4][a] = kp[3 + a];
      }
      P[3][3] = kk[0];
      P[3][4] = kk[1];
      P[4][3] = kk[2];
      P[4][4] = kk[3];
      const double dist = assoc_dist(P, pose, xk[0], xk[1], z0, z1, r_noise);
      key = dist < INFINITY ? dist : INFINITY;  // NaN never wins (strict <, k_assoc)
    }
    int kbest = valid ? k : INT_MAX;
    wave_argmin(key, kbest);
    AM_STAMP(c, 1);
    if (G > 1 && !full)
      exchange(gran, G, g, c, tagbase | static_cast<unsigned>(c + 1), key, kbest, &timeout, loc,
               B.spin, B.drop && c == 0 && g == G - 1);
    key = __longlong_as_double(static_cast<long long>(__builtin_amdgcn_readfirstlane(
              static_cast<int>(__double_as_longlong(key))) & 0xffffffffull) |
          (static_cast<long long>(__builtin_amdgcn_readfirstlane(
               static_cast<int>(__double_as_longlong(key) >> 32))) << 32));
    kbest = __builtin_amdgcn_readfirstlane(kbest);  // (every lane holds the same argmin)
    AM_STAMP(c, 2);
    // ---- decision (slam.cpp:418-440): the new slot (index s, d = gate) wins only over a strictly
    // larger existing minimum; a full map is the reference's out-of-range state index ----
    int j;
    bool isnew = false;
    if (full) {
      j = -1;
      status |= EKF_FLAG_RANGE_D;
    } else if (!(key <= gate)) {
      {
        j = static_cast<int>(s);
        isnew = true;
        ++s;
        any_new = true;
      }
    } else {
      j = kbest;
    }
    if (lane == 0) {
      sh.jl[c] = j;
      if (g == 0) {
        const int slot = (d.assoc_slot + c) & (kMaxAssoc - 1);
        ctl->assoc_j[slot] = j;
        ctl->assoc_new[slot] = isnew ? 1 : 0;
      }
    }
    double Kk[2][2] = {{0.0, 0.0}, {0.0, 0.0}}, Mk[2][2] = {{0.0, 0.0}, {0.0, 0.0}};
    double Kp[3][2] = {{0.0, 0.0}, {0.0, 0.0}, {0.0, 0.0}}, Mp[2][3] = {{0.0, 0.0, 0.0},
                                                                         {0.0, 0.0, 0.0}};
    // Joseph: V = Σ·Hᵀ − K·S at the pose (Vp) and at this lane's slot (Vk), and S (Sv)
    double Vp[3][2] = {{0.0, 0.0}, {0.0, 0.0}, {0.0, 0.0}}, Vk[2][2] = {{0.0, 0.0}, {0.0, 0.0}};
    double Sv[4] = {0.0, 0.0, 0.0, 0.0};
    // the new landmark's state (slam.cpp:351-354, the pose before this marker's correction)
    double nx = 0.0, ny = 0.0;
    double rkj[4] = {0.0, 0.0, 0.0, 0.0}, rjk[4] = {0.0, 0.0, 0.0, 0.0};
    if (j >= 0) {
      const int jx = 3 + 2 * j;
      if (isnew) {  // (uniform)
        nx = pose[1] + z0 * cos(z1 + pose[0]);
        ny = pose[2] + z0 * sin(z1 + pose[0]);
        if (k == j) {
          xk[0] = nx;
          xk[1] = ny;
        }
      }
      // ---- j's block, state and history (one round of sc1 loads), crosses from Σ_in ----
      constexpr int kJL = (18 + HW * (kMaxChunk - 1) + 63) / 64;  // 3 (Joseph: 4)
      double v[kJL];
      const unsigned jco = static_cast<unsigned>((c * Np + j) * sizeof(AmCur));
#pragma unroll
      for (int i = 0; i < kJL; ++i) {
        const int e = lane + 64 * i;  // 0..17: the AmCur fields; then HW per earlier step
        v[i] = 0.0;
        if (G > 1 && e < 18) {
          v[i] = ld_xf64(cur_r, jco + 8 * e);
        } else if (G > 1 && e < 18 + HW * c) {
          const int cc = (e - 18) / HW, t = (e - 18) % HW;  // AmHist: k[4], m[4] (, v[4])
          v[i] = ld_xf64(hist_r, static_cast<unsigned>((cc * Np + j) * sizeof(AmHist) + 8 * t));
        }
      }
      // Σ_in crosses of this lane's slot with j (no predict term between landmarks)
      const T* q0 = S + static_cast<size_t>(ix) * ld;
      const T* p0 = S + static_cast<size_t>(jx) * ld;
      rkj[0] = static_cast<double>(q0[jx]);
      rkj[1] = static_cast<double>(q0[jx + 1]);
      rkj[2] = static_cast<double>(q0[ld + jx]);
      rkj[3] = static_cast<double>(q0[ld + jx + 1]);
      rjk[0] = static_cast<double>(p0[ix]);
      rjk[1] = static_cast<double>(p0[ix + 1]);
      rjk[2] = static_cast<double>(p0[ld + ix]);
      rjk[3] = static_cast<double>(p0[ld + ix + 1]);
      if (G > 1) {
#pragma unroll
        for (int i = 0; i < kJL; ++i) {
          const int e = lane + 64 * i;
          if (e < 18) sh.jc[e] = v[i];
          else if (e < 18 + HW * c) sh.jh[(e - 18) / HW][(e - 18) % HW] = v[i];
        }
      } else {  // one workgroup: j's lane holds its block (v_readlane), its history is in LDS
        const int lj = j;
        double jv[18];
#pragma unroll
        for (int t = 0; t < 4; ++t) jv[t] = readlane_f64(kk[t], lj);
#pragma unroll
        for (int t = 0; t < 6; ++t) jv[4 + t] = readlane_f64(kp[t], lj);
#pragma unroll
        for (int t = 0; t < 6; ++t) jv[10 + t] = readlane_f64(pk[t], lj);
        jv[16] = readlane_f64(xk[0], lj);
        jv[17] = readlane_f64(xk[1], lj);
        if (lane == 0) {
#pragma unroll
          for (int t = 0; t < 18; ++t) sh.jc[t] = jv[t];
        }
        for (int e = lane; e < HW * c; e += 64) {
          const int cc = e / HW, t = e % HW;
          sh.jh[cc][t] = sh.hkm[cc][lj][t];
        }
      }
    }
    // ---- the step (slam.cpp:443-488): wave 0 forms what every lane shares (ẑ, H, S, S⁻¹, ν,
    // K / M at the pose) while waves 1-2 (history_helper) sum this step's history terms of every
    // lane's crosses with j, between barriers A and B (both waves pass both at every step) ----
    lds_barrier();  // A: sh.jl[c], sh.jc and j's history sh.jh published to waves 1-2
    AM_STAMP(c, 3);
    double H0[5], H1[5], Si[4], nu0 = 0.0, nu1 = 0.0;
    bool sok = false;
    if (j >= 0) {
      double jkk[4], jkp[6], jpk[6], xj[2];
#pragma unroll
      for (int t = 0; t < 4; ++t) jkk[t] = sh.jc[t];
#pragma unroll
      for (int t = 0; t < 6; ++t) jkp[t] = sh.jc[4 + t];
#pragma unroll
      for (int t = 0; t < 6; ++t) jpk[t] = sh.jc[10 + t];
      xj[0] = isnew ? nx : sh.jc[16];
      xj[1] = isnew ? ny : sh.jc[17];
      double zhat[2], braw;
      bool bok;
      range_bearing(pose, xj[0], xj[1], zhat, H0, H1, &braw, &bok);
      if (!bok) zhat[1] = normalize_angle(braw);
      double P5[5][5];
#pragma unroll
      for (int a = 0; a < 3; ++a) {
#pragma unroll
        for (int b = 0; b < 3; ++b) P5[a][b] = Pp[a][b];
        P5[a][3] = jpk[2 * a];
        P5[a][4] = jpk[2 * a + 1];
        P5[3][a] = jkp[a];
        P5[4][a] = jkp[3 + a];
      }
      P5[3][3] = jkk[0];
      P5[3][4] = jkk[1];
      P5[4][3] = jkk[2];
      P5[4][4] = jkk[3];
      // H's shape (range_bearing): H0 = [0, h1, h2, −h1, −h2], H1 = [−1, g1, g2, −g1, −g2] (exact
      // negations), so a row times H is two fmas on (v1 − v3, v2 − v4), as in the chain's step
      const double h1 = H0[1], h2 = H0[2], g1 = H1[1], g2 = H1[2];
      double Gt[5][2];  // (Σ·Hᵀ)[pA]
#pragma unroll
      for (int a = 0; a < 5; ++a) {
        const double d1 = P5[a][1] - P5[a][3], d2 = P5[a][2] - P5[a][4];
        Gt[a][0] = fma(h2, d2, h1 * d1);
        Gt[a][1] = fma(g2, d2, fma(g1, d1, -P5[a][0]));
      }
      double Sm[4];  // S = H·(Σ·Hᵀ)[pA] + R (slam.cpp:476)
      {
        const double t1 = Gt[1][0] - Gt[3][0], t2 = Gt[2][0] - Gt[4][0];
        const double u1 = Gt[1][1] - Gt[3][1], u2 = Gt[2][1] - Gt[4][1];
        Sm[0] = fma(h2, t2, h1 * t1) + r_noise;
        Sm[1] = fma(h2, u2, h1 * u1);
        Sm[2] = fma(g2, t2, fma(g1, t1, -Gt[0][0]));
        Sm[3] = fma(g2, u2, fma(g1, u1, -Gt[0][1])) + r_noise;
      }
      sok = inv2(Sm, Si);
      if (!sok) {
        status |= EKF_FLAG_NUMERIC_D;  // Armadillo's inv throws; this marker is skipped
      } else {
        nu0 = z0 - zhat[0];
        nu1 = normalize_angle(z1 - zhat[1]);
#pragma unroll
        for (int a = 0; a < 3; ++a) {
          Kp[a][0] = Gt[a][0] * Si[0] + Gt[a][1] * Si[2];
          Kp[a][1] = Gt[a][0] * Si[1] + Gt[a][1] * Si[3];
          if (J) {  // (k_chain's V expression)
            Vp[a][0] = Gt[a][0] - (Kp[a][0] * Sm[0] + Kp[a][1] * Sm[2]);
            Vp[a][1] = Gt[a][1] - (Kp[a][0] * Sm[1] + Kp[a][1] * Sm[3]);
          }
        }
        if (J)
#pragma unroll
          for (int t = 0; t < 4; ++t) Sv[t] = Sm[t];
#pragma unroll
        for (int b = 0; b < 3; ++b) {  // (H·Σ)[:, pose b]
          const double e1 = P5[1][b] - P5[3][b], e2 = P5[2][b] - P5[4][b];
          Mp[0][b] = fma(h2, e2, h1 * e1);
          Mp[1][b] = fma(g2, e2, fma(g1, e1, -P5[0][b]));
        }
      }
    }
    lds_barrier();  // B: waves 1 / 2's sums in sh.es
    AM_STAMP(c, 5);
    if (sok) {
      // this lane's crosses with j at step c: Σ_c[k, j] = Σ_p[k, j] − Σ_cc K_cc[k]·M_cc[:, j] and
      // Σ_c[j, k] likewise (the sums from waves 1-2)
      if (k == j) {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          rkj[t] = kk[t];
          rjk[t] = kk[t];
        }
      } else {
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          rkj[t] = rkj[t] - (sh.es[0][t][lane] + sh.es[1][t][lane]);
          rjk[t] = rjk[t] - (sh.es[0][4 + t][lane] + sh.es[1][4 + t][lane]);
        }
      }
      {
        // ---- this lane's slot: K[k], M[:, k] from its crosses with j ----
        // (H's shape as above: two fmas on the differences)
        const double h1 = H0[1], h2 = H0[2], g1 = H1[1], g2 = H1[2];
#pragma unroll
        for (int a = 0; a < 2; ++a) {  // (Σ·Hᵀ)[k_a] over pA
          const double d1 = kp[3 * a + 1] - rkj[2 * a], d2 = kp[3 * a + 2] - rkj[2 * a + 1];
          const double q0 = fma(h2, d2, h1 * d1);
          const double q1 = fma(g2, d2, fma(g1, d1, -kp[3 * a]));
          Kk[a][0] = q0 * Si[0] + q1 * Si[2];
          Kk[a][1] = q0 * Si[1] + q1 * Si[3];
          if (J) {
            Vk[a][0] = q0 - (Kk[a][0] * Sv[0] + Kk[a][1] * Sv[2]);
            Vk[a][1] = q1 - (Kk[a][0] * Sv[1] + Kk[a][1] * Sv[3]);
          }
        }
#pragma unroll
        for (int b = 0; b < 2; ++b) {  // (H·Σ)[:, k_b]
          const double e1 = pk[2 + b] - rjk[b], e2 = pk[4 + b] - rjk[2 + b];
          Mk[0][b] = fma(h2, e2, h1 * e1);
          Mk[1][b] = fma(g2, e2, fma(g1, e1, -pk[b]));
        }
        // ---- Σ ← Σ − K·M on the lane's block and the pose block; x += K·ν (slam.cpp:482-488) ----
        // (Joseph: then − V·Kᵀ)
        double nkk[4], nkp[6], npk[6];
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            nkk[2 * a + b] = rank2_sub(kk[2 * a + b], Kk[a][0], Kk[a][1], Mk[0][b], Mk[1][b]);
            if (J) nkk[2 * a + b] = rank2_sub(nkk[2 * a + b], Vk[a][0], Vk[a][1], Kk[b][0], Kk[b][1]);
          }
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < 3; ++b) {
            nkp[3 * a + b] = rank2_sub(kp[3 * a + b], Kk[a][0], Kk[a][1], Mp[0][b], Mp[1][b]);
            if (J) nkp[3 * a + b] = rank2_sub(nkp[3 * a + b], Vk[a][0], Vk[a][1], Kp[b][0], Kp[b][1]);
          }
#pragma unroll
        for (int a = 0; a < 3; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            npk[2 * a + b] = rank2_sub(pk[2 * a + b], Kp[a][0], Kp[a][1], Mk[0][b], Mk[1][b]);
            if (J) npk[2 * a + b] = rank2_sub(npk[2 * a + b], Vp[a][0], Vp[a][1], Kk[b][0], Kk[b][1]);
          }
#pragma unroll
        for (int t = 0; t < 4; ++t) kk[t] = nkk[t];
#pragma unroll
        for (int t = 0; t < 6; ++t) {
          kp[t] = nkp[t];
          pk[t] = npk[t];
        }
        xk[0] = xk[0] + (Kk[0][0] * nu0 + Kk[0][1] * nu1);
        xk[1] = xk[1] + (Kk[1][0] * nu0 + Kk[1][1] * nu1);
        double nP[3][3];
#pragma unroll
        for (int a = 0; a < 3; ++a)
#pragma unroll
          for (int b = 0; b < 3; ++b) {
            nP[a][b] = rank2_sub(Pp[a][b], Kp[a][0], Kp[a][1], Mp[0][b], Mp[1][b]);
            if (J) nP[a][b] = rank2_sub(nP[a][b], Vp[a][0], Vp[a][1], Kp[b][0], Kp[b][1]);
          }
#pragma unroll
        for (int a = 0; a < 3; ++a) {
#pragma unroll
          for (int b = 0; b < 3; ++b) Pp[a][b] = nP[a][b];
          pose[a] = pose[a] + (Kp[a][0] * nu0 + Kp[a][1] * nu1);
        }
        pose[0] = normalize_angle(pose[0]);  // slam.cpp:488
      }
    }
    AM_STAMP(c, 4);
    // ---- the step's factors: history (LDS + write-through table), Kcat / Mcat rows ----
    // (Joseph: Kcat / Mcat rows 2 + 2m + 2c + e hold V_c / K_c, the V·Kᵀ term's factors)
    const int jr = 2 + 2 * m + 2 * c;
    {
      const double hrow[12] = {Kk[0][0], Kk[0][1], Kk[1][0], Kk[1][1], Mk[0][0], Mk[0][1],
                               Mk[1][0], Mk[1][1], Vk[0][0], Vk[0][1], Vk[1][0], Vk[1][1]};
      double2* hl = reinterpret_cast<double2*>(sh.hkm[c][lane]);
#pragma unroll
      for (int t = 0; t < HW / 2; ++t) hl[t] = make_double2(hrow[2 * t], hrow[2 * t + 1]);
      if (valid) {
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          kc[(2 + 2 * c + e) * ldk + ix] = static_cast<T>(Kk[0][e]);
          kc[(2 + 2 * c + e) * ldk + ix + 1] = static_cast<T>(Kk[1][e]);
          mc[(2 + 2 * c + e) * ldk + ix] = static_cast<T>(Mk[e][0]);
          mc[(2 + 2 * c + e) * ldk + ix + 1] = static_cast<T>(Mk[e][1]);
          if (J) {
            kc[(jr + e) * ldk + ix] = static_cast<T>(Vk[0][e]);
            kc[(jr + e) * ldk + ix + 1] = static_cast<T>(Vk[1][e]);
            mc[(jr + e) * ldk + ix] = static_cast<T>(Kk[0][e]);
            mc[(jr + e) * ldk + ix + 1] = static_cast<T>(Kk[1][e]);
          }
        }
        if (G > 1 && c + 1 < m)
          put_hist(hist + static_cast<size_t>(c) * Np + g * kAmSlots, lane, hrow, HW, loc);
      }
    }
    if (g == 0 && lane < 3) {
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        const double kv = lane == 0 ? Kp[0][e] : (lane == 1 ? Kp[1][e] : Kp[2][e]);
        const double mv = lane == 0 ? Mp[e][0] : (lane == 1 ? Mp[e][1] : Mp[e][2]);
        kc[(2 + 2 * c + e) * ldk + lane] = static_cast<T>(kv);
        mc[(2 + 2 * c + e) * ldk + lane] = static_cast<T>(mv);
        if (J) {
          const double vv = lane == 0 ? Vp[0][e] : (lane == 1 ? Vp[1][e] : Vp[2][e]);
          kc[(jr + e) * ldk + lane] = static_cast<T>(vv);
          mc[(jr + e) * ldk + lane] = static_cast<T>(kv);
        }
      }
    }
    if (valid && G > 1 && c + 1 < m)  // the slot's block and state as step c + 1 starts
      put_cur(cur + static_cast<size_t>(c + 1) * Np + g * kAmSlots, lane, kk, kp, pk, xk, loc);
  }

  AM_STAMP(kMaxChunk, 1);
  // ---- the chunk's remaining factor rows: the predict's two rank-1 terms (slam.cpp:198, as
  // k_factors writes them), zero rows up to the pass's rank kw ----
  const int rank = 2 + (J ? 4 : 2) * m, kw = ((rank + 3) / 4) * 4;
  if (valid) {
    // Σ_in[ix + e][0] and Σ_in[0][ix + e] (raw, as slot_block read them)
    const double c0[2] = {static_cast<double>(S[static_cast<size_t>(ix) * ld]),
                          static_cast<double>(S[static_cast<size_t>(ix + 1) * ld])};
    const double r0[2] = {static_cast<double>(S[ix]), static_cast<double>(S[ix + 1])};
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      kc[0 * ldk + ix + e] = static_cast<T>(0.0);                  // −α_i = 0 for landmark rows
      kc[1 * ldk + ix + e] = static_cast<T>(first ? -c0[e] : 0.0);  // −(Σ[i][0] + α_i·Σ[0][0])
      mc[0 * ldk + ix + e] = static_cast<T>(first ? r0[e] : 0.0);   // Σ[0][j]
      mc[1 * ldk + ix + e] = static_cast<T>(0.0);                  // α_j = 0
      for (int rr = rank; rr < kw; ++rr) {
        kc[rr * ldk + ix + e] = static_cast<T>(0.0);
        mc[rr * ldk + ix + e] = static_cast<T>(0.0);
      }
    }
    xout[ix] = xk[0];
    xout[ix + 1] = xk[1];
  }
  if (g == 0 && lane < 3) {
    const double al = alpha_of(lane, a1, a2);
    const double rc0 = static_cast<double>(S[lane * ld]), r0c = static_cast<double>(S[lane]);
    const double s00 = static_cast<double>(S[0]);
    kc[0 * ldk + lane] = static_cast<T>(first ? -al : 0.0);
    kc[1 * ldk + lane] = static_cast<T>(first ? -(rc0 + al * s00) : 0.0);
    mc[0 * ldk + lane] = static_cast<T>(first ? r0c : 0.0);
    mc[1 * ldk + lane] = static_cast<T>(first ? al : 0.0);
    for (int rr = rank; rr < kw; ++rr) {
      kc[rr * ldk + lane] = static_cast<T>(0.0);
      mc[rr * ldk + lane] = static_cast<T>(0.0);
    }
    xout[lane] = pose[lane];
  }
  if (g == 0 && lane == 0) {
    ctl->counter = s;
    if (flags & kLast) {  // posterior t_map_odom = T(x, y, θ)·t_odom_robot⁻¹ (slam.cpp:490-494)
      const Pose2 tmo = compose(Pose2{pose[0], pose[1], pose[2]},
                                inverse(Pose2{d.odom[0], d.odom[1], d.odom[2]}));
      ctl->tmo[0] = tmo.theta;
      ctl->tmo[1] = tmo.x;
      ctl->tmo[2] = tmo.y;
    }
  }
  if (lane == 0 && g == 0 && status) atomicOr(&ctl->status, status);
  if (lane == 0 && timeout) flag_timeout(&ctl->status, A.fatal);

  // ---- fp32 Σ: the final Σ[U, U] in fp64 over the pass's block when a landmark was committed
  // (k_patch_stage; its first sighting cancels 1e7 − (1e7 − δ) in fp32) ----
  if (sizeof(T) != 4) return;
  ChunkRec* rec = A.rec + static_cast<size_t>(d.parity) * A.rec_stride + f;
  if (!any_new) {
    if (g == 0 && lane == 0) rec->flags = 0;
    return;
  }
  if (G > 1) {  // the final blocks (cur[m]) and every history row published; then workgroup 0 only
    if (valid) {
      put_hist(hist + static_cast<size_t>(m - 1) * Np + g * kAmSlots, lane, sh.hkm[m - 1][lane],
               HW, loc);
      put_cur(cur + static_cast<size_t>(m) * Np + g * kAmSlots, lane, kk, kp, pk, xk, loc);
    }
    double dd = 0.0;
    int kd = 0;
    bool late = false;
    exchange(gran, G, g, m, tagbase | static_cast<unsigned>(m + 1), dd, kd, &late, loc, B.spin);
    if (late && lane == 0) flag_timeout(&ctl->status, A.fatal);
    if (g != 0) return;
  }
  // workgroup 0: U = {θ, x, y, jx, jy per marker} (a skipped marker maps onto θ: never a first
  // position, never patched); every marker's landmark's final block (pb) and, with G > 1, its
  // factor history staged into the no longer needed own-history LDS (ph[c][cc][8])
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
  const int nu = 3 + 2 * m;
  double* ph = &sh.hkm[0][0][0];  // G > 1: [m][m][HW] ≤ 3 072 doubles (the region holds 64·HW·16)
  if (G > 1) {
    for (int e = lane; e < m * 18; e += 64) {
      const int c = e / 18, t = e - c * 18;
      sh.pb[c][t] = ld_xf64(
          cur_r, static_cast<unsigned>((m * Np + max(sh.jl[c], 0)) * sizeof(AmCur) + 8 * t));
    }
    for (int e = lane; e < m * m * HW; e += 64) {
      const int c = e / (HW * m), cc = (e / HW) % m, t = e % HW;
      const double v = ld_xf64(
          hist_r, static_cast<unsigned>((cc * Np + max(sh.jl[c], 0)) * sizeof(AmHist) + 8 * t));
      __builtin_amdgcn_wave_barrier();  // every lane's loads issued before any lane overwrites
      ph[e] = v;
    }
  } else {
    for (int c = 0; c < m; ++c) {
      const int j = __builtin_amdgcn_readfirstlane(max(sh.jl[c], 0));
      double jv[18];
#pragma unroll
      for (int t = 0; t < 4; ++t) jv[t] = readlane_f64(kk[t], j);
#pragma unroll
      for (int t = 0; t < 6; ++t) jv[4 + t] = readlane_f64(kp[t], j);
#pragma unroll
      for (int t = 0; t < 6; ++t) jv[10 + t] = readlane_f64(pk[t], j);
      jv[16] = readlane_f64(xk[0], j);
      jv[17] = readlane_f64(xk[1], j);
      if (lane == 0) {
#pragma unroll
        for (int t = 0; t < 18; ++t) sh.pb[c][t] = jv[t];
      }
    }
  }
  if (lane == 0) {
#pragma unroll
    for (int a = 0; a < 3; ++a)
#pragma unroll
      for (int b = 0; b < 3; ++b) sh.pp[3 * a + b] = Pp[a][b];
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
  // the history of marker position c's landmark at step cc: K (t < 4), M (t < 8), V (t < 12)
  auto hv = [&](int c, int cc, int t) -> double {
    if (G > 1) return ph[(c * m + cc) * HW + t];
    const int j = max(sh.jl[c], 0);
    return sh.hkm[cc][j][t];
  };
  for (int e = lane; e < nu * nu; e += 64) {
    const int a = e / nu, b = e - a * nu;
    const int ca = a < 3 ? -1 : (a - 3) >> 1, ea = (a - 3) & 1;
    const int cb = b < 3 ? -1 : (b - 3) >> 1, eb = (b - 3) & 1;
    const bool sa = ca >= 0 && sh.jl[ca] < 0, sb = cb >= 0 && sh.jl[cb] < 0;
    double v;
    if (sa || sb) {
      v = 0.0;  // a skipped marker's position (its column maps onto θ and is never patched)
    } else if (ca < 0 && cb < 0) {
      v = sh.pp[3 * a + b];
    } else if (ca < 0) {  // Σ[pose a][landmark]: pk
      v = sh.pb[cb][10 + 2 * a + eb];
    } else if (cb < 0) {  // Σ[landmark][pose b]: kp
      v = sh.pb[ca][4 + 3 * ea + b];
    } else if (sh.jl[ca] == sh.jl[cb]) {
      v = sh.pb[ca][2 * ea + eb];
    } else {  // two landmarks: Σ_in minus the chunk's rank-2 terms, as the lanes' crosses
      const int ja = 3 + 2 * sh.jl[ca] + ea, jb = 3 + 2 * sh.jl[cb] + eb;
      v = static_cast<double>(S[static_cast<size_t>(ja) * ld + jb]);
      for (int cc = 0; cc < m; ++cc) {
        v = rank2_sub(v, hv(ca, cc, 2 * ea), hv(ca, cc, 2 * ea + 1), hv(cb, cc, 4 + eb),
                      hv(cb, cc, 4 + 2 + eb));
        if (J)  // − V_cc[a]·K_cc[b]ᵀ
          v = rank2_sub(v, hv(ca, cc, 8 + 2 * ea), hv(ca, cc, 8 + 2 * ea + 1), hv(cb, cc, 2 * eb),
                        hv(cb, cc, 2 * eb + 1));
      }
    }
    rec->Pend[a][b] = v;
  }
  for (int a = lane; a < kMaxU + 1; a += 64) {
    int u = 0;
    if (a < 3) {
      u = a;
    } else if (a < nu) {
      const int jj = sh.jl[(a - 3) >> 1];
      u = jj < 0 ? 0 : 3 + 2 * jj + ((a - 3) & 1);
    }
    rec->u[a] = u;
  }
  if (lane == 0) {
    rec->nu = nu;
    rec->m = m;
    rec->flags = kPendValid;
  }
}

#ifdef EKF_DIAG_STAMPS
}  // namespace ekfslam
extern "C" int ekfslam_diag_read_am_stamps(unsigned long long* out) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(ekfslam::g_am_stamps), sizeof(ekfslam::g_am_stamps)) ==
                 hipSuccess ? 0 : -5;
}
namespace ekfslam {
#endif

template <typename T>
hipError_t launch_assoc_msg(const PassArgs<T>& a, const AmArgs& b, int nf, hipStream_t s,
                            hipEvent_t e0, hipEvent_t e1) {
  const dim3 grid(b.xcd ? 8 * b.G : b.G, nf);
  auto k = a.joseph ? k_assoc_msg<T, true> : k_assoc_msg<T, false>;
  if (e0 && e1)
    hipExtLaunchKernelGGL(k, grid, dim3(kAmThreads), 0, s, e0, e1, 0, a, b);
  else
    hipLaunchKernelGGL(k, grid, dim3(kAmThreads), 0, s, a, b);
  return hipGetLastError();
}

int assoc_msg_blocks_per_cu(bool f32, bool joseph) {
  int nb = 0;
  auto occ = [&](auto kern) { return hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kern, kAmThreads, 0); };
  const hipError_t e = f32 ? (joseph ? occ(k_assoc_msg<float, true>) : occ(k_assoc_msg<float, false>))
                           : (joseph ? occ(k_assoc_msg<double, true>) : occ(k_assoc_msg<double, false>));
  return e == hipSuccess ? nb : 0;
}

template hipError_t launch_assoc_msg<double>(const PassArgs<double>&, const AmArgs&, int,
                                             hipStream_t, hipEvent_t, hipEvent_t);
template hipError_t launch_assoc_msg<float>(const PassArgs<float>&, const AmArgs&, int, hipStream_t,
                                            hipEvent_t, hipEvent_t);

}  // namespace ekfslam
