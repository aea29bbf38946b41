// HIP kernels (gfx950 / CDNA4) for the EKF-SLAM predict → correct* → posterior path of
// maxipalay/ekf-slam nuslam/src/slam.cpp.
//
// A chunk (one message, up to kMaxChunk markers) runs as three kernels:
//
//   k_chain       One workgroup per filter. The m corrections of a chunk only couple through the
//                 rows/columns the chunk touches, U = {θ, x, y} ∪ {jx, jy per marker} (|U| ≤ 3+2m).
//                 The chain replays them on the |U|×|U| block in LDS (predict folded in) — the only
//                 sequential part — and hands the factor kernel the row / column maps Z (|U|×2m) and
//                 Y (2m×|U|) plus x[U] through a write-through record (ChunkRec).
//   k_factors     Kcat = Σ_pred[:, U]·Z and Mcat = Y·Σ_pred[U, :] for every row / column on f64
//                 MFMA (v_mfma_f64_16x16x4f64), plus the new state x.
//   k_sigma_pass  Σ_out = Σ_in + Q̄ − Σ_k Kcat[k]ᵀ ⊗ Mcat[k], a rank-(2+2m) update of the dense
//                 covariance: the predict's two rank-1 terms (A Σ Aᵀ, slam.cpp:198) and one rank-2
//                 term per correction ((I − KH)Σ, slam.cpp:264-265). It streams Σ once per chunk
//                 through MFMA (v_mfma_f32_32x32x2f32 for fp32 Σ, v_mfma_f64_16x16x4f64 for fp64),
//                 so the HBM cost of a correction is 2·n²·w / m instead of 2·n²·w.
//
// Equal to the reference's sequential dense algebra in exact arithmetic; the summation order
// differs (tolerances in tests/). Unknown association adds k_assoc before each single-marker chunk.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cfloat>
#include <climits>
#include <cstdint>
#include <type_traits>

#include "ekf_device.hpp"
#include "ekf_launch.hpp"
#include "ekf_math.hpp"
#include "geom.hpp"

namespace ekfslam {

// Diagnostic build only (tools/chain_stamps.py): s_memtime stamps of k_chain's block (0,0), thread
// 0, in a ring of the last four chunks (by seq & 3).
#ifdef EKF_DIAG_STAMPS
__device__ unsigned long long g_stamps[4 * 512];
#define EKF_STAMP(i)                                                              \
  do {                                                                            \
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)                   \
      g_stamps[512 * (seq & 3) + (i)] = __builtin_amdgcn_s_memtime();             \
  } while (0)
#define EKF_STAMPT(i, t)                                                          \
  do {                                                                            \
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == (t))                 \
      g_stamps[512 * (seq & 3) + (i)] = __builtin_amdgcn_s_memtime();             \
  } while (0)
#define EKF_STAMPV(i, v)                                                          \
  do {                                                                            \
    if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)                   \
      g_stamps[512 * (seq & 3) + (i)] = (v);                                      \
  } while (0)
#else
#define EKF_STAMPT(i, t) \
  do {                   \
  } while (0)
#define EKF_STAMPV(i, v) \
  do {                   \
  } while (0)
#define EKF_STAMP(i) \
  do {               \
  } while (0)
#endif
#ifdef EKF_DIAG_STAMPS
}  // namespace ekfslam
extern "C" int ekfslam_diag_read_stamps(unsigned long long* out, int n) {
  using ekfslam::g_stamps;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(unsigned long long) * (n < 2048 ? n : 2048)) == hipSuccess ? 0 : -5;
}
namespace ekfslam {
#endif

// Diagnostic build only (tools/diag_blocks.py): filter 0's chain block Σ[U, U] and x[U] as the
// corrections start (predict folded in), per chunk sequence number mod 64.
#ifdef EKF_DIAG_STAMPS
__device__ double g_blocks[64][kMaxU][kMaxU + 1];
__device__ double g_blockx[64][kMaxU];
}  // namespace ekfslam
extern "C" int ekfslam_diag_read_blocks(double* blocks, double* xs) {
  using namespace ekfslam;
  if (hipMemcpyFromSymbol(blocks, HIP_SYMBOL(g_blocks), sizeof(g_blocks)) != hipSuccess) return -5;
  return hipMemcpyFromSymbol(xs, HIP_SYMBOL(g_blockx), sizeof(g_blockx)) == hipSuccess ? 0 : -5;
}
namespace ekfslam {
#define EKF_DUMP_BLOCK(seq)                                                         \
  do {                                                                              \
    __syncthreads();                                                                \
    if (blockIdx.y == 0) {                                                          \
      for (int e = threadIdx.x; e < kMaxU * (kMaxU + 1); e += blockDim.x)           \
        (&g_blocks[(seq) & 63][0][0])[e] = (&P[0][0])[e];                             \
      if (threadIdx.x < kMaxU) g_blockx[(seq) & 63][threadIdx.x] = sh.xU[0][threadIdx.x]; \
    }                                                                               \
    __syncthreads();                                                                \
  } while (0)
#else
#define EKF_DUMP_BLOCK(seq) \
  do {                      \
  } while (0)
#endif


// Diagnostic build only (tools/sigma_bench.hip): s_memrealtime (100 MHz) per Σ-pass workgroup.
#ifdef EKF_DIAG_STAMPS
__device__ unsigned long long g_sig_stamps[4096][5];
#define SIG_STAMP(i)                                                                   \
  do {                                                                                 \
    if (threadIdx.x == 0 && blockIdx.y == 0 && blockIdx.x < 4096) {                    \
      g_sig_stamps[blockIdx.x][i] = __builtin_amdgcn_s_memrealtime();                  \
      if (i == 0)                                                                      \
        g_sig_stamps[blockIdx.x][4] =                                                  \
            (static_cast<unsigned long long>(__builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (15 << 11))) << 32) | \
            __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));                \
    }                                                                                  \
  } while (0)
#else
#define SIG_STAMP(i) \
  do {               \
  } while (0)
#endif

// f64 MFMA 16×16×4: A[i = lane&15][k = lane>>4], B[k = lane>>4][j = lane&15],
// D[row = (lane>>4) + 4r][col = lane&15] (the f64 C/D map differs from the f32 one).
typedef double d4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ d4 mfma_f64(double a, double b, d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}



// J: the Joseph-form instantiation (round 6: a whole message of ≤ 16 markers per chunk): its row
// maps Z hold Zv beside Z (4m ≤ 64 columns) and V, S, C', D' are kept per step; the simple form's
// instantiation keeps the round-5 layout (ZC = 32 columns, one unused slot for the Joseph arrays).
template <bool J>
struct ChainSharedT {
  static constexpr int ZC = J ? kZJ : kZC;     // Z columns (the chain's and the rebuilt pv.Z / pv.K)
  static constexpr int JM = J ? kMaxJoseph : 1;  // Joseph steps kept
  int u[kMaxU];
  int skip[kMaxChunk];
  double alphaU[kMaxU];
  double row0raw[kMaxU];  // Σ_in[0][u_b]
  double col0raw[kMaxU];  // Σ_in[u_a][0]
  double xU[1][kMaxU];    // x[U], owned by wave 0 during the corrections
  double P[1][kMaxU][kMaxU + 1];    // Σ[U,U] (rows all, columns live)
  double Cz[kMaxChunk][4];  // wave 1, step c: C_k = M_k[:, pA_c]·Hᵀ·S⁻¹ (2×2) for k < c
  double Dy[kMaxChunk][4];  // wave 2, step c: D_k = H·K_k[pA_c] (2×2) for k < c
  double KU[kMaxChunk][kMaxU][2];
  double MU[kMaxChunk][kMaxU][2];
  double Z[kMaxU][ZC + 1];       // K_c[i] = r_0(i)[U] · Z[:, 2c..2c+1] (Joseph: Zv in 32 + 2c..)
  double Y[kZC][kMaxU + 1];      // M_c[:, j] = Y[2c..2c+1, :] · c_0(j)[U]
  double Zx[kMaxU];              // Σ_c Z_c ν_c: x_i += r_0(i)[U] · Zx
  double nu[kMaxChunk][2];
  double Hs[kMaxChunk][2][5];    // H_c over pA (published for waves 1–2)
  double Sis[kMaxChunk][4];      // S_c⁻¹
  // Joseph chunks (m ≤ kMaxJoseph): V_c = (Σ_c·Hᵀ − K_c·S_c)[U] and S_c per step (wave 0), wave 1's
  // C'_k = K_k[pA_c]ᵀ·Hᵀ and wave 2's D'_k = H·V_k[pA_c]
  double VU[JM][kMaxU][2];
  double Ss[JM][4];
  double Cv[JM][4];
  double Dv[JM][4];
  // kLook: the previous chunk's record and the blocks rebuilt from it
  struct {
    int u[kMaxU];
    int nu, m, first, joseph;
    double a1, a2, s00;
    double xU[kMaxU], Zx[kMaxU];
    // k (over U') padded to kMaxU + 1 = 36 with zeros, so MFMA operand reads need no predicate
    double Z[kMaxU + 1][ZC + 1];
    double Y[kZC][kMaxU + 1];
    double R[kMaxU][kMaxU + 1];       // Σ_pred'[U][U']  (U' = previous chunk's index set)
    double C[kMaxU + 1][kMaxU + 1];   // Σ_pred'[U'][U]
    double K[kMaxU][ZC + 1];      // R·Z'  = the previous K_c at U (Joseph: and V_c at U)
    double M[kZC][kMaxU + 1];     // Y'·C  = the previous M_c at U
    double r0U[kMaxU], c0U[kMaxU], r0P[kMaxU], c0P[kMaxU];
    double xg[kMaxU];             // x_in'[u] for this chunk's U (rows the previous chunk missed)
  } pv;
  double junk[4][64];             // per-wave sink of masked-off LDS stores (no divergent branch)
  double junk2[64][2];
  double pose[3];
  double xpose[3];  // x_in pose (posterior of the previous chunk)
  double npose[3], na1, na2;  // the next chunk's predicted pose and At entries (wave 3, ahead)
  int npose_ci;               // the chunk index they belong to (−1: none)
  double tmo[3];    // t_map_odom
  double a1, a2, s00;
  int nu_cnt;
  unsigned status;
  int pub;    // steps whose K, M, H, S⁻¹ wave 0 has published
  int pdone;  // steps wave 3 has applied outside the cross
  int any_init;  // a correction of this chunk initialised its landmark (slam.cpp:213-216)
  int zdone;     // Joseph: steps whose Z_c, Zv_c wave 1 has stored (wave 2 reads them)
};


#include "ekf_sync.hpp"  // (hand-off protocol and buffer-descriptor helpers)

// A workgroup barrier that orders LDS only: global loads in flight stay in flight across it
// (__syncthreads waits vmcnt(0), and vmcnt counts loads too).
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Intra-workgroup hand-off through LDS (waves on different SIMDs; no s_barrier).
// The LDS executes one wave's accesses in issue order, so a flag stored after the data is seen
// after it by any wave: no s_waitcnt before the flag (a release would drain every LDS op of the
// wave first), only a compiler fence that keeps the data stores ahead of it.
__device__ __forceinline__ void lds_publish(int* flag, int v) {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __hip_atomic_store(flag, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_wait_ge(const int* flag, int v) {
  while (__builtin_amdgcn_readfirstlane(
             __hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) < v)
    __builtin_amdgcn_s_sleep(1);
}

// Wave 0's corrections (see k_chain, A2): a function of its own, so that its register allocation
// is not the one of the kernel's four wave programs together (the shared allocation spilled
// SGPRs, and their reloads sat in this loop). LDS through address-space-3 references.
template <bool J>
using LdsChain = __attribute__((address_space(3))) ChainSharedT<J>;
typedef __attribute__((address_space(3))) const MsgDesc LdsDesc;
typedef __attribute__((address_space(3))) double ldsd;
__device__ __forceinline__ void lds_publish3(__attribute__((address_space(3))) int* flag, int v) {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __hip_atomic_store(flag, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}
__device__ __forceinline__ void lds_wait_ge3(const __attribute__((address_space(3))) int* flag,
                                             int v) {
  while (__builtin_amdgcn_readfirstlane(
             __hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) < v)
    __builtin_amdgcn_s_sleep(1);
}

// J: a Joseph chunk (m ≤ kMaxJoseph). Every step then also subtracts V_c·K_cᵀ, V_c = Σ_c·Hᵀ − K_c·S_c
// (slam.cpp:264-265's update as (I − KH)Σ(I − KH)ᵀ + K·R·Kᵀ expanded), always after the K_c·M_c term
// — the order wave 3 uses, so an entry both waves compute has the same bits.
// The diagnostic build (EKF_DIAG_STAMPS, libekfslam_diag.so) also carries the hand-off
// instrumentation behind PassArgs::dbg (EKF_DBG_ORDER, tools/diag_handover.py, tools/diag_dlog.py);
// in the product library every such branch folds away.
#ifdef EKF_DIAG_STAMPS
constexpr bool kDiagBuild = true;
#else
constexpr bool kDiagBuild = false;
#endif

// dev only (PassArgs::dbg & 16): order-independent wrapping sums of the bit patterns a kernel read
// or wrote, A.dlog[kind][seq % 64][f % 64][slot]
__device__ __forceinline__ unsigned long long dbits(double v) {
  return static_cast<unsigned long long>(__double_as_longlong(v));
}
__device__ __forceinline__ unsigned long long dbits(float v) { return __float_as_uint(v); }
template <typename T>
__device__ __forceinline__ void dlog_add(const PassArgs<T>& A, int kind, unsigned seq, int f,
                                         int slot, unsigned long long v) {
  atomicAdd(A.dlog + ((static_cast<size_t>(kind) * 64 + (seq & 63u)) * 64 + (f & 63)) * 8 + slot, v);
}

// dev only (PassArgs::dbg & 16): step c's wrapping sums at lg[(kChainLogKind + c)·64·64·8 + slot]
constexpr int kChainLogKind = 5;
__device__ __forceinline__ unsigned long long dbits0(double v) {
  return static_cast<unsigned long long>(__double_as_longlong(v));
}
__device__ __forceinline__ void steplog(unsigned long long* lg, int c, int slot, unsigned long long v) {
  atomicAdd(lg + static_cast<size_t>(kChainLogKind + c) * 64 * 64 * 8 + slot, v);
}

template <bool J>
__device__ __noinline__ void chain_wave0(LdsChain<J>* shp, LdsDesc* dp, int pb, int m, int nu,
                                         double r_noise, unsigned seq, unsigned long long* lg) {
  LdsChain<J>& sh = *shp;
  constexpr int JM = ChainSharedT<J>::JM;
  LdsDesc& d = *dp;
  const int lane = threadIdx.x & 63;
  (void)seq;  // (diagnostic stamps)
  // Lane ℓ carries row ℓ of the step's block columns (pk = Σ[ℓ, pA]) and column ℓ of its block
  // rows (pm = Σ[pA, ℓ]) in registers from one step to the next: the cross update of step c
  // produces exactly step c+1's pk (and pm for the later columns). S needs no block read:
  // (Σ·Hᵀ)[ℓ] is the first half of K anyway, and S = H·(Σ·Hᵀ)[pA] takes five lanes' values by
  // v_readlane. The pose / landmark x of a step come by v_readlane from the lane that updated
  // them. Lanes ≥ |U| carry a clamped row and never store.
  const int lr = lane < kMaxU ? lane : kMaxU - 1;
  const int ul = sh.u[lr];
  double pk[5], pm[5];
  double xl = sh.xU[0][lr];
#pragma unroll
  for (int a = 0; a < 5; ++a) {
    const int col = a < 3 ? a : 3 + a - 3;  // pA of step 0 = {0, 1, 2, 3, 4}
    pk[a] = sh.P[pb][lr][col];
    pm[a] = sh.P[pb][col][lr];
  }
  // Look-ahead operands of the next marker's cross (see the step): rn = Σ[ℓ, nx..nx+1] and
  // qn = Σ[nx..nx+1, ℓ] one step old, and the previous step's K (kp) and M (mp) of this lane.
  double rn[2], qn[2], kp0 = 0.0, kp1 = 0.0, mp0 = 0.0, mp1 = 0.0, vp0 = 0.0, vp1 = 0.0;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int col = min(5 + j, kMaxU - 1);
    rn[j] = sh.P[pb][lr][col];
    qn[j] = sh.P[pb][col][lr];
  }
  // A step's geometry (first sighting, ẑ, H) needs only x after the step before. It is computed
  // right after that step's state update, ahead of the step's cross update, so the two
  // independent chains (f64 ALU vs LDS round trips) interleave in one basic block.
  double lx = 0.0, ly = 0.0, H0[5], H1[5], zhat[2], braw = 0.0;
  bool init = false, bok = true;
  // the marker's measurement and skip flag, read one step ahead (the descriptor and the skip list
  // are constant during the chunk): their LDS round trip stays off the step's dependent chain
  const bool noinit = (d.flags & kNoInit) != 0;
  double zn0 = 0.0, zn1 = 0.0;
  int skn = 0;
  if (m > 0) {
    zn0 = d.z[0][0];
    zn1 = d.z[0][1];
    skn = sh.skip[0];
  }
  auto geometry = [&](int c) {
    const int pj = 3 + 2 * c;
    const double pose[3] = {readlane_f64(xl, 0), readlane_f64(xl, 1), readlane_f64(xl, 2)};
    lx = readlane_f64(xl, pj);
    ly = readlane_f64(xl, pj + 1);
    init = false;
    // slam.cpp:213-216 (zn, skn: marker c); a wave-uniform test, so a scalar branch
    if (__builtin_amdgcn_readfirstlane(!skn && !noinit && lx == 0.0 && ly == 0.0)) {
      init = true;
      sh.any_init = 1;
      lx = pose[1] + zn0 * cos(zn1 + pose[0]);
      ly = pose[2] + zn0 * sin(zn1 + pose[0]);
    }
    range_bearing(pose, lx, ly, zhat, H0, H1, &braw, &bok);
  };
  if (m > 0) geometry(0);
  for (int c = 0; c < m; ++c) {
    const int pj = 3 + 2 * c, nx = pj + 2;
    const bool more = c + 1 < m;
    EKF_STAMP(64 + 8 * c);
    const double z0 = zn0, z1 = zn1;
    bool sk = skn != 0;
    if (more) {  // marker c + 1's, for geometry(c + 1) and the next step
      zn0 = d.z[c + 1][0];
      zn1 = d.z[c + 1][1];
      skn = sh.skip[c + 1];
    }
    double Si[4], nv0, nv1, Sm_keep[4];
    EKF_STAMP(65 + 8 * c);
    // (Σ·Hᵀ)[ℓ] and (H·Σ)[:, ℓ]. H's shape (range_bearing): H0 = [0, h1, h2, −h1, −h2],
    // H1 = [−1, g1, g2, −g1, −g2] — a row times H is two FMAs on (v1 − v3, v2 − v4) (exact negations)
    const double dk1 = pk[1] - pk[3], dk2 = pk[2] - pk[4];
    const double dm1 = pm[1] - pm[3], dm2 = pm[2] - pm[4];
    double ka = fma(H0[2], dk2, H0[1] * dk1), kb = fma(H1[2], dk2, fma(H1[1], dk1, -pk[0]));
    double mm0 = fma(H0[2], dm2, H0[1] * dm1), mm1 = fma(H1[2], dm2, fma(H1[1], dm1, -pm[0]));
    {
      double Sm[4];  // S = H·(Σ·Hᵀ)[pA] + R (slam.cpp:252), the same shape
      {
        double ta[5], tb[5];
#pragma unroll
        for (int a = 0; a < 5; ++a) {
          const int l = a < 3 ? a : pj + a - 3;
          ta[a] = readlane_f64(ka, l);
          tb[a] = readlane_f64(kb, l);
        }
        const double ta1 = ta[1] - ta[3], ta2 = ta[2] - ta[4], tb1 = tb[1] - tb[3], tb2 = tb[2] - tb[4];
        Sm[0] = fma(H0[2], ta2, H0[1] * ta1) + r_noise;
        Sm[1] = fma(H0[2], tb2, H0[1] * tb1);
        Sm[2] = fma(H1[2], ta2, fma(H1[1], ta1, -ta[0]));
        Sm[3] = fma(H1[2], tb2, fma(H1[1], tb1, -tb[0])) + r_noise;
      }
      for (int k = 0; k < 4; ++k) Sm_keep[k] = Sm[k];
      // The common case without a branch (so the step's scalar chain is one basic block): a
      // finite, nonsingular S and a bearing / innovation within normalize_angle_near's range.
      // Anything else — a skipped marker, a singular S (arma's inv throws), an angle beyond it —
      // redoes these scalars on the generic path below, in the reference's order; the common
      // case's values are that path's bit for bit.
      const double det = inv2_calc(Sm, Si);
      nv0 = z0 - zhat[0];
      bool nok;
      nv1 = normalize_angle_near(z1 - zhat[1], &nok);
      const bool good = !sk && bok && nok && inv2_ok(det, Si);
      if (!__builtin_amdgcn_readfirstlane(good)) {  // (uniform: every lane has the same scalars)
        if (!bok) zhat[1] = normalize_angle(braw);  // |θ| > π: the generic fmod path
        if (!sk && inv2(Sm, Si)) {
          nv0 = z0 - zhat[0];
          bool nok2;
          const double nn = normalize_angle_near(z1 - zhat[1], &nok2);
          nv1 = nok2 ? nn : normalize_angle(z1 - zhat[1]);
        } else {
          if (!sk) sh.status |= EKF_FLAG_NUMERIC_D;  // same value from every lane
          sk = true;
#pragma unroll
          for (int a = 0; a < 5; ++a) H0[a] = H1[a] = 0.0;
          Si[0] = Si[1] = Si[2] = Si[3] = 0.0;
          nv0 = nv1 = 0.0;
          ka = kb = mm0 = mm1 = 0.0;
        }
      }
    }
    if (kDiagBuild && lg) {
      if (lane == 0) {
        steplog(lg, c, 0, dbits0(Sm_keep[0]) + dbits0(Sm_keep[1]) + dbits0(Sm_keep[2]) +
                              dbits0(Sm_keep[3]) + dbits0(Si[0]) + dbits0(Si[3]));
        steplog(lg, c, 1, dbits0(nv0) + dbits0(nv1) + dbits0(zhat[0]) + dbits0(zhat[1]) +
                              dbits0(H0[1]) + dbits0(H1[2]));
      }
      if (lane < nu) steplog(lg, c, 2, dbits0(ka) + dbits0(kb) + dbits0(mm0) + dbits0(mm1));
    }
    // The next marker's cross operands (Bx = {0, 1, 2, nx, nx+1}) after step c−1. Pose columns /
    // rows: pk / pm (pA ⊃ pose). The nx columns / rows were read one step back (rn / qn, after
    // step c−2) and get step c−1's rank-2 term here from registers: K_{c−1} of this lane (kp)
    // and of the nx rows (v_readlane), M_{c−1} of this column (mp) and of the nx columns
    // (v_readlane) — the writers' expression, operands and order (wave 3's, or this wave's cross
    // update), so the same bits. Step 0 has kp = mp = 0: rank2_sub(v, 0, 0, 0, 0) = v.
    double xr[5], xq[5];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      xr[k] = pk[k];
      xq[k] = pm[k];
    }
    // wave 3's progress, read here (≈ 1 000 cycles into the step, when it has normally finished
    // step c − 1) and tested below: the flag's LDS round trip off the chain's path
    const int pd_early = __hip_atomic_load(&sh.pdone, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    {  // K_{c−1} and M_{c−1} of the nx rows / columns: broadcast LDS reads of what step c−1
       // stored (the stored values are the registers' values; two reads instead of 8 readlanes)
      const int l0 = more ? nx : 0, cp = c > 0 ? c - 1 : 0;
      const double mqx = sh.MU[cp][l0][0], mqy = sh.MU[cp][l0][1];
      const double mq2x = sh.MU[cp][l0 + 1][0], mq2y = sh.MU[cp][l0 + 1][1];
      const double kqx = sh.KU[cp][l0][0], kqy = sh.KU[cp][l0][1];
      const double kq2x = sh.KU[cp][l0 + 1][0], kq2y = sh.KU[cp][l0 + 1][1];
      // step 0: kp = mp = 0 and the (stale, finite) reads multiply zeros: rank2_sub returns v
      xr[3] = rank2_sub(rn[0], kp0, kp1, mqx, mqy);
      xr[4] = rank2_sub(rn[1], kp0, kp1, mq2x, mq2y);
      xq[3] = rank2_sub(qn[0], kqx, kqy, mp0, mp1);
      xq[4] = rank2_sub(qn[1], kq2x, kq2y, mp0, mp1);
      if (J) {  // − V_{c−1}·K_{c−1}ᵀ (step 0: vp = kp = 0)
        const int cj = min(cp, JM - 1);
        const double vqx = sh.VU[cj][l0][0], vqy = sh.VU[cj][l0][1];
        const double vq2x = sh.VU[cj][l0 + 1][0], vq2y = sh.VU[cj][l0 + 1][1];
        xr[3] = rank2_sub(xr[3], vp0, vp1, kqx, kqy);
        xr[4] = rank2_sub(xr[4], vp0, vp1, kq2x, kq2y);
        xq[3] = rank2_sub(xq[3], vqx, vqy, kp0, kp1);
        xq[4] = rank2_sub(xq[4], vq2x, vq2y, kp0, kp1);
      }
    }
    EKF_STAMP(66 + 8 * c);
    // the cross after next (nx + 2): read once wave 3 has applied step c−1 outside this step's
    // cross, before this step's cross update writes its Bx rows (wave 3 writes these entries for
    // step c only after the publish below, whose release waits for the reads)
    if (c + 2 < m) {
      // the LDS serves this wave's accesses in order, and wave 3 stored its entries before the
      // flag: once a flag value ≥ c has been read, later reads see the entries (a compiler fence
      // keeps them after the test)
      if (__builtin_amdgcn_readfirstlane(pd_early) < c) lds_wait_ge3(&sh.pdone, c);
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        rn[j] = sh.P[pb][lr][nx + 2 + j];
        qn[j] = sh.P[pb][nx + 2 + j][lr];
      }
    }
    if (kDiagBuild && lg && lane < nu) {
      unsigned long long v = 0;
      for (int k = 0; k < 5; ++k) v += dbits0(xr[k]) + dbits0(xq[k]);
      steplog(lg, c, 3, v);
      steplog(lg, c, 7, dbits0(rn[0]) + dbits0(rn[1]) + dbits0(qn[0]) + dbits0(qn[1]));
    }
    const int jx = __builtin_amdgcn_readlane(ul, pj);  // sh.u[pj] (ul = sh.u[lane], pj < kMaxU)
    EKF_STAMP(67 + 8 * c);
    const double K0 = ka * Si[0] + kb * Si[2];  // K = Σ·Hᵀ·S⁻¹
    const double K1 = ka * Si[1] + kb * Si[3];
    // Joseph: V = Σ·Hᵀ − K·S of this lane's row (zero in exact arithmetic; the form's rounding)
    const double V0 = J ? ka - (K0 * Sm_keep[0] + K1 * Sm_keep[2]) : 0.0;
    const double V1 = J ? kb - (K0 * Sm_keep[1] + K1 * Sm_keep[3]) : 0.0;
    {
      double xt = xl;
      xt = (init && ul == jx) ? lx : ((init && ul == jx + 1) ? ly : xt);
      xt = xt + (K0 * nv0 + K1 * nv1);              // slam.cpp:261
      bool tok;                                     // slam.cpp:267 on lane 0, branch-free
      const double tn = normalize_angle_near(xt, &tok);
      const double xraw = xt;
      xt = lane == 0 ? tn : xt;
      // lane 0's θ beyond normalize_angle_near's range: the generic path (a scalar branch)
      if (__builtin_amdgcn_ballot_w64(!tok) & 1ull) {
        if (lane == 0) xt = normalize_angle(xraw);
      }
      xl = xt;
      *(lane < nu ? &sh.xU[0][lane] : &sh.junk[0][lane]) = xt;
      if (kDiagBuild && lg && lane < nu) {
        steplog(lg, c, 4, dbits0(K0) + dbits0(K1));
        steplog(lg, c, 5, dbits0(xt));
      }
    }
    {
      const bool in = lane < nu, st = lane < kMaxU;
      ldsd* kd = st ? &sh.KU[c][lane][0] : &sh.junk2[lane][0];
      ldsd* md = st ? &sh.MU[c][lane][0] : &sh.junk2[lane][0];
      kd[0] = in ? K0 : 0.0;
      kd[1] = in ? K1 : 0.0;
      md[0] = in ? mm0 : 0.0;
      md[1] = in ? mm1 : 0.0;
      if (J) {  // V and S of the step, for waves 1–3 and the fp32 block patch
        const int cj = min(c, JM - 1);
        ldsd* vd = st ? &sh.VU[cj][lane][0] : &sh.junk2[lane][0];
        vd[0] = in ? V0 : 0.0;
        vd[1] = in ? V1 : 0.0;
        if (lane == 0)
          for (int k = 0; k < 4; ++k) sh.Ss[cj][k] = sk ? 0.0 : Sm_keep[k];
      }
    }
    if (lane == 0) {
#pragma unroll
      for (int a = 0; a < 5; ++a) {
        sh.Hs[c][0][a] = H0[a];
        sh.Hs[c][1][a] = H1[a];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) sh.Sis[c][k] = Si[k];
      sh.nu[c][0] = nv0;
      sh.nu[c][1] = nv1;
    }
    lds_publish3(&sh.pub, c + 1);
    EKF_STAMP(68 + 8 * c);
    if (more) {
      // K and M of the five Bx rows / columns: broadcast LDS reads of what this step stored
      // above (issued before geometry(c + 1), so its latency hides; ds_read_b128 each)
      double kx0[5], kx1[5], mx0[5], mx1[5], vx0[5], vx1[5];
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        const int l = k < 3 ? k : nx + k - 3;
        const double kkx = sh.KU[c][l][0], kky = sh.KU[c][l][1];
        const double mkx = sh.MU[c][l][0], mky = sh.MU[c][l][1];
        kx0[k] = kkx;
        kx1[k] = kky;
        mx0[k] = mkx;
        mx1[k] = mky;
        if (J) {
          const int cj = min(c, JM - 1);
          vx0[k] = sh.VU[cj][l][0];
          vx1[k] = sh.VU[cj][l][1];
        }
      }
      geometry(c + 1);
      // wave 3's step c−1 writes outside this step's cross must land before this cross update
      // overwrites the nx columns / rows (waited for above already when c + 2 < m)
      if (c + 2 >= m && __builtin_amdgcn_readfirstlane(pd_early) < c) lds_wait_ge3(&sh.pdone, c);
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      // all rows × Bx columns: next step's pk
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        const int col = k < 3 ? k : nx + k - 3;
        pk[k] = rank2_sub(xr[k], K0, K1, mx0[k], mx1[k]);
        if (J) pk[k] = rank2_sub(pk[k], V0, V1, kx0[k], kx1[k]);
        *(lane < nu ? &sh.P[pb][lane][col] : &sh.junk[0][lane]) = pk[k];
      }
      // Bx rows × every other column (the block is kept whole so that the chunk's final Σ[U,U]
      // can seed the next chunk): next step's pm there
      const bool later = lane >= 3 && lane < nu && lane != nx && lane != nx + 1;
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        const int row = k < 3 ? k : nx + k - 3;
        double v = rank2_sub(xq[k], kx0[k], kx1[k], mm0, mm1);
        if (J) v = rank2_sub(v, vx0[k], vx1[k], K0, K1);
        pm[k] = v;
        *(later ? &sh.P[pb][row][lane] : &sh.junk[0][lane]) = v;
      }
      if (kDiagBuild && lg && lane < nu) {
        unsigned long long v = 0;
        for (int k = 0; k < 5; ++k) v += dbits0(pk[k]) + dbits0(pm[k]);
        steplog(lg, c, 6, v);
      }
      // (the Bx × Bx entries: lane `row` stored the same value as its pk, same operands)
      kp0 = K0;
      kp1 = K1;
      mp0 = mm0;
      mp1 = mm1;
      vp0 = V0;
      vp1 = V1;
    }
    EKF_STAMP(70 + 8 * c);
  }
}


// The previous chunk's predict on the gathered rebuild operands: v + α_i·Σ[0][j] +
// (Σ[i][0] + α_i·Σ00)·α_j + Q̄, for D = Σ_in'[U, U] → P, R = Σ_in'[U, U'] → pv.R and
// C = Σ_in'[U', U] → pv.C (R / C columns k ≥ |U'| up to 36 zeroed: MFMA k padding). Thread tid's
// entries e = tid + i·256 of the 36 × 36 block. Reads sh.u (U), sh.pv.u (U'), the staged row 0 /
// column 0 (pv.r0U, c0U, r0P, c0P) and the previous predict (pv.first, a1, a2).
constexpr int kChainThreads = 256;
constexpr int kRebW = kMaxU + 1;                                      // 36: entry e = a·36 + b
constexpr int kRebPer = (kRebW * kRebW + kChainThreads - 1) / kChainThreads;  // 6
// The predict (slam.cpp:198) changes an entry of a block over U × U' only in rows / columns 1 and 2
// (α_i = 0 unless u_i ∈ {1, 2}, and u_i = i for the pose positions of U and U') and on the pose
// diagonal (Q̄): 4·36 − 3 entries of the 36 × 36 block. Special entry s → (a, b): s < 72 rows 1, 2
// (b = 0..35); s < 140 columns 1, 2 (a = 0, 3..35); s = 140 the (0, 0) entry.
constexpr int kSpec = 141;
__device__ __forceinline__ void special_entry(int s, int& a, int& b) {
  if (s < 72) {
    a = 1 + (s >= 36);
    b = s - (s >= 36 ? 36 : 0);
  } else if (s < 140) {
    const int r = s - 72, h = r >= 34;
    b = 1 + h;
    const int a2 = r - (h ? 34 : 0);
    a = a2 == 0 ? 0 : a2 + 2;
  } else {
    a = 0;
    b = 0;
  }
}

template <typename T, typename Shared>
__device__ __forceinline__ void rebuild_rcd(Shared& sh, double (&P)[kMaxU][kMaxU + 1],
                                            const T (&vd)[kRebPer], const T (&vr)[kRebPer],
                                            const T (&vc)[kRebPer], int tid, int nu, int np,
                                            double q) {
  constexpr int kW = kRebW, kPer = kRebPer;
  // the raw blocks: no LDS read
#pragma unroll
  for (int i = 0; i < kPer; ++i) {
    const int e = tid + i * kChainThreads;
    const int a = e / kW, b = e % kW;
    if (a < nu && b < nu) P[a][b] = static_cast<double>(vd[i]);
    if (a < nu) {  // b = k over U' (36: the MFMA k padding, zero)
      sh.pv.R[a][b] = b < np ? static_cast<double>(vr[i]) : 0.0;
      sh.pv.C[b][a] = b < np ? static_cast<double>(vc[i]) : 0.0;
    }
  }
  if (sh.pv.first == 0) return;  // (uniform)
  // The previous predict on the special entries, by the thread that gathered them (its raw values
  // are in registers, so no barrier): a thread's entries e = tid + 256·i have b = (tid % 36 + 4·i)
  // mod 36, so besides position 0 (rows 1, 2 are e ∈ [36, 108); (0, 0) is e = 0) at most one
  // position ic ≥ 1 falls in column 1 or 2. Both are rewritten over the raw stores above (same
  // thread, same address: LDS order), with one wait for all operand reads and no branch.
  const int r = tid % kW;
  int ic = 0;
#pragma unroll
  for (int i = 1; i < kPer; ++i) {
    const int bb = (r + 4 * i) % kW;
    ic = (bb == 1 || bb == 2) && tid + i * kChainThreads < kW * kW ? i : ic;
  }
  double sv[2][3];
  sv[0][0] = static_cast<double>(vd[0]);
  sv[0][1] = static_cast<double>(vr[0]);
  sv[0][2] = static_cast<double>(vc[0]);
  sv[1][0] = sv[1][1] = sv[1][2] = 0.0;
#pragma unroll
  for (int i = 1; i < kPer; ++i) {
    sv[1][0] = ic == i ? static_cast<double>(vd[i]) : sv[1][0];
    sv[1][1] = ic == i ? static_cast<double>(vr[i]) : sv[1][1];
    sv[1][2] = ic == i ? static_cast<double>(vc[i]) : sv[1][2];
  }
  const double s00 = sh.pv.r0U[0], qa1 = sh.pv.a1, qa2 = sh.pv.a2;
  int pa[2], pb[2];
  bool sp[2];
  double r0u_b[2], c0u_a[2], r0p_b[2], r0u_a[2], c0p_b[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int e = tid + (j ? ic : 0) * kChainThreads;
    const int a = e / kW, b = e % kW;
    pa[j] = a;
    pb[j] = b;
    sp[j] = j ? ic > 0 : (a == 1 || a == 2 || b == 1 || b == 2 || e == 0);
    const int ac = min(a, kMaxU - 1), bc = min(b, kMaxU - 1);
    r0u_b[j] = sh.pv.r0U[bc];
    c0u_a[j] = sh.pv.c0U[ac];
    r0p_b[j] = sh.pv.r0P[bc];
    r0u_a[j] = sh.pv.r0U[ac];
    c0p_b[j] = sh.pv.c0P[bc];
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int a = pa[j], b = pb[j];
    const double ai = alpha_of(a, qa1, qa2), aj = alpha_of(b, qa1, qa2);
    const bool qd = a == b && a < 3;
    double v = sv[j][0] + ai * r0u_b[j];  // D = Σ_in'[U, U] → P
    v = v + (c0u_a[j] + ai * s00) * aj;
    double v2 = sv[j][1] + ai * r0p_b[j];  // R = Σ_in'[U, U'] (b = k over U')
    v2 = v2 + (c0u_a[j] + ai * s00) * aj;
    double w2 = sv[j][2] + aj * r0u_a[j];  // C = Σ_in'[U', U]
    w2 = w2 + (c0p_b[j] + aj * s00) * ai;
    const bool okd = sp[j] && a < nu && b < nu, okr = sp[j] && a < nu && b < np;
    *(okd ? &P[a][b] : &sh.junk[0][tid & 63]) = qd ? v + q : v;
    *(okr ? &sh.pv.R[a][b] : &sh.junk[1][tid & 63]) = qd ? v2 + q : v2;
    *(okr ? &sh.pv.C[b][a] : &sh.junk[2][tid & 63]) = qd ? w2 + q : w2;
  }
}

template <bool J>
struct FactorSharedT {
  static constexpr int ZC = J ? kZJ : kZC;  // the record's Z columns in use (Joseph: Z and Zv)
  int u[kMaxU + 1];
  double alphaU[kMaxU], row0raw[kMaxU], col0raw[kMaxU], Zx[kMaxU], xU[kMaxU];
  double Z[kMaxU][ZC + 1];
  double Y[kZC][kMaxU + 1];
  double a1, a2, s00;
  int nu;
};

// The factor kernel's two halves: a chunk's record into LDS, then one wave's 16 indices of Kcat = R_pred·Z (rows) and
// Mcat = Y·C_pred (columns) on f64 MFMA, plus the new state.
// R_pred(i)[b] = Σ_pred[i][u_b], C_pred(j)[a] = Σ_pred[u_a][j].
template <bool J>
__device__ __forceinline__ void factor_record(const ChunkRec* rec, FactorSharedT<J>& sh, int tid) {
  constexpr int ZC = FactorSharedT<J>::ZC;
  {  // the record into LDS: every load of a thread issued before its first LDS store
    constexpr int kPer = (kMaxU * kZC + 255) / 256;  // 5
    constexpr int kPerZ = (kMaxU * ZC + 255) / 256;  // 5 (Joseph: 9)
    double vz[kPerZ], vy[kPer];
#pragma unroll
    for (int i = 0; i < kPerZ; ++i) {  // (the record's rows are kZJ wide)
      const int e = min(tid + 256 * i, kMaxU * ZC - 1);
      vz[i] = rec->Z[e / ZC][e % ZC];
    }
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int e = min(tid + 256 * i, kMaxU * kZC - 1);
      vy[i] = (&rec->Y[0][0])[e];
    }
#pragma unroll
    for (int i = 0; i < kPerZ; ++i) {
      const int e = tid + 256 * i;
      if (e < kMaxU * ZC) {
        const int b = e / ZC, k = e - b * ZC;
        sh.Z[b][k] = vz[i];
      }
    }
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int e = tid + 256 * i;
      if (e < kMaxU * kZC) {
        const int k2 = e / kMaxU, b2 = e - k2 * kMaxU;
        sh.Y[k2][b2] = vy[i];
      }
    }
  }
  if (tid < kMaxU) {
    sh.u[tid] = rec->u[tid];
    sh.alphaU[tid] = rec->alphaU[tid];
    sh.row0raw[tid] = rec->row0raw[tid];
    sh.col0raw[tid] = rec->col0raw[tid];
    sh.Zx[tid] = rec->Zx[tid];
    sh.xU[tid] = rec->xU[tid];
  }
  if (tid == 0) {
    sh.a1 = rec->a1;
    sh.a2 = rec->a2;
    sh.s00 = rec->s00;
    sh.nu = rec->nu;
  }
}

template <typename T, bool J>
__device__ __forceinline__ void factor_wave(const PassArgs<T>& A, const MsgDesc& d, int f, int wg,
                                            const FactorSharedT<J>& sh, int lane) {
  constexpr int NG = FactorSharedT<J>::ZC / 16;  // 16-column groups of Z: 2 (Joseph: 4)
  const int n = A.n, ld = A.ld, ldk = A.ldk;
  const T* S = A.sig[d.parity] + f * A.sig_stride;
  const double* xin = A.x[d.parity] + f * A.x_stride;
  double* xout = A.x[d.parity ^ 1] + f * A.x_stride;
  T* kc = A.kcat + f * A.km_stride;
  T* mc = A.mcat + f * A.km_stride;
  const bool first = (d.flags & kFirst) != 0;
  const bool joseph = J && (d.flags & kJoseph) != 0;
  // Joseph: Mcat rows 2 + 2m .. 2 + 4m − 1 hold K_c (the V_c·K_cᵀ term's column factor), written
  // by the row waves; the column waves leave them alone
  const int jk0 = joseph ? 2 * d.m : kZC, jk1 = joseph ? 4 * d.m : kZC;
  const int nu = sh.nu;
  const double* xfin = sh.xU;
  // ---- phase B: Kcat = R_pred·Z, Mcat = Y·C_pred on f64 MFMA, 16 rows (or columns) per wave ----
  // R_pred(i)[b] = Σ_pred[i][u_b], C_pred(j)[a] = Σ_pred[u_a][j] (predict folded in as above).
  const int row_tiles = (n + 15) / 16;
  const int ks = lane >> 4, l16 = lane & 15;
  const double s00 = sh.s00;
  // Mcat columns j = C0 + l16 of a wave from Σ_in[U, j] (raw) and Σ_in[0, j] (c0t)
  auto columns = [&](int j, const T (&raw)[9], T c0t) {
    const bool vj = j < n;
    const double c0raw = vj ? static_cast<double>(c0t) : 0.0;
    const double aj = first ? alpha_of(j, sh.a1, sh.a2) : 0.0;
    double bv[9];
#pragma unroll
    for (int s = 0; s < 9; ++s) {
      const int k = 4 * s + ks;
      double v = (vj && k < nu) ? static_cast<double>(raw[s]) : 0.0;
      if (first && vj && k < nu) {
        v = v + sh.alphaU[k] * c0raw;
        v = v + (sh.col0raw[k] + sh.alphaU[k] * s00) * aj;
        if (sh.u[k] == j && j < 3) v += A.q;
      }
      bv[s] = v;
    }
    d4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < 9; ++s) {
      const int k = 4 * s + ks;
      const double y0 = k < kMaxU ? sh.Y[l16][k] : 0.0;
      const double y1 = k < kMaxU ? sh.Y[16 + l16][k] : 0.0;
      acc0 = mfma_f64(y0, bv[s], acc0);
      acc1 = mfma_f64(y1, bv[s], acc1);
    }
    if (vj && ks == 0) {
      mc[0 * ldk + j] = static_cast<T>(first ? c0raw : 0.0);
      mc[1 * ldk + j] = static_cast<T>(first ? aj : 0.0);
    }
    if (vj) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int kr = ks + 4 * r;
        if (kr < jk0 || kr >= jk1) mc[(2 + kr) * ldk + j] = static_cast<T>(acc0[r]);
        if (16 + kr < jk0 || 16 + kr >= jk1) mc[(18 + kr) * ldk + j] = static_cast<T>(acc1[r]);
      }
    }
  };
  // fp64: Σ_in is symmetric, so a row wave's Σ_in[U, i] are also its columns' — one wave per 16
  // indices builds both Kcat rows and Mcat columns (half the waves and half the Σ_in reads of
  // separate row and column waves, the same values)
  constexpr bool merged = sizeof(T) == 8;
  if (wg < row_tiles) {
    const int R0 = wg * 16;
    const int i = R0 + l16;
    const bool vi = i < n;
    const T* rowp = S + static_cast<size_t>(vi ? i : 0) * ld;
    // every gather issued unconditionally (clamped index; padding u = 0 stays in bounds), then
    // masked: a predicated load would be a branch with its own wait, one round trip per load
    T raw[9];
    T r0t;
    if (sizeof(T) == 8) {
      // fp64 Σ is symmetric (the symmetric Σ pass mirrors every element below the diagonal), so
      // Σ_in[i, U] is read as Σ_in[U, i]: 16 consecutive i per row of U (128 B) instead of one
      // scattered element per lane and column of U
      r0t = S[vi ? i : 0];
#pragma unroll
      for (int s = 0; s < 9; ++s)
        raw[s] = S[static_cast<size_t>(sh.u[min(4 * s + ks, kMaxU - 1)]) * ld + (vi ? i : 0)];
    } else {
      r0t = rowp[0];
#pragma unroll
      for (int s = 0; s < 9; ++s) raw[s] = rowp[sh.u[min(4 * s + ks, kMaxU - 1)]];
    }
    const double r0raw = vi ? static_cast<double>(r0t) : 0.0;
    const double ai = first ? alpha_of(i, sh.a1, sh.a2) : 0.0;
    double av[9];
#pragma unroll
    for (int s = 0; s < 9; ++s) {
      const int k = 4 * s + ks;
      double v = (vi && k < nu) ? static_cast<double>(raw[s]) : 0.0;
      if (first && vi && k < nu) {
        v = v + ai * sh.row0raw[k];
        v = v + (r0raw + ai * s00) * sh.alphaU[k];
        if (i == sh.u[k] && i < 3) v += A.q;
      }
      av[s] = v;
    }
    d4 acc[NG], acc2 = {0, 0, 0, 0};
#pragma unroll
    for (int g = 0; g < NG; ++g) acc[g] = d4{0, 0, 0, 0};
#pragma unroll
    for (int s = 0; s < 9; ++s) {
      const int k = 4 * s + ks;
      const double zx = (k < kMaxU && l16 == 0) ? sh.Zx[k] : 0.0;
      // Zᵀ·R rather than R·Z: the lane then holds Kcat[c = ks + 4r][i = R0 + l16], so each store
      // covers 4 factor rows × 128 B instead of 16 rows × 32 B (the same products and sums)
#pragma unroll
      for (int g = 0; g < NG; ++g)
        acc[g] = mfma_f64(k < kMaxU ? sh.Z[k][16 * g + l16] : 0.0, av[s], acc[g]);
      acc2 = mfma_f64(zx, av[s], acc2);
    }
    if (kDiagBuild && (A.dbg & 16)) {  // Σ_in as read, x_in as read
      unsigned long long s2 = 0;
#pragma unroll
      for (int s = 0; s < 9; ++s) s2 += dbits(raw[s]);
      s2 += dbits(r0t);
      dlog_add(A, 4, A.seq, f, 2, s2);
    }
    if (vi && ks == 0) {  // the predict's two rank-1 factors (slam.cpp:198)
      kc[0 * ldk + i] = static_cast<T>(first ? -ai : 0.0);
      kc[1 * ldk + i] = static_cast<T>(first ? -(r0raw + ai * s00) : 0.0);
      // rows of U take the chain's x (first position of the row in U)
      int pos = kMaxU;
#pragma unroll
      for (int k = kMaxU - 1; k >= 0; --k) pos = (k < nu && sh.u[k] == i) ? k : pos;
      xout[i] = pos < nu ? xfin[pos] : xin[i] + acc2[0];
      if (kDiagBuild && (A.dbg & 16)) {
        dlog_add(A, 4, A.seq, f, 3, dbits(xin[i]));
        dlog_add(A, 4, A.seq, f, 4, dbits(pos < nu ? xfin[pos] : xin[i] + acc2[0]));
      }
    }
    if (vi) {
#pragma unroll
      for (int g = 0; g < NG; ++g)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = 16 * g + ks + 4 * r;
          // Joseph: Z columns 0 .. 2m − 1 (the first two groups) are K, which is also the column
          // factor of the (ΣHᵀ − K·S)·Kᵀ term (Mcat rows 2 + 2m + c); columns 32 + c are V, Kcat
          // rows 2 + 2m + c — the rank-(2 + 4m) factors packed, zero columns not stored
          if (!joseph) {
            if (g < 2) kc[(2 + c) * ldk + i] = static_cast<T>(acc[g][r]);
          } else if (g < 2) {
            if (c < jk0) {
              kc[(2 + c) * ldk + i] = static_cast<T>(acc[g][r]);
              mc[(2 + jk0 + c) * ldk + i] = static_cast<T>(acc[g][r]);
            }
          } else if (c - kZC < jk0 + 2) {  // (+ the two zero rows up to kw = 4m + 4: the
            // pass reads them, and a longer chunk before may have left V rows there)
            kc[(2 + jk0 + c - kZC) * ldk + i] = static_cast<T>(acc[g][r]);
          }
        }
    }
    if (merged) columns(i, raw, r0t);
  } else if (!merged && wg < 2 * row_tiles) {
    const int C0 = (wg - row_tiles) * 16;
    const int j = C0 + l16;
    const bool vj = j < n;
    const int jj = vj ? j : 0;
    T raw[9];
    const T c0t = S[jj];
#pragma unroll
    for (int s = 0; s < 9; ++s)
      raw[s] = S[static_cast<size_t>(sh.u[min(4 * s + ks, kMaxU - 1)]) * ld + jj];
    columns(j, raw, c0t);
  }
}

// 16 rows or 16 columns per wave (fp64: both), per_filter workgroups of 4 waves per filter
template <typename T>
__host__ __device__ inline int factor_waves(const PassArgs<T>& a) {
  return (sizeof(T) == 8 ? 1 : 2) * ((a.n + 15) / 16);
}

// One workgroup per filter, persistent over the `nchunks` chunks of a launch (descriptors
// A.desc[i·desc_stride + filter]): per chunk the m sequential corrections on the |U|×|U| block.
// Every chunk of a launch after the first rebuilds its block from the chunk before (kLook): the
// previous Σ_in (complete) and the record, the factor kernel's formulas at U. (Carrying the
// chain's own final block into the next chunk instead was 6 % faster but let the chain's block and
// the HBM Σ drift apart — two roundings of the 1e7-prior first sightings — until a survey replay
// went non-finite; the rebuild keeps every schedule bit-identical)
// dev only (PassArgs::dbg & 8): kernel `k` (0 chain, 1 factors, 2 Σ pass) of filter f runs with
// launch epoch e; the launches of a kind are stream-ordered, so e must exceed the last one seen
// (a kernel that runs with an older launch's arguments counts at sync[kSyncDbg + 3 + k])
template <typename T>
__device__ void dbg_seq_check(const PassArgs<T>& A, int k, int f, unsigned e) {
  unsigned* last = A.sync + kSyncChain + (1 + k) * A.rec_stride + f;
  if (static_cast<int>(e - *last) <= 0) atomicAdd(A.sync + kSyncDbg + 3 + k, 1u);
  *last = e;
}

template <typename T, bool J>
__global__ __launch_bounds__(kChainThreads) void k_chain(PassArgs<T> A, int nchunks) {
  __shared__ ChainSharedT<J> sh;
  constexpr int ZC = ChainSharedT<J>::ZC, JM = ChainSharedT<J>::JM;
  // The descriptor is read every step: keep it in LDS. Two buffers: a chunk's epilogue prefetches
  // the next one's (and computes its predicted pose from it).
  __shared__ MsgDesc sdesc[2];
  static_assert(sizeof(MsgDesc) % 16 == 0, "MsgDesc copied as uint4");
  const int fy = blockIdx.y;
  const int f = A.f0 + fy;
  const int tid = threadIdx.x;
  const int ld = A.ld;
  FilterCtl* ctl = A.ctl + f;
  // LDS starts as whatever the CU's previous kernel left (possibly NaN bit patterns): zero it once,
  // so padding rows / columns that feed MFMA or dot products as zeros really are zeros
  for (int e = tid; e < static_cast<int>(sizeof(sh) / 8); e += blockDim.x)
    reinterpret_cast<double*>(&sh)[e] = 0.0;
  // Every wave's zeroing stores must land before the one below: the word npose_ci lives in is
  // zeroed by a thread of another wave, and without the barrier that store could come after this
  // one (npose_ci = 0 made chunk 0 copy a never-computed predicted pose, (0, 0, 0)). The race
  // showed where the chain's waves run at different paces — on CUs shared with the bulk stream's
  // kernels (two streams without CU masks: > 32 filters with EKF_SERIAL=0), DESIGN.md §5.
  __syncthreads();
  if (tid == 0) sh.npose_ci = -1;  // (ordered before its first reader by the chunk loop's barriers)
  if (kDiagBuild && (A.dbg & 1)) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  bool pre = false;        // sdesc[ci & 1] was prefetched by the previous chunk's epilogue
  unsigned pending = 0;    // chain epoch of the previous chunk, not yet published (its record
                           // stores are still in flight; see the epilogue)
  for (int ci = 0; ci < nchunks; ++ci) {
  if (!pre) {
    const MsgDesc& gd = A.desc[static_cast<size_t>(ci) * A.desc_stride + fy];
    // planned on the bulk stream beside this launch: the planner's count covers every descriptor
    if (ci == 0 && A.need_plan && tid == 0 && !epoch_wait_acquire(A.sync + kSyncPlan, A.need_plan))
      flag_timeout(&ctl->status, A.fatal);
    __syncthreads();
    if (threadIdx.x < sizeof(MsgDesc) / 16)
      reinterpret_cast<uint4*>(&sdesc[ci & 1])[threadIdx.x] =
          reinterpret_cast<const uint4*>(&gd)[threadIdx.x];
    __syncthreads();
  }
  pre = false;
  const MsgDesc& d = sdesc[ci & 1];
  auto& P = sh.P[0];
  const bool active = (d.flags & kActive) != 0;
  const bool look = (d.flags & kLook) != 0 && !A.gather;
  // Publish the previous chunk's record before this chunk waits on anything the bulk stream
  // produces (its factor kernel needs that record).
  if (pending) {
    drain_stores();
    __syncthreads();
    if (tid == 0) epoch_store(A.sync + kSyncChain + f, pending);
    pending = 0;
  }
  if (!active) continue;  // this filter sits the chunk out
  const unsigned seq = A.seq + static_cast<unsigned>(ci);
  if ((kDiagBuild && (A.dbg & 8)) && tid == 0) dbg_seq_check(A, 0, f, seq + 1u);
  // Σ_in / x / records a rebuilding chain reads come from the Σ pass two launches back (bulk
  // stream), and this record parity is free again once that pass is done (its factor kernel read
  // it); a chunk that gathers its own Σ_in needs the pass one back.
  const unsigned need = look ? (seq >= 2 ? seq - 1 : 0u) : seq;
  if ((kDiagBuild && (A.dbg & 4)) && need && tid == 0) {
    if (static_cast<int>(epoch_load(A.sync + kSyncSigma) - need) < 0) atomicAdd(A.sync + kSyncDbg, 1u);
    atomicAdd(A.sync + kSyncDbg + 2, 1u);
  }
  // A0's associated ids (k_assoc, earlier on this stream), loaded unconditionally (clamped) and
  // here, so that the barrier below completes them: under A0's branch the load was waited for,
  // vmcnt(0), together with every early load below
  const int cA = tid >= 3 && tid < 3 + 2 * d.m ? (tid - 3) >> 1 : 0;
  const int aj = ctl->assoc_j[min(max(d.assoc_slot + cA, 0), kMaxAssoc - 1)];
  // first_ready: the host joined the bulk stream before this launch, so every pass before it is
  // complete (epochs ≤ A.seq), published or not — the launch's second chunk needs the pass just
  // before the launch, whose epoch the flush that issued it did not publish (waiting for a later
  // epoch instead held that chunk until this launch's first pass: ≈ 27 µs)
  if (A.polls && need && tid == 0 && !(A.first_ready && need <= A.seq) &&
      !epoch_wait_acquire(A.sync + kSyncSigma, need))
    flag_timeout(&ctl->status, A.fatal);
  EKF_STAMP(305);
  // (Z, Φ are set up by wave 1 and Y, Ψ by wave 2 at the start of their step loops)
  if (tid == 0) sh.status = 0;
  __syncthreads();
  EKF_STAMP(0);
  const T* S = A.sig[d.parity] + f * A.sig_stride;
  const double* xin = A.x[d.parity] + f * A.x_stride;
  const int m = d.m;
  const bool first = (d.flags & kFirst) != 0;
  // Joseph (≤ kMaxJoseph markers per chunk): Σ ← Σ − K_c·M_c − (Σ_cHᵀ − K_c·S_c)·K_cᵀ per step,
  // i.e. (I−KH)Σ(I−KH)ᵀ + K·R·Kᵀ expanded (slam.cpp:264-265's update in Joseph form). Row factor
  // V_c = G_c − K_c·S_c beside K_c, column factor K_cᵀ beside M_c: the record's Z carries V_c's
  // row map in columns 32 + 2c.. (kZC + 2c), the chain's block gets the term step by step.
  const bool joseph = J && (d.flags & kJoseph) != 0;
  if ((kDiagBuild && (A.dbg & 16)) && tid < static_cast<int>(sizeof(MsgDesc) / 8))
    dlog_add(A, 0, seq, f, 0, reinterpret_cast<const unsigned long long*>(&d)[tid]);

  // kLook: this chunk's Σ_in is still being written by the previous chunk's Σ pass. Rebuild what
  // the chain needs from the chunk before: Σ_in' (the other buffer, complete) and its record.
  const ChunkRec* rp = A.rec + static_cast<size_t>(d.parity ^ 1) * A.rec_stride + f;

  constexpr int kW = kMaxU + 1;  // block entries are indexed e = a·36 + b (constant divisor)
  constexpr int kPer = (kW * kW + kChainThreads - 1) / kChainThreads;  // 6
  // the previous record's Z (|U| rows of ZC, the record's rows kZJ wide) and Y (kZC rows)
  constexpr int kPerZ = (kMaxU * ZC + kChainThreads - 1) / kChainThreads;  // 5 (Joseph: 9)
  // kLook with staged operands: the loads do not depend on A0's index sets, so they are issued
  // here and land during A0 (whose barrier orders LDS only)
  const bool early = look && (d.flags & kStageIn);
  double vz[kPerZ], vy[kPer];
  T vd[kPer], vr[kPer], vc[kPer];  // (as stored: half the registers at fp32 while A0 runs)
  double r0u = 0.0, c0u = 0.0, r0p = 0.0, c0p = 0.0, x2 = 0.0;
  double x0 = 0.0, x1 = 0.0, pa1 = 0.0, pa2 = 0.0, tq = 0.0;
  int pflags = 0;
  {
    // staged by the k_patch_stage two chunks back, right behind the Σ pass that wrote Σ_in':
    // the same values as the gather below, contiguous (≈ 5 000 cycles less than the ≈ 1 900
    // scattered lines of the gather through one CU). Issued unconditionally, through buffer
    // descriptors of size 0 unless `early` (zeros, no access): a load under a branch is waited for
    // at the branch's join on the path that skipped it — vmcnt(0) before A0's first use of `aj`
    const int tc = tid < kMaxU ? tid : 0;
    const StageRec<T>* sg = A.stage + static_cast<size_t>(d.parity) * A.rec_stride + f;
    const auto rs = buf_rsrc(sg, early ? static_cast<unsigned>(sizeof(StageRec<T>)) : 0u);
    const auto rr = buf_rsrc(rp, early ? static_cast<unsigned>(sizeof(ChunkRec)) : 0u);
    constexpr unsigned oZ = offsetof(ChunkRec, Z), oY = offsetof(ChunkRec, Y);
    constexpr unsigned oV = offsetof(StageRec<T>, v), oT = kW * kW * sizeof(T);
#pragma unroll
    for (int i = 0; i < kPerZ; ++i) {
      const int e = tid + i * kChainThreads, ez = e < kMaxU * ZC ? e : 0;
      vz[i] = ld_f64(rr, oZ + 8u * ((ez / ZC) * kZJ + ez % ZC), 0);
    }
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int e = tid + i * kChainThreads, es = min(e, kW * kW - 1);
      vy[i] = ld_f64(rr, oY + 8u * (e < kZC * kMaxU ? e : 0), 0);
      vd[i] = ld_t(rs, oV + sizeof(T) * es, T{});
      vr[i] = ld_t(rs, oV + oT + sizeof(T) * es, T{});
      vc[i] = ld_t(rs, oV + 2 * oT + sizeof(T) * es, T{});
    }
    r0u = ld_f64(rs, offsetof(StageRec<T>, r0u) + 8u * tc, 0);
    c0u = ld_f64(rs, offsetof(StageRec<T>, c0u) + 8u * tc, 0);
    r0p = ld_f64(rs, offsetof(StageRec<T>, r0p) + 8u * tc, 0);
    c0p = ld_f64(rs, offsetof(StageRec<T>, c0p) + 8u * tc, 0);
    x2 = ld_f64(rs, offsetof(StageRec<T>, xg) + 8u * tc, 0);
    x0 = ld_f64(rr, offsetof(ChunkRec, xU) + 8u * tc, 0);
    x1 = ld_f64(rr, offsetof(ChunkRec, Zx) + 8u * tc, 0);
    pflags = static_cast<int>(__builtin_amdgcn_raw_buffer_load_b32(rr, offsetof(ChunkRec, flags), 0, 0));
    pa1 = ld_f64(rr, offsetof(ChunkRec, a1), 0);
    pa2 = ld_f64(rr, offsetof(ChunkRec, a2), 0);
    tq = ctl->tmo[tid < 3 ? tid : 0];
  }

  EKF_STAMP(14);
  // ---- A0: index sets U (this chunk) and U' (kLook: the previous chunk, from the descriptor) ----
  if (tid < kMaxU) {  // u[3+2c], u[4+2c] = the columns of marker c's landmark (bad id → slot 0's)
    int u = tid < 3 ? tid : 0;  // padding 0: loads stay in bounds
    if (tid >= 3 && tid < 3 + 2 * m) {
      const int c = (tid - 3) >> 1, idd = d.ids[c];
      const int id = idd >= 0 ? idd : aj;
      const bool bad = id < 0 || id >= A.N;
      u = (bad ? 3 : 3 + 2 * id) + ((tid - 3) & 1);
      if (((tid - 3) & 1) == 0) {
        sh.skip[c] = bad ? 1 : 0;
        if (bad && idd >= 0) atomicOr(&sh.status, EKF_FLAG_RANGE_D);  // association: flagged already
      }
    }
    sh.u[tid] = u;
  }
  if (tid == 0) sh.nu_cnt = 3 + 2 * m;
  if (look && tid < kMaxU) {  // the previous chain's mapping of its ids (bad → slot 0)
    const int pm = d.prev_m;
    int u = 0;
    if (tid < 3) {
      u = tid;
    } else if (tid < 3 + 2 * pm) {
      const int c = (tid - 3) >> 1, id = d.prev_ids[c];
      u = (id < 0 || id >= A.N ? 3 : 3 + 2 * id) + ((tid - 3) & 1);
    }
    sh.pv.u[tid] = u;
    if (tid == 0) {
      sh.pv.nu = 3 + 2 * pm;
      sh.pv.m = pm;
    }
  }
  lds_barrier();
  EKF_STAMP(1);
  const int nu = sh.nu_cnt;

  // ---- A1: every global load of the prologue in one round ---------------------------------------
  // Each thread issues all of its loads before its first LDS store: indices are clamped rather
  // than predicated (a predicated load becomes a branch with its own wait), so the loads of a
  // thread are in flight together instead of one memory round trip per loop iteration.
  const int wv = tid >> 6, ln = tid & 63, i16 = ln & 15, k4 = ln >> 4;
  if (look) {
    // Σ_in[U,U] = Σ_pred'[U,U] − K'·M' with Σ_pred' = A'·Σ_in'·A'ᵀ + Q̄' (the previous chunk's
    // predict, if it had one), K'[a] = Σ_pred'[u_a, U']·Z', M'[:, b] = Y'·Σ_pred'[U', u_b]: the
    // factor kernel's formulas evaluated at U only.
    const T* Sp = A.sig[d.parity ^ 1] + f * A.sig_stride;
    const double* xp = A.x[d.parity ^ 1] + f * A.x_stride;
    const int np = sh.pv.nu;
    const int tc = tid < kMaxU ? tid : 0;
    if (!early) {  // (early: the staged operands and the record's values are in registers)
#pragma unroll
      for (int i = 0; i < kPerZ; ++i) {
        const int e = tid + i * kChainThreads, ez = e < kMaxU * ZC ? e : 0;
        vz[i] = rp->Z[ez / ZC][ez % ZC];
      }
#pragma unroll
      for (int i = 0; i < kPer; ++i) {
        const int e = tid + i * kChainThreads;
        vy[i] = (&rp->Y[0][0])[e < kZC * kMaxU ? e : 0];
        const int a = min(e / kW, kMaxU - 1), b = min(e % kW, kMaxU - 1);  // clamped: in bounds
        const size_t ua = static_cast<size_t>(sh.u[a]) * ld, pa = static_cast<size_t>(sh.pv.u[b]);
        vd[i] = Sp[ua + sh.u[b]];
        vr[i] = Sp[ua + pa];
        vc[i] = Sp[pa * ld + sh.u[a]];
      }
      // raw row 0 / column 0 of Σ_in' at U and U' (for the previous predict), x'
      const int uu = sh.u[tc], pu = sh.pv.u[tc];
      r0u = static_cast<double>(Sp[uu]);
      c0u = static_cast<double>(Sp[static_cast<size_t>(uu) * ld]);
      r0p = static_cast<double>(Sp[pu]);
      c0p = static_cast<double>(Sp[static_cast<size_t>(pu) * ld]);
      x2 = xp[uu];
      // record scalars
      x0 = rp->xU[tc];
      x1 = rp->Zx[tc];
      pflags = rp->flags;
      pa1 = rp->a1;
      pa2 = rp->a2;
      tq = ctl->tmo[tid < 3 ? tid : 0];
    }
    if (kDiagBuild && (A.dbg & 16)) {
      unsigned long long s2 = 0, s4 = 0;
#pragma unroll
      for (int i = 0; i < kPer; ++i) {
        s2 += dbits(vd[i]) + dbits(vr[i]) + dbits(vc[i]);
        s4 += dbits(vy[i]);
      }
#pragma unroll
      for (int i = 0; i < kPerZ; ++i) s4 += dbits(vz[i]);
      if (tid < kMaxU) {
        s2 += dbits(r0u) + dbits(c0u) + dbits(r0p) + dbits(c0p);
        s4 += dbits(x0) + dbits(x1);
        dlog_add(A, 0, seq, f, 3, dbits(x2));
      }
      if (tid == 0) s4 += static_cast<unsigned>(pflags) + dbits(pa1) + dbits(pa2);
      if (tid < 3) dlog_add(A, 0, seq, f, 1, dbits(tq));
      dlog_add(A, 0, seq, f, 2, s2);
      dlog_add(A, 0, seq, f, 4, s4);
    }
#pragma unroll
    for (int i = 0; i < kPerZ; ++i) {
      const int e = tid + i * kChainThreads;
      if (e < kMaxU * ZC) (&sh.pv.Z[0][0])[(e / ZC) * (ZC + 1) + e % ZC] = vz[i];
    }
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int e = tid + i * kChainThreads;
      if (e < kZC * kMaxU) (&sh.pv.Y[0][0])[(e / kMaxU) * (kMaxU + 1) + e % kMaxU] = vy[i];
    }
    if (tid < ZC) sh.pv.Z[kMaxU][tid] = 0.0;  // the 36th k row / column
    if (tid < kZC) sh.pv.Y[tid][kMaxU] = 0.0;
    if (tid < kMaxU) {
      sh.pv.r0U[tid] = r0u;
      sh.pv.c0U[tid] = c0u;
      sh.pv.r0P[tid] = r0p;
      sh.pv.c0P[tid] = c0p;
      sh.pv.xU[tid] = x0;
      sh.pv.Zx[tid] = x1;
      sh.pv.xg[tid] = x2;
    }
    if (tid == 0) {
      sh.pv.first = (pflags & kFirst) != 0;
      sh.pv.joseph = (pflags & kJoseph) != 0;
      sh.pv.a1 = pa1;
      sh.pv.a2 = pa2;
    }
    if (tid < 3) sh.tmo[tid] = tq;
    __syncthreads();
    EKF_STAMP(21);
    rebuild_rcd<T>(sh, P, vd, vr, vc, tid, nu, np, A.q);
    __syncthreads();
    EKF_STAMP(3);
    EKF_STAMP(4);
    // K' = R·Z' (35 × 32) and M' = Y'·C (32 × 35) on f64 MFMA. Their 32 × 32 cores are 8 tiles,
    // two per wave; the 3-wide bands K'[32..34][·] and M'[·][32..34] (16 × 16 tiles there would be
    // 13/16 padding) are VALU dot products, one output per thread of waves 0–2, and wave 3 forms
    // x_in[U] instead. Operand reads are unconditional (clamped rows / columns feed only discarded
    // outputs, k ≥ |U'| is zero-padded in both operands, so every k-step runs: its MFMA adds exact
    // zeros). A wave's tiles and its VALU work are one basic block (operand reads first, then two
    // interleaved accumulation chains beside the dot product): the MFMA and VALU pipes overlap.
    if constexpr (!J) {
    auto kmphase = [&](auto w3c) {
      constexpr bool W3 = decltype(w3c)::value;
      double av[2][9], bv[2][9];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int tt = wv + 4 * q;  // 0..3 K' tiles, 4..7 M' tiles
        const bool kt = tt < 4;
        const int ti = (kt ? tt : tt - 4) >> 1, tj = (kt ? tt : tt - 4) & 1;
        // A: R[row][k] (K') or Y'[row][k] (M'), k contiguous; B: Z'[k][col] (stride kZC + 1) or
        // C[k][col] (stride kMaxU + 1)
        const double* pa = kt ? &sh.pv.R[16 * ti + i16][0] : &sh.pv.Y[16 * ti + i16][0];
        const double* pb = kt ? &sh.pv.Z[0][16 * tj + i16] : &sh.pv.C[0][16 * tj + i16];
        const int sb = kt ? kZC + 1 : kMaxU + 1;
#pragma unroll
        for (int s0 = 0; s0 < 9; ++s0) {
          av[q][s0] = pa[4 * s0 + k4];
          bv[q][s0] = pb[(4 * s0 + k4) * sb];
        }
      }
      // the VALU share: a band output (waves 0–2) or x_in[U] (wave 3)
      double bacc[4] = {0.0, 0.0, 0.0, 0.0};
      int brow = 0, bcol = 0;
      bool bk = false;
      double xres = 0.0;
      if (!W3) {
        if (tid < 96) {  // K'[32 + t/32][t%32] = R[row]·Z'[:, col]
          bk = true;
          brow = 32 + (tid >> 5);
          bcol = tid & 31;
        } else {  // M'[u/3][32 + u%3] = Y'[row]·C[:, col]
          const int u = tid - 96;
          brow = u / 3;
          bcol = 32 + (u - 3 * (u / 3));
        }
        const double* ra = bk ? &sh.pv.R[min(brow, kMaxU - 1)][0] : &sh.pv.Y[brow][0];
        const double* cb = bk ? &sh.pv.Z[0][bcol] : &sh.pv.C[0][min(bcol, kMaxU)];
        const int sc = bk ? kZC + 1 : kMaxU + 1;
#pragma unroll
        for (int k = 0; k < kMaxU + 1; ++k) bacc[k & 3] = fma(ra[k], cb[k * sc], bacc[k & 3]);
      } else {
        // x_in[U]: the previous chunk's x[U'] where it has it, else x' + r'(i)·Zx'
        const int l = ln < kMaxU ? ln : kMaxU - 1;
        const int u = sh.u[l];
        int pos = -1;
#pragma unroll
        for (int k = kMaxU - 1; k >= 0; --k) pos = (k < np && sh.pv.u[k] == u) ? k : pos;
#pragma unroll
        for (int k = 0; k < kMaxU; ++k) bacc[k & 3] = fma(sh.pv.R[l][k], sh.pv.Zx[k], bacc[k & 3]);
        const double r = (bacc[0] + bacc[1]) + (bacc[2] + bacc[3]);  // R[·][k ≥ |U'|] = 0
        xres = pos >= 0 ? sh.pv.xU[pos] : sh.pv.xg[l] + r;
      }
      d4 acc[2] = {{0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}};
#pragma unroll
      for (int s0 = 0; s0 < 9; ++s0)
#pragma unroll
        for (int q = 0; q < 2; ++q) acc[q] = mfma_f64(av[q][s0], bv[q][s0], acc[q]);
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int tt = wv + 4 * q;
        const bool kt = tt < 4;
        const int ti = (kt ? tt : tt - 4) >> 1, tj = (kt ? tt : tt - 4) & 1;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const double v = acc[q][r];
          if (kt) sh.pv.K[16 * ti + k4 + 4 * r][16 * tj + i16] = v;
          else sh.pv.M[16 * ti + k4 + 4 * r][16 * tj + i16] = v;
        }
      }
      if (!W3) {
        const double v = (bacc[0] + bacc[1]) + (bacc[2] + bacc[3]);
        if (bk) sh.pv.K[brow][bcol] = v;
        else if (bcol < kMaxU) sh.pv.M[brow][bcol] = v;
      } else {
        if (ln < nu) sh.xU[0][ln] = xres;
        if (ln < 3) sh.xpose[ln] = sh.pv.xU[ln];  // pose ∈ U' always
      }
    };
    if (wv == 3)
      kmphase(std::true_type{});
    else
      kmphase(std::false_type{});
    EKF_STAMP(7);
    __syncthreads();
    EKF_STAMP(5);
    // P = D − K'·M' on the 48×48 padded block: 9 tiles over the 4 waves (K' columns and M' rows
    // ≥ 2m' are zero because Z' / Y' are; a Joseph chunk's are ≥ 4m')
    // (every k-step runs: K' columns and M' rows beyond the chunk's rank are zero, so their MFMAs
    // add exact zeros.) The 32 × 32 core of P on MFMA, one 16 × 16 tile per wave; the 3-wide bands
    // (rows 32..34 and columns 32..34, 201 entries) as VALU dot products, one per thread, in the same
    // basic block.
    {
      const int ti = wv >> 1, tj = wv & 1;
      const int col = 16 * tj + i16, ar = 16 * ti + i16;
      double av[8], bv[8];
#pragma unroll
      for (int s0 = 0; s0 < 8; ++s0) {
        av[s0] = -sh.pv.K[ar][4 * s0 + k4];
        bv[s0] = sh.pv.M[4 * s0 + k4][col];
      }
      d4 acc;
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[r] = P[16 * ti + k4 + 4 * r][col];
      // band entry: t < 105 → rows 32..34 × columns 0..34, then rows 0..31 × columns 32..34
      const int t = tid < 201 ? tid : 200;
      const int brow = t < 105 ? 32 + t / 35 : (t - 105) / 3;
      const int bcol = t < 105 ? t - 35 * (t / 35) : 32 + (t - 105) - 3 * ((t - 105) / 3);
      const int br = min(brow, kMaxU - 1), bc = min(bcol, kMaxU - 1);
      double bs[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int k = 0; k < kZC; ++k) bs[k & 3] = fma(sh.pv.K[br][k], sh.pv.M[k][bc], bs[k & 3]);
      const double bv0 = P[br][bc];
#pragma unroll
      for (int s0 = 0; s0 < 8; ++s0) acc = mfma_f64(av[s0], bv[s0], acc);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * ti + k4 + 4 * r;
        if (row < nu && col < nu) P[row][col] = acc[r];
      }
      if (tid < 201 && brow < nu && bcol < nu) P[brow][bcol] = bv0 - ((bs[0] + bs[1]) + (bs[2] + bs[3]));
    }
    } else {
    // Joseph form (ZC = 64): K' = R·Z' is 35 × 4m' (K' then V' columns), M' = Y'·C is 2m' × 35.
    // Their 16 × 16 cores are 12 tiles, three per wave (one after another, each operand read waited
    // for once); the bands K'[32..34][·] (192 outputs) and M'[·][32..34] (96) are VALU dot products
    // of waves 0–2 (two per thread for the first 96), wave 3 forms x_in[U] as in the simple form.
    auto kmphase = [&](auto w3c) {
      constexpr bool W3 = decltype(w3c)::value;
#pragma unroll 1
      for (int q = 0; q < 3; ++q) {
        const int tt = wv + 4 * q;  // 0..7 K' tiles (2 × 4), 8..11 M' tiles (2 × 2)
        const bool kt = tt < 8;
        const int ti = kt ? tt >> 2 : (tt - 8) >> 1, tj = kt ? tt & 3 : (tt - 8) & 1;
        const double* pa = kt ? &sh.pv.R[16 * ti + i16][0] : &sh.pv.Y[16 * ti + i16][0];
        const double* pb = kt ? &sh.pv.Z[0][16 * tj + i16] : &sh.pv.C[0][16 * tj + i16];
        const int sb = kt ? ZC + 1 : kMaxU + 1;
        double av[9], bv[9];
#pragma unroll
        for (int s0 = 0; s0 < 9; ++s0) {
          av[s0] = pa[4 * s0 + k4];
          bv[s0] = pb[(4 * s0 + k4) * sb];
        }
        d4 acc = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int s0 = 0; s0 < 9; ++s0) acc = mfma_f64(av[s0], bv[s0], acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (kt) sh.pv.K[16 * ti + k4 + 4 * r][16 * tj + i16] = acc[r];
          else sh.pv.M[16 * ti + k4 + 4 * r][16 * tj + i16] = acc[r];
        }
      }
      if (!W3) {
#pragma unroll 1
        for (int t = tid; t < 288; t += 192) {
          const bool bk = t < 192;  // K'[32 + t/64][t%64] = R[row]·Z'[:, col], else M'[u/3][32 + u%3]
          const int u = t - 192;
          const int brow = bk ? 32 + (t >> 6) : u / 3, bcol = bk ? (t & 63) : 32 + u % 3;
          const double* ra = bk ? &sh.pv.R[min(brow, kMaxU - 1)][0] : &sh.pv.Y[brow][0];
          const double* cb = bk ? &sh.pv.Z[0][bcol] : &sh.pv.C[0][min(bcol, kMaxU)];
          const int sc = bk ? ZC + 1 : kMaxU + 1;
          double bacc[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int k = 0; k < kMaxU + 1; ++k) bacc[k & 3] = fma(ra[k], cb[k * sc], bacc[k & 3]);
          const double v = (bacc[0] + bacc[1]) + (bacc[2] + bacc[3]);
          if (bk) sh.pv.K[brow][bcol] = v;
          else if (bcol < kMaxU) sh.pv.M[brow][bcol] = v;
        }
      } else {
        // x_in[U]: the previous chunk's x[U'] where it has it, else x' + r'(i)·Zx'
        const int l = ln < kMaxU ? ln : kMaxU - 1;
        const int u = sh.u[l];
        int pos = -1;
#pragma unroll
        for (int k = kMaxU - 1; k >= 0; --k) pos = (k < np && sh.pv.u[k] == u) ? k : pos;
        double bacc[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int k = 0; k < kMaxU; ++k) bacc[k & 3] = fma(sh.pv.R[l][k], sh.pv.Zx[k], bacc[k & 3]);
        const double r = (bacc[0] + bacc[1]) + (bacc[2] + bacc[3]);  // R[·][k ≥ |U'|] = 0
        const double xres = pos >= 0 ? sh.pv.xU[pos] : sh.pv.xg[l] + r;
        if (ln < nu) sh.xU[0][ln] = xres;
        if (ln < 3) sh.xpose[ln] = sh.pv.xU[ln];  // pose ∈ U' always
      }
    };
    if (wv == 3)
      kmphase(std::true_type{});
    else
      kmphase(std::false_type{});
    EKF_STAMP(7);
    __syncthreads();
    EKF_STAMP(5);
    // P = D − K'·M'full with M'full = [M' (rows 0..31); K'[:, 0..32)ᵀ (rows 32..63: a Joseph chunk
    // before, its V'·K'ᵀ terms, V' = K' columns 32..63)] — zero beyond each part's rank 2m', and
    // the K'ᵀ part zero after a simple-form chunk (its record's columns ≥ 32 are not V'). The
    // 48 × 48 padded block as 9 tiles on f64 MFMA, k < 64 in 16 k-steps: waves 0–2 one row tile
    // each (its K' rows read once) × the three column tiles, interleaved. Rows / columns ≥ kMaxU
    // are clamped on read and never stored; a wave reads and writes only its own rows.
    if (wv < 3) {
      const bool pj = sh.pv.joseph != 0;
      const int ar = min(16 * wv + i16, kMaxU - 1);
      double av[16];
#pragma unroll
      for (int s0 = 0; s0 < 16; ++s0) av[s0] = -sh.pv.K[ar][4 * s0 + k4];
      d4 acc[3];
#pragma unroll
      for (int tj = 0; tj < 3; ++tj) {
        const int bc = min(16 * tj + i16, kMaxU - 1);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[tj][r] = P[min(16 * wv + k4 + 4 * r, kMaxU - 1)][bc];
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {  // k < 32 (M' rows), then k ≥ 32 (K'ᵀ)
        double bv[3][8];
#pragma unroll
        for (int tj = 0; tj < 3; ++tj) {
          const int bc = min(16 * tj + i16, kMaxU - 1);
#pragma unroll
          for (int s0 = 0; s0 < 8; ++s0)
            bv[tj][s0] = h == 0 ? sh.pv.M[4 * s0 + k4][bc] : (pj ? sh.pv.K[bc][4 * s0 + k4] : 0.0);
        }
#pragma unroll
        for (int s0 = 0; s0 < 8; ++s0)
#pragma unroll
          for (int tj = 0; tj < 3; ++tj) acc[tj] = mfma_f64(av[8 * h + s0], bv[tj][s0], acc[tj]);
      }
#pragma unroll
      for (int tj = 0; tj < 3; ++tj) {
        const int col = 16 * tj + i16;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = 16 * wv + k4 + 4 * r;
          if (row < nu && col < nu) P[row][col] = acc[tj][r];
        }
      }
    }
    }
    EKF_STAMPT(10, 64);
    EKF_STAMPT(11, 128);
    EKF_STAMPT(13, 192);
    // wave 2: the predicted pose
    if (wv == 2 && ln == 0) {  // the predicted pose (slam.cpp:184-196) from x' of the pose
      if (sh.npose_ci == ci) {  // computed ahead by the chunk before (wave 3)
        sh.pose[0] = sh.npose[0];
        sh.pose[1] = sh.npose[1];
        sh.pose[2] = sh.npose[2];
        sh.a1 = sh.na1;
        sh.a2 = sh.na2;
      } else {
        double a1, a2;
        const double xp[3] = {sh.pv.xU[0], sh.pv.xU[1], sh.pv.xU[2]};
        predicted_pose(sh.tmo, d, xp, sh.pose, &a1, &a2);
        sh.a1 = a1;
        sh.a2 = a2;
      }
      EKF_STAMPT(8, 128);
    }
    EKF_STAMPT(9, 192);  // (x_in[U]: wave 3 in the K' / M' phase)
  } else {
    double vd[kPer];
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int e = tid + i * kChainThreads;
      const int a = min(e / kW, kMaxU - 1), b = min(e % kW, kMaxU - 1);
      vd[i] = static_cast<double>(S[static_cast<size_t>(sh.u[a]) * ld + sh.u[b]]);
    }
    const double xv = xin[sh.u[tid < nu ? tid : 0]];
    const double xq = xin[tid < 3 ? tid : 0];
    const double tq = ctl->tmo[tid < 3 ? tid : 0];
    if (kDiagBuild && (A.dbg & 16)) {
      unsigned long long s2 = 0;
#pragma unroll
      for (int i = 0; i < kPer; ++i) s2 += dbits(vd[i]);
      dlog_add(A, 0, seq, f, 2, s2);
      dlog_add(A, 0, seq, f, 3, dbits(xv) + dbits(xq));
      if (tid < 3) dlog_add(A, 0, seq, f, 1, dbits(tq));
    }
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int e = tid + i * kChainThreads;
      const int a = e / kW, b = e % kW;
      if (a < nu && b < nu) P[a][b] = vd[i];
    }
    if (tid < nu) sh.xU[0][tid] = xv;
    if (tid < 3) {
      sh.xpose[tid] = xq;
      sh.tmo[tid] = tq;
    }
    __syncthreads();
    if (tid == 192) {
      double a1, a2;
      predicted_pose(sh.tmo, d, sh.xpose, sh.pose, &a1, &a2);
      sh.a1 = a1;
      sh.a2 = a2;
    }
  }
  EKF_STAMP(6);
  // ---- A3: x[U] pose, α, this chunk's predict folded in: P ← A P Aᵀ + Q̄ (slam.cpp:198) --------
  __syncthreads();
  {
    // α, row 0, column 0 to LDS for the record; the predict (slam.cpp:198) changes only the
    // special entries (rows / columns 1, 2 and the pose diagonal, special_entry): one per thread,
    // its raw value, row 0 and column 0 read before any is written
    const double a1 = sh.a1, a2 = sh.a2, s00 = P[0][0];
    if (tid < nu) {
      if (tid < 3) sh.xU[0][tid] = sh.pose[tid];
      sh.alphaU[tid] = first ? alpha_of(sh.u[tid], a1, a2) : 0.0;
      sh.row0raw[tid] = P[0][tid];
      sh.col0raw[tid] = P[tid][0];
    }
    if (tid == 0) sh.s00 = s00;
    if (first) {
      int a, b;
      special_entry(min(tid, kSpec - 1), a, b);
      const bool ok = tid < kSpec && a < nu && b < nu;
      a = min(a, kMaxU - 1);
      b = min(b, kMaxU - 1);
      const double pr = P[a][b], r0 = P[0][b], c0 = P[a][0];
      lds_barrier();  // every raw read done before the first write
      const double ai = alpha_of(a, a1, a2), aj = alpha_of(b, a1, a2);
      double v = pr + ai * r0;
      v = v + (c0 + ai * s00) * aj;
      v = (a == b && a < 3) ? v + A.q : v;
      if (ok) P[a][b] = v;
    }
  }
  __syncthreads();
  EKF_STAMP(2);
  EKF_DUMP_BLOCK(seq);
  EKF_STAMP(18);

  // ---- A2: the m corrections -----------------------------------------------------------------
  // The dependent chain (ẑ, H, S⁻¹, ν → K, M, x → next marker) runs on wave 0 alone, with no
  // workgroup barrier. After step c it publishes K_c, M_c, H_c, S_c⁻¹ and applies the step's rank-2
  // term only to the "cross" of the next marker (all rows × its 5 columns, its 5 rows × the later
  // columns) — the entries step c+1 reads. The other waves follow through LDS flags:
  //   wave 3  the rest of P (rows ∉ next, columns of markers ≥ c+2), one step behind wave 0;
  //   wave 1  Z_c = Φ_c[:, pA]·Hᵀ·S⁻¹, then Φ −= Z_c·M_c (live columns);
  //   wave 2  Y_c = H·Ψ_c[pA, :],      then Ψ −= K_c·Y_c (live rows).
  // Φ, Ψ, Z, Y feed only the factor kernel, so waves 1–2 may lag the chain freely. "Live" = what
  // later steps still read (pose and later markers).
  const int wave = tid >> 6, lane = tid & 63;
  if (tid == 0) {
    sh.pub = 0;
    sh.pdone = 0;
    sh.zdone = 0;
    sh.any_init = 0;
  }
  if (pending) drain_stores();
  __syncthreads();
  if (pending) {
    if (tid == 0) epoch_store(A.sync + kSyncChain + f, pending);
    pending = 0;
  }
  EKF_STAMP(19);
  if (wave == 0) {
    unsigned long long* lg =
        (kDiagBuild && (A.dbg & 16)) ? A.dlog + (static_cast<size_t>(seq & 63u) * 64 + (f & 63)) * 8 : nullptr;
    chain_wave0<J>((LdsChain<J>*)(&sh), (LdsDesc*)(&d), 0, m, nu, A.r, seq, lg);
  } else if (wave == 3) {  // P outside the cross: rows and columns ∉ the next marker's Bx
    // lane → column 3+(lane&31), rows 3.. of parity lane>>5. The lane's 16 entries stay in
    // registers for the whole chunk: every step's rank-2 term is applied to all of them — also to
    // those in the next marker's cross, which wave 0 updates (and stores) itself with the same
    // operands in the same order, so the register copy keeps the block's bits — and only the
    // entries outside that cross are stored (what wave 0 reads ahead, and the block's final state).
    const int hb = lane & 31, hr = lane >> 5;
    const int b = min(3 + hb, kMaxU - 1);
    auto rest = [&](auto jc) {  // (Joseph: V_c[a]·K_c[b] after the K·M term, as wave 0 does)
      constexpr bool JR = decltype(jc)::value;
      double pv[16];
#pragma unroll
      for (int i = 0; i < 16; ++i) pv[i] = P[min(3 + hr + 2 * i, kMaxU - 1)][b];  // clamped rows
      for (int c = 0; c + 1 < m; ++c) {
        lds_wait_ge(&sh.pub, c + 1);
        EKF_STAMPT(192 + 2 * c, 192);
        const int nx = 5 + 2 * c, cj = min(c, JM - 1);
        const bool colok = 3 + hb < nu && b != nx && b != nx + 1;
        const double mb0 = sh.MU[c][b][0], mb1 = sh.MU[c][b][1];
        const double kb0 = JR ? sh.KU[c][b][0] : 0.0, kb1 = JR ? sh.KU[c][b][1] : 0.0;
        double k0[16], k1[16], w0[16], w1[16];
#pragma unroll
        for (int i = 0; i < 16; ++i) {  // clamped rows: unconditional reads, no per-row wait
          const int a = min(3 + hr + 2 * i, kMaxU - 1);
          k0[i] = sh.KU[c][a][0];
          k1[i] = sh.KU[c][a][1];
          if (JR) {
            w0[i] = sh.VU[cj][a][0];
            w1[i] = sh.VU[cj][a][1];
          }
        }
        // every lane stores every row (masked-off entries to its junk slot): no divergent
        // branches, so the reads above are waited for once, not once per predicated store
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const int a = 3 + hr + 2 * i;
          const bool ok = colok && a < nu && a != nx && a != nx + 1;
          double v = rank2_sub(pv[i], k0[i], k1[i], mb0, mb1);
          if (JR) v = rank2_sub(v, w0[i], w1[i], kb0, kb1);
          pv[i] = v;
          *(ok ? &P[a][b] : &sh.junk[3][lane]) = v;
        }
        lds_publish(&sh.pdone, c + 1);
        EKF_STAMPT(193 + 2 * c, 192);
      }
    };
    rest(std::integral_constant<bool, J>{});
    // The posterior t_map_odom = T(x, y, θ)·t_odom_robot⁻¹ (slam.cpp:273-277) as soon as wave 0 has
    // published the last step (its x is stored before that), beside waves 1–2's last Z / Y and off
    // the epilogue (a pose composition's sin / cos on one lane)
    if (lane == 0 && (d.flags & kLast)) {
      lds_wait_ge(&sh.pub, m);
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      const Pose2 tmo = compose(Pose2{sh.xU[0][0], sh.xU[0][1], sh.xU[0][2]},
                                inverse(Pose2{d.odom[0], d.odom[1], d.odom[2]}));
      ctl->tmo[0] = tmo.theta;
      ctl->tmo[1] = tmo.x;
      ctl->tmo[2] = tmo.y;
      if (kDiagBuild && (A.dbg & 16))
        dlog_add(A, 0, A.seq + static_cast<unsigned>(ci), f, 6,
                 dbits(tmo.theta) + dbits(tmo.x) + dbits(tmo.y));
      sh.tmo[0] = tmo.theta;
      sh.tmo[1] = tmo.x;
      sh.tmo[2] = tmo.y;
    }
    // ... and the next chunk's predicted pose (slam.cpp:184-196), beside waves 1–2's last Z / Y
    // instead of in its prologue: its inputs are this chunk's final pose (the record's x[U] there,
    // which the next chunk would read), the t_map_odom after this chunk (the word it would load)
    // and its descriptor's odometry — the same values, so the same bits
    if (lane == 0 && ci + 1 < nchunks) {
      const MsgDesc& nd = A.desc[static_cast<size_t>(ci + 1) * A.desc_stride + fy];
      const int nfl = nd.flags;
      const double od[3] = {nd.odom[0], nd.odom[1], nd.odom[2]};
      if ((nfl & kActive) && (nfl & kLook) && !A.gather) {
        lds_wait_ge(&sh.pub, m);
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        const double xp[3] = {sh.xU[0][0], sh.xU[0][1], sh.xU[0][2]};
        const double tm[3] = {sh.tmo[0], sh.tmo[1], sh.tmo[2]};
        double np_[3], a1, a2;
        predicted_pose(tm, nfl, od, xp, np_, &a1, &a2);
        sh.npose[0] = np_[0];
        sh.npose[1] = np_[1];
        sh.npose[2] = np_[2];
        sh.na1 = a1;
        sh.na2 = a2;
        sh.npose_ci = ci + 1;
      }
    }
  } else if (wave == 1) {  // Z_c: K_c[i] = r_0(i)·Z_c for every row i
    // Σ_c[i, pA_c] = r_0(i)·(E_c − Σ_{k<c} Z_k·M_k[:, pA_c]) (E_c selects the positions pA_c), so
    // Z_c = E_c·G − Σ_{k<c} Z_k·C_k with G = Hᵀ·S⁻¹ (5×2) and C_k = M_k[:, pA_c]·G (2×2): lane k
    // forms C_k, lane i its row of Z_c — 4c FMAs a row instead of a |U|×|U| row map updated per
    // step. The record parity this chunk writes was last written two chunks back: the prologue's
    // poll (that chunk's Σ-pass epoch) has made the bulk stream done with it. Z_c goes to the
    // record as soon as it is computed (write-through, off the chain's path).
    ChunkRec* rec = A.rec + static_cast<size_t>(d.parity) * A.rec_stride + f;
    const __amdgpu_buffer_rsrc_t rr =
        __builtin_amdgcn_make_buffer_rsrc(rec, 0, static_cast<int>(sizeof(ChunkRec)), 0x00020000);
    constexpr int oZ = static_cast<int>(offsetof(ChunkRec, Z));
    {  // columns ≥ 2m of the record's Z are zero (the factor kernel and a rebuilding chain read
       // them); Joseph: columns 2m..32 and 32 + 2m..64 (V in 32..32 + 2m)
      const int zw = kZC - 2 * m, nz = J ? 2 : 1;
      for (int e = lane; e < kMaxU * zw * nz; e += 64) {
        const int h = e >= kMaxU * zw ? 1 : 0, e2 = e - h * kMaxU * zw;
        const int b = e2 / zw, k = 2 * m + (e2 - b * zw) + kZC * h;
        st_wt(&rec->Z[b][k], 0.0);
      }
    }
    const int li = lane < kMaxU ? lane : kMaxU - 1;
    double zxa = 0.0;  // Σ_c Z_c ν_c of row `lane`, accumulated as the Z_c come (the record's Zx)
    if constexpr (!J) {
    for (int c = 0; c < m; ++c) {
      lds_wait_ge(&sh.pub, c + 1);
      const int pj = 3 + 2 * c;
      double H0[5], H1[5], Si[4], G0[5], G1[5];
#pragma unroll
      for (int a = 0; a < 5; ++a) {
        H0[a] = sh.Hs[c][0][a];
        H1[a] = sh.Hs[c][1][a];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) Si[k] = sh.Sis[c][k];
#pragma unroll
      for (int a = 0; a < 5; ++a) {
        G0[a] = H0[a] * Si[0] + H1[a] * Si[2];
        G1[a] = H0[a] * Si[1] + H1[a] * Si[3];
      }
      {  // lane k < c: C_k (lanes ≥ c store to a junk slot: no divergent branch)
        const int k = lane < c ? lane : 0;
        double m0[5], m1[5];
#pragma unroll
        for (int a = 0; a < 5; ++a) {
          const int pa = a < 3 ? a : pj + a - 3;
          m0[a] = sh.MU[k][pa][0];
          m1[a] = sh.MU[k][pa][1];
        }
        double c00 = 0.0, c01 = 0.0, c10 = 0.0, c11 = 0.0;
#pragma unroll
        for (int a = 0; a < 5; ++a) {
          c00 = fma(m0[a], G0[a], c00);
          c01 = fma(m0[a], G1[a], c01);
          c10 = fma(m1[a], G0[a], c10);
          c11 = fma(m1[a], G1[a], c11);
        }
        double* cd = lane < c ? &sh.Cz[lane][0] : &sh.junk[1][0];
        cd[0] = c00;
        cd[1] = c01;
        cd[2] = c10;
        cd[3] = c11;
      }
      __atomic_signal_fence(__ATOMIC_SEQ_CST);  // (one wave: LDS keeps its order)
      {  // row li of Z_c
        const int pos = li < 3 ? li : (li == pj ? 3 : (li == pj + 1 ? 4 : -1));
        double z0 = 0.0, z1 = 0.0;
#pragma unroll
        for (int a = 0; a < 5; ++a) {
          z0 = pos == a ? G0[a] : z0;
          z1 = pos == a ? G1[a] : z1;
        }
        // the history in groups of 4 terms: a group's 12 LDS reads are issued together and
        // waited for once (one term per read-wait-FMA round trip was ≈ 135 cycles)
        int k = 0;
        for (; k + 4 <= c; k += 4) {
          double zz[4][2], cz[4][4];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            zz[q][0] = sh.Z[li][2 * (k + q)];
            zz[q][1] = sh.Z[li][2 * (k + q) + 1];
#pragma unroll
            for (int e = 0; e < 4; ++e) cz[q][e] = sh.Cz[k + q][e];
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            z0 = fma(-zz[q][1], cz[q][2], fma(-zz[q][0], cz[q][0], z0));
            z1 = fma(-zz[q][1], cz[q][3], fma(-zz[q][0], cz[q][1], z1));
          }
        }
        for (; k < c; ++k) {
          const double zk0 = sh.Z[li][2 * k], zk1 = sh.Z[li][2 * k + 1];
          const double c00 = sh.Cz[k][0], c01 = sh.Cz[k][1], c10 = sh.Cz[k][2], c11 = sh.Cz[k][3];
          z0 = fma(-zk1, c10, fma(-zk0, c00, z0));
          z1 = fma(-zk1, c11, fma(-zk0, c01, z1));
        }
        const bool in = lane < nu;
        const double Z0 = in ? z0 : 0.0, Z1 = in ? z1 : 0.0;
        const double t = Z0 * sh.nu[c][0] + Z1 * sh.nu[c][1];
        zxa += t;
        if (lane < kMaxU) {
          sh.Z[lane][2 * c] = Z0;
          sh.Z[lane][2 * c + 1] = Z1;
          st_wt2(rr, oZ + 8 * (kZJ * lane + 2 * c), Z0, Z1);
        }
      }
      EKF_STAMPT(320 + c, 64);
    }
    } else {
    // Joseph: Σ_c[i, U] = r_0(i)·Φ_c with Φ_{c+1} = Φ_c − Z_c·M_c[:, U] − Zv_c·K_c[U]ᵀ, so
    // W_c = Φ_c[:, pA]·Hᵀ = E_c·Hᵀ − Σ_{k<c} (Z_k·C_k + Zv_k·C'_k), C_k = M_k[:, pA_c]·Hᵀ and
    // C'_k = K_k[pA_c]ᵀ·Hᵀ (2×2 each); then Z_c = W_c·S_c⁻¹ (K_c = G_c·S⁻¹, G_c[i] = r_0(i)·W_c) and
    // Zv_c = W_c − Z_c·S_c (V_c = G_c − K_c·S_c). One marker: Z_0 = E·Hᵀ·S⁻¹, as the simple form.
    constexpr int cols = kZC;  // V_c in columns 32 + 2c.. (fixed: the rebuild's K'ᵀ rows start at 32)
    for (int c = 0; c < m && c < kMaxJoseph; ++c) {
      lds_wait_ge(&sh.pub, c + 1);
      EKF_STAMPT(460 + c, 64);
      const int pj = 3 + 2 * c;
      double H0[5], H1[5], Si[4], Sc[4];
#pragma unroll
      for (int a = 0; a < 5; ++a) {
        H0[a] = sh.Hs[c][0][a];
        H1[a] = sh.Hs[c][1][a];
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        Si[k] = sh.Sis[c][k];
        Sc[k] = sh.Ss[c][k];
      }
      {  // lane k < c: C_k and C'_k
        const int k = lane < c ? lane : 0;
        double m0[5], m1[5], q0[5], q1[5];
#pragma unroll
        for (int a = 0; a < 5; ++a) {
          const int pa = a < 3 ? a : pj + a - 3;
          m0[a] = sh.MU[k][pa][0];
          m1[a] = sh.MU[k][pa][1];
          q0[a] = sh.KU[k][pa][0];
          q1[a] = sh.KU[k][pa][1];
        }
        double c00 = 0.0, c01 = 0.0, c10 = 0.0, c11 = 0.0;
        double e00 = 0.0, e01 = 0.0, e10 = 0.0, e11 = 0.0;
#pragma unroll
        for (int a = 0; a < 5; ++a) {
          c00 = fma(m0[a], H0[a], c00);
          c01 = fma(m0[a], H1[a], c01);
          c10 = fma(m1[a], H0[a], c10);
          c11 = fma(m1[a], H1[a], c11);
          e00 = fma(q0[a], H0[a], e00);
          e01 = fma(q0[a], H1[a], e01);
          e10 = fma(q1[a], H0[a], e10);
          e11 = fma(q1[a], H1[a], e11);
        }
        double* cd = lane < c ? &sh.Cz[lane][0] : &sh.junk[1][0];
        double* ed = lane < c ? &sh.Cv[lane][0] : &sh.junk[1][4];
        cd[0] = c00;
        cd[1] = c01;
        cd[2] = c10;
        cd[3] = c11;
        ed[0] = e00;
        ed[1] = e01;
        ed[2] = e10;
        ed[3] = e11;
      }
      __atomic_signal_fence(__ATOMIC_SEQ_CST);  // (one wave: LDS keeps its order)
      EKF_STAMPT(480 + c, 64);
      {  // row li of W_c, then of Z_c and Zv_c
        const int pos = li < 3 ? li : (li == pj ? 3 : (li == pj + 1 ? 4 : -1));
        double w0 = 0.0, w1 = 0.0;
#pragma unroll
        for (int a = 0; a < 5; ++a) {
          w0 = pos == a ? H0[a] : w0;
          w1 = pos == a ? H1[a] : w1;
        }
        // the history in groups of 4 terms, each group's 24 LDS reads issued together (one
        // read-wait round trip per term made this wave the chunk's last, ≈ 200 cycles a term)
        auto jterm = [&](const double* zz, const double* cz) {
          w0 = fma(-zz[1], cz[2], fma(-zz[0], cz[0], w0));
          w1 = fma(-zz[1], cz[3], fma(-zz[0], cz[1], w1));
          w0 = fma(-zz[3], cz[6], fma(-zz[2], cz[4], w0));
          w1 = fma(-zz[3], cz[7], fma(-zz[2], cz[5], w1));
        };
        int k = 0;
        for (; k + 4 <= c; k += 4) {
          double zz[4][4], cz[4][8];
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            zz[q][0] = sh.Z[li][2 * (k + q)];
            zz[q][1] = sh.Z[li][2 * (k + q) + 1];
            zz[q][2] = sh.Z[li][cols + 2 * (k + q)];
            zz[q][3] = sh.Z[li][cols + 2 * (k + q) + 1];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              cz[q][e] = sh.Cz[k + q][e];
              cz[q][4 + e] = sh.Cv[k + q][e];
            }
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int q = 0; q < 4; ++q) jterm(zz[q], cz[q]);
        }
        for (; k < c; ++k) {
          double zz[4], cz[8];
          zz[0] = sh.Z[li][2 * k];
          zz[1] = sh.Z[li][2 * k + 1];
          zz[2] = sh.Z[li][cols + 2 * k];
          zz[3] = sh.Z[li][cols + 2 * k + 1];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            cz[e] = sh.Cz[k][e];
            cz[4 + e] = sh.Cv[k][e];
          }
          jterm(zz, cz);
        }
        const bool in = lane < nu;
        const double Z0 = in ? w0 * Si[0] + w1 * Si[2] : 0.0;
        const double Z1 = in ? w0 * Si[1] + w1 * Si[3] : 0.0;
        const double V0 = in ? w0 - (Z0 * Sc[0] + Z1 * Sc[2]) : 0.0;
        const double V1 = in ? w1 - (Z0 * Sc[1] + Z1 * Sc[3]) : 0.0;
        zxa += Z0 * sh.nu[c][0] + Z1 * sh.nu[c][1];
        if (lane < kMaxU) {
          sh.Z[lane][2 * c] = Z0;
          sh.Z[lane][2 * c + 1] = Z1;
          sh.Z[lane][cols + 2 * c] = V0;
          sh.Z[lane][cols + 2 * c + 1] = V1;
          st_wt2(rr, oZ + 8 * (kZJ * lane + 2 * c), Z0, Z1);
          st_wt2(rr, oZ + 8 * (kZJ * lane + cols + 2 * c), V0, V1);
        }
      }
      lds_publish(&sh.zdone, c + 1);  // (wave 2 reads Z_c, Zv_c)
      EKF_STAMPT(320 + c, 64);
    }
    }
    if (lane < kMaxU) sh.Zx[lane] = zxa;
  } else {  // wave 2: Y_c: M_c[:, j] = Y_c·c_0(j) for every column j; Y_c to the record at once
    // Σ_c[pA_c, j] = (E_cᵀ − Σ_{k<c} K_k[pA_c]·Y_k)·c_0(j), so Y_c = H·E_cᵀ − Σ_{k<c} D_k·Y_k with
    // D_k = H·K_k[pA_c] (2×2): lane k forms D_k, lane j its column of Y_c.
    ChunkRec* rec = A.rec + static_cast<size_t>(d.parity) * A.rec_stride + f;
    for (int e = lane; e < (kZC - 2 * m) * kMaxU; e += 64)  // rows ≥ 2m of the record's Y are zero
      st_wt(&(&rec->Y[2 * m][0])[e], 0.0);
    const int lj = lane < kMaxU ? lane : kMaxU - 1;
    // Joseph: Σ_{c+1}[·, j] also loses V_c·K_c[j]ᵀ, and K_c[j] = r_0(j)·Z_c = Z_cᵀ·c_0(j) (Σ_pred is
    // symmetric in exact arithmetic; fp64 Σ exactly): Y_c = H·E_cᵀ − Σ_{k<c} (D_k·Y_k + D'_k·Z_kᵀ),
    // D'_k = H·V_k[pA_c], with wave 1's Z_k (flag zdone)
    for (int c = 0; c < m; ++c) {
      lds_wait_ge(&sh.pub, c + 1);
      EKF_STAMPT(400 + c, 128);
      if (joseph && c > 0) lds_wait_ge(&sh.zdone, min(c, kMaxJoseph));
      EKF_STAMPT(420 + c, 128);
      const int pj = 3 + 2 * c;
      double H0[5], H1[5];
#pragma unroll
      for (int a = 0; a < 5; ++a) {
        H0[a] = sh.Hs[c][0][a];
        H1[a] = sh.Hs[c][1][a];
      }
      {  // lane k < c: D_k (Joseph: and D'_k)
        const int k = lane < c ? lane : 0;
        double k0[5], k1[5];
#pragma unroll
        for (int a = 0; a < 5; ++a) {
          const int pa = a < 3 ? a : pj + a - 3;
          k0[a] = sh.KU[k][pa][0];
          k1[a] = sh.KU[k][pa][1];
        }
        double d00 = 0.0, d01 = 0.0, d10 = 0.0, d11 = 0.0;
#pragma unroll
        for (int a = 0; a < 5; ++a) {
          d00 = fma(H0[a], k0[a], d00);
          d01 = fma(H0[a], k1[a], d01);
          d10 = fma(H1[a], k0[a], d10);
          d11 = fma(H1[a], k1[a], d11);
        }
        double* dd = lane < c ? &sh.Dy[lane][0] : &sh.junk[2][0];
        dd[0] = d00;
        dd[1] = d01;
        dd[2] = d10;
        dd[3] = d11;
        if (joseph) {
          const int kj = min(k, JM - 1);
          double v0[5], v1[5];
#pragma unroll
          for (int a = 0; a < 5; ++a) {
            const int pa = a < 3 ? a : pj + a - 3;
            v0[a] = sh.VU[kj][pa][0];
            v1[a] = sh.VU[kj][pa][1];
          }
          double e00 = 0.0, e01 = 0.0, e10 = 0.0, e11 = 0.0;
#pragma unroll
          for (int a = 0; a < 5; ++a) {
            e00 = fma(H0[a], v0[a], e00);
            e01 = fma(H0[a], v1[a], e01);
            e10 = fma(H1[a], v0[a], e10);
            e11 = fma(H1[a], v1[a], e11);
          }
          double* ed = lane < c ? &sh.Dv[kj][0] : &sh.junk[2][4];
          ed[0] = e00;
          ed[1] = e01;
          ed[2] = e10;
          ed[3] = e11;
        }
      }
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      EKF_STAMPT(440 + c, 128);
      {  // column lj of Y_c
        const int pos = lj < 3 ? lj : (lj == pj ? 3 : (lj == pj + 1 ? 4 : -1));
        double y0 = 0.0, y1 = 0.0;
#pragma unroll
        for (int a = 0; a < 5; ++a) {
          y0 = pos == a ? H0[a] : y0;
          y1 = pos == a ? H1[a] : y1;
        }
        int k0 = 0;
        if (joseph) {  // (uniform) groups of 4 terms with D'_k·Z_kᵀ, reads issued together
          for (; k0 + 4 <= c; k0 += 4) {
            double yy[4][4], dy[4][8];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const int kj = min(k0 + q, JM - 1);
              yy[q][0] = sh.Y[2 * (k0 + q)][lj];
              yy[q][1] = sh.Y[2 * (k0 + q) + 1][lj];
              yy[q][2] = sh.Z[lj][2 * (k0 + q)];
              yy[q][3] = sh.Z[lj][2 * (k0 + q) + 1];
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                dy[q][e] = sh.Dy[k0 + q][e];
                dy[q][4 + e] = sh.Dv[kj][e];
              }
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              y0 = fma(-dy[q][1], yy[q][1], fma(-dy[q][0], yy[q][0], y0));
              y1 = fma(-dy[q][3], yy[q][1], fma(-dy[q][2], yy[q][0], y1));
              y0 = fma(-dy[q][5], yy[q][3], fma(-dy[q][4], yy[q][2], y0));
              y1 = fma(-dy[q][7], yy[q][3], fma(-dy[q][6], yy[q][2], y1));
            }
          }
        } else {  // (uniform) groups of 4 terms, reads issued together (as wave 1's Z)
          for (; k0 + 4 <= c; k0 += 4) {
            double yy[4][2], dy[4][4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              yy[q][0] = sh.Y[2 * (k0 + q)][lj];
              yy[q][1] = sh.Y[2 * (k0 + q) + 1][lj];
#pragma unroll
              for (int e = 0; e < 4; ++e) dy[q][e] = sh.Dy[k0 + q][e];
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              y0 = fma(-dy[q][1], yy[q][1], fma(-dy[q][0], yy[q][0], y0));
              y1 = fma(-dy[q][3], yy[q][1], fma(-dy[q][2], yy[q][0], y1));
            }
          }
        }
#pragma unroll 4
        for (int k = k0; k < c; ++k) {
          const double yk0 = sh.Y[2 * k][lj], yk1 = sh.Y[2 * k + 1][lj];
          const double d00 = sh.Dy[k][0], d01 = sh.Dy[k][1], d10 = sh.Dy[k][2], d11 = sh.Dy[k][3];
          y0 = fma(-d01, yk1, fma(-d00, yk0, y0));
          y1 = fma(-d11, yk1, fma(-d10, yk0, y1));
          if (joseph) {
            const int kj = min(k, JM - 1);
            const double zk0 = sh.Z[lj][2 * k], zk1 = sh.Z[lj][2 * k + 1];
            const double e00 = sh.Dv[kj][0], e01 = sh.Dv[kj][1], e10 = sh.Dv[kj][2], e11 = sh.Dv[kj][3];
            y0 = fma(-e01, zk1, fma(-e00, zk0, y0));
            y1 = fma(-e11, zk1, fma(-e10, zk0, y1));
          }
        }
        if (lane < kMaxU) {
          const bool in = lane < nu;
          sh.Y[2 * c][lane] = in ? y0 : 0.0;
          sh.Y[2 * c + 1][lane] = in ? y1 : 0.0;
          st_wt(&rec->Y[2 * c][lane], in ? y0 : 0.0);
          st_wt(&rec->Y[2 * c + 1][lane], in ? y1 : 0.0);
        }
      }
      EKF_STAMPT(360 + c, 128);
    }
  }
  __syncthreads();
  // fp32 Σ: the last step's rank-2 term on the whole block (earlier steps are applied), the final
  // Σ[U, U] in fp64, to the record (write-through) for k_patch_stage (the Σ pass's U × U entries).
  // Only a chunk that initialises a landmark has the 1e7 − (1e7 − δ) cancellation the patch is
  // for (slam.cpp:130's prior has no cross terms; an untouched landmark's rows stay exact): a first
  // sighting, or an association chunk (its new landmark is written by k_assoc). Other chunks keep
  // the pass's own values and skip this.
  const bool pend = sizeof(T) == 4 && (sh.any_init || (d.flags & kNoInit));
  if (pend) {
    const int c = max(m - 1, 0);
    ChunkRec* rec = A.rec + static_cast<size_t>(d.parity) * A.rec_stride + f;
    for (int e = tid; e < kMaxU * kMaxU; e += blockDim.x) {
      const int a = e / kMaxU, b = e - a * kMaxU;
      double v = P[a][b];
      if (m > 0)
        v = rank2_sub(v, sh.KU[c][a][0], sh.KU[c][a][1], sh.MU[c][b][0], sh.MU[c][b][1]);
      if (m > 0 && joseph) {  // − V_c[a]·K_c[b]ᵀ
        const int cj = min(c, JM - 1);
        v = rank2_sub(v, sh.VU[cj][a][0], sh.VU[cj][a][1], sh.KU[c][b][0], sh.KU[c][b][1]);
      }
      if (a < nu && b < nu) st_wt(&rec->Pend[a][b], v);
    }
  }
  __syncthreads();
  EKF_STAMP(12);
  // ---- epilogue -----------------------------------------------------------------------------
  // Waves 0–2 prefetch the next chunk's descriptor and store the record write-through. The record's epoch is published at the next
  // chunk's start (or the kernel's end): the stores drain behind the next prologue instead of
  // stalling this one. The record parity's release (the bulk stream done with it) was awaited by
  // the prologue's poll.
  const double* xfin = sh.xU[0];
  const bool pre_next = ci + 1 < nchunks;
  if (wave == 3) {
    // (the posterior t_map_odom: wave 3 after the last step, above)
  } else {
    if (pre_next && tid >= 128 && tid < 128 + static_cast<int>(sizeof(MsgDesc) / 16))
      reinterpret_cast<uint4*>(&sdesc[(ci + 1) & 1])[tid - 128] = reinterpret_cast<const uint4*>(
          &A.desc[static_cast<size_t>(ci + 1) * A.desc_stride + fy])[tid - 128];
    if (tid == 0 && sh.status) atomicOr(&ctl->status, sh.status);
    // hand the chunk to the factor kernel (and the next chain): write-through record
    ChunkRec* rec = A.rec + static_cast<size_t>(d.parity) * A.rec_stride + f;
    if (tid < kMaxU) {  // state weights: x_i += r_0(i)[U] · Σ_c Z_c ν_c
      const double zx = sh.Zx[tid];  // (wave 1's sum over the corrections)
      const bool in = tid < nu;
      st_wt(&rec->Zx[tid], zx);
      if (kDiagBuild && (A.dbg & 16)) dlog_add(A, 0, seq, f, 5, dbits(zx) + dbits(in ? xfin[tid] : 0.0));
      st_wt(&rec->u[tid], sh.u[tid]);
      st_wt(&rec->alphaU[tid], in ? sh.alphaU[tid] : 0.0);
      st_wt(&rec->row0raw[tid], in ? sh.row0raw[tid] : 0.0);
      st_wt(&rec->col0raw[tid], in ? sh.col0raw[tid] : 0.0);
      st_wt(&rec->xU[tid], in ? xfin[tid] : 0.0);
    }
    if (tid == 0) {
      st_wt(&rec->m, m);
      st_wt(&rec->nu, nu);
      st_wt(&rec->flags, d.flags | (pend ? kPendValid : 0));
      st_wt(&rec->a1, sh.a1);
      st_wt(&rec->a2, sh.a2);
      st_wt(&rec->s00, sh.s00);
    }
    EKF_STAMP(16);
  }
  pending = seq + 1u;
  pre = pre_next;
  __syncthreads();
  EKF_STAMP(40);
  EKF_STAMPV(307, __builtin_amdgcn_s_memrealtime());
  }  // chunk loop
  if (pending) {
    drain_stores();
    __syncthreads();
    if (tid == 0) epoch_store(A.sync + kSyncChain + f, pending);
  }
  if (kDiagBuild && (A.dbg & 2)) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
}

template <typename T, bool J>
__global__ __launch_bounds__(256) void k_factors(PassArgs<T> A, int xcd_b, int nf) {
  __shared__ FactorSharedT<J> sh;
  constexpr int ZC = FactorSharedT<J>::ZC;
  // xcd_b = 0: grid (blocks per filter, filters). xcd_b = B > 0 (swarms): the Σ pass's XCD-aware
  // 1-D grid — block L on XCD L % 8 takes filter 8·⌊(L/8)/B⌋ + L % 8, block (L/8) % B — so a
  // filter's record is fetched into one L2 instead of eight. Placement only changes speed.
  int fb = blockIdx.y, bx = blockIdx.x;
  if (xcd_b > 0) {
    const int L = blockIdx.x, j = L >> 3;
    fb = (L & 7) + 8 * (j / xcd_b);
    bx = j % xcd_b;
  }
  // the previous chunk's Σ pass ended before this launch (same stream): its epoch, for the chains
  if (A.pub_sigma && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)
    epoch_store(A.sync + kSyncSigma, A.pub_sigma);
  if (kDiagBuild && (A.dbg & 1)) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  if (fb >= nf) return;
  const MsgDesc& d = A.desc[fb];
  if (!(d.flags & kActive)) return;
  const int f = A.f0 + fb;
  const int tid = threadIdx.x;
  if ((kDiagBuild && (A.dbg & 4)) && tid == 0 &&
      static_cast<int>(epoch_load(A.sync + kSyncChain + f) - (A.seq + 1u)) < 0)
    atomicAdd(A.sync + kSyncDbg + 1, 1u);
  if ((kDiagBuild && (A.dbg & 8)) && tid == 0 && bx == 0) dbg_seq_check(A, 1, f, A.seq + 1u);
  const ChunkRec* rec = A.rec + static_cast<size_t>(d.parity) * A.rec_stride + f;
  // the chain of this chunk runs on the other stream: wait for its record
  if (A.polls && tid == 0 && !epoch_wait_acquire(A.sync + kSyncChain + f, A.seq + 1u))
    flag_timeout(&A.ctl[f].status, A.fatal);
  drain_stores();
  __syncthreads();
  factor_record(rec, sh, tid);
  __syncthreads();
  if ((kDiagBuild && (A.dbg & 16)) && bx == 0) {  // the record as this kernel read it
    unsigned long long s1 = 0;
    for (int e = tid; e < kMaxU * ZC; e += 256) s1 += dbits(sh.Z[e / ZC][e % ZC]);
    for (int e = tid; e < kMaxU * kZC; e += 256) s1 += dbits(sh.Y[e / kMaxU][e % kMaxU]);
    if (tid < kMaxU)
      s1 += static_cast<unsigned>(sh.u[tid]) + dbits(sh.alphaU[tid]) + dbits(sh.row0raw[tid]) +
            dbits(sh.col0raw[tid]) + dbits(sh.Zx[tid]) + dbits(sh.xU[tid]);
    if (tid == 0) s1 += dbits(sh.a1) + dbits(sh.a2) + dbits(sh.s00) + static_cast<unsigned>(sh.nu);
    dlog_add(A, 4, A.seq, f, 1, s1);
    if (tid < static_cast<int>(sizeof(MsgDesc) / 8))
      dlog_add(A, 4, A.seq, f, 0, reinterpret_cast<const unsigned long long*>(&d)[tid]);
  }
  factor_wave<T, J>(A, d, f, bx * (blockDim.x >> 6) + (tid >> 6), sh, tid & 63);
  if (kDiagBuild && (A.dbg & 2)) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
}

// ---- Σ pass on MFMA -------------------------------------------------------------------------
// Σ_out = Σ_in + Q̄ − Σ_k Kcat[k]ᵀ ⊗ Mcat[k], one tile per wave, four waves per workgroup.
//   fp32  32×32 tile, v_mfma_f32_32x32x2_f32: D[row = (r&3) + 8(r>>2) + 4(lane>>5)][col = lane&31]
//         → each load / store instruction covers 2 rows × 128 B
//   fp64  32×16 tile, two v_mfma_f64_16x16x4_f64 blocks: D[row = 16ti + (lane>>4) + 4r][col = lane&15]
//         → 4 rows × 128 B per instruction
// A/B lane maps: 16x16x4 A[i = lane&15][k = lane>>4]; 32x32x2 A[i = lane&31][k = lane>>5].
// Memory goes through buffer descriptors with 32-bit offsets (no 64-bit address per load):
//   - Σ: the wave's 32-row panel (up to row n); a row ≥ n lies past the end, a column ≥ n gets
//     the offset kOOB, so the range check returns 0 for its loads and drops its stores (no masks,
//     no waits);
//   - Kcat / Mcat: the factor rows are uniform (SGPR soffset), the lane's column in voffset.
// Order: operands (L2-hot) first, then Σ_in. The MFMAs start from zero as soon as the operands
// land and run while Σ_in is still in flight; Σ_in (+ Q̄) is added once, before the store.
typedef float f16v __attribute__((ext_vector_type(16)));
constexpr unsigned kOOB = 0x80000000u;  // voffset past any Σ panel descriptor (32·ld·w < 2 GiB)


template <typename T>
struct SigmaTile;

// The simple form's factor rank is at most 2 + 2·kMaxChunk = 34: 17 k-steps of the 32×32×2 MFMA.
// (kw, the rank rounded up to 4 for the fp64 tiles, would make it 18, the last one on the two zero
// rows 34–35.) A Joseph chunk's rank 2 + 4m ≤ 66 (kw ≤ 68) takes a second block of 17 k-steps
// (KB = 2): the operand registers are loaded again for it, so the tile keeps its register count.
constexpr int kSteps = (2 + 2 * kMaxChunk + 1) / 2;
static_assert(kMaxKW <= 4 * kSteps, "Joseph rank within two blocks of fp32 k-steps");
struct F32TileRegs {  // one fp32 tile's loads
  float a[kSteps], b[kSteps], sv[16];
};
template <>
struct SigmaTile<float> {
  static constexpr int kRows = 32, kCols = 32;
  // descriptors based at the wave's row panel: offsets stay 32-bit for any n (a filter's Σ may
  // exceed 4 GiB), and the records end at row n
  static __device__ __forceinline__ __amdgpu_buffer_rsrc_t panel(const float* S, int n, int ld,
                                                                 int R0) {
    return buf_rsrc(S + static_cast<size_t>(R0) * ld,
                    static_cast<unsigned>(min(n - R0, kRows)) * ld * 4u);
  }
  static __device__ __forceinline__ unsigned soff(int n, int ld, int C0, int lane) {
    const int col = C0 + (lane & 31);
    return col < n ? static_cast<unsigned>(4 * (lane >> 5) * ld + col) * 4u : kOOB;
  }
  // every load of the tile: the operands (L2-hot) first, then Σ_in
  static __device__ __forceinline__ void load(F32TileRegs& g, const float* Sin, const float* kc,
                                              const float* mc, int n, int ld, int ldk, int R0,
                                              int C0, int lane) {
    load_ops(g, kc, mc, n, ldk, R0, C0, lane);
    // keep the operand loads ahead of Σ_in's: the MFMAs then wait for vmcnt(16), not vmcnt(0)
    __builtin_amdgcn_sched_barrier(0);
    load_sig(g, Sin, n, ld, R0, C0, lane);
  }
  // block kb: factor rows 2·kSteps·kb + 2s + (lane ≥ 32)
  static __device__ __forceinline__ void load_ops(F32TileRegs& g, const float* kc, const float* mc,
                                                  int n, int ldk, int R0, int C0, int lane,
                                                  int kb = 0) {
    const int kr = lane >> 5, kcol = lane & 31;
    const unsigned kbytes = static_cast<unsigned>(kMaxKW) * ldk * 4u;
    const auto rk = buf_rsrc(kc, kbytes), rm = buf_rsrc(mc, kbytes);
    const int k0 = 2 * kSteps * kb;
    const unsigned ko = static_cast<unsigned>((k0 + kr) * ldk + R0 + kcol) * 4u;
    const unsigned mo = static_cast<unsigned>((k0 + kr) * ldk + min(C0 + kcol, n - 1)) * 4u;
    const unsigned kstep = 2u * ldk * 4u;
#pragma unroll
    for (int s = 0; s < kSteps; ++s) {
      g.a[s] = ld_f32(rk, ko, s * kstep);
      g.b[s] = ld_f32(rm, mo, s * kstep);
    }
  }
  static __device__ __forceinline__ void load_sig(F32TileRegs& g, const float* Sin, int n, int ld,
                                                  int R0, int C0, int lane) {
    const auto rin = panel(Sin, n, ld, R0);
    const unsigned so = soff(n, ld, C0, lane);
    const unsigned rstride = static_cast<unsigned>(ld) * 4u;
#pragma unroll
    for (int r = 0; r < 16; ++r) g.sv[r] = ld_f32(rin, so + ((r & 3) + 8 * (r >> 2)) * rstride, 0);
  }
  static __device__ __forceinline__ void run(const float* Sin, float* Sout, const float* kc,
                                             const float* mc, int n, int ld, int ldk, int kw,
                                             bool first, double qd, int R0, int C0, int lane,
                                             float*) {
    F32TileRegs g;
    load(g, Sin, kc, mc, n, ld, ldk, R0, C0, lane);
    finish(g, Sout, n, ld, kw, first, qd, R0, C0, lane);
  }
  // the MFMAs on the tile's operands, Σ_in − K·M (+ Q̄), the stores
  // pm (≠ null: the chunk's record holds the chain's fp64 Σ[U, U], kPendValid): the first position
  // in U of each tile row (pm[0..32)) and column (pm[32..64)), > kMaxU − 1 for none — those
  // entries take the record's value instead (what k_patch_stage wrote after the pass before)
  static __device__ __forceinline__ void finish(const F32TileRegs& g, float* Sout, int n, int ld,
                                                int kw, bool first, double qd, int R0, int C0,
                                                int lane, const int* pm = nullptr,
                                                const ChunkRec* rec = nullptr) {
    f16v acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
    mma(g, kw, 0, acc);
    store(g, acc, Sout, n, ld, first, qd, R0, C0, lane, pm, rec);
  }
  // the k-steps of one operand block (k0: its first factor row): every MFMA issued, factor rows
  // ≥ kw (stale) zeroed by a select — a branch per k-step let the compiler sink each operand load
  // into its branch behind a vmcnt(0)
  static __device__ __forceinline__ void mma(const F32TileRegs& g, int kw, int k0, f16v& acc) {
#pragma unroll
    for (int s = 0; s < kSteps; ++s) {
      const bool live = k0 + 2 * s < kw;
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(live ? g.a[s] : 0.0f, live ? g.b[s] : 0.0f, acc,
                                                 0, 0, 0);
    }
  }
  // Joseph: the two operand blocks (the first loaded before Σ_in, the second after its MFMAs)
  static __device__ __forceinline__ void finish2(F32TileRegs& g, const float* kc, const float* mc,
                                                 int ldk, float* Sout, int n, int ld, int kw,
                                                 bool first, double qd, int R0, int C0, int lane,
                                                 const int* pm, const ChunkRec* rec) {
    f16v acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.0f;
    mma(g, kw, 0, acc);
    load_ops(g, kc, mc, n, ldk, R0, C0, lane, 1);
    mma(g, kw, 2 * kSteps, acc);
    store(g, acc, Sout, n, ld, first, qd, R0, C0, lane, pm, rec);
  }
  static __device__ __forceinline__ void store(const F32TileRegs& g, const f16v& acc, float* Sout,
                                               int n, int ld, bool first, double qd, int R0,
                                               int C0, int lane, const int* pm,
                                               const ChunkRec* rec) {
    const int kr = lane >> 5, col = C0 + (lane & 31);
    const auto rout = panel(Sout, n, ld, R0);
    const unsigned so = soff(n, ld, C0, lane);
    const unsigned rstride = static_cast<unsigned>(ld) * 4u;
    const float* sv = g.sv;
    SIG_STAMP(2);
    const float q = static_cast<float>(qd);
    if (!pm) {  // (two loops: the common one keeps the plain store sequence)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = R0 + (r & 3) + 8 * (r >> 2) + 4 * kr;
        float v = sv[r] - acc[r];
        if (first && row == col && row < 3) v += q;
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rout,
                                              so + ((r & 3) + 8 * (r >> 2)) * rstride, 0, 0);
      }
      return;
    }
    const int pc = pm[32 + (lane & 31)];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int rl = (r & 3) + 8 * (r >> 2) + 4 * kr, row = R0 + rl;
      float v = sv[r] - acc[r];
      if (first && row == col && row < 3) v += q;
      const int pr = pm[rl];
      if (pr < kMaxU && pc < kMaxU) v = static_cast<float>(rec->Pend[pr][pc]);
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), rout,
                                            so + ((r & 3) + 8 * (r >> 2)) * rstride, 0, 0);
    }
  }
};

// fp64 tile of 32 × 16·TJ: TJ = 2 for a few filters (more waves per filter), TJ = 4 for swarms
// (≥ 16 filters): the M operand rows are read once per 64 columns instead of per 32 — the
// operand loads are the pass's VMEM bottleneck there (swarm pass 589 → 564 µs; one filter's pass
// 5.2 → 7.6 µs, so it keeps TJ = 2)
// 2 = nt: the swarm's 2.2 GB of Σ stream through HBM once per message (≫ the 256 MB MALL), so its
// Σ_in loads and Σ_out stores skip cache retention — swarm 1.09e7 → 1.15e7 corrections/s
// (profiles/r2/r2z_*, two alternating runs each). The MALL-resident single-filter tiles keep the default.
#ifndef EKF_SIG_POL
#define EKF_SIG_POL 2
#endif
// Symmetric: Σ_out is symmetric (Σ_in + Q̄ − Kcatᵀ·Mcat is, the predict's A·Σ·Aᵀ and every
// correction's K·S·Kᵀ are), so an fp64 pass computes only the tiles holding an element on or above
// the diagonal (first tile column of tile row tr: ⌊32·tr / kCols⌋) and writes every element (r, c),
// r > c, as the mirror of (c, r): Σ_in is read in those tiles only (≈ 0.58 of Σ at the swarm's n),
// the MFMA work of the strictly-lower tiles is skipped, and Σ_out stays exactly symmetric. The
// mirror goes out through the wave's LDS (the tile transposed, then row by row: a direct
// transposed store is 16 rows × 32 B per instruction, measured 1.5× slower than the whole pass).
// Swarm pass 445 → 379 µs standalone, bit-identical in the upper triangle (tools/pass64_lab.hip).
constexpr int kTS = 34;  // transposed tile row stride (doubles; 16 B aligned rows)
template <int TJ_>
struct SigmaTile64 {
  static constexpr int TJ = TJ_;
  // cache policy of the swarm tile's Σ_in loads / Σ_out stores (the swarm's Σ streams through HBM)
  static constexpr int kPol = TJ == 4 ? EKF_SIG_POL : 0;
  static constexpr int kRows = 32, kCols = 16 * TJ;
  static constexpr int kLds = kCols * kTS;  // doubles of the wave's transposed tile
  // KB operand blocks of 36 factor rows (Joseph: 2, rank 2 + 4m ≤ 66; the second block's operands
  // reuse the first's registers after its MFMAs)
  template <int KB = 1>
  static __device__ __forceinline__ void run(const double* Sin, double* Sout, const double* kc,
                                             const double* mc, int n, int ld, int ldk, int kw,
                                             bool first, double q, int R0, int C0, int lane,
                                             double* tT) {
    const int kr = lane >> 4, kcol = lane & 15;
    // descriptors based at the wave's row panel: offsets stay 32-bit for any n (a filter's Σ
    // may exceed 4 GiB), and the records end at row n
    const size_t pbase = static_cast<size_t>(R0) * ld;
    const unsigned sbytes = static_cast<unsigned>(min(n - R0, kRows)) * ld * 8u;
    const unsigned kbytes = static_cast<unsigned>(kMaxKW) * ldk * 8u;
    const auto rin = buf_rsrc(Sin + pbase, sbytes), rout = buf_rsrc(Sout + pbase, sbytes);
    // the mirror: rows C0 … C0 + kCols − 1 of Σ_out from column R0
    const auto rmir = buf_rsrc(Sout + static_cast<size_t>(C0) * ld + R0,
                               static_cast<unsigned>(min(n - C0, kCols)) * ld * 8u);
    const auto rk = buf_rsrc(kc, kbytes), rm = buf_rsrc(mc, kbytes);
    double a[2][9], b[TJ][9], sv[2][TJ][4];
    const unsigned ko = static_cast<unsigned>(kr * ldk + R0 + kcol) * 8u;
    unsigned mo[TJ], so[TJ];
    const unsigned rstride = static_cast<unsigned>(ld) * 8u;
#pragma unroll
    for (int tj = 0; tj < TJ; ++tj) {
      const int col = C0 + 16 * tj + kcol;
      mo[tj] = static_cast<unsigned>(kr * ldk + min(col, n - 1)) * 8u;
      so[tj] = col < n ? static_cast<unsigned>(kr * ld + col) * 8u : kOOB;
    }
    const unsigned kstep = 4u * ldk * 8u;
    auto load_ops = [&](int kb) {
#pragma unroll
      for (int s = 0; s < 9; ++s) {
        a[0][s] = ld_f64(rk, ko, (9 * kb + s) * kstep);
        a[1][s] = ld_f64(rk, ko + 16 * 8, (9 * kb + s) * kstep);
#pragma unroll
        for (int tj = 0; tj < TJ; ++tj) b[tj][s] = ld_f64(rm, mo[tj], (9 * kb + s) * kstep);
      }
    };
    load_ops(0);
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
      for (int tj = 0; tj < TJ; ++tj)
#pragma unroll
        for (int r = 0; r < 4; ++r)
          sv[ti][tj][r] = __builtin_bit_cast(
              double, __builtin_amdgcn_raw_buffer_load_b64(rin, so[tj] + (16 * ti + 4 * r) * rstride, 0, kPol));
    d4 acc[2][TJ];
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
      for (int tj = 0; tj < TJ; ++tj) acc[ti][tj] = d4{0, 0, 0, 0};
    auto mma = [&](int kb) {
#pragma unroll
      for (int s = 0; s < 9; ++s) {  // unconditional, stale rows ≥ kw zeroed (see the fp32 tile)
        const bool live = 36 * kb + 4 * s < kw;
#pragma unroll
        for (int ti = 0; ti < 2; ++ti)
#pragma unroll
          for (int tj = 0; tj < TJ; ++tj)
            acc[ti][tj] = mfma_f64(live ? a[ti][s] : 0.0, live ? b[tj][s] : 0.0, acc[ti][tj]);
      }
    };
    mma(0);
    if (KB == 2) {
      load_ops(1);
      mma(1);
    }
    SIG_STAMP(2);
#pragma unroll
    for (int ti = 0; ti < 2; ++ti)
#pragma unroll
      for (int tj = 0; tj < TJ; ++tj)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int rl = 16 * ti + kr + 4 * r, cl = 16 * tj + kcol;
          const int row = R0 + rl, col = C0 + cl;
          double v = sv[ti][tj][r] - acc[ti][tj][r];
          if (first && row == col && row < 3) v += q;
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, v), rout,
                                                col >= row ? so[tj] + (16 * ti + 4 * r) * rstride : kOOB,
                                                0, kPol);
          tT[cl * kTS + rl] = v;
        }
    // the mirror, two rows of the transposed tile per store (LDS in order within the wave)
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const int rl = lane & 31;
#pragma unroll
    for (int i = 0; i < kCols / 2; ++i) {
      const int cl = 2 * i + (lane >> 5);
      const double v = tT[cl * kTS + rl];
      const int row = R0 + rl, col = C0 + cl;
      const unsigned mo2 = col > row && col < n ? static_cast<unsigned>(cl * ld + rl) * 8u : kOOB;
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, v), rmir, mo2, 0, kPol);
    }
  }
};
// the tiles of a symmetric pass: tile row tr holds tile columns ⌊32·tr / kCols⌋ … tcols − 1
template <int kCols>
__host__ __device__ inline int sym_first(int tr) { return 32 * tr / kCols; }
template <int kCols>
__host__ __device__ inline int sym_tiles(int trows, int tcols) {
  int t = 0;
  for (int tr = 0; tr < trows; ++tr) t += tcols - sym_first<kCols>(tr);
  return t;
}
// the t-th of them, row-major (wave-uniform t: a scalar walk over the tile rows)
template <int kCols>
__device__ __forceinline__ bool sym_tile(int t, int trows, int tcols, int& tr, int& tc) {
  int base = 0;
  for (tr = 0; tr < trows; ++tr) {
    const int c = tcols - sym_first<kCols>(tr);
    if (t < base + c) break;
    base += c;
  }
  tc = tr < trows ? sym_first<kCols>(tr) + (t - base) : 0;
  return tr < trows;
}
template <>
struct SigmaTile<double> : SigmaTile64<2> {};
// the tile a Σ pass of T runs: WIDE (swarms) takes the 32 × 64 fp64 tile
template <typename T, bool WIDE>
using PassTile = typename std::conditional<sizeof(T) == 8 && WIDE, SigmaTile64<4>, SigmaTile<T>>::type;

// xcd_b = 0: grid (blocks per filter, filters). xcd_b = B > 0 (many filters): a 1-D grid whose
// block L runs on XCD L % 8 (dispatch deals blocks round-robin over the XCDs); it is given filter
// 8·⌊(L/8)/B⌋ + L % 8, tile block (L/8) % B, so all of a filter's blocks share one XCD and its
// Kcat/Mcat are fetched into one L2 instead of eight. Placement only changes speed.
// Waves take tiles row-major over a trows × tcols grid.
// xcd_b = −1 (few filters, one per blockIdx.y): the tile grid is cut 2 × 4 into regions, block L
// takes region L % 8 (so XCD L % 8 does): each XCD's L2 then fetches half of Kcat and a quarter
// of Mcat instead of both whole (the fetch beyond Σ: 8 × (Kcat + Mcat) → 4 × Kcat + 2 × Mcat).
constexpr int kRegRows = 2, kRegCols = 4;
__host__ __device__ inline int region_tiles(int trows, int tcols) {  // the largest region's tiles
  return ((trows + kRegRows - 1) / kRegRows) * ((tcols + kRegCols - 1) / kRegCols);
}
// An explicit occupancy target (the one the registers allowed anyway: 2 waves/SIMD for the wide
// fp64 tile, 4–5 for the narrow one, 6–7 for fp32) makes the allocator keep the MFMA accumulators
// in VGPRs instead of AGPRs (no v_accvgpr_read before the Σ_in subtraction and the stores): swarm
// message 0.719 → 0.703 ms, N = 1024 fp64 pass 16.4 → 15.9 µs, fp32 unchanged
// (profiles/r3/p3r_vgpr_acc_ab.txt, two alternating runs each)
// KB: operand blocks of the rank (the Joseph form's instantiation: 2)
template <typename T, bool WIDE, int KB>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WIDE ? 2 : (sizeof(T) == 8 ? 4 : 6)))) void k_sigma_pass(PassArgs<T> A, int tcols, int xcd_b, int nf) {
  using Tile = PassTile<T, WIDE>;
  SIG_STAMP(0);
  if (kDiagBuild && (A.dbg & 1)) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  int fb = blockIdx.y, bx = blockIdx.x;
  if (xcd_b > 0) {
    const int L = blockIdx.x, j = L >> 3;
    fb = (L & 7) + 8 * (j / xcd_b);
    bx = j % xcd_b;
    if (fb >= nf) return;
  }
  const MsgDesc& d = A.desc[fb];
  constexpr bool kSym = sizeof(T) == 8;  // fp64: the symmetric tiles (SigmaTile64)
  __shared__ int cmap[4][64];  // per wave (fp32 patch): tile row / column → first position in U
  __shared__ double tT[kSym ? 4 : 1][kSym ? 16 * (WIDE ? 4 : 2) * kTS : 1];  // (SigmaTile64::kLds)
  const int lane = threadIdx.x & 63;
  const int trows = (A.n + Tile::kRows - 1) / Tile::kRows;
  // the wave's tile index, provably wave-uniform (readfirstlane): the buffer descriptors built
  // from it stay in SGPRs instead of a waterfall loop around every buffer access
  int t = __builtin_amdgcn_readfirstlane(bx * (blockDim.x >> 6) + (threadIdx.x >> 6));
  int tr = 0, tc = 0;
  bool ok;
  if constexpr (kSym) {
    // the upper tiles row-major; xcd_b < 0: XCD x takes the x-th eighth of them
    if (xcd_b < 0) {
      const int x = blockIdx.x & 7, w = (blockIdx.x >> 3) * (blockDim.x >> 6) + (threadIdx.x >> 6);
      const int T8 = sym_tiles<Tile::kCols>(trows, tcols);
      const int lo = x * T8 / 8, hi = (x + 1) * T8 / 8;
      t = __builtin_amdgcn_readfirstlane(lo + w);
      ok = t < hi;
    } else {
      ok = true;
    }
    ok = ok && sym_tile<Tile::kCols>(t, trows, tcols, tr, tc);
  } else if (xcd_b < 0) {
    const int x = blockIdx.x & 7, w = (blockIdx.x >> 3) * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int hx = x / kRegCols, qx = x % kRegCols;
    const int r0 = hx * trows / kRegRows, r1 = (hx + 1) * trows / kRegRows;
    const int c0 = qx * tcols / kRegCols, c1 = (qx + 1) * tcols / kRegCols;
    const int cw = c1 - c0;
    const int tt = __builtin_amdgcn_readfirstlane(w);
    ok = tt < (r1 - r0) * cw;
    tr = r0 + tt / cw;
    tc = c0 + tt % cw;
  } else {
    ok = t < trows * tcols;
    tr = t / tcols;
    tc = t - tr * tcols;
  }
  if constexpr (std::is_same<Tile, SigmaTile<float>>::value) {
    // fp32: the operand loads depend only on the filter and the tile, so they go out before the
    // descriptor's scalar round trips (flags, parity, m, then the Σ pointer it selects) instead of
    // behind them (≈ 0.3 µs of a 9 µs pass, tools/pass_lab.hip)
    if (!ok) return;
    const int f = A.f0 + fb;
    // the patch test's record flags of both parities, issued with the operands (not a scalar round
    // trip behind the descriptor's parity: that wait cost ≈ 0.4 µs of the pass)
    const int rf0 = A.rec[f].flags, rf1 = A.rec[A.rec_stride + f].flags;
    F32TileRegs g;
    Tile::load_ops(g, A.kcat + f * A.km_stride, A.mcat + f * A.km_stride, A.n, A.ldk,
                   tr * Tile::kRows, tc * Tile::kCols, lane);
    __builtin_amdgcn_sched_barrier(0);
    if (d.flags & kActive) {
      SIG_STAMP(1);
      const int kw = ((2 + ((d.flags & kJoseph) ? 4 : 2) * d.m + 3) / 4) * 4;
      Tile::load_sig(g, A.sig[d.parity] + f * A.sig_stride, A.n, A.ld, tr * Tile::kRows,
                     tc * Tile::kCols, lane);
      // the fp32 patch (see k_patch_stage): the chain's fp64 Σ[U, U] over this tile's entries
      // there, for the chunks that initialised a landmark (the pass's 1e7 − (1e7 − δ) loses δ)
      const ChunkRec* rec = A.rec + static_cast<size_t>(d.parity) * A.rec_stride + f;
      const int* pm = nullptr;
      if ((d.parity ? rf1 : rf0) & kPendValid) {  // wave-uniform
        const int R0 = tr * Tile::kRows, C0 = tc * Tile::kCols;
        int* map = cmap[threadIdx.x >> 6];
        map[lane] = kMaxU;
        const int nu = rec->nu, u = rec->u[min(lane, kMaxU - 1)];
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        if (lane < nu && u >= R0 && u < R0 + 32) atomicMin(&map[u - R0], lane);
        if (lane < nu && u >= C0 && u < C0 + 32) atomicMin(&map[32 + u - C0], lane);
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
        pm = map;
      }
      if constexpr (KB == 1)
        Tile::finish(g, A.sig[d.parity ^ 1] + f * A.sig_stride, A.n, A.ld, kw,
                     (d.flags & kFirst) != 0, A.q, tr * Tile::kRows, tc * Tile::kCols, lane, pm,
                     rec);
      else
        Tile::finish2(g, A.kcat + f * A.km_stride, A.mcat + f * A.km_stride, A.ldk,
                      A.sig[d.parity ^ 1] + f * A.sig_stride, A.n, A.ld, kw,
                      (d.flags & kFirst) != 0, A.q, tr * Tile::kRows, tc * Tile::kCols, lane, pm,
                      rec);
    }
  } else if ((d.flags & kActive) && ok) {
    SIG_STAMP(1);
    const int f = A.f0 + fb;
    if ((kDiagBuild && (A.dbg & 8)) && t == 0 && lane == 0) dbg_seq_check(A, 2, f, A.seq + 1u);
    // this filter's rank (Joseph: K·M and V·Kᵀ per marker); rows beyond are stale
    const int kw = ((2 + ((d.flags & kJoseph) ? 4 : 2) * d.m + 3) / 4) * 4;
    Tile::template run<KB>(A.sig[d.parity] + f * A.sig_stride, A.sig[d.parity ^ 1] + f * A.sig_stride,
              A.kcat + f * A.km_stride, A.mcat + f * A.km_stride, A.n, A.ld, A.ldk, kw,
              (d.flags & kFirst) != 0, A.q, tr * Tile::kRows, tc * Tile::kCols, lane,
              tT[threadIdx.x >> 6]);
  }
  if (kDiagBuild && (A.dbg & 2)) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  SIG_STAMP(3);
}


// Right behind the Σ pass on its stream, for chunks that stage (kStageOut, either dtype): the
// rebuild operands of the filter's chunk after next (StageRec), gathered from the Σ_out / x_out
// just completed — off the chain's critical path, where the same gather at the chain's start cost
// ≈ 10 µs of a 47 µs message (≈ 1 900 scattered lines through one CU). One workgroup per filter.
// The fp32 patch this kernel also did until round 4 — the chain's fp64 Σ[U, U] (rec->Pend, rounded
// once) over the pass's values, because the pass's 1e7 − (1e7 − δ) at a first sighting (the
// reference's prior, slam.cpp:130) loses δ in fp32 — now happens in the pass's tiles
// (SigmaTile<float>::finish), so Σ_out is already patched here; the patch branches below are off.
template <typename T>
__global__ __launch_bounds__(256) void k_patch_stage(PassArgs<T> A) {
  // (the fp32 patch itself now happens in the Σ pass's tiles, SigmaTile<float>::finish: the
  // staging below reads the patched Σ_out)
  constexpr bool kPatch = false;
  const MsgDesc& d = A.desc[blockIdx.x];
  const int flags = d.flags;
  if (!(flags & kActive)) return;
  const bool stage = (flags & kStageOut) != 0;
  if (!kPatch && !stage) return;
  const int f = A.f0 + blockIdx.x;
  const int tid = threadIdx.x;
  const ChunkRec* rec = A.rec + static_cast<size_t>(d.parity) * A.rec_stride + f;
  // the chain wrote Pend only for chunks that initialised a landmark (k_chain: `pend`)
  const bool patch = kPatch && (rec->flags & kPendValid);
  if (!patch && !stage) return;
  __shared__ int su[kMaxU];
  __shared__ int sfirst[kMaxU];           // position is its index's first in this chunk's U
  __shared__ double spend[kMaxU][kMaxU + 1];
  __shared__ int sgu[kStW], sgp[kStW];    // staged chain's U and U' (columns)
  __shared__ int sgfu[kStW], sgfp[kStW];  // their first positions in this chunk's U (patched), −1
  // ---- one global round trip: the record's block and U, the staged chunks' ids ----
  constexpr int kPer = (kMaxU * kMaxU + 255) / 256;
  double pv[kPer];
  if (patch) {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int e = min(tid + 256 * i, kMaxU * kMaxU - 1);
      pv[i] = rec->Pend[e / kMaxU][e % kMaxU];
    }
  }
  const int nu = rec->nu;
  const int myu = rec->u[min(tid, kMaxU - 1)];
  // stage threads: a = tid (U of the chunk after next) or tid − 64 (U', the next chunk's)
  const bool isp = tid >= 64;
  const int sa = isp ? tid - 64 : tid;
  const int sm = isp ? d.stg_pm : d.stg_m;
  const int sid = (isp ? d.stg_pids : d.stg_ids)[min(max(sa - 3, 0) >> 1, kMaxChunk - 1)];
  if (tid < kMaxU) su[tid] = myu;
  if (patch) {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int e = tid + 256 * i;
      if (e < kMaxU * kMaxU) spend[e / kMaxU][e % kMaxU] = pv[i];
    }
  }
  __syncthreads();
  // ---- first positions: every lane takes all of U into registers (one LDS wait) ----
  int uall[kMaxU];
#pragma unroll
  for (int k = 0; k < kMaxU; ++k) uall[k] = su[k];
  if (tid < kMaxU) {
    bool fp = tid < nu;
#pragma unroll
    for (int k = 0; k < kMaxU; ++k) fp = fp && !(k < tid && uall[k] == myu);
    sfirst[tid] = fp;
  }
  if (stage && sa < kStW && (tid < kStW || (isp && tid < 64 + kStW))) {
    int col = 0;
    if (sa < 3) col = sa;
    else if (sa < 3 + 2 * sm && sa < kMaxU)
      // k_chain's A0 mapping: marker c → 3 + 2·id (+1), a bad id → slot 0's, padding → 0
      col = (sid < 0 || sid >= A.N ? 3 : 3 + 2 * sid) + ((sa - 3) & 1);
    int fpos = -1;  // the first position of col in this chunk's U = its patched entry
    if (patch) {
#pragma unroll
      for (int k = kMaxU - 1; k >= 0; --k) fpos = (k < nu && uall[k] == col) ? k : fpos;
    }
    (isp ? sgp : sgu)[sa] = col;
    (isp ? sgfp : sgfu)[sa] = fpos;
  }
  __syncthreads();
  T* S = A.sig[d.parity ^ 1] + f * A.sig_stride;
  if (patch) {
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
      const int e = tid + 256 * i, a = e / kMaxU, b = e % kMaxU;
      if (e < kMaxU * kMaxU && sfirst[a] && sfirst[b])
        S[static_cast<size_t>(su[a]) * A.ld + su[b]] = static_cast<T>(pv[i]);
    }
  }
  if (!stage) return;
  // ---- stage: the chunk after next's rebuild operands (the second global round trip) ----
  const double* xo = A.x[d.parity ^ 1] + f * A.x_stride;
  StageRec<T>* sg = A.stage + static_cast<size_t>(d.parity) * A.rec_stride + f;
  // Σ_out[r][c] as the chain would read it after the patch (the load of a patched entry races
  // the scatter above and is discarded)
  auto val = [&](int r, int fr, int c, int fc) -> T {
    const T g = S[static_cast<size_t>(r) * A.ld + c];
    return (patch && fr >= 0 && fc >= 0) ? static_cast<T>(spend[fr][fc]) : g;
  };
  constexpr int kSPer = (kStW * kStW + 255) / 256;  // 6
  T od[kSPer], orr[kSPer], oc[kSPer];
#pragma unroll
  for (int i = 0; i < kSPer; ++i) {
    const int e = min(tid + 256 * i, kStW * kStW - 1);
    const int a = min(e / kStW, kMaxU - 1), b = min(e % kStW, kMaxU - 1);
    od[i] = val(sgu[a], sgfu[a], sgu[b], sgfu[b]);
    orr[i] = val(sgu[a], sgfu[a], sgp[b], sgfp[b]);
    oc[i] = val(sgp[b], sgfp[b], sgu[a], sgfu[a]);
  }
  const int t = min(tid, kMaxU - 1);
  const int z = sgfu[0];  // position 0 of U is the pose θ column
  const T r0u = val(0, z, sgu[t], sgfu[t]), c0u = val(sgu[t], sgfu[t], 0, z);
  const T r0p = val(0, z, sgp[t], sgfp[t]), c0p = val(sgp[t], sgfp[t], 0, z);
  const double xg = xo[sgu[t]];
  if (tid < kStW) {
    sg->r0u[tid] = static_cast<double>(r0u);
    sg->c0u[tid] = static_cast<double>(c0u);
    sg->r0p[tid] = static_cast<double>(r0p);
    sg->c0p[tid] = static_cast<double>(c0p);
    sg->xg[tid] = xg;
  }
#pragma unroll
  for (int i = 0; i < kSPer; ++i) {
    const int e = tid + 256 * i;
    if (e < kStW * kStW) {
      sg->v[0][e] = od[i];
      sg->v[1][e] = orr[i];
      sg->v[2][e] = oc[i];
    }
  }
}

// Σ-pass epoch for the chains on the other stream, launched right behind the Σ pass on its stream:
// the kernel boundary's release has written the pass's Σ_out (and the factor kernel's x, Kcat,
// Mcat) back before this store, so the pass itself keeps plain stores and no per-block release.
__global__ void k_sigma_epoch(unsigned* sync, unsigned epoch) {
  if (threadIdx.x == 0) epoch_store(sync + kSyncSigma, epoch);
}

// ---- association ------------------------------------------------------------------------------
// slam.cpp:344-440 for the marker in desc.z[0]: d_k = νᵀψ_k⁻¹ν over the known landmarks k < counter
// (predict folded in when pending), the new slot's d forced to the gate (:406-408), first-index
// argmin (arma::index_min), then commit (new landmark written into x_in, counter++) or roll back.
constexpr int kAssocThreads = 1024;  // one known landmark per lane up to counter 1024: the gathers
                                     // of every landmark in flight in one round
template <typename T>
__global__ __launch_bounds__(kAssocThreads) void k_assoc(PassArgs<T> A) {
  __shared__ double s_pose[3], s_a[2], s_P33[3][3];
  __shared__ double s_bd[kAssocThreads / 64];
  __shared__ int s_bk[kAssocThreads / 64];
  __shared__ int s_abort;
  const MsgDesc& d = A.desc[blockIdx.y];
  if (!(d.flags & kActive) || d.m == 0) return;
  const int f = A.f0 + blockIdx.y;
  const int tid = threadIdx.x;
  const int ld = A.ld;
  const T* S = A.sig[d.parity] + f * A.sig_stride;
  double* x = A.x[d.parity] + f * A.x_stride;
  FilterCtl* ctl = A.ctl + f;
  // device epochs: Σ_in and x are the last Σ pass's (bulk stream), its epoch A.need_sigma
  if (A.polls && A.need_sigma) {
    if (tid == 0 && !epoch_wait_acquire(A.sync + kSyncSigma, A.need_sigma))
      flag_timeout(&ctl->status, A.fatal);
    __syncthreads();
  }
  const unsigned s = ctl->counter;
  const int slot = d.assoc_slot;
  if (tid == 0) {
    double a1, a2;
    predicted_pose(ctl->tmo, d, x, s_pose, &a1, &a2);
    s_a[0] = a1;
    s_a[1] = a2;
    double raw[3][3];
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) raw[a][b] = static_cast<double>(S[a * ld + b]);
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) {
        const double aa = (d.flags & kFirst) ? alpha_of(a, a1, a2) : 0.0;
        const double ab = (d.flags & kFirst) ? alpha_of(b, a1, a2) : 0.0;
        double v = raw[a][b] + aa * raw[0][b];
        v = v + (raw[a][0] + aa * raw[0][0]) * ab;
        if ((d.flags & kFirst) && a == b) v += A.q;
        s_P33[a][b] = v;
      }
    s_abort = 0;
    if (s >= static_cast<unsigned>(A.N)) {  // the reference indexes state(3+2·counter) out of range
      s_abort = 1;
      atomicOr(&ctl->status, EKF_FLAG_RANGE_D);
      ctl->assoc_j[slot] = -1;
      ctl->assoc_new[slot] = 0;
    }
  }
  __syncthreads();
  if (s_abort) return;
  const double z0 = d.z[0][0], z1 = d.z[0][1];
  const double a1 = s_a[0], a2 = s_a[1];
  const bool first = (d.flags & kFirst) != 0;
  double bestd = INFINITY;
  int bestk = INT_MAX;
  for (unsigned k = tid; k < s; k += blockDim.x) {
    const int j = 3 + 2 * static_cast<int>(k);
    double P[5][5];
    for (int a = 0; a < 3; ++a)
      for (int b = 0; b < 3; ++b) P[a][b] = s_P33[a][b];
    const double r0j0 = static_cast<double>(S[j]), r0j1 = static_cast<double>(S[j + 1]);
    for (int a = 0; a < 3; ++a) {
      const double aa = first ? alpha_of(a, a1, a2) : 0.0;
      P[a][3] = static_cast<double>(S[a * ld + j]) + aa * r0j0;
      P[a][4] = static_cast<double>(S[a * ld + j + 1]) + aa * r0j1;
    }
    for (int e = 0; e < 2; ++e) {
      const T* row = S + static_cast<size_t>(j + e) * ld;
      const double rj0 = static_cast<double>(row[0]);
      for (int b = 0; b < 3; ++b) {
        const double ab = first ? alpha_of(b, a1, a2) : 0.0;
        P[3 + e][b] = static_cast<double>(row[b]) + rj0 * ab;
      }
      P[3 + e][3] = static_cast<double>(row[j]);
      P[3 + e][4] = static_cast<double>(row[j + 1]);
    }
    const double dist = assoc_dist(P, s_pose, x[j], x[j + 1], z0, z1, A.r);
    if (dist < bestd) {  // strict: first index kept, NaN never selected
      bestd = dist;
      bestk = static_cast<int>(k);
    }
  }
  wave_argmin(bestd, bestk);  // 64 lanes, ties → lower index (DPP, ekf_math.hpp)
  const int wv = tid >> 6;
  if ((tid & 63) == 0) {
    s_bd[wv] = bestd;
    s_bk[wv] = bestk;
  }
  __syncthreads();
  if (tid == 0) {
    for (int w = 1; w < static_cast<int>(blockDim.x >> 6); ++w)
      if (s_bd[w] < bestd || (s_bd[w] == bestd && s_bk[w] < bestk)) {
        bestd = s_bd[w];
        bestk = s_bk[w];
      }
    // the new slot (index s, d = gate) wins only over a strictly larger existing minimum
    if (!(bestd <= A.gate)) {
      const int js = 3 + 2 * static_cast<int>(s);
      x[js] = s_pose[1] + z0 * cos(z1 + s_pose[0]);      // slam.cpp:351-354
      x[js + 1] = s_pose[2] + z0 * sin(z1 + s_pose[0]);
      ctl->counter = s + 1;
      ctl->assoc_j[slot] = static_cast<int>(s);
      ctl->assoc_new[slot] = 1;
    } else {
      ctl->assoc_j[slot] = bestk;
      ctl->assoc_new[slot] = 0;
    }
  }
}

template <typename T>
__global__ void k_posterior(PassArgs<T> A, int nf) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nf) return;
  const MsgDesc& d = A.desc[k];
  if (!(d.flags & kActive)) return;
  const int f = A.f0 + k;
  const double* x = A.x[d.parity] + f * A.x_stride;
  FilterCtl* ctl = A.ctl + f;
  const Pose2 tmo = compose(Pose2{x[0], x[1], x[2]}, inverse(Pose2{d.odom[0], d.odom[1], d.odom[2]}));
  ctl->tmo[0] = tmo.theta;
  ctl->tmo[1] = tmo.x;
  ctl->tmo[2] = tmo.y;
}

template <typename T>
__global__ void k_init_diag(T* sig, size_t stride, int n, int ld, double v, int nf) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x + 3;
  if (i >= n) return;
  for (int f = blockIdx.y; f < nf; f += gridDim.y)
    sig[f * stride + static_cast<size_t>(i) * ld + i] = static_cast<T>(v);
}

// dev only (PassArgs::dbg & 16): one workgroup per filter sums what the surrounding kernels left in
// memory (launch_dbg_sum's kinds), in stream order
template <typename T>
__global__ __launch_bounds__(256) void k_dbg_sum(PassArgs<T> A, int kind, int nf) {
  const int fb = blockIdx.x;
  if (fb >= nf) return;
  const MsgDesc& d = A.desc[fb];
  if (!(d.flags & kActive)) return;
  const int f = A.f0 + fb, p = d.parity, n = A.n, tid = threadIdx.x;
  unsigned long long s[6] = {0, 0, 0, 0, 0, 0};
  if (kind == 1) {
    const double* xo = A.x[p ^ 1] + f * A.x_stride;
    for (int i = tid; i < n; i += 256) s[0] += dbits(xo[i]);
    const int kw = ((2 + ((d.flags & kJoseph) ? 4 : 2) * d.m + 3) / 4) * 4;
    const T* kc = A.kcat + f * A.km_stride;
    const T* mc = A.mcat + f * A.km_stride;
    for (int e = tid; e < kw * n; e += 256) {
      const size_t o = static_cast<size_t>(e / n) * A.ldk + e % n;
      s[1] += dbits(kc[o]);
      s[2] += dbits(mc[o]);
    }
  } else if (kind == 2) {
    const T* so = A.sig[p ^ 1] + f * A.sig_stride;
    for (int e = tid; e < n * n; e += 256) s[0] += dbits(so[static_cast<size_t>(e / n) * A.ld + e % n]);
  } else {
    const T* sp = A.sig[p ^ 1] + f * A.sig_stride;
    const T* si = A.sig[p] + f * A.sig_stride;
    for (int e = tid; e < n * n; e += 256) {
      const size_t o = static_cast<size_t>(e / n) * A.ld + e % n;
      s[0] += dbits(sp[o]);
      s[4] += dbits(si[o]);
    }
    const double* xp = A.x[p ^ 1] + f * A.x_stride;
    const double* xi = A.x[p] + f * A.x_stride;
    for (int i = tid; i < n; i += 256) {
      s[1] += dbits(xp[i]);
      s[5] += dbits(xi[i]);
    }
    const unsigned long long* rw = reinterpret_cast<const unsigned long long*>(
        A.rec + static_cast<size_t>(p ^ 1) * A.rec_stride + f);
    for (int e = tid; e < static_cast<int>(sizeof(ChunkRec) / 8); e += 256) s[2] += rw[e];
    if (tid < 3) s[3] += dbits(A.ctl[f].tmo[tid]);
  }
#pragma unroll
  for (int k = 0; k < 6; ++k)
    if (s[k]) dlog_add(A, kind, A.seq, f, k, s[k]);
}

template <typename T>
hipError_t launch_dbg_sum(const PassArgs<T>& a, int nf, int kind, hipStream_t s) {
  hipLaunchKernelGGL(k_dbg_sum<T>, dim3(nf), dim3(256), 0, s, a, kind, nf);
  return hipGetLastError();
}
template hipError_t launch_dbg_sum<double>(const PassArgs<double>&, int, int, hipStream_t);
template hipError_t launch_dbg_sum<float>(const PassArgs<float>&, int, int, hipStream_t);

// ---- launchers ------------------------------------------------------------------------------
// With events, the launch carries them in its dispatch (hipExtLaunchKernelGGL): they time the
// kernel's own execution, not the queueing / dispatch latency around it.
template <typename K, typename... Args>
void launch(K kernel, dim3 grid, dim3 block, hipStream_t s, hipEvent_t e0, hipEvent_t e1,
            Args... args) {
  if (e0 && e1)
    hipExtLaunchKernelGGL(kernel, grid, block, 0, s, e0, e1, 0, args...);
  else
    hipLaunchKernelGGL(kernel, grid, block, 0, s, args...);
}

template <typename T>
hipError_t launch_chain(const PassArgs<T>& a, int nf, int nchunks, hipStream_t s, hipEvent_t e0,
                        hipEvent_t e1) {
  // (the Joseph form's instantiation: a handle's chunks are all of its form, ekf_set_joseph)
  launch(a.joseph ? k_chain<T, true> : k_chain<T, false>, dim3(1, nf), dim3(kChainThreads), s, e0,
         e1, a, nchunks);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_factors(const PassArgs<T>& a, int nf, hipStream_t s, hipEvent_t e0,
                          hipEvent_t e1) {
  const int per_filter = (factor_waves(a) + 3) / 4;
  // (the Joseph form's instantiation: Z's 4m columns; a handle's chunks are all of its form)
  auto k = a.joseph ? k_factors<T, true> : k_factors<T, false>;
  if (nf >= 16) {  // XCD-aware 1-D grid, as the swarm's Σ pass
    launch(k, dim3(8 * ((nf + 7) / 8) * per_filter), dim3(256), s, e0, e1, a, per_filter, nf);
  } else {
    launch(k, dim3(per_filter, nf), dim3(256), s, e0, e1, a, 0, nf);
  }
  return hipGetLastError();
}

template <typename T>
hipError_t launch_sigma_pass(const PassArgs<T>& a, int nf, bool publish, bool stage, hipStream_t s,
                             hipEvent_t e0, hipEvent_t e1) {
  constexpr int wpb = 4;  // waves per workgroup
  // the tiles per filter: all of them, or (fp64, symmetric) those on or above the diagonal
  auto tiles = [](int trows, int tcols, auto tile) {
    using Tile = decltype(tile);
    return sizeof(T) == 8 ? sym_tiles<Tile::kCols>(trows, tcols) : trows * tcols;
  };
  if (nf >= 16) {  // XCD-aware 1-D grid (see k_sigma_pass), wide fp64 tiles
    using Tile = PassTile<T, true>;
    const int trows = (a.n + Tile::kRows - 1) / Tile::kRows;
    const int tcols = (a.n + Tile::kCols - 1) / Tile::kCols;
    const int per_filter = (tiles(trows, tcols, Tile{}) + wpb - 1) / wpb;
    const dim3 grid(8 * ((nf + 7) / 8) * per_filter);
    launch(a.joseph ? k_sigma_pass<T, true, 2> : k_sigma_pass<T, true, 1>, grid, dim3(64 * wpb), s, e0, e1, a, tcols, per_filter, nf);
  } else {
    using Tile = PassTile<T, false>;
    const int trows = (a.n + Tile::kRows - 1) / Tile::kRows;
    const int tcols = (a.n + Tile::kCols - 1) / Tile::kCols;
    if (trows >= 2 * kRegRows && tcols >= 2 * kRegCols) {  // XCD regions (k_sigma_pass)
      const int per_x = sizeof(T) == 8 ? (tiles(trows, tcols, Tile{}) + 7) / 8 : region_tiles(trows, tcols);
      const dim3 grid(8 * ((per_x + wpb - 1) / wpb), nf);
      launch(a.joseph ? k_sigma_pass<T, false, 2> : k_sigma_pass<T, false, 1>, grid, dim3(64 * wpb), s, e0, e1, a, tcols, -1, nf);
    } else {
      const int per_filter = (tiles(trows, tcols, Tile{}) + wpb - 1) / wpb;
      const dim3 grid(per_filter, nf);
      launch(a.joseph ? k_sigma_pass<T, false, 2> : k_sigma_pass<T, false, 1>, grid, dim3(64 * wpb), s, e0, e1, a, tcols, 0, nf);
    }
  }
  if (stage) hipLaunchKernelGGL(k_patch_stage<T>, dim3(nf), dim3(256), 0, s, a);
  // the pass's epoch (otherwise published by the next chunk's factor kernel, PassArgs::pub_sigma)
  if ((publish && a.polls) || (a.dbg & 4))
    hipLaunchKernelGGL(k_sigma_epoch, dim3(1), dim3(64), 0, s, a.sync, a.seq + 1u);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_assoc(const PassArgs<T>& a, int nf, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
  launch(k_assoc<T>, dim3(1, nf), dim3(kAssocThreads), s, e0, e1, a);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_posterior(const PassArgs<T>& a, int nf, hipStream_t s) {
  hipLaunchKernelGGL(k_posterior<T>, dim3((nf + 63) / 64), dim3(64), 0, s, a, nf);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_init_diag(T* sig, size_t stride, int n, int ld, double v, int nf, hipStream_t s) {
  hipLaunchKernelGGL(k_init_diag<T>, dim3((n + 255) / 256, nf < 65535 ? nf : 65535), dim3(256), 0,
                     s, sig, stride, n, ld, v, nf);
  return hipGetLastError();
}

// Diagnostics (ekf_debug_poison_lds): overwrite a workgroup's whole LDS allocation with a NaN bit
// pattern. Launched over every CU several times, it leaves LDS the way an arbitrary previous kernel
// may, so a kernel that reads LDS it never wrote shows it deterministically (tests/).
__global__ __launch_bounds__(256) void k_poison_lds(unsigned long long pattern) {
  extern __shared__ unsigned long long lds_poison[];
  for (int e = threadIdx.x; e < kPoisonLdsBytes / 8; e += blockDim.x) lds_poison[e] = pattern;
  __syncthreads();
  // keep the stores: one lane publishes a word the compiler cannot prove dead
  if (threadIdx.x == 0 && lds_poison[blockIdx.x % (kPoisonLdsBytes / 8)] == 0x1ull)
    lds_poison[0] = 0;
}

hipError_t launch_poison_lds(unsigned long long pattern, int n_blocks, hipStream_t s) {
  hipLaunchKernelGGL(k_poison_lds, dim3(n_blocks), dim3(256), kPoisonLdsBytes, s, pattern);
  return hipGetLastError();
}

#define EKF_INSTANTIATE(T)                                                              \
  template hipError_t launch_chain<T>(const PassArgs<T>&, int, int, hipStream_t, hipEvent_t,        \
                                      hipEvent_t);                                                 \
  template hipError_t launch_factors<T>(const PassArgs<T>&, int, hipStream_t, hipEvent_t,          \
                                        hipEvent_t);                                               \
  template hipError_t launch_sigma_pass<T>(const PassArgs<T>&, int, bool, bool, hipStream_t, hipEvent_t, \
                                           hipEvent_t);                                            \
  template hipError_t launch_assoc<T>(const PassArgs<T>&, int, hipStream_t, hipEvent_t, hipEvent_t); \
  template hipError_t launch_posterior<T>(const PassArgs<T>&, int, hipStream_t);              \
  template hipError_t launch_init_diag<T>(T*, size_t, int, int, double, int, hipStream_t);
EKF_INSTANTIATE(double)
EKF_INSTANTIATE(float)

}  // namespace ekfslam

