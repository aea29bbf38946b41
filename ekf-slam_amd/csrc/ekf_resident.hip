// Register-resident filter kernel (gfx950) for small maps: n = 3 + 2N ≤ kResidentMaxN, fp64.
//
// The low-rank pipeline of ekf_kernels.hip (chain → factors → Σ pass per chunk, an association
// kernel per marker) is built for covariances that live in HBM. At the reference's own map size
// (N = 50 slots, n = 103: basic_world and the rosbag drive, BASELINE configs[0] and [4]) the whole
// Σ is 83 KB, and that pipeline is launch- and hand-off-bound (≈ 94 µs per associated marker).
// Here one 256-thread workgroup (4 waves) owns one filter for an entire upload (every message of a
// replay): Σ stays in VGPRs (wave w holds rows w, w+4, …; lane ℓ holds columns ℓ, ℓ+64), x with it,
// and each correction is
//   gather   the owners of rows / columns {θ, x, y, jx, jy} write them to LDS (10·n doubles);
//   barrier  (one per correction: the gather buffers are double-buffered);
//   update   every thread forms ẑ, H, S = HΣHᵀ + R, S⁻¹, ν from the gathered values (the same
//            operands in every thread, so the same bits) and applies Σ ← Σ − K·(HΣ) and x += Kν
//            to the elements it owns: 2 FMAs per element, no LDS traffic for Σ itself.
// The Mahalanobis association of a marker (slam.cpp:344-440) is one wavefront: lane k scores
// landmark k from the gathered pose rows / columns, the 2×2 landmark blocks and x, then a
// 64-lane shuffle argmin (first index wins, like arma::index_min).
//
// Numerics follow the chain kernel's helpers (range_bearing, inv2, rank2_sub, normalize_angle_near)
// and k_assoc's distance expression, so decisions match the HBM pipeline's; Σ differs from it by
// summation order only (Σ_ij − K_i0·M_0j − K_i1·M_1j as two FMAs; tests/test_gpu_resident.py: both
// paths against the oracle).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <climits>

#include "ekf_device.hpp"
#include "ekf_launch.hpp"
#include "ekf_math.hpp"
#include "geom.hpp"

namespace ekfslam {

// Diagnostic build only (libekfslam_diag.so, tools/resident_stamps.py): s_memtime of thread 0 of
// the first workgroup at RS_STAMP points, 8 slots per correction for the first 64 corrections.
#ifdef EKF_DIAG_STAMPS
__device__ unsigned long long g_res_stamps[512];
#define RS_STAMP(k, i)                                                        \
  do {                                                                        \
    if (blockIdx.x == 0 && threadIdx.x == 0 && (k) < 64)                      \
      g_res_stamps[8 * (k) + (i)] = __builtin_amdgcn_s_memtime();             \
  } while (0)
}  // namespace ekfslam
extern "C" int ekfslam_res_read_stamps(unsigned long long* out, int n) {
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(ekfslam::g_res_stamps),
                             sizeof(unsigned long long) * (n < 512 ? n : 512)) == hipSuccess ? 0 : -5;
}
namespace ekfslam {
#else
#define RS_STAMP(k, i) \
  do {                 \
  } while (0)
#endif

namespace {

typedef unsigned u2 __attribute__((ext_vector_type(2)));
// a voffset past the descriptor's num_records: the access is dropped (loads return 0); the range
// check is on voffset, so rows past n (the SGPR offset) must use it too
constexpr int kOOB = 0x7ffffff0;


// The prefix of a MsgDesc the kernel reads (m … z), staged in LDS a block of plan entries at a time.
struct alignas(16) ResMsg {
  int m, flags, parity, assoc_slot;
  double odom[3];
  int prev_m, pad1;
  int ids[kMaxChunk];
  double z[kMaxChunk][2];
};
static_assert(offsetof(ResMsg, odom) == offsetof(MsgDesc, odom) &&
                  offsetof(ResMsg, ids) == offsetof(MsgDesc, ids) &&
                  offsetof(ResMsg, z) == offsetof(MsgDesc, z) && sizeof(ResMsg) % 16 == 0,
              "ResMsg is MsgDesc's prefix");
constexpr int kMsgQ = sizeof(ResMsg) / 16;  // 16-byte pieces per staged descriptor
constexpr int kBlk = 16;                    // plan entries staged per block

template <int W, int RS, int CS>
struct ResShared {
  ResMsg msg[kBlk];
  int kind[kBlk];  // the entry's kind, −1: it does not name this filter
  double grow[2][5][64 * CS];  // Σ[idx_a][c]  (idx = {0, 1, 2, j, j+1})
  double gcol[2][5][W * RS];   // Σ[r][idx_a]
  double gx[2][8];             // x[idx_a]
  double blk[(W * RS) / 2][4];  // association: Σ[jk..jk+1][jk..jk+1] of landmark k
  double xall[W * RS];          // association: x
  int dec[2];                   // association decision: slot j, is_new
  int decj[kMaxAssoc], decn[kMaxAssoc];  // decisions by slot, stored to FilterCtl at the end
  double junk[64];                        // sink of the branch-free block gather
  double kw[W][RS][4];          // per wave: K[row(s)] (and Joseph: (Σ·Hᵀ)[row(s)]), wave-private
};

__device__ __forceinline__ int pos5(int r, int j) {
  return r < 3 ? r : (r == j ? 3 : (r == j + 1 ? 4 : -1));
}

}  // namespace

// One workgroup per filter flo + blockIdx.x; walks the whole plan (PlanEntry list, in order) and
// applies the entries that name its filter. Σ / x are loaded on the first active entry from the
// entry's parity and written back once, to the parity the host's plan ends on.
template <int W, int RS, int CS, bool JOSEPH>
__global__ __launch_bounds__(W * 64) void k_resident(PassArgs<double> A, const PlanEntry* plan,
                                                     int nplan, int flo) {
  constexpr int kRW = W;
  static_assert(RS <= 32 && RS <= 64, "jump-table gather covers 32 slots; x is lane-distributed");
  __shared__ ResShared<W, RS, CS> sh;
  const int f = flo + blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform: row offsets in SGPRs
  const int n = A.n, ld = A.ld, N = A.N;
  FilterCtl* ctl = A.ctl + f;

  double sg[RS][CS];
  // x and per-row scalars live lane-distributed: lane s < RS holds row w + kRW·s (its own row rl)
  const int rl = w + kRW * (lane < RS ? lane : RS - 1);
  const bool rown = lane < RS;
  double xl = 0.0;
  double tmo[3];
  // posterior deferred to the next gather of the pose (the next message's predict gathers it
  // anyway; nothing moves the pose in between): one barrier per message instead of two
  bool post = false;
  double podom[3] = {0.0, 0.0, 0.0};
  unsigned counter = 0, status = 0;
  unsigned long long dslots = 0;  // association slots decided in this launch (sh.decj/decn)
  int par = -1;          // current parity (−1: not loaded yet)
  bool dirty = false;    // Σ / x changed (a chunk entry ran)
  int b = 0;             // gather buffer

  // wq: the wave index re-materialised per correction (an opaque copy), so the compiler recomputes
  // the per-row conditions in a few scalar ops instead of hoisting them out of the plan loop into
  // (spilled) SGPRs
  int wq = w;
  auto row = [&](int s) __attribute__((always_inline)) { return wq + kRW * s; };
  auto col = [&](int t) __attribute__((always_inline)) { return lane + 64 * t; };

  // rows / columns idx_a with a ≥ amin (j < 0: pose only) and their x into gather buffer bb
  auto gather = [&](int bb, int j, int amin) __attribute__((always_inline)) {
    asm volatile("" : "+s"(wq));
    // rows: θ, x, y are slot 0 of waves 0-2; jx, jy sit in slot r / W of wave r % W, picked by
    // one jump-table switch each (a few scalar ops and one indirect branch: the scalar unit is
    // shared by the CU's waves, a test per slot costs more)
    if (amin == 0 && wq < 3) {
#pragma unroll
      for (int t = 0; t < CS; ++t) sh.grow[bb][wq][col(t)] = sg[0][t];
    }
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      const int r = j + e;
      if (j >= 0 && r < n && r % kRW == wq) {
        double* dst = &sh.grow[bb][3 + e][0];
        switch (r / kRW) {
#define RES_SLOT(q)                                                      \
  case q:                                                                \
    if constexpr (q < RS) {                                              \
      _Pragma("unroll") for (int t = 0; t < CS; ++t) dst[col(t)] = sg[q][t]; \
    }                                                                    \
    break;
          RES_SLOT(0) RES_SLOT(1) RES_SLOT(2) RES_SLOT(3) RES_SLOT(4) RES_SLOT(5) RES_SLOT(6)
          RES_SLOT(7) RES_SLOT(8) RES_SLOT(9) RES_SLOT(10) RES_SLOT(11) RES_SLOT(12) RES_SLOT(13)
          RES_SLOT(14) RES_SLOT(15) RES_SLOT(16) RES_SLOT(17) RES_SLOT(18) RES_SLOT(19)
          RES_SLOT(20) RES_SLOT(21) RES_SLOT(22) RES_SLOT(23) RES_SLOT(24) RES_SLOT(25)
          RES_SLOT(26) RES_SLOT(27) RES_SLOT(28) RES_SLOT(29) RES_SLOT(30) RES_SLOT(31)
#undef RES_SLOT
          default:
            break;
        }
      }
    }
    {
      const int a = pos5(rl, j);
      if (rown && a >= amin && rl < n) sh.gx[bb][a] = xl;
    }
#pragma unroll
    for (int t = 0; t < CS; ++t) {
      const int c = col(t), a = pos5(c, j);
      if (a >= amin && c < n) {
#pragma unroll
        for (int s = 0; s < RS; ++s) sh.gcol[bb][a][row(s)] = sg[s][t];
      }
    }
  };
  // x[r] ← v on the owner of row r
  auto set_x = [&](int r, double v) __attribute__((always_inline)) {
    if (rown && rl == r) xl = v;
  };

  // One correction against landmark column j = 3 + 2·id (slam.cpp:219-267 / :443-488). The
  // gather of idx into buffer b is done and the barrier passed.
  // posterior t_map_odom = T(x, y, θ)·t_odom_robot⁻¹ (slam.cpp:273-291) from a gathered pose
  auto posterior_from = [&](double p0, double p1, double p2) __attribute__((always_inline)) {
    const Pose2 t = compose_sc(Pose2{p0, p1, p2}, inverse_sc(Pose2{podom[0], podom[1], podom[2]}));
    tmo[0] = t.theta;
    tmo[1] = t.x;
    tmo[2] = t.y;
    post = false;
  };
  auto posterior_now = [&]() __attribute__((always_inline)) {
    b ^= 1;
    if (rown && rl < 3) sh.gx[b][rl] = xl;
    __syncthreads();
    posterior_from(sh.gx[b][0], sh.gx[b][1], sh.gx[b][2]);
  };
  [[maybe_unused]] int ncorr = 0;  // corrections so far (diagnostic stamps)
  auto correct = [&](int j, double z0, double z1, bool noinit) __attribute__((always_inline)) {
    RS_STAMP(ncorr, 1);
    asm volatile("" : "+s"(wq));
    const double pose[3] = {sh.gx[b][0], sh.gx[b][1], sh.gx[b][2]};
    double lx = sh.gx[b][3], ly = sh.gx[b][4];
    if (!noinit && lx == 0.0 && ly == 0.0) {  // first sighting, slam.cpp:213-216
      double sn, cs;
      sincos(z1 + pose[0], &sn, &cs);
      lx = pose[1] + z0 * cs;
      ly = pose[2] + z0 * sn;
      set_x(j, lx);
      set_x(j + 1, ly);
    }
    double zhat[2], H0[5], H1[5], braw;
    bool bok;
    range_bearing(pose, lx, ly, zhat, H0, H1, &braw, &bok);
    if (!bok) zhat[1] = normalize_angle(braw);
    RS_STAMP(ncorr, 2);
    double mc0[CS], mc1[CS];  // (H·Σ)[:, c] of this lane's columns
#pragma unroll
    for (int t = 0; t < CS; ++t) {
      double m0 = 0.0, m1 = 0.0;
#pragma unroll
      for (int a = 0; a < 5; ++a) {
        const double v = sh.grow[b][a][col(t)];
        m0 += H0[a] * v;
        m1 += H1[a] * v;
      }
      mc0[t] = m0;
      mc1[t] = m1;
    }
    // S = (H·Σ)[:, idx]·Hᵀ + R (slam.cpp:252, left to right like arma); (H·Σ)[:, idx] from the
    // lanes that own those columns
    double Sm[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int bb = 0; bb < 5; ++bb) {
      const int c = bb < 3 ? bb : j + bb - 3;
      double v0 = mc0[0], v1 = mc1[0];
#pragma unroll
      for (int t = 1; t < CS; ++t)
        if ((c >> 6) == t) {
          v0 = mc0[t];
          v1 = mc1[t];
        }
      const double h0 = readlane_f64(v0, c & 63), h1 = readlane_f64(v1, c & 63);
      Sm[0] += h0 * H0[bb];
      Sm[1] += h0 * H1[bb];
      Sm[2] += h1 * H0[bb];
      Sm[3] += h1 * H1[bb];
    }
    Sm[0] += A.r;
    Sm[3] += A.r;
    double Si[4];
    if (!inv2(Sm, Si)) {  // arma::inv throws in the reference: skip the marker, flag it
      status |= EKF_FLAG_NUMERIC_D;
      return;
    }
    const double nv0 = z0 - zhat[0];
    bool nok;
    const double nn = normalize_angle_near(z1 - zhat[1], &nok);
    const double nv1 = nok ? nn : normalize_angle(z1 - zhat[1]);
    RS_STAMP(ncorr, 3);
    // K[rl] = (Σ·Hᵀ)[rl]·S⁻¹ on the lane that holds row rl, then every lane takes its rows' K
    double K0, K1, ka = 0.0, kb = 0.0;
    {
#pragma unroll
      for (int a = 0; a < 5; ++a) {
        const double v = sh.gcol[b][a][rl];
        ka += v * H0[a];
        kb += v * H1[a];
      }
      K0 = ka * Si[0] + kb * Si[2];
      K1 = ka * Si[1] + kb * Si[3];
    }
    // the wave's rows' K through its own LDS slots (one wave: LDS ops complete in issue order)
    if (rown) {
      sh.kw[w][lane][0] = K0;
      sh.kw[w][lane][1] = K1;
      sh.kw[w][lane][2] = ka;
      sh.kw[w][lane][3] = kb;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if constexpr (!JOSEPH) {  // Σ ← Σ − K·(HΣ), slam.cpp:264-265
#pragma unroll
      for (int s = 0; s < RS; ++s) {
        const double k0 = sh.kw[w][s][0], k1 = sh.kw[w][s][1];  // broadcast reads
#pragma unroll
        for (int t = 0; t < CS; ++t) sg[s][t] = fma(-k1, mc1[t], fma(-k0, mc0[t], sg[s][t]));
      }
    } else {
      // Joseph form (opt-in): Σ ← (I−KH)Σ(I−KH)ᵀ + KRKᵀ = Σ − K·(HΣ) − (ΣHᵀ)·Kᵀ + K·S·Kᵀ. Per
      // column c: K[c] from (ΣHᵀ)[c] (the gathered columns at row c) and u = S·K[c]ᵀ; then each
      // element takes Σ_rc − K_r·(M_c − u_c) − (ΣHᵀ)_r·K_cᵀ, four FMAs
      double kc0[CS], kc1[CS];
#pragma unroll
      for (int t = 0; t < CS; ++t) {
        const int c = min(col(t), kRW * RS - 1);  // columns ≥ n: never stored
        double pa = 0.0, pb = 0.0;
#pragma unroll
        for (int a = 0; a < 5; ++a) {
          const double v = sh.gcol[b][a][c];
          pa += v * H0[a];
          pb += v * H1[a];
        }
        kc0[t] = pa * Si[0] + pb * Si[2];
        kc1[t] = pa * Si[1] + pb * Si[3];
        mc0[t] -= Sm[0] * kc0[t] + Sm[1] * kc1[t];
        mc1[t] -= Sm[2] * kc0[t] + Sm[3] * kc1[t];
      }
#pragma unroll
      for (int s = 0; s < RS; ++s) {
        const double k0 = sh.kw[w][s][0], k1 = sh.kw[w][s][1];
        const double p0 = sh.kw[w][s][2], p1 = sh.kw[w][s][3];
#pragma unroll
        for (int t = 0; t < CS; ++t)
          sg[s][t] = fma(-p1, kc1[t], fma(-p0, kc0[t],
                         fma(-k1, mc1[t], fma(-k0, mc0[t], sg[s][t]))));
      }
    }
    double xt = xl + (K0 * nv0 + K1 * nv1);  // slam.cpp:261
    if (rl == 0) {                            // slam.cpp:267
      bool tok;
      const double tn = normalize_angle_near(xt, &tok);
      xt = tok ? tn : normalize_angle(xt);
    }
    xl = xt;
    RS_STAMP(ncorr, 4);
    ++ncorr;
  };

  for (int l0 = 0; l0 < nplan; l0 += kBlk) {
  // stage the block's descriptors: every thread fetches 16-byte pieces (plan entry → descriptor,
  // one dependent pair of loads per thread, all in flight together), one barrier
  const int nb = min(kBlk, nplan - l0);
  __syncthreads();  // the previous block's entries are consumed
  for (int t = tid; t < nb * kMsgQ; t += kRW * 64) {
    const int e = t / kMsgQ, q = t - e * kMsgQ;
    const PlanEntry L = plan[l0 + e];
    const bool mine = f >= L.f0 && f < L.f0 + L.nf;
    if (q == 0) sh.kind[e] = mine ? L.kind : -1;
    if (mine)
      reinterpret_cast<uint4*>(&sh.msg[e])[q] =
          reinterpret_cast<const uint4*>(A.desc + L.off + (f - L.f0))[q];
  }
  __syncthreads();
  for (int e = 0; e < nb; ++e) {
    const int kind = sh.kind[e];
    if (kind < 0) continue;
    const ResMsg& d = sh.msg[e];
    const int flags = d.flags;
    if (!(flags & kActive)) continue;
    const PlanEntry L{0, 0, 0, kind};
    if (par < 0) {  // first entry naming this filter: load it
      par = d.parity;
      const double* S = A.sig[par] + f * A.sig_stride;
      const double* X = A.x[par] + f * A.x_stride;
      // buffer loads: row offset in the SGPR operand, column in the VGPR one; out-of-range
      // rows / columns read 0 (the descriptor covers exactly n rows)
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(S), 0, n * ld * 8, 0x00020000);
#pragma unroll
      for (int s = 0; s < RS; ++s) {
        const int r = row(s);
#pragma unroll
        for (int t = 0; t < CS; ++t) {
          const int c = col(t);
          const double v = __builtin_bit_cast(
              double, __builtin_amdgcn_raw_buffer_load_b64(rs, r < n && c < n ? c * 8 : kOOB, r * ld * 8, 0));
          sg[s][t] = (r < n && c < n) ? v : 0.0;
        }
      }
      xl = (rown && rl < n) ? X[rl] : 0.0;
      tmo[0] = ctl->tmo[0];
      tmo[1] = ctl->tmo[1];
      tmo[2] = ctl->tmo[2];
      counter = ctl->counter;
    }
    if (post && L.kind != 2 && !(flags & kFirst)) posterior_now();  // corrections follow
    if (L.kind != 2) {
      if (flags & kFirst) {  // predict, slam.cpp:184-198: Σ = AΣAᵀ + Q̄, A = I + α·e0ᵀ
        b ^= 1;
        gather(b, -8, 0);
        __syncthreads();
        const double prev[3] = {sh.gx[b][0], sh.gx[b][1], sh.gx[b][2]};
        if (post) posterior_from(prev[0], prev[1], prev[2]);  // the last message's posterior
        const Pose2 cur = compose_sc(Pose2{tmo[0], tmo[1], tmo[2]},
                                     Pose2{d.odom[0], d.odom[1], d.odom[2]});
        const double a1 = -(cur.y - prev[2]), a2 = cur.x - prev[1];
        const double s00 = sh.grow[b][0][0];
#pragma unroll
        for (int s = 0; s < RS; ++s) {
          const int r = row(s);
          const double aa = alpha_of(r, a1, a2);
          const double cr0 = sh.gcol[b][0][r];  // Σ[r][0], broadcast
#pragma unroll
          for (int t = 0; t < CS; ++t) {
            const int c = col(t);
            const double ab = alpha_of(c, a1, a2);
            double v = sg[s][t] + aa * sh.grow[b][0][c];
            v = v + (cr0 + aa * s00) * ab;
            if (r == c && r < 3) v += A.q;
            sg[s][t] = v;
          }
        }
        set_x(0, normalize_angle(cur.theta));
        set_x(1, cur.x);
        set_x(2, cur.y);
      }
      if (L.kind == 0) {  // known association, slam.cpp:201-271
        for (int c = 0; c < d.m; ++c) {
          const int id = d.ids[c];
          if (id < 0 || id >= N) continue;  // validated on the host; never reached
          RS_STAMP(ncorr, 0);
          b ^= 1;
          gather(b, 3 + 2 * id, 0);
          RS_STAMP(ncorr, 5);
          __syncthreads();
          correct(3 + 2 * id, d.z[c][0], d.z[c][1], (flags & kNoInit) != 0);
        }
      } else if (d.m > 0) {  // association + correction, slam.cpp:344-488
        const double z0 = d.z[0][0], z1 = d.z[0][1];
        const int slot = d.assoc_slot;
        if (counter >= static_cast<unsigned>(N)) {  // the reference indexes out of range
          status |= EKF_FLAG_RANGE_D;
          if (tid == 0) {
            sh.decj[slot] = -1;
            sh.decn[slot] = 0;
          }
          dslots |= 1ull << slot;
        } else {
          RS_STAMP(ncorr, 0);
          b ^= 1;
          gather(b, -8, 0);  // pose rows / columns and pose x
          // landmark 2×2 blocks of the seen landmarks (rows < 3 + 2·counter): every (slot,
          // column) element stores — to its block entry when it is one, else to this lane's junk
          // slot. The row index is taken as a vector value (tid >> 6 unmerged), so the index
          // math runs on each SIMD's VALU, not on the CU's one scalar unit.
          {
            const int wv = static_cast<int>(threadIdx.x) >> 6;
            const int rmax = 3 + 2 * static_cast<int>(counter);
#pragma unroll
            for (int s = 0; s < RS; ++s) {
              if (row(s) >= rmax) break;  // rows grow with s
              const int r = wv + kRW * s;
              const int k = (r - 3) >> 1, e = (r - 3) & 1;
#pragma unroll
              for (int t = 0; t < CS; ++t) {
                const int dc = col(t) - (3 + 2 * k);
                const bool in = r >= 3 && (dc == 0 || dc == 1);
                *(in ? &sh.blk[k < 0 ? 0 : k][2 * e + dc] : &sh.junk[lane]) = sg[s][t];
              }
            }
          }
          if (rown && rl >= 3 && rl < n) sh.xall[rl] = xl;
          __syncthreads();
          RS_STAMP(ncorr, 6);
          if (w == 0) {
            const double pose[3] = {sh.gx[b][0], sh.gx[b][1], sh.gx[b][2]};
            double bestd = INFINITY;
            int bestk = INT_MAX;
            for (unsigned k = lane; k < counter; k += 64) {
              const int j = 3 + 2 * static_cast<int>(k);
              // Σ over {θ, x, y, j, j+1}, read where it is used
              auto P = [&](int a, int c) __attribute__((always_inline)) -> double {
                if (a < 3) return sh.grow[b][a][c < 3 ? c : j + c - 3];
                if (c < 3) return sh.gcol[b][c][j + a - 3];
                return sh.blk[k][2 * (a - 3) + (c - 3)];
              };
              double zhat[2], H0[5], H1[5], braw;
              bool bok;
              range_bearing(pose, sh.xall[j], sh.xall[j + 1], zhat, H0, H1, &braw, &bok);
              if (!bok) zhat[1] = normalize_angle(braw);
              double HP0[5], HP1[5];
#pragma unroll
              for (int bb = 0; bb < 5; ++bb) {
                double s0 = 0.0, s1 = 0.0;
#pragma unroll
                for (int a = 0; a < 5; ++a) {
                  const double v = P(a, bb);
                  s0 += H0[a] * v;
                  s1 += H1[a] * v;
                }
                HP0[bb] = s0;
                HP1[bb] = s1;
              }
              double psi[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
              for (int bb = 0; bb < 5; ++bb) {
                psi[0] += HP0[bb] * H0[bb];
                psi[1] += HP0[bb] * H1[bb];
                psi[2] += HP1[bb] * H0[bb];
                psi[3] += HP1[bb] * H1[bb];
              }
              psi[0] += A.r;
              psi[3] += A.r;
              const double nu0 = z0 - zhat[0];
              const double nu1 = normalize_angle(z1 - zhat[1]);
              double dist = NAN;
              const double det = psi[0] * psi[3] - psi[1] * psi[2];
              if (fabs(det) > 0.0) {  // (z_diffᵀ·ψ⁻¹)·z_diff, slam.cpp:401 (assoc_dist's form)
                const double t0 = nu0 * psi[3] - nu1 * psi[2];
                const double t1 = nu1 * psi[0] - nu0 * psi[1];
                dist = (t0 * nu0 + t1 * nu1) / det;
              }
              if (dist < bestd) {  // strict: first index kept, NaN never selected
                bestd = dist;
                bestk = static_cast<int>(k);
              }
            }
            wave_argmin(bestd, bestk);  // (DPP, ekf_math.hpp; every lane holds the result)
            if (lane == 0) {
              // the new slot (d = gate, slam.cpp:406-408) wins only over a larger minimum
              const bool nw = !(bestd <= A.gate);
              const int jsel = nw ? static_cast<int>(counter) : bestk;
              sh.dec[0] = jsel;
              sh.dec[1] = nw;
              sh.decj[slot] = jsel;
              sh.decn[slot] = nw;
            }
          }
          __syncthreads();
          dslots |= 1ull << slot;
          const int k = sh.dec[0];
          const int j = 3 + 2 * k;
          if (sh.dec[1]) {  // slam.cpp:351-356, kept (:421)
            const double p0 = sh.gx[b][0], p1 = sh.gx[b][1], p2 = sh.gx[b][2];
            double sn, cs;
            sincos(z1 + p0, &sn, &cs);
            set_x(j, p1 + z0 * cs);
            set_x(j + 1, p2 + z0 * sn);
            ++counter;
          }
          RS_STAMP(ncorr, 7);
          gather(b, j, 3);  // the pose rows / columns are in b already
          RS_STAMP(ncorr, 5);
          __syncthreads();
          correct(j, z0, z1, true);
        }
      }
      par ^= 1;
      dirty = true;
    }
    if ((flags & kLast) || L.kind == 2) {  // posterior, slam.cpp:273-291 (deferred)
      post = true;
      podom[0] = d.odom[0];
      podom[1] = d.odom[1];
      podom[2] = d.odom[2];
    }
  }
  }
  if (par < 0) return;  // the plan does not name this filter
  if (post) posterior_now();
  __syncthreads();  // the decisions in LDS
  if (tid < kMaxAssoc && (dslots >> tid & 1)) {
    ctl->assoc_j[tid] = sh.decj[tid];
    ctl->assoc_new[tid] = sh.decn[tid];
  }
  if (dirty) {
    double* S = A.sig[par] + f * A.sig_stride;
    double* X = A.x[par] + f * A.x_stride;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(S, 0, n * ld * 8, 0x00020000);
#pragma unroll
    for (int s = 0; s < RS; ++s) {
      const int r = row(s);
      if (r >= n) continue;
#pragma unroll
      for (int t = 0; t < CS; ++t) {
        const int c = col(t);  // columns ≥ n go out of the descriptor's range (dropped)
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, sg[s][t]), rs,
                                              c < n ? c * 8 : kOOB, r * ld * 8, 0);
      }
    }
    if (rown && rl < n) X[rl] = xl;
  }
  if (tid == 0) {
    ctl->tmo[0] = tmo[0];
    ctl->tmo[1] = tmo[1];
    ctl->tmo[2] = tmo[2];
    ctl->counter = counter;
    if (status) atomicOr(&ctl->status, status);
  }
}

hipError_t launch_resident(const PassArgs<double>& a, const PlanEntry* plan, int nplan, int flo,
                           int nfil, hipStream_t s, hipEvent_t e0, hipEvent_t e1) {
  if (a.n > kResidentMaxN || nfil <= 0) return hipErrorInvalidValue;
  const dim3 grid(nfil);
  auto go = [&](auto kernel, int waves) {
    const dim3 block(64 * waves);
    if (e0 && e1)
      hipExtLaunchKernelGGL(kernel, grid, block, 0, s, e0, e1, 0, a, plan, nplan, flo);
    else
      hipLaunchKernelGGL(kernel, grid, block, 0, s, a, plan, nplan, flo);
  };
  // 4 waves (one per SIMD): the per-correction scalar work (geometry, S, gather control) runs
  // once per wave on the CU's one scalar unit, so fewer, wider waves finish a step sooner
  // Joseph form is its own instantiation: the default update keeps its register budget
  if (a.n <= 64)
    a.joseph ? go(k_resident<4, 16, 1, true>, 4) : go(k_resident<4, 16, 1, false>, 4);
  else if (a.n <= 4 * 26)  // N = 50 (n = 103): no idle row slots
    a.joseph ? go(k_resident<4, 26, 2, true>, 4) : go(k_resident<4, 26, 2, false>, 4);
  else
    a.joseph ? go(k_resident<4, 32, 2, true>, 4) : go(k_resident<4, 32, 2, false>, 4);
  return hipGetLastError();
}

}  // namespace ekfslam
