// Device-side data layout shared by the kernels (ekf_kernels.hip) and the host runtime (ekf_api.cpp).
//
// HBM layout per filter f (row-major, fp64 or fp32 per ekf_config.dtype):
//   Σ[2]      : two n × ld ping-pong copies (ld = n rounded up to 128 bytes). One launch pair reads
//               Σ_in and writes Σ_out, so no workgroup ever reads a row another one is rewriting.
//   x[2]      : state, n doubles each (state math is always fp64).
//   Kcat,Mcat : KW × ldk low-rank factors of one chunk: Σ_out = Σ_in + Q − Kcatᵀ·Mcat.
//   FilterCtl : t_map_odom, counter_obstacles, status, association results.
#pragma once
#include <cstddef>
#include <cstdint>

namespace ekfslam {

constexpr int kMaxChunk = 16;                    // markers folded into one Σ pass (EKF_MAX_CHUNK)
constexpr int kMaxU = 3 + 2 * kMaxChunk;         // touched rows/cols of one chunk: pose + 2 per marker
constexpr int kMaxAssoc = 64;                    // association slots per filter per upload
constexpr int kZC = 2 * kMaxChunk;               // correction columns of Z / rows of Y
constexpr int kMaxJoseph = kMaxChunk;            // markers of a Joseph-form chunk (round 6: a whole
                                                 // message, one Σ pass); its row map Z holds K's and
                                                 // V's columns, 4 per marker
constexpr int kZJ = 4 * kMaxJoseph;              // the record's Z columns (Joseph: Z then Zv)
// rank of the fused update, padded to 4: 2 + 2m (simple form), 2 + 4m (Joseph form)
constexpr int kMaxKW = ((2 + 4 * kMaxJoseph + 3) / 4) * 4;

// Device epochs (unsigned words of the handle's sync buffer, each polled word on its own line):
constexpr int kSyncSigma = 0;    // epoch (seq + 1) of the last complete Σ pass (k_sigma_epoch)
constexpr int kSyncPlan = 32;    // (t, f) descriptors device replays have planned so far (a count;
                                 // its own 128-B line: the planner waves' fetch_adds do not contend
                                 // with the polls of the Σ epoch in word 0)
constexpr int kSyncChain = 64;   // [F]: epoch of each filter's last complete chain
constexpr int kSyncDbg = 48;     // dev only (PassArgs::dbg & 4): [0] chains, [1] factor kernels that
                                 // started before their producer's epoch was visible, [2] checks

// MsgDesc.flags
constexpr int kFirst = 1;    // chunk carries the predict (slam.cpp:184-198) for this message
constexpr int kLast = 2;     // chunk ends the message: posterior t_map_odom (slam.cpp:273-291)
constexpr int kNoInit = 4;   // association path: no first-sighting init in the correction
constexpr int kActive = 8;   // filter takes part in this launch
constexpr int kLook = 16;    // Σ_in not materialised yet: rebuild the chain's block from the
                             // previous chunk's Σ_in (other buffer) and ChunkRec
constexpr int kJoseph = 128; // Joseph-form Σ update (ekf_set_joseph): ≤ kMaxJoseph markers per
                             // chunk, the factor rank 2 + 4m (K·M and (ΣHᵀ − K·S)·Kᵀ, see k_chain)
constexpr int kStageOut = 256;  // behind this chunk's Σ pass (k_patch_stage): gather the rebuild
                                // operands of the filter's chunk after next (stg_*) into StageRec
constexpr int kStageIn = 512;   // kLook chain: read its rebuild operands from StageRec (contiguous)
                                // instead of gathering them from Σ_in' at the chunk's start
constexpr int kStW = kMaxU + 1;  // chain block stride (entry e = a·kStW + b)
constexpr int kPendValid = 1024;  // ChunkRec::flags only: Pend holds the chain's final Σ[U, U]
                                  // (fp32 chunks with a first sighting or an association)

// One chunk of one message for one filter (uploaded by the host, read by every kernel of the pair).
struct alignas(16) MsgDesc {
  int m;             // markers in this chunk (≤ kMaxChunk)
  int flags;
  int parity;        // which Σ / x copy is "in"
  int assoc_slot;    // association: index into FilterCtl::assoc_j for ids[c] < 0
  double odom[3];    // t_odom_robot (θ, x, y) at this message
  int prev_m;        // kLook: markers of the previous chunk
  int pad1;
  int ids[kMaxChunk];        // landmark ids; < 0 ⇒ taken from FilterCtl::assoc_j[assoc_slot + c]
  double z[kMaxChunk][2];    // measured (range, bearing), computed on the host like slam.cpp:208-210
  int prev_ids[kMaxChunk];   // kLook: the previous chunk's ids (its index set U', known up front)
  int stg_m, stg_pm;            // kStageOut: markers of the filter's chunk after next / next chunk
  int pad3[2];
  int stg_ids[kMaxChunk];       // kStageOut: the chunk after next's ids (its U)
  int stg_pids[kMaxChunk];      // kStageOut: the next chunk's ids (U' of the chunk after next)
};

struct alignas(16) FilterCtl {
  double tmo[3];       // t_map_odom (θ, x, y), slam.cpp:659
  unsigned counter;    // counter_obstacles, slam.cpp:670
  unsigned status;     // EKF_FLAG_* bits
  int assoc_j[kMaxAssoc];
  int assoc_new[kMaxAssoc];
};

// What the chain kernel (the sequential part of a chunk) hands to the factor kernel: with
// r(i) = Σ_pred[i][U] and c(j) = Σ_pred[U][j], K_c[i] = r(i)·Z[:, 2c..2c+1] and
// M_c[:, j] = Y[2c..2c+1, :]·c(j); x_i += r(i)·Zx for rows outside U, xU for rows in U.
// A Joseph chunk (kJoseph, m ≤ kMaxJoseph) adds V_c[i] = (Σ_c·Hᵀ − K_c·S_c)[i] = r(i)·Z[:, 32+2c..]
// (the row factor of the V_c·K_cᵀ term; its column factor is K_c itself).
struct alignas(16) ChunkRec {
  int m, nu, flags, pad;
  int u[kMaxU + 1];
  double a1, a2, s00;                // predict: At(1,0) = a1, At(2,0) = a2; Σ_in[0][0]
  double alphaU[kMaxU];
  double row0raw[kMaxU];             // Σ_in[0][u_b]
  double col0raw[kMaxU];             // Σ_in[u_a][0]
  double Zx[kMaxU];
  double xU[kMaxU];
  double Z[kMaxU][kZJ];   // columns 0..2m−1: Z; Joseph also 2m..4m−1: Zv (the rest zero)
  double Y[kZC][kMaxU];
  double Pend[kMaxU][kMaxU];         // the chain's final Σ[U, U] (fp64): written over the Σ pass's
                                     // block so fp32 Σ keeps first sightings (1e7 − (1e7 − δ))
};
// the chain stores Z, Y and Pend in 16-byte pairs
static_assert(offsetof(ChunkRec, Z) % 16 == 0 && offsetof(ChunkRec, Y) % 16 == 0 &&
                  offsetof(ChunkRec, Pend) % 16 == 0 && sizeof(ChunkRec) % 16 == 0,
              "ChunkRec payload 16-byte aligned");

// The rebuild operands of a kLook chain (k_chain's prologue), gathered off the chain's path by the
// k_patch_stage of the chunk two back, right behind the Σ pass that wrote them: with U this chunk's
// index set and U' the previous chunk's, Σ = Σ_in' (the previous chunk's Σ_in), x = x_in',
//   v[0][e] = Σ[u_a][u_b], v[1][e] = Σ[u_a][u'_b], v[2][e] = Σ[u'_b][u_a]   (a, b clamped to kMaxU−1)
//   r0u[t] = Σ[0][u_t], c0u[t] = Σ[u_t][0], r0p[t] = Σ[0][u'_t], c0p[t] = Σ[u'_t][0], xg[t] = x[u_t]
// — the very values the chain would gather (the fp32 block patch included), stored contiguously.
// [2][F] by the chain's Σ parity.
template <typename T>
struct alignas(16) StageRec {
  double r0u[kStW], c0u[kStW], r0p[kStW], c0p[kStW], xg[kStW];
  T v[3][kStW * kStW];
};

// ---- unknown association of a whole chunk in one launch (k_assoc_msg, ekf_assoc.hip) ----
constexpr int kAmSlots = 64;  // landmark slots per workgroup: one wave, one slot per lane
// One slot's factors of one correction c: K_c at its rows {kx, ky} (k[2a + e] = K_c[a][e]) and
// M_c at its columns (m[2e + b] = M_c[e][b]); written by the slot's lane, read by every workgroup
// of the filter whenever the slot is a later marker's landmark. Joseph form: also
// V_c = Σ_c·Hᵀ − K_c·S_c at its rows (v[2a + e] = V_c[a][e]).
struct alignas(16) AmHist {
  double k[4], m[4], v[4];
};
// One slot's 16 entries of Σ over {θ, x, y, kx, ky} (kk = Σ[k][k], kp = Σ[k][pose],
// pk = Σ[pose][k]) and its state, as correction c starts.
struct alignas(16) AmCur {
  double kk[4], kp[6], pk[6], x[2], pad[2];
};
static_assert(sizeof(AmHist) == 96 && sizeof(AmCur) == 160, "AmHist / AmCur 16-byte rows");

}  // namespace ekfslam
